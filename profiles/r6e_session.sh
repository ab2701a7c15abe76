#!/bin/bash
# Tail scans: lists of at most 12 entries that go past entry 3 scanned by one lane each (all entries in
# flight) instead of 8 lanes per candidate. GPU tests on this build, then an A/B against HEAD 981c874's
# build (libfgi_base) on configs[0] (layered, 8-entry lists), configs[1] and configs[2]'s graph.
set -u
out=gpurun_out/r6e
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6e_ab0 3 --args --config layered_1m -- $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6e_ab24 3 $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6e_ab27 1 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi.so || exit 1
