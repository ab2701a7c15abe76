#!/bin/bash
# (a) Tail queue entries carry the candidate's slot (index | slot - block's first slot << 16), so a tail
# pass requests the entry and its dependency list together (one round trip fewer per pass); (b) a pull block's
# segment bounds and survivor counts are requested at k_level's entry with the level counters. GPU tests,
# then an A/B against HEAD (libfgi_base) on configs[0], configs[1] and configs[2]'s graph.
set -u
out=gpurun_out/r6h
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6h_ab0 3 --args --config layered_1m -- $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6h_ab24 3 $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6h_ab27 2 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi.so || exit 1
