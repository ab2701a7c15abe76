#!/bin/bash
# Pull geometry in whole rounds of resident blocks (at most 36 tiles per block): R-MAT 27 runs 3 rounds
# of 3,745 blocks x 35 tiles instead of 4,096 x 32 (the last 256 ran as a fourth round); R-MAT 26 2 rounds
# of 2,521 x 26 instead of 2,048 x 32. GPU tests, then an A/B against HEAD (libfgi_base).
set -u
out=gpurun_out/r6j
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6j_ab27 2 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6j_ab26 2 --args --config rmat26 -- $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6j_ab24 2 $L/libfgi_base.so $L/libfgi.so || exit 1
