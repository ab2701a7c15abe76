#!/bin/bash
# Small-pull-level trims on HEAD f6a6fd3's kernels (the r6b head-bitmap variants were all slower and are
# reverted): libfgi = only changed visit words written back + hot snapshot staged only by blocks with
# >= 1,024 candidates; libfgi_stageall = the write-back trim alone; libfgi_alldirty = neither (f6a6fd3's
# behaviour in this build). GPU tests on libfgi, then an A/B on configs[1] and configs[2]'s graph.
set -u
out=gpurun_out/r6c
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6c_ab24 3 $L/libfgi_base.so $L/libfgi_alldirty.so $L/libfgi_stageall.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6c_ab27 1 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi_alldirty.so $L/libfgi_stageall.so $L/libfgi.so || exit 1
