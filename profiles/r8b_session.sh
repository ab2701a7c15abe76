#!/bin/bash
# round 4: partitioned mutation tests, then the hot-heads count A/B at configs[2]'s size
# (262,144 heads = one per 512 handles, the default; 524,288; 1,048,576) on one box.
set -u
out=gpurun_out/r8b
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_part_mutations.py tests/test_gpu_part_rccl.py > $out/mut.log 2>&1 \
    || { echo "mut rc=$?"; tail -30 $out/mut.log; exit 1; }
tail -2 $out/mut.log
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r8b_ab27 2 --args --config rmat27 -- $L/libfgi.so $L/libfgi_hot524288d256.so $L/libfgi_hot1048576d128.so || exit 1
