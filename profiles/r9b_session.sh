#!/bin/bash
# round 4: the spin wait and wall-clock span extended to the partitioned paths (all-reduce results
# published to host memory; no event pair unless per-level timing). GPU suite, then A/B against the
# stream-synchronised build: bench --partition at N = 1, then the headline
set -u
L=stl.fusion_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r9b_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r9b_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r5_ab.sh r9b_part 3 --args --partition -- $L/libfgi.so $L/libfgi_nospin.so || exit 1
bash profiles/r5_ab.sh r9b_head 2 $L/libfgi.so $L/libfgi_nospin.so || exit 1
