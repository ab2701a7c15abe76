#!/bin/bash
# fgi_run_batch's checks and staging copies split over 3 host threads (FGI_HOST_THREADS, default 3):
# batch / stream / host GPU tests, then the streaming mix alternating FGI_HOST_THREADS=0 and the
# default, with the host phases (FGI_BATCH_TIMES=1).
set -u
out=gpurun_out/r6zg
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_host.py tests/test_gpu_scenarios.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2 3; do
  for t in 0 3; do
    FGI_HOST_THREADS=$t TAG=r6zg/t${t}_$r bash profiles/r6y_session.sh | sed "s/^/threads=$t run $r: /" || exit 1
  done
done
