#!/bin/bash
# (r6z2: validation fused into the staging copy, one pass over the caller arrays)
# Batch argument checks as vectorisable reductions + a byte-per-slot duplicate test: batch / stream
# GPU tests, then the host phases of fgi_run_batch in the streaming mix (FGI_BATCH_TIMES=1).
set -u
out=gpurun_out/r6z2
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
TAG=r6z2 bash profiles/r6y_session.sh
