#!/bin/bash
# Cascade grid default 128 blocks: batch / stream / scenario / host GPU tests, then 64 / 96 / 128 blocks
# alternating on the streaming mix.
set -u
out=gpurun_out/r6zm
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_scenarios.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2; do
  for b in 128 96 64; do
    FGI_COOP_BLOCKS=$b timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream_b${b}_$r.jsonl" 2> "$out/stream_b${b}_$r.err" \
      || { echo "stream rc=$?"; tail -20 "$out/stream_b${b}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/stream_b${b}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('blocks=$b', $r, 'ms/round', round(d['ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4), 'wave kernel ms/round', round(d['wave_kernel_ms_per_round'], 4), 'Mnodes/s', round(d['value'] / 1e6, 1))"
  done
done
