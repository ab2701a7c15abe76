#!/bin/bash
# Cascades (k_wave_coop) size their push chunks so that a level is one round of chunks over the grid
# (level_mult_one_round): batch / stream / scenario GPU tests, then the streaming mix alternating
# FGI_COOP_CHUNKS=0 (the plain waves' level_mult) and the default.
set -u
out=gpurun_out/r6zj
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_scenarios.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2 3; do
  for c in 0 1; do
    FGI_COOP_CHUNKS=$c timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream_c${c}_$r.jsonl" 2> "$out/stream_c${c}_$r.err" \
      || { echo "stream rc=$?"; tail -20 "$out/stream_c${c}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/stream_c${c}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('one_round=$c', $r, 'ms/round', round(d['ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4), 'wave kernel ms/round', round(d['wave_kernel_ms_per_round'], 4), 'Mnodes/s', round(d['value'] / 1e6, 1))"
  done
done
