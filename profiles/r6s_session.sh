#!/bin/bash
# Streaming mix (configs[4]): cooperative wave grid of 256 (default, one block per CU) / 512 / 1024 blocks,
# alternating (FGI_COOP_BLOCKS, measurement knob): the 100-hub wave's 391 push chunks take two rounds of 256 blocks.
set -u
out=gpurun_out/r6s
mkdir -p "$out"
for r in 1 2; do
  for b in 0 512 1024; do
    FGI_COOP_BLOCKS=$b timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream_${b}_$r.jsonl" 2> "$out/stream_${b}_$r.err" \
      || { echo "stream $b rc=$?"; tail -20 "$out/stream_${b}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/stream_${b}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('blocks', $b or 256, 'round', $r, 'ms/round', round(d['ms_per_round'], 4), 'wave kernel ms/round', round(d['wave_kernel_ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4))"
  done
done
