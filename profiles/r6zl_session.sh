#!/bin/bash
# Cascade grid size with the software barrier (FGI_COOP_BLOCKS measurement knob): 128 / 256 blocks,
# streaming mix alternating.
set -u
out=gpurun_out/r6zl
mkdir -p "$out"
for r in 1 2 3; do
  for b in 256 128; do
    FGI_COOP_BLOCKS=$b timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream_b${b}_$r.jsonl" 2> "$out/stream_b${b}_$r.err" \
      || { echo "stream rc=$?"; tail -20 "$out/stream_b${b}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/stream_b${b}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('blocks=$b', $r, 'ms/round', round(d['ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4), 'wave kernel ms/round', round(d['wave_kernel_ms_per_round'], 4), 'Mnodes/s', round(d['value'] / 1e6, 1))"
  done
done
