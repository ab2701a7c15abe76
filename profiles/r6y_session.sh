#!/bin/bash
# Host phases of fgi_run_batch (TAG=<name>: output under gpurun_out/<name>) in the streaming mix (FGI_BATCH_TIMES=1): staging copy into the pinned
# buffer, enqueue, wait, unpacking; medians over the timed rounds.
set -u
out=gpurun_out/${TAG:-r6y}
mkdir -p "$out"
FGI_BATCH_TIMES=1 timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream.jsonl" 2> "$out/stream.err" \
    || { echo "stream rc=$?"; tail -20 "$out/stream.err"; exit 1; }
python - <<PY
import json, re, statistics as st
rows = [l for l in open('$out/stream.err') if l.startswith('[fgi] batch')]
print(len(rows), 'batches')
keys = ['check', 'cap', 'stage', 'pack', 'enqueue', 'wait', 'unpack', 'total']
vals = {k: [] for k in keys}
for l in rows[len(rows) // 4:]:
    for k in keys:
        vals[k].append(float(re.search(k + r' ([0-9.]+)', l).group(1)))
print({k: round(st.median(v), 1) for k, v in vals.items()})
for l in open('$out/stream.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('ms/round', round(d['ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4), 'call ms/round', round(d['run_batch_call_ms_per_round'], 4))
PY
