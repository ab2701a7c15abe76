#!/bin/bash
# Round-4 HEAD after the host spin: bench_configs.py (configs[0], [2], [3], [4])
set -u
out=gpurun_out/r9c
mkdir -p "$out"
timeout -k 10 1000 python -u bench_configs.py > "$out/configs.jsonl" 2> "$out/configs.err" || { echo "configs rc=$?"; tail -20 "$out/configs.err"; exit 1; }
python -c "
import json
for l in open('$out/configs.jsonl'):
    l = l.strip()
    if not l.startswith('{'): continue
    d = json.loads(l)
    print({k: v for k, v in d.items() if not isinstance(v, (dict, list))})
    for k in ('gpu', 'prune', 'wave_before_prune'):
        if k in d: print(' ', k, d[k])
"
