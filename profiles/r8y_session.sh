#!/bin/bash
# Round-4 HEAD (final) on a fresh box, part 2: the rocprofv3 kernel trace + PMC passes of bench.py
# (profiles/run_profile.sh -> summarize.py) and bench_configs.py's secondary configurations.
set -u
out=gpurun_out/r8y
mkdir -p "$out"
bash profiles/run_profile.sh r8y --steps 20 --warmup 3 --no-cpu --no-e2e || { echo "profile rc=$?"; exit 1; }
python profiles/summarize.py gpurun_out/prof_r8y r8y --steps 20 > "$out/summarize.log" 2>&1 || { echo "summarize rc=$?"; tail -5 "$out/summarize.log"; }
[ "${CONFIGS:-0}" = 1 ] || exit 0
timeout -k 10 900 python -u bench_configs.py > "$out/configs.jsonl" 2> "$out/configs.err" || { echo "configs rc=$?"; tail -20 "$out/configs.err"; exit 1; }
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
