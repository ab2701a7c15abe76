#!/bin/bash
# Round-4 HEAD (final) on a fresh box: GPU tests, the bench line (with the CPU baseline), the rocprofv3 kernel
# trace + PMC passes of bench.py (profiles/run_profile.sh -> summarize.py), and bench_configs.py's
# secondary configurations (configs[0], [3], [4]).
set -u
out=gpurun_out/r8z
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 400 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench rc=$?"; tail -20 "$out/bench.err"; exit 1; }
python -c "
import json; d = json.load(open('$out/bench.json')); r = d['roofline']
print('bench', round(d['value'] / 1e9, 2), 'G nodes/s', round(d['ms_per_step'], 4), 'ms/step; k_level', round(r['avg_launch_ms'] * 1e3, 2), 'us/launch, frac', round(r['frac'], 4), '; e2e', round(d['e2e_ms_per_step'], 3), 'ms; cpu', d['cpu_baseline'].get('value'))"
bash profiles/run_profile.sh r8z --steps 20 --warmup 3 --no-cpu --no-e2e || { echo "profile rc=$?"; exit 1; }
python profiles/summarize.py gpurun_out/prof_r8z r8z --steps 20 > "$out/summarize.log" 2>&1 || { echo "summarize rc=$?"; tail -5 "$out/summarize.log"; }
timeout -k 10 600 python -u bench_configs.py > "$out/configs.jsonl" 2> "$out/configs.err" || { echo "configs rc=$?"; tail -20 "$out/configs.err"; exit 1; }
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
