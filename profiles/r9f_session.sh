#!/bin/bash
# round 4's last HEAD: smoke + the default bench line (CPU baseline and e2e included)
set -u
mkdir -p gpurun_out/r9f
timeout -k 10 200 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > gpurun_out/r9f/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r9f/smoke.log; exit 1; }
tail -1 gpurun_out/r9f/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r9f/bench.json 2> gpurun_out/r9f/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r9f/bench.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/r9f/bench.json')); r = d['roofline']
print('bench', round(d['value'] / 1e9, 2), 'G nodes/s', round(d['ms_per_step'], 4), 'ms/step; k_level', round(r['avg_launch_ms'] * 1e3, 2), 'us/launch, frac', round(r['frac'], 4), '; e2e', round(d['e2e_ms_per_step'], 3), 'ms; cpu', round(d['cpu_baseline'].get('value')))"
