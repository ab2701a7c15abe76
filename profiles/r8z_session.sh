#!/bin/bash
# Round-4 HEAD (final) on a fresh box, part 1: the GPU suite and the bench line (with the CPU baseline).
set -u
out=gpurun_out/${1:-r8z}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 150 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 400 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench rc=$?"; tail -20 "$out/bench.err"; exit 1; }
python -c "
import json; d = json.load(open('$out/bench.json')); r = d['roofline']
print('bench', round(d['value'] / 1e9, 2), 'G nodes/s', round(d['ms_per_step'], 4), 'ms/step; k_level', round(r['avg_launch_ms'] * 1e3, 2), 'us/launch, frac', round(r['frac'], 4), '; e2e', round(d['e2e_ms_per_step'], 3), 'ms; cpu', d['cpu_baseline'].get('value'))"
