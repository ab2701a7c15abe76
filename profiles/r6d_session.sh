#!/bin/bash
# Prune fast path (entry liveness recorded at list build + a bitmap of current nodes instead of a
# node-word gather per entry): GPU tests, configs[3] with and without FGI_PRUNE_GATHER (alternating),
# then HEAD's bench line and a rocprofv3 kernel-trace summary of bench.py.
set -u
out=gpurun_out/r6d
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
for r in 1 2; do
  for mode in fast gather; do
    if [ $mode = gather ]; then export FGI_PRUNE_GATHER=1; else unset FGI_PRUNE_GATHER; fi
    timeout -k 10 300 python -u bench_configs.py --only churn --no-cpu > "$out/churn_${mode}_$r.json" 2> "$out/churn_${mode}_$r.err" \
      || { echo "churn $mode rc=$?"; tail -20 "$out/churn_${mode}_$r.err"; exit 1; }
    python -c "
import json; d = json.loads(open('$out/churn_${mode}_$r.json').read().strip().splitlines()[-1]); p = d['prune']
print('$mode', $r, 'prune kernel ms', round(p['kernel_ms'], 3), 'edges', p['old_edges'], '->', p['new_edges'], 'wave after', round(d['wave_after_prune']['ms_per_step'], 4))"
  done
done
unset FGI_PRUNE_GATHER
timeout -k 10 400 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench rc=$?"; tail -20 "$out/bench.err"; exit 1; }
python -c "
import json; d = json.load(open('$out/bench.json')); r = d['roofline']
print('bench', round(d['value'] / 1e9, 2), 'G nodes/s', round(d['ms_per_step'], 4), 'ms/step; k_level', round(r['avg_launch_ms'] * 1e3, 2), 'us/launch, frac', round(r['frac'], 4), '; e2e', round(d['e2e_ms_per_step'], 3), 'ms; cpu', d['cpu_baseline'].get('value'))"
mkdir -p "$out/prof"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --no-e2e --steps 20 --warmup 3 > "$GRAFT_REPO_ROOT/$out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$out/prof_bench.err" ) \
    || echo "rocprof rc=$? (see prof_bench.err)"
find "$out/prof" -name "*kernel_stats.csv" | head -3
