#!/bin/bash
# Round 6: async waves (clean start, collect plan, host roots / host ids, pull_pushed), host mirror
# WhenInvalidated / OnAccess; the GPU suite and a short bench line (pipelined leg)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14c; mkdir -p $out
T="timeout -k 10"
cd $R
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
$T 300 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python -c "
import json; d = json.load(open('$out/bench.json'))
print('ms/step', d['ms_per_step'], 'pipe', d.get('pipelined_ms_per_step'), 'frac', d['roofline']['frac'])"
