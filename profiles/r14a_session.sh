#!/bin/bash
# Round 6: GPU suite (new async/tail failure tests included), smoke, a short bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14a; mkdir -p $out
T="timeout -k 10"
cd $R
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
$T 400 python bench.py --no-cpu --no-e2e > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python -c "
import json; d = json.load(open('$out/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'c2', d.get('configs2_single_gpu', {}).get('ms_per_step'), 'pipe', d.get('pipelined_ms_per_step'))"
