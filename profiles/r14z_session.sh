#!/bin/bash
# Round 6 close: the whole GPU suite, smoke(), the default bench line (N = 1)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14zz; mkdir -p $out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('traffic_source'), d.get('pipelined_ms_per_step'), d.get('configs2_single_gpu',{}).get('ms_per_step'))"
