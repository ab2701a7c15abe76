#!/bin/bash
# Round 5 (HEAD with 4,096 LDS hot words): the driver's own bench line (N = 1, CPU legs included), and smoke().
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13b; mkdir -p $out
cd $R
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $out/smoke.log; exit 1; }
tail -3 $out/smoke.log
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
cut -c1-3000 $out/bench.json
