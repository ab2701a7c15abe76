#!/bin/bash
# Round 6: bench --partition at N = 1 (the partitioned engine on one device) with partition codes forced vs host
# numbering, configs[1] and [2] (the run also held a debug step, profiles/r14_replica_debug.txt)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14l; mkdir -p $out
cd $R
for cfg in rmat24 rmat27; do
  for lab in 1 -1; do
    FGI_LABELS=$lab timeout -k 10 300 python bench.py --partition --config $cfg --steps 20 --warmup 3 --no-cpu --no-e2e --no-secondary > $out/part_${cfg}_$lab.json 2> $out/part_${cfg}_$lab.err || { echo "bench rc=$?"; tail -5 $out/part_${cfg}_$lab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$out/part_${cfg}_$lab.json')); print('$cfg labels=$lab', round(d['ms_per_step'],4), d['v_inv_per_step'], d['roofline'].get('pull_levels'), d['roofline'].get('push_levels'))"
  done
done
