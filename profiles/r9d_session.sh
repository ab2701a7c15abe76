#!/bin/bash
# round 4 HEAD after the host spin: configs[2]'s whole R-MAT 27 graph on one GPU (single engine)
set -u
mkdir -p gpurun_out/r9d
timeout -k 10 500 python -u bench.py --config rmat27 --no-cpu --no-e2e --steps 20 --warmup 3 > gpurun_out/r9d/bench_rmat27.json 2> gpurun_out/r9d/bench_rmat27.err || { echo "rc=$?"; tail -5 gpurun_out/r9d/bench_rmat27.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r9d/bench_rmat27.json')); r=d['roofline']
print(round(d['value']/1e9,2), 'G nodes/s', round(d['ms_per_step'],4), 'ms/step; pull', round(r['pull_levels']['ms_per_step'],4), 'push', round(r['push_levels']['ms_per_step'],4))"
