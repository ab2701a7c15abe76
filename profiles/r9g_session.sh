#!/bin/bash
# round 4: a planned round's counters published to fine-grained host memory ahead of the all-reduce
# (no copy command); the GPU suite and bench --partition at N = 1
set -u
mkdir -p gpurun_out/r9g
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r9g/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r9g/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --partition --no-cpu --no-e2e --steps 50 --warmup 5 > gpurun_out/r9g/bench_partition.json 2> gpurun_out/r9g/bench_partition.err || { echo "rc=$?"; tail -5 gpurun_out/r9g/bench_partition.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r9g/bench_partition.json')); print('partition N=1', round(d['ms_per_step'],4), 'ms/step', round(d['value']/1e9,2), 'G nodes/s, syncs', d['host_syncs_per_step'], 'kernel', round(d['wave_kernel_ms'],4))"
