#!/bin/bash
# round 4: partition tests, then bench.py --partition at N=1 (planned waves; the frontier bitmap
# aliased to the invalidated bitmap at one rank without collectives), three runs
set -u
out=gpurun_out/r8e
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_part.py tests/test_gpu_part_plan.py \
    tests/test_gpu_part_rccl.py tests/test_gpu_part_load.py tests/test_gpu_part_mutations.py tests/test_gpu_probe_summary.py > $out/tests.log 2>&1 \
    || { echo "tests rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --partition --no-cpu --no-e2e --steps 50 --warmup 5 > $out/part_$r.json 2> $out/part_$r.err || { echo "bench rc=$?"; tail -5 $out/part_$r.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/part_$r.json'))
print('partition N=1', $r, round(d['ms_per_step'], 4), 'ms/step', d.get('host_syncs_per_step'), 'syncs/step', round(d['value']/1e9, 2), 'G nodes/s')"
done
