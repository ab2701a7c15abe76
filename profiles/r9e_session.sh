#!/bin/bash
# round 4: a batch's end (fgi_run_batch) waiting on a published sequence word behind its result copies
# instead of a stream synchronisation; GPU suite, then configs[4] A/B against the synchronised build
set -u
L=stl.fusion_amd/lib
mkdir -p gpurun_out/r9e
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r9e/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r9e/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in libfgi libfgi_nospin; do
    FGI_LIBRARY=$PWD/$L/$lib.so timeout -k 10 200 python -u bench_configs.py --only stream --no-cpu > gpurun_out/r9e/${lib}_$r.jsonl 2> gpurun_out/r9e/${lib}_$r.err || { echo "$lib rc=$?"; exit 1; }
    python -c "
import json
for l in open('gpurun_out/r9e/${lib}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('$lib', $r, round(d['ms_per_round'], 4), 'ms/round; call', round(d['run_batch_call_ms_per_round'], 4), 'kernels', round(d['batch_kernel_ms_per_round'], 4))"
  done
done
