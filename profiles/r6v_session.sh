#!/bin/bash
# Cooperative waves launched as plain kernels with a software grid barrier (soft_grid_sync) instead of
# hipLaunchCooperativeKernel: the GPU tests, the streaming mix alternating with FGI_COOP_LAUNCH=1 (the
# cooperative launch), then a kernel trace of the plain-launch build (dispatch gaps).
set -u
out=gpurun_out/r6v
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2 3; do
  for mode in coop soft; do
    if [ $mode = coop ]; then export FGI_COOP_LAUNCH=1; else unset FGI_COOP_LAUNCH; fi
    timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream_${mode}_$r.jsonl" 2> "$out/stream_${mode}_$r.err" \
      || { echo "stream $mode rc=$?"; tail -20 "$out/stream_${mode}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/stream_${mode}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('$mode', $r, 'ms/round', round(d['ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4), 'wave kernel ms/round', round(d['wave_kernel_ms_per_round'], 4), 'Mnodes/s', round(d['value'] / 1e6, 1))"
  done
done
unset FGI_COOP_LAUNCH
bash profiles/trace_stream.sh r6v 20 && python profiles/kernel_table.py gpurun_out/trace_r6v/trace/run_kernel_trace.csv > "$out/stream_kernels.txt" 2>&1; tail -25 "$out/stream_kernels.txt"
