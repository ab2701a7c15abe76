#!/bin/bash
# The prune as two plain launches, each phase on its own kernel's resident block count: prune GPU
# tests, configs[3] alternating with HEAD's library (libfgi_base: one cooperative launch), then a
# kernel trace of configs[3] for each library.
set -u
out=gpurun_out/r6x
mkdir -p "$out"
L=$PWD/stl.fusion_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2 3; do
  for lib in libfgi_base libfgi; do
    FGI_LIBRARY=$L/$lib.so timeout -k 10 300 python -u bench_configs.py --only stream,churn --no-cpu > "$out/cfg_${lib}_$r.jsonl" 2> "$out/cfg_${lib}_$r.err" \
      || { echo "configs $lib rc=$?"; tail -20 "$out/cfg_${lib}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/cfg_${lib}_$r.jsonl'):
    if not l.startswith('{'): continue
    d = json.loads(l)
    if d['config'] == 'stream':
        print('$lib', $r, 'stream ms/round', round(d['ms_per_round'], 4), 'Mnodes/s', round(d['value'] / 1e6, 1))
    else:
        p = d['prune']; print('$lib', $r, 'prune ms', round(p['s'] * 1e3, 3), 'kernel ms', round(p['kernel_ms'], 3), 'new', p['new_edges'], 'wave after ms', round(d['wave_after_prune']['ms_per_step'], 4))"
  done
done
for lib in libfgi_base libfgi; do
  FGI_LIBRARY=$L/$lib.so bash profiles/trace_configs.sh r6x_$lib --only churn --no-cpu || { echo "trace $lib failed"; exit 1; }
  python profiles/kernel_table.py gpurun_out/trace_r6x_$lib/trace/run_kernel_trace.csv 0 > "$out/churn_kernels_$lib.txt" 2>&1
  echo "== $lib"; grep -E "prune|build_cur|span" "$out/churn_kernels_$lib.txt"
done
