#!/bin/bash
# No cooperative launches left: streaming cascades as plain launches with soft_grid_sync, the prune as
# two plain launches (k_prune_rows, k_prune_chunks). GPU tests; configs[3] (prune) and configs[4]
# (streaming) alternating with HEAD's library (libfgi_base: cooperative launches); then the headline
# profile under rocprofv3 (does the exit-time fault still happen without a cooperative queue?).
set -u
out=gpurun_out/r6w
mkdir -p "$out"
L=$PWD/stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2; do
  for lib in libfgi_base libfgi; do
    FGI_LIBRARY=$L/$lib.so timeout -k 10 300 python -u bench_configs.py --only churn,stream --no-cpu > "$out/cfg_${lib}_$r.jsonl" 2> "$out/cfg_${lib}_$r.err" \
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
bash profiles/trace_stream.sh r6w 20; echo "trace_stream rc=$?"; tail -3 gpurun_out/trace_r6w/stream.err
[ -s gpurun_out/trace_r6w/trace/run_kernel_trace.csv ] && python profiles/kernel_table.py gpurun_out/trace_r6w/trace/run_kernel_trace.csv > "$out/stream_kernels.txt" 2>&1; head -4 "$out/stream_kernels.txt"
