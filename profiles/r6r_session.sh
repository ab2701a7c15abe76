#!/bin/bash
# Cooperative waves fold the statistics rows of their own grid only (one load per thread instead of a
# 16-deep chain over 4,096 rows, ~25 us on block 0 per cascade in r6q's phase stamps). Streaming GPU
# tests, the streaming mix against HEAD (libfgi_base) alternating, then the phase stamps again.
set -u
out=gpurun_out/r6r
mkdir -p "$out"
L=$PWD/stl.fusion_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_batch.py tests/test_gpu_scenarios.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2 3; do
  for lib in libfgi_base libfgi; do
    FGI_LIBRARY=$L/$lib.so timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > "$out/stream_${lib}_$r.jsonl" 2> "$out/stream_${lib}_$r.err" \
      || { echo "stream $lib rc=$?"; tail -20 "$out/stream_${lib}_$r.err"; exit 1; }
    python -c "
import json
for l in open('$out/stream_${lib}_$r.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('$lib', $r, 'ms/round', round(d['ms_per_round'], 4), 'batch kernel ms/round', round(d['batch_kernel_ms_per_round'], 4), 'wave kernel ms/round', round(d['wave_kernel_ms_per_round'], 4))"
  done
done
FGI_LIBRARY=$L/libfgi_probe.so FGI_TRACE=1 timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu --rounds 12 \
    > "$out/probe.jsonl" 2> "$out/probe.err" || { echo "probe rc=$?"; exit 1; }
grep "\[coop\]" "$out/probe.err" | grep "1:" | tail -6
