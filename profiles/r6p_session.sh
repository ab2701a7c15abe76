#!/bin/bash
# (a) AddUsed kernels: one candidate reservation per block (was one per wave on a single counter) and one
# row-slot reservation per run of equal used nodes in a wave (was one atomic per pair on the used
# node's row length: a hub's thousand dependants serialised); (b) the cooperative wave folds its visits
# grid-wide, one lane per handle (was per block, bit by bit). GPU tests, then the streaming mix
# (configs[4], 100 k AddUsed per round) against HEAD (libfgi_base), alternating.
set -u
out=gpurun_out/r6p
mkdir -p "$out"
L=$PWD/stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
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
