#!/bin/bash
# round 4: batch kernels folded (begin_compute's check into the classify launch's last block, add_used's
# size and pool check into the reserve launch's last block) — streaming tests (fault injection, full-size
# configs[4]), then configs[4] A/B against the previous build (libfgi_prev.so), alternating
set -u
out=gpurun_out/r8o
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_stream.py \
    tests/test_gpu_full_size.py::test_configs4_full_size_batches_match_oracle tests/test_gpu_parity.py tests/test_gpu_scenarios.py > $out/tests.log 2>&1 \
    || { echo "tests rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
L=$PWD/stl.fusion_amd/lib
for r in 1 2 3; do
  for lib in libfgi_prev libfgi; do
    FGI_LIBRARY=$L/$lib.so timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu > $out/${lib}_$r.jsonl 2> $out/${lib}_$r.err \
        || { echo "bench rc=$?"; tail -5 $out/${lib}_$r.err; exit 1; }
    python -c "
import json
for l in open('$out/${lib}_$r.jsonl'):
    l = l.strip()
    if l.startswith('{'):
        d = json.loads(l); print('$lib', $r, round(d['ms_per_round'], 4), 'ms/round', round(d['value'] / 1e6, 1), 'M/s', round(d['batch_kernel_ms_per_round'], 4), 'batch kernel ms')"
  done
done
