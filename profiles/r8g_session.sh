#!/bin/bash
# round 4: single-pass final collect (FGI_FINAL_ONE=1) — GPU tests with it, then an alternating bench A/B
set -u
out=gpurun_out/r8g
mkdir -p $out
FGI_FINAL_ONE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_part.py tests/test_gpu_host.py > $out/tests.log 2>&1 \
    || { echo "tests rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  for one in 0 1; do
    FGI_FINAL_ONE=$one timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 100 --warmup 5 > $out/b${one}_$r.json 2> $out/b${one}_$r.err || { echo "bench rc=$?"; tail -5 $out/b${one}_$r.err; exit 1; }
    python -c "
import json; d = json.load(open('$out/b${one}_$r.json'))
print('final_one', $one, $r, round(d['ms_per_step'], 4), 'ms/step', round(d['wave_kernel_ms'], 4), 'wave kernel ms')"
  done
done
