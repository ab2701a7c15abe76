#!/bin/bash
# round 4: partitioned mutation tests (LocalComm and RCCL world 1), the probe-summary tests, then at
# configs[2]'s size: the probe summary on / off, and the hot-heads count A/B (262,144 heads = one per
# 512 handles, the default; 1,048,576; 2,097,152) on one box.
set -u
out=gpurun_out/r8b
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_part_mutations.py \
    tests/test_gpu_part_rccl.py tests/test_gpu_probe_summary.py > $out/tests.log 2>&1 \
    || { echo "tests rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
L=stl.fusion_amd/lib
for r in 1 2; do
  for sm in -1 524288; do
    FGI_PROBE_SUMMARY=$sm timeout -k 10 240 python bench.py --config rmat27 --no-cpu --no-e2e --steps 30 --warmup 3 \
        > $out/sum${sm}_$r.json 2> $out/sum${sm}_$r.err || { echo "bench rc=$?"; tail -5 $out/sum${sm}_$r.err; exit 1; }
    python -c "
import json; d = json.load(open('$out/sum${sm}_$r.json')); r = d['roofline']
print('summary', '$sm', $r, round(d['ms_per_step'], 4), round(r['pull_levels']['ms_per_step'], 4), round(r['push_levels']['ms_per_step'], 4), round(d['wave_kernel_ms'], 4), flush=True)"
  done
done
bash profiles/r5_ab.sh r8b_ab27 1 --args --config rmat27 -- $L/libfgi.so $L/libfgi_hot1048576d128.so $L/libfgi_hot2097152d64.so || exit 1
