#!/bin/bash
# Bench variants on the GPU box (measurement knobs, one line each): parity tests first, then
# bench.py under each environment setting. Usage: profiles/variants.sh <tag> ["ENV=.. ENV2=.." ...]
TAG=${1:-exp}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
i=0
for v in "$@"; do
  i=$((i+1))
  timeout -k 10 200 env $v python bench.py --no-cpu --steps 20 --warmup 3 > "$O/v$i.json" 2> "$O/v$i.err" || { echo "variant $v failed"; exit 30; }
  python3 -c "import json,sys; d=json.load(open('$O/v$i.json')); r=d['roofline']; print('$v', 'ms/step %.4f wave %.4f value %.3e push %.4f pull %.4f frac %.3f' % (d['ms_per_step'], d['wave_kernel_ms'], d['value'], r['push_levels']['ms_per_step'], r['pull_levels']['ms_per_step'], r['frac']))"
done
