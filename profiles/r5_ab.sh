#!/bin/bash
# A/B of engine builds on one box (alternating, same graph build each run):
#   bash profiles/r5_ab.sh <tag> <rounds> [bench args --] lib1.so lib2.so ...
# Prints one line per run: lib, round, ms/step, pull-level ms/step, push-level ms/step, wave kernel ms.
set -u
tag=$1; rounds=$2; shift 2
extra=()
if [ "${1:-}" = "--args" ]; then shift; while [ "$1" != "--" ]; do extra+=("$1"); shift; done; shift; fi
out=gpurun_out/$tag; mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    FGI_LIBRARY=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu --no-e2e --steps 50 --warmup 5 "${extra[@]}" \
      > "$out/${name}_$r.json" 2> "$out/${name}_$r.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$lib rc=$rc"; exit $rc; fi
    python -c "
import json; d = json.load(open('$out/${name}_$r.json')); r = d['roofline']
print('$name', $r, round(d['ms_per_step'], 4), round(r['pull_levels']['ms_per_step'], 4), round(r['push_levels']['ms_per_step'], 4), round(d['wave_kernel_ms'], 4), flush=True)"
  done
done
