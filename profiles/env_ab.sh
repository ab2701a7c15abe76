#!/bin/bash
# A/B of engine settings on one box (alternating, same build): bash profiles/env_ab.sh <tag> <rounds> [bench args --] "VAR=v ..." ...
# ("-" = no extra setting). One line per run: setting, round, ms/step, pull ms/step, push ms/step, wave kernel ms.
set -u
tag=$1; rounds=$2; shift 2
extra=()
if [ "${1:-}" = "--args" ]; then shift; while [ "$1" != "--" ]; do extra+=("$1"); shift; done; shift; fi
out=gpurun_out/$tag; mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu --no-e2e --steps 50 --warmup 5 "${extra[@]}" \
      > "$out/s${i}_$r.json" 2> "$out/s${i}_$r.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$setting rc=$rc"; exit $rc; fi
    python -c "
import json; d = json.load(open('$out/s${i}_$r.json')); r = d['roofline']
print('$setting', $r, round(d['ms_per_step'], 4), round(r['pull_levels']['ms_per_step'], 4), round(r['push_levels']['ms_per_step'], 4), round(d['wave_kernel_ms'], 4), flush=True)"
  done
done
