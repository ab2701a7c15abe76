#!/bin/bash
# Round 5: hot prefix in slot order (FGI_EXP_RELABEL_ORDER=1) against weight order, configs[2]'s graph.
set -u
out=gpurun_out/r10b; mkdir -p $out
for cfg in rmat27; do
for r in 1 2; do
  i=0
  for setting in "-" "FGI_EXP_RELABEL=-1" "FGI_EXP_RELABEL=8388608 FGI_EXP_RELABEL_ORDER=1" "FGI_EXP_RELABEL=16777216 FGI_EXP_RELABEL_ORDER=1" "FGI_EXP_RELABEL=33554432 FGI_EXP_RELABEL_ORDER=1" "FGI_EXP_RELABEL=16777216 FGI_EXP_RELABEL_ORDER=1 FGI_EXP_RELABEL_W=1"; do
    i=$((i + 1))
    envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --config $cfg \
      > "$out/${cfg}_s${i}_$r.json" 2> "$out/${cfg}_s${i}_$r.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$setting rc=$rc"; tail -5 "$out/${cfg}_s${i}_$r.err"; exit $rc; fi
    python -c "
import json; d = json.load(open('$out/${cfg}_s${i}_$r.json')); r = d['roofline']
print('$cfg', '$setting', $r, round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'lv', d['levels_per_step'], 'npull', d['pull_levels_per_step'], flush=True)"
  done
done
done
