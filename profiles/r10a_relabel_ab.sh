#!/bin/bash
# Round 5: does packing heavy slots into a label prefix pay? (FGI_EXP_RELABEL, synth.hip) — configs[2] and [1]
# graphs relabelled at generation (isomorphic graphs; roots re-picked by the same rule), alternating on one box.
set -u
out=gpurun_out/r10a; mkdir -p $out
for cfg in rmat27 rmat24; do
for r in 1 2; do
  i=0
  for setting in "-" "FGI_EXP_RELABEL=-1" "FGI_EXP_RELABEL=-1 FGI_EXP_RELABEL_W=1" "FGI_EXP_RELABEL=4194304" "FGI_EXP_RELABEL=16777216"; do
    i=$((i + 1))
    envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --config $cfg \
      > "$out/${cfg}_s${i}_$r.json" 2> "$out/${cfg}_s${i}_$r.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$setting rc=$rc"; tail -5 "$out/${cfg}_s${i}_$r.err"; exit $rc; fi
    python -c "
import json; d = json.load(open('$out/${cfg}_s${i}_$r.json')); r = d['roofline']
print('$cfg', '$setting', $r, round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'lv', d['levels_per_step'], 'first', round(d['first_wave_s'],3), flush=True)"
  done
done
done
