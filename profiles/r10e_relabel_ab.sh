#!/bin/bash
# Round 5: labels ordered by (weight class, slot): 4 / 1 / 8 classes per octave (FGI_EXP_RELABEL_ORDER=3 / 4 / 5)
set -u
out=gpurun_out/r10e; mkdir -p $out
run() {  # cfg round idx setting
  local cfg=$1 r=$2 i=$3 setting=$4
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --config $cfg \
    > "$out/${cfg}_s${i}_$r.json" 2> "$out/${cfg}_s${i}_$r.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "$setting rc=$rc"; tail -5 "$out/${cfg}_s${i}_$r.err"; exit $rc; fi
  python -c "
import json; d = json.load(open('$out/${cfg}_s${i}_$r.json')); r = d['roofline']
print('$cfg', '$setting', $r, round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'lv', d['levels_per_step'], 'c2', round(d.get('configs2_single_gpu', {}).get('ms_per_step', 0), 4), flush=True)"
}
for r in 1 2; do
  i=0
  for setting in "-" "FGI_EXP_RELABEL=-1 FGI_EXP_RELABEL_W=1" "FGI_EXP_RELABEL=-1 FGI_EXP_RELABEL_ORDER=3 FGI_EXP_RELABEL_W=1" "FGI_EXP_RELABEL=-1 FGI_EXP_RELABEL_ORDER=4 FGI_EXP_RELABEL_W=1" "FGI_EXP_RELABEL=-1 FGI_EXP_RELABEL_ORDER=5 FGI_EXP_RELABEL_W=1" "FGI_EXP_RELABEL=-1 FGI_EXP_RELABEL_ORDER=3"; do
    i=$((i + 1)); run rmat27 $r $i "$setting"
  done
done
