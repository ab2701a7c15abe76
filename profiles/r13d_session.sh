#!/bin/bash
# Round 5: push levels' pool reads — streaming (nontemporal, default) vs plain loads (FGI_PUSH_NT=0):
# configs[1] bench A/B (3 rounds) and the probe variant's level-0 phases for both.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13d; mkdir -p $out
T="timeout -k 10"
cd $R
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], flush=True)"
}
for r in 1 2 3; do
  bench c1_$r rmat24 "-"
  bench c1_nt0_$r rmat24 "FGI_PUSH_NT=0"
done
bench c2_nt0 rmat27 "FGI_PUSH_NT=0"
bench c2 rmat27 "-"
for nt in 1 0; do
  FGI_PUSH_NT=$nt FGI_TRACE=1 FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_probe.so $T 200 python profiles/wave_levels.py rmat24 > $out/probe_nt$nt.log 2>&1 || { echo "probe rc=$?"; exit 1; }
  echo "nt=$nt"; grep -E "probe\] level [0-5]" $out/probe_nt$nt.log | tail -6
done
