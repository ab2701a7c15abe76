#!/bin/bash
# Round 5: Beamer's beta (stay in pull while F > n / beta): configs[2]'s level 3 frontier (5.80 M) sits 4% above
# n / 24 = 5.59 M, and a build whose level-2 pull found slightly more (r13q) pushed level 3 at +0.25 ms. A/B of
# beta 24 (HEAD) / 32 / 48 on configs[1] and configs[2], and the 4,096-word tail queue build with beta 32 / 48.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13r; mkdir -p $out
T="timeout -k 10"
cd $R
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$tag', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], flush=True)"
}
Q="FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_cpl4_4096_2048.so"
for r in 1 2; do
  bench c1_b24_$r rmat24 "-"
  bench c1_b32_$r rmat24 "FGI_PULL_BETA=32"
  bench c1_b48_$r rmat24 "FGI_PULL_BETA=48"
  bench c2_b24_$r rmat27 "-"
  bench c2_b32_$r rmat27 "FGI_PULL_BETA=32"
  bench c2_b48_$r rmat27 "FGI_PULL_BETA=48"
  bench c2_q_b32_$r rmat27 "$Q FGI_PULL_BETA=32"
  bench c1_q_b32_$r rmat24 "$Q FGI_PULL_BETA=32"
done
