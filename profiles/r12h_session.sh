#!/bin/bash
# Round 5: with hub-first labels, does configs[2] want a different hot-heads snapshot? Default (524,288
# heads max, one per 512 handles, 2,048 words in LDS) against 4,096 LDS words (libfgi_ldshot4096) and
# 1 M heads at one per 128 handles (libfgi_hot1048576d128). One box, two rounds.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12h; mkdir -p $out
T="timeout -k 10"
L=$R/stl.fusion_amd/lib
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 20 --warmup 3 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '${setting##*/}', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], flush=True)"
}
for r in 1 2; do
  bench c2_$r rmat27 "-"
  bench c2_lds_$r rmat27 "FGI_LIBRARY=$L/libfgi_ldshot4096.so"
  bench c2_hot_$r rmat27 "FGI_LIBRARY=$L/libfgi_hot1048576d128.so"
done
bench c1_lds rmat24 "FGI_LIBRARY=$L/libfgi_ldshot4096.so"
bench c1 rmat24 "-"
