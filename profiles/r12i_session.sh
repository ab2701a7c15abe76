#!/bin/bash
# Round 5: the hot snapshot's LDS share per pull block (FGI_LDS_HOT words: 2,048 default, 4,096, 8,192)
# on configs[1] and configs[2], alternating, two rounds, one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12i; mkdir -p $out
T="timeout -k 10"
L=$R/stl.fusion_amd/lib
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '${setting##*/}', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), flush=True)"
}
for r in 1 2; do
  bench c1_$r rmat24 "-"
  bench c1_4k_$r rmat24 "FGI_LIBRARY=$L/libfgi_ldshot4096.so"
  bench c1_8k_$r rmat24 "FGI_LIBRARY=$L/libfgi_ldshot8192.so"
  bench c2_$r rmat27 "-"
  bench c2_4k_$r rmat27 "FGI_LIBRARY=$L/libfgi_ldshot4096.so"
  bench c2_8k_$r rmat27 "FGI_LIBRARY=$L/libfgi_ldshot8192.so"
done
