#!/bin/bash
# Round 5 (r13k): 4 candidates per lane with a 4,096-word tail queue and 2,048 hot words (HEAD's LDS), against HEAD.
# From r13i: candidates per lane per pull step — HEAD (4 per lane, 2,048-word tail queue, 4,096 hot words) against
# 8 per lane (4,096-word queue, 2,048 hot words: the same LDS) and 6 per lane (HEAD's LDS), configs[1] x3 and
# configs[2] x1 on one box; the parity suite on the 8-per-lane build first
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13k; mkdir -p $out
T="timeout -k 10"
cd $R
L8="FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_cpl4_4096_2048.so"
L6="FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_cpl6_2048_4096.so"
env $L8 $T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_labels.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/parity_q4096.log 2>&1 || { echo "parity rc=$?"; tail -30 $out/parity_q4096.log; exit 1; }
tail -1 $out/parity_q4096.log
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$tag', '$cfg', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'frac', round(r['frac'], 4), flush=True)"
}
for r in 1 2; do
  bench c1_head_$r rmat24 "-"
  bench c1_q4096_$r rmat24 "$L8"
  bench c2_head_$r rmat27 "-"
  bench c2_q4096_$r rmat27 "$L8"
done

