#!/bin/bash
# Round 5: A/B on one box — configs[1] with the default (separate publish kernel, predicted collect grids,
# test-before-atomic visits) against FGI_LIST_PUBLISH=1 (the list kernel publishes), 3 rounds; then the
# per-level PMC passes of configs[2]'s wave with labels (level-1 FETCH).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12d; mkdir -p $out
T="timeout -k 10"
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), 'frac', round(r['frac'], 4), flush=True)"
}
for r in 1 2 3; do
  bench c1_$r rmat24 "-"
  bench c1_lp_$r rmat24 "FGI_LIST_PUBLISH=1"
done
bench c2_1 rmat27 "-"
bash profiles/pmc_levels.sh r12d rmat27 > $out/pmc_levels.log 2>&1 || { echo "pmc levels rc=$?"; tail -5 $out/pmc_levels.log; exit 1; }
python3 profiles/pmc_levels.py gpurun_out/pmcl_r12d > $out/pmc_levels.txt 2>&1 || true
head -40 $out/pmc_levels.txt
