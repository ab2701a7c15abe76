#!/bin/bash
# Round 5: the whole GPU suite and the suite with labels forced on every graph, after the fold rewrite;
# then the benches (configs[2] labels on / off, configs[1]).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r11l; mkdir -p $out
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -8 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests rc=$rc"; exit 1; }
FGI_LABELS=1 $T 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $out/gpu_tests_labels.log 2>&1
rc=$?; tail -8 $out/gpu_tests_labels.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "forced-label gpu tests rc=$rc"; exit 1; }
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), 'frac', round(r['frac'], 4), flush=True)"
}
for r in 1 2; do
  bench c2_on_$r rmat27 "-"
  bench c2_off_$r rmat27 "FGI_LABELS=-1"
  bench c1_$r rmat24 "-"
done
