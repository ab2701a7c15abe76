#!/bin/bash
# Round 5: test-before-atomic visits, the list kernel publishing the counters, predicted collect grids:
# the whole GPU suite, then configs[1] / configs[2] benches (3 rounds) and a kernel trace of configs[1].
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12c; mkdir -p $out
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -6 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests rc=$rc"; exit 1; }
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
done
bench c2_1 rmat27 "-"
cd /tmp && export TMPDIR=/tmp
$T 200 rocprofv3 --kernel-trace --stats -T -d $out/trace_c1 -o run --output-format csv -- python3 $R/bench.py --config rmat24 --no-secondary --no-cpu --no-e2e --steps 10 --warmup 2 > $out/trace_c1.json 2> $out/trace_c1.err || { echo "trace rc=$?"; exit 1; }
grep -E "k_" $out/trace_c1/run_kernel_stats.csv | cut -c1-110
