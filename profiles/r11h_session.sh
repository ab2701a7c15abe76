#!/bin/bash
# Round 5: fold table tile-major (k_final_count at configs[2]): labels / configs tests, a kernel trace of
# the configs[2] bench, then configs[2] labels on / off and configs[1] benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r11h; mkdir -p $out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_labels.py tests/test_gpu_configs.py "tests/test_gpu_parity.py::test_deep_waves_through_the_tail" -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit 1; }
(cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats -T -d $out/trace_c2 -o run --output-format csv -- python3 $R/bench.py --config rmat27 --no-secondary --no-cpu --no-e2e --steps 10 --warmup 2 > $out/trace_c2_bench.json 2> $out/trace_c2_bench.err) || { echo "trace rc=$?"; exit 1; }
grep -E "k_final|k_level|k_collect|k_wave_init|k_roots|k_publish" $out/trace_c2/*/run_kernel_stats.csv $out/trace_c2/run_kernel_stats.csv 2>/dev/null | cut -c1-200
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'lv', d['levels_per_step'], 'pl', d['pull_levels_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), 'frac', round(r['frac'], 4), 'traffic', r['traffic'], flush=True)"
}
for r in 1 2; do
  bench c2_on_$r rmat27 "-"
  bench c2_off_$r rmat27 "FGI_LABELS=-1"
  bench c1_$r rmat24 "-"
done
# per-level trace of configs[1] and configs[2] (FGI_TRACE: direction, frontier, edges, k_level ms per level)
cd $R && FGI_TRACE=1 $T 120 python bench.py --no-cpu --no-e2e --no-secondary --steps 2 --warmup 1 --config rmat24 > $out/trace_levels_c1.json 2> $out/trace_levels_c1.err || { echo "trace c1 rc=$?"; exit 1; }
grep -E "^\[fgi\] (level|wave|tail)" $out/trace_levels_c1.err | tail -16
