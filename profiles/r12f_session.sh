#!/bin/bash
# Round 5: the tail's totals summed in registers and its group levels read in parallel; small push levels
# without the dead-filter trip and with speculative row gathers (A/B: FGI_PUSH_SMALL=0). Tests that run the
# tail (deep waves, async, labels, batches), then configs[1] / configs[2] benches (sync and pipelined).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12f; mkdir -p $out
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_labels.py tests/test_gpu_batch.py tests/test_gpu_configs.py -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit 1; }
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), d.get('pipelined', {}).get('same_counts_as_sync'), 'frac', round(r['frac'], 4), flush=True)"
}
for r in 1 2 3; do
  bench c1_$r rmat24 "-"
  bench c1_ps0_$r rmat24 "FGI_PUSH_SMALL=0"
done
bench c2_1 rmat27 "-"
