#!/bin/bash
# Round 5: the deep-wave tail test, parity / labels / async / configs tests, then benches: configs[2]
# labels on / off, configs[1] (adaptive tail) and FGI_TAIL=0, two rounds (one box).
set -u
out=gpurun_out/r11f; mkdir -p $out
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_labels.py tests/test_gpu_async.py tests/test_gpu_configs.py tests/test_gpu_scale.py -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit 1; }
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'lv', d['levels_per_step'], 'pl', d['pull_levels_per_step'], 'syncs', d['host_syncs_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), d.get('pipelined', {}).get('same_counts_as_sync'), 'first', round(d['first_wave_s'], 3), flush=True)"
}
for r in 1 2; do
  bench c2_on_$r rmat27 "-"
  bench c2_off_$r rmat27 "FGI_LABELS=-1"
  bench c1_$r rmat24 "-"
  bench c1_notail_$r rmat24 "FGI_TAIL=0"
done
