#!/bin/bash
# Round 5: the wave tail's shape on configs[1] (one box): default (no tail: the level after the last
# pull stays in the group), the tail running the post-pull level too (FGI_TAIL_HEAD=1) at 32 / 128 / 256
# blocks. Then the deep-wave test with a 256-block tail.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12g; mkdir -p $out
T="timeout -k 10"
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$cfg', '$setting', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'pipe', round(d.get('pipelined_ms_per_step', 0), 4), d.get('pipelined', {}).get('same_counts_as_sync'), 'syncs', d['host_syncs_per_step'], flush=True)"
}
for r in 1 2; do
  bench c1_$r rmat24 "-"
  bench c1_h1_32_$r rmat24 "FGI_TAIL_HEAD=1"
  bench c1_h1_128_$r rmat24 "FGI_TAIL_HEAD=1 FGI_TAIL_BLOCKS=128"
  bench c1_h1_256_$r rmat24 "FGI_TAIL_HEAD=1 FGI_TAIL_BLOCKS=256"
done
FGI_TAIL_BLOCKS=256 $T 200 python -u -m pytest "tests/test_gpu_parity.py::test_deep_waves_through_the_tail" -q --timeout 150 --timeout-method thread > $out/deep.log 2>&1
rc=$?; tail -2 $out/deep.log
