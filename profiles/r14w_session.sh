#!/bin/bash
# Round 6: the synchronous wave publishes its counters from k_final_count (the host turns round while
# k_final_write writes the list; no k_publish launch): GPU suite, configs[1] / configs[2] A/B against
# the previous build (libfgi_base.so), then a kernel trace of configs[1] (launches and gaps per wave)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14w; mkdir -p $out
T="timeout -k 10"
cd $R
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
bench() {  # tag config setting
  local tag=$1 cfg=$2 setting=$3
  envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
  env "${envs[@]}" $T 240 python bench.py --no-cpu --no-e2e --no-secondary --steps 30 --warmup 5 --config $cfg > $out/$tag.json 2> $out/$tag.err || { echo "bench rc=$?"; tail -5 $out/$tag.err; exit 1; }
  python -c "
import json; d = json.load(open('$out/$tag.json')); r = d['roofline']
print('$tag', '$cfg', round(d['ms_per_step'], 4), 'pull', round(r['pull_levels']['ms_per_step'], 4), 'push', round(r['push_levels']['ms_per_step'], 4), 'kern', round(d['wave_kernel_ms'], 4), 'vinv', d['v_inv_per_step'], 'frac', round(r['frac'], 4), flush=True)"
}
BASE="FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_base.so"
for r in 1 2 3; do
  bench c1_new_$r rmat24 "-"
  bench c1_base_$r rmat24 "$BASE"
done
bench c2_new rmat27 "-"
bench c2_base rmat27 "$BASE"
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -T -d $out/trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-secondary > $out/trace_bench.json 2> $out/trace_bench.err || { echo "trace rc=$?"; exit 1; }
echo trace ok
python3 $R/profiles/wave_gaps.py $out/trace
