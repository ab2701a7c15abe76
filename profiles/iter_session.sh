#!/bin/bash
# Iteration check on the GPU box (repo root): the GPU tests, a short bench without the CPU leg, and
# the per-level k_level times of configs[1] and configs[0]. Stops at the first crash-like exit.
# Usage: profiles/iter_session.sh <tag>
TAG=${1:-it}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-e2e > "$O/bench.json" 2> "$O/bench.err" || exit 22
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],4), 'ms', 'k_level', round(d['roofline']['avg_launch_ms']*1e3,1), 'us')" "$O/bench.json"
for cfg in rmat24 layered_1m; do
    FGI_TRACE=1 timeout -k 10 120 python profiles/wave_levels.py $cfg > "$O/levels_$cfg.log" 2>&1 || exit 23
    echo "$cfg: $(grep "level [0-9] " "$O/levels_$cfg.log" | tail -6 | awk '{print $3, $4, $NF, $(NF-1)}' | tr '\n' ';')"
done
