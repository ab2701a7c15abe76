#!/bin/bash
# A/B of an environment knob on one box: bench.py (no CPU leg, no e2e) alternately without and with
# the given VAR=VALUE, three times each. Usage: profiles/ab_bench.sh <tag> VAR=VALUE [bench args]
TAG=${1:-ab}; KV=$2; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
for i in 1 2 3; do
    for mode in base knob; do
        if [ $mode = knob ]; then env $KV timeout -k 10 300 python bench.py --no-cpu --no-e2e "$@" > "$O/$mode$i.json" 2> "$O/$mode$i.err" || exit 1
        else timeout -k 10 300 python bench.py --no-cpu --no-e2e "$@" > "$O/$mode$i.json" 2> "$O/$mode$i.err" || exit 1; fi
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],4), round(d['wave_kernel_ms'],4))" "$O/$mode$i.json" "$mode$i"
    done
done
