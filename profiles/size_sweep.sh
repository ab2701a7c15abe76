#!/bin/bash
# One-device graph-size sweep: bench.py (no CPU leg, no e2e) on R-MAT 24/25/26 (edge factor 16) and
# configs[2]'s R-MAT 27 (edge factor 8), single engine; then configs[2] through the partitioned engine
# at one rank. Usage (repo root, GPU box): profiles/size_sweep.sh <tag>
O=gpurun_out/${1:-size}
mkdir -p "$O"
for c in rmat24 rmat25 rmat26 rmat27; do
    timeout -k 10 400 python bench.py --config $c --no-cpu --no-e2e --steps 10 > "$O/$c.json" 2> "$O/$c.err" || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['config']['nodes'], d['config']['edges'], d['v_inv_per_step'], round(d['ms_per_step'],4), round(d['value']/1e9,2), round(d['gteps'],1), d['pull_levels_per_step'])" "$O/$c.json" $c
done
timeout -k 10 400 python bench.py --config rmat27 --partition --no-cpu --no-e2e --steps 10 > "$O/rmat27_partition.json" 2> "$O/rmat27_partition.err" || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('rmat27 --partition', round(d['ms_per_step'],4), round(d['value']/1e9,2), round(d['gteps'],1))" "$O/rmat27_partition.json"
