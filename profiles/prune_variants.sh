#!/bin/bash
# Prune kernel time of the measurement variants (stl.fusion_amd/lib/libfgi_pexp*.so, wrong results)
# next to the real build, on configs[3]. Usage: profiles/prune_variants.sh <tag>
TAG=${1:-x}
O=gpurun_out/pexp_$TAG
mkdir -p "$O"
for lib in stl.fusion_amd/lib/libfgi.so stl.fusion_amd/lib/libfgi_pexp*.so stl.fusion_amd/lib/libfgi_sp*.so; do
    [ -f "$lib" ] || continue
    n=$(basename "$lib" .so)
    FGI_LIBRARY=$PWD/$lib timeout -k 10 150 python bench_configs.py --only churn --no-cpu > "$O/$n.jsonl" 2> "$O/$n.err" || exit 1
    echo "== $n $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(d['prune']['kernel_ms'], d['prune']['new_edges'])" "$O/$n.jsonl")"
done
