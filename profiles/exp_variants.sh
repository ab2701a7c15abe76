#!/bin/bash
# Level timings of the measurement variants (stl.fusion_amd/lib/libfgi_exp*.so, wrong results) next to
# the real build: which part of a pull level its time goes to. Usage: profiles/exp_variants.sh <tag>
TAG=${1:-x}
O=gpurun_out/exp_$TAG
mkdir -p "$O"
for lib in stl.fusion_amd/lib/libfgi.so stl.fusion_amd/lib/libfgi_exp*.so stl.fusion_amd/lib/libfgi_pv*.so; do
    [ -f "$lib" ] || continue
    n=$(basename "$lib" .so)
    FGI_LIBRARY=$PWD/$lib FGI_TRACE=1 timeout -k 10 120 python profiles/wave_levels.py ${CFG:-rmat24} > "$O/$n.log" 2>&1 || exit 1
    echo "== $n"; grep "level [0-5] " "$O/$n.log" | tail -6 | awk '{print $3, $4, $NF, $(NF-1)}' | tr '\n' ';'; echo
done
