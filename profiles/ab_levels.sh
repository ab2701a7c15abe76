#!/bin/bash
# A/B on one box: bench.py pairs (profiles/ab_bench.sh) and the configs[1] per-level k_level times of
# the in-tree build against another build of the engine (FGI_LIBRARY=<lib>).
# Usage (repo root, GPU box): profiles/ab_levels.sh <tag> <other lib path>
TAG=${1:-abl}; OTHER=$2
profiles/ab_bench.sh $TAG FGI_LIBRARY=$OTHER || exit 1
for lib in $PWD/stl.fusion_amd/lib/libfgi.so $OTHER; do
  FGI_LIBRARY=$lib FGI_TRACE=1 timeout -k 10 120 python profiles/wave_levels.py rmat24 > gpurun_out/$TAG/lv.log 2>&1 || exit 1
  echo "$(basename $lib): $(grep "level [0-9] " gpurun_out/$TAG/lv.log | tail -6 | awk '{print $3, $4, $NF, $(NF-1)}' | tr '\n' ';')"
done
