#!/bin/bash
# A/B of the in-process 8-rank partitioned wave (profiles/part_local_timing.py) between the in-tree
# build and another build (FGI_LIBRARY), alternating three times on one box.
# Usage (repo root, GPU box): profiles/ab_part_local.sh <tag> <other lib> [scale] [P]
TAG=${1:-abp}; OTHER=$2; SCALE=${3:-22}; P=${4:-8}
mkdir -p gpurun_out/$TAG
for i in 1 2 3; do
  for lib in $PWD/stl.fusion_amd/lib/libfgi.so $OTHER; do
    FGI_LIBRARY=$lib timeout -k 10 150 python profiles/part_local_timing.py $SCALE $P 20 >> gpurun_out/$TAG/ab.txt 2>> gpurun_out/$TAG/ab.err || exit 1
  done
done
cat gpurun_out/$TAG/ab.txt
