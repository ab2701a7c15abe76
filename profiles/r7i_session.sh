#!/bin/bash
# round 4: fused-wave barrier variants (A/B on one box): FGI_BAR_MODE 0/1, init in the head or not,
# fused grid 64/128/256, against the level-group path; plus the barrier microbenchmark
set -e
out=gpurun_out/${1:-r7i}
mkdir -p $out
timeout -k 10 120 ./profiles/micro/grid_barrier > $out/grid_barrier.txt 2>&1 || true
b() { timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $out/$1.json 2> $out/$1.err; }
FGI_FUSED=0 b nofuse
FGI_BAR_MODE=0 FGI_FUSED_INIT=1 b m0_init
FGI_BAR_MODE=1 FGI_FUSED_INIT=1 b m1_init
FGI_BAR_MODE=1 b m1
FGI_BAR_MODE=1 FGI_FUSED_BLOCKS=128 b m1_g128
FGI_BAR_MODE=1 FGI_FUSED_BLOCKS=64 b m1_g64
FGI_FUSED=0 b nofuse2
