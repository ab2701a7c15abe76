#!/bin/bash
# round 4: the partitioned engine at N = 1 (planned waves vs the host-driven levels), alternating
set -e
out=gpurun_out/${1:-r7k}
mkdir -p $out
p() { timeout -k 10 200 python -u bench.py --partition --steps 20 --warmup 3 --no-cpu > $out/$1.json 2> $out/$1.err; }
p plan_a
FGI_PART_PLAN=0 p noplan_a
p plan_b
FGI_PART_PLAN=0 p noplan_b
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $out/single.json 2> $out/single.err
