#!/bin/bash
# round 4: streaming mix (configs[4]) with the cascades' grid barrier fenced by every thread (mode 0,
# round 3) or by one wave per block (mode 1), alternating on one box; the cascade grid 128 / 64
set -e
out=gpurun_out/${1:-r7j}
mkdir -p $out
s() { timeout -k 10 200 python -u bench_configs.py --only stream --rounds 100 > $out/$1.json 2> $out/$1.err; }
FGI_BAR_MODE=0 s m0_a
FGI_BAR_MODE=1 s m1_a
FGI_BAR_MODE=0 s m0_b
FGI_BAR_MODE=1 s m1_b
FGI_BAR_MODE=1 FGI_COOP_BLOCKS=64 s m1_g64
FGI_BAR_MODE=1 FGI_COOP_BLOCKS=256 s m1_g256
