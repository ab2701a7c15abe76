#!/bin/bash
# Round 5: attribute k_final_count's time at configs[2] with labels (FGI_FOLD_EXP, measurement only:
# 1 = no hot labels folded, 2 = no cold words copied, 3 = neither) — kernel trace per setting.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r11k; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for x in 0 4; do
  FGI_FOLD_EXP=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $out/t$x -o run --output-format csv -- python3 $R/bench.py --config rmat27 --no-secondary --no-cpu --no-e2e --steps 5 --warmup 1 > $out/t$x.json 2> $out/t$x.err || { echo "trace $x rc=$?"; tail -5 $out/t$x.err; exit 1; }
  echo "FGI_FOLD_EXP=$x"; grep -E "k_final" $out/t$x/run_kernel_stats.csv | cut -c1-120
done
