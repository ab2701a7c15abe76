#!/bin/bash
# Round 5: configs[1]'s level-0 push phases with the dead-edge filter on (default) and off (probe variant)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13f; mkdir -p $out
cd $R
for df in 1 0; do
  WL_OPTS="1=$df" FGI_TRACE=1 FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_probe.so timeout -k 10 200 python profiles/wave_levels.py rmat24 > $out/probe_df$df.log 2>&1 || { echo "probe rc=$?"; exit 1; }
  echo "dead_filter=$df"; grep -E "probe\] level [0-5]|^wave" $out/probe_df$df.log | tail -7
done
