#!/bin/bash
# Round 5: configs[1]'s level phases with row records (default) and without (FGI_ROW_REC=0), probe variant
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13o; mkdir -p $out
cd $R
for rr in 1 0 1 0; do
  FGI_ROW_REC=$rr FGI_TRACE=1 FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_probe.so timeout -k 10 200 python profiles/wave_levels.py rmat24 > $out/probe_rr$rr.log 2>&1 || { echo "probe rc=$?"; exit 1; }
  echo "row_rec=$rr"; grep -E "probe\] level [0-5]|^wave 2" $out/probe_rr$rr.log | tail -7
done
