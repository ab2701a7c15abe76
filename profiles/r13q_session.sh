#!/bin/bash
# Round 5: configs[2]'s per-level trace with HEAD and with the 4,096-word tail queue / 2,048 LDS hot words build
# (r13l's variant), to see which levels its extra 0.29 ms of push time sits in
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13q; mkdir -p $out
cd $R
FGI_TRACE=1 timeout -k 10 300 python profiles/wave_levels.py rmat27 > $out/head.log 2>&1 || { echo "head rc=$?"; tail -5 $out/head.log; exit 1; }
FGI_TRACE=1 FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_cpl4_4096_2048.so timeout -k 10 300 python profiles/wave_levels.py rmat27 > $out/q4096.log 2>&1 || { echo "variant rc=$?"; tail -5 $out/q4096.log; exit 1; }
for f in head q4096; do echo "== $f"; grep -E "\[fgi\] (level|tail|wave)|^wave" $out/$f.log | tail -14; done
