#!/bin/bash
# Round 5: the 8-rank partitioned wave of configs[2]'s graph (in-process, one GPU) with beta 32 (HEAD) and 24
# (the previous build): per-level directions and the wave's wall time
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13t; mkdir -p $out
cd $R
for v in b32 b24; do
  if [ $v = b24 ]; then export FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_base.so; else unset FGI_LIBRARY; fi
  FGI_TRACE=1 timeout -k 10 400 python profiles/part_local_timing.py 27 8 3 > $out/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $out/$v.log; exit 1; }
  echo "== $v"; grep -E "level [0-9]+ (pull|push)" $out/$v.log | tail -7; grep -v "^\[fgi\]" $out/$v.log | tail -3
done
