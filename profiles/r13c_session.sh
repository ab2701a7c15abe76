#!/bin/bash
# Round 5: per-block phase stamps of configs[1]'s pull levels (make variant-probe; FGI_TRACE=1 prints the
# per-level medians), HEAD's kernels with 4,096 LDS hot words.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13c; mkdir -p $out
cd $R
FGI_TRACE=1 FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_probe.so timeout -k 10 200 python profiles/wave_levels.py rmat24 > $out/probe_c1.log 2>&1 || { echo "probe rc=$?"; tail -20 $out/probe_c1.log; exit 1; }
grep -v "^\[fgi\] labels" $out/probe_c1.log | tail -40
