#!/bin/bash
# Round 6: partition codes vs none on configs[2] (8 in-process ranks on one GPU). A counter pass serialises
# the dispatches, so its kernel trace gives each rank's k_level alone (no other rank's kernels beside it)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14h; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for lab in 0 -1; do
  FGI_LABELS=$lab timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $out/kt_$lab -o run --output-format csv -- \
      python3 $R/profiles/part_local_timing.py 27 8 2 8 > $out/kt_$lab.out 2> $out/kt_$lab.err || { echo "kt rc=$?"; tail -5 $out/kt_$lab.err; exit 1; }
  cat $out/kt_$lab.out
done
