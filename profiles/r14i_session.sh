#!/bin/bash
# Round 6: partition codes dealt over the pull blocks' runs (default) vs contiguous (FGI_PC_STRIPE=0) vs none
# (FGI_LABELS=-1) on configs[2] in 8 in-process ranks on one GPU: wall time, then a counter pass's serialised
# kernel trace (each rank's k_level alone)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14i; mkdir -p $out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_part_load.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for mode in stripe contig none; do
    case $mode in stripe) E="";; contig) E="FGI_PC_STRIPE=0";; none) E="FGI_LABELS=-1";; esac
    env $E timeout -k 10 300 python profiles/part_local_timing.py 27 8 5 8 | sed "s/^/$mode /" >> $out/ab.txt 2>> $out/ab.err || { echo "timing rc=$?"; tail -5 $out/ab.err; exit 1; }
  done
done
cat $out/ab.txt
cd /tmp && export TMPDIR=/tmp
for mode in stripe none; do
  case $mode in stripe) L=0;; none) L=-1;; esac
  FGI_LABELS=$L timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $out/kt_$mode -o run --output-format csv -- \
      python3 $R/profiles/part_local_timing.py 27 8 2 8 > $out/kt_$mode.out 2> $out/kt_$mode.err || { echo "kt rc=$?"; tail -5 $out/kt_$mode.err; exit 1; }
done
