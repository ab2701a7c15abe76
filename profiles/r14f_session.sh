#!/bin/bash
# Round 6: partition codes vs none on configs[2] (8 in-process ranks on one GPU): per-kernel stats, kernels
# serialised (AMD_SERIALIZE_KERNEL=3) so that each dispatch runs alone
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14g; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for lab in 0 -1; do
  AMD_SERIALIZE_KERNEL=3 FGI_LABELS=$lab timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_$lab -o run --output-format csv -- \
      python3 $R/profiles/part_local_timing.py 27 8 5 8 > $out/kt_$lab.out 2> $out/kt_$lab.err || { echo "kt rc=$?"; tail -5 $out/kt_$lab.err; exit 1; }
  cat $out/kt_$lab.out
done
