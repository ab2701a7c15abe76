#!/bin/bash
# FETCH_SIZE calibration passes (run on the GPU box from the repo root); one counter group per pass
set -e
R=$PWD
O=$R/gpurun_out/fc
mkdir -p $O
timeout -k 10 60 tools/fetch_calib > $O/run.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_MISS_sum TCC_HIT_sum" "TCC_BUBBLE_sum"; do
  n=$(echo $c | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- $R/tools/fetch_calib > $O/$n.log 2>&1
done
