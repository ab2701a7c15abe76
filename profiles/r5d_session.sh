#!/bin/bash
# rocprofv3 evidence (second half of the r5b measurements): kernel trace + HBM counters of bench.py
# (configs[1]), the per-level PMC of configs[2]'s single-GPU wave, and last the exit-crash
# investigation (a rocprofv3 run with cooperative launches; /proc/self/maps written before exit).
set -u
tag=$1
R=$(pwd)
out=$R/gpurun_out/$tag
mkdir -p "$out"
bash profiles/run_profile.sh $tag --steps 5 --warmup 1 --no-cpu --no-e2e > "$out/run_profile.out" 2>&1 || { echo "run_profile rc=$?"; exit 1; }
echo "profile done"
bash profiles/pmc_levels.sh ${tag}27 rmat27 > "$out/pmc_levels.out" 2>&1 || { echo "pmc_levels rc=$?"; exit 1; }
echo "pmc levels done"
cd /tmp && export TMPDIR=/tmp
FGI_MAPS_OUT=$out/maps_stream.txt timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$out/stream_trace" -o run --output-format csv -- \
  python3 "$R/bench_configs.py" --only stream --no-cpu > "$out/stream_trace.out" 2> "$out/stream_trace.err"
echo "stream trace rc=$?"
