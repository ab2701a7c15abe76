#!/bin/bash
# Round-3 measurement session (GPU box, repo root): per-level traces of configs[0]/[1]/[2], the
# rocprofv3 kernel trace + HBM counters of bench.py (configs[1]), the per-level PMC of configs[2]'s
# single-GPU wave, the other configs' GPU legs, and last the exit-crash investigation (a rocprofv3
# run with cooperative launches, /proc/self/maps written before exit).
set -u
R=$(pwd)
out=$R/gpurun_out/r5b
mkdir -p "$out"
for cfg in rmat24 rmat27 layered_1m; do
  FGI_TRACE=1 timeout -k 10 180 python profiles/wave_levels.py $cfg > "$out/levels_$cfg.out" 2> "$out/levels_$cfg.err" || { echo "levels $cfg rc=$?"; exit 1; }
done
echo "levels done"
timeout -k 10 300 python bench_configs.py --no-cpu > "$out/configs.jsonl" 2> "$out/configs.err" || { echo "configs rc=$?"; exit 1; }
echo "configs done"
bash profiles/run_profile.sh r5b --steps 5 --warmup 1 --no-cpu --no-e2e > "$out/run_profile.out" 2>&1 || { echo "run_profile rc=$?"; exit 1; }
echo "profile done"
bash profiles/pmc_levels.sh r5b27 rmat27 > "$out/pmc_levels.out" 2>&1 || { echo "pmc_levels rc=$?"; exit 1; }
echo "pmc levels done"
cd /tmp && export TMPDIR=/tmp
FGI_MAPS_OUT=$out/maps_stream.txt timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$out/stream_trace" -o run --output-format csv -- \
  python3 "$R/bench_configs.py" --only stream --no-cpu > "$out/stream_trace.out" 2> "$out/stream_trace.err"
echo "stream trace rc=$?"
