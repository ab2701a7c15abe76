#!/bin/bash
# GPU tests on the current build, then pull-level floor measurements (the probe-rate microbenchmark,
# profiles/micro/probe_rate.hip), the per-level phase probes of configs[1]'s wave (variant-probe)
# and an A/B of the current build against HEAD's (libfgi_base.so).
set -u
R=$(pwd)
out=$R/gpurun_out/r5f
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 120 ./profiles/micro/probe_rate > "$out/probe_rate.txt" 2>&1 || { echo "probe_rate rc=$?"; exit 1; }
cat "$out/probe_rate.txt"
FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_probe.so FGI_TRACE=1 timeout -k 10 240 python -u profiles/wave_levels.py \
    > "$out/probe.log" 2>&1 || { echo "probe rc=$?"; exit 1; }
grep -E "^\[probe\]|^wave" "$out/probe.log" | tail -12
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r5f_ab24 3 $L/libfgi_base.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r5f_ab27 1 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi.so || exit 1
