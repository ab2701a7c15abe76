#!/bin/bash
# Round 3 re-entry: HEAD's GPU tests and bench on a fresh box.
set -u
out=gpurun_out/r6a
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 400 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench rc=$?"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 120 ./profiles/micro/probe_mix > "$out/probe_mix.txt" 2>&1 || { echo "probe_mix rc=$?"; exit 1; }
cat "$out/probe_mix.txt"
