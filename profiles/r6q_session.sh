#!/bin/bash
# Phase stamps of the streaming mix's cooperative waves (make variant-probe, FGI_TRACE=1: block 0's
# times per launch: roots done, level barriers, final counts, prefix barrier, ids written, cleaned up).
set -u
out=gpurun_out/r6q
mkdir -p "$out"
FGI_LIBRARY=$PWD/stl.fusion_amd/lib/libfgi_probe.so FGI_TRACE=1 timeout -k 10 300 python -u bench_configs.py --only stream --no-cpu --rounds 12 \
    > "$out/stream.jsonl" 2> "$out/stream.err" || { echo "rc=$?"; tail -20 "$out/stream.err"; exit 1; }
grep "\[coop\]" "$out/stream.err" | tail -24
