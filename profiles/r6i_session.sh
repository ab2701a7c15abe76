#!/bin/bash
# Per-level phase probes (make variant-probe; FGI_TRACE=1) of configs[2]'s graph (R-MAT 27) on one GPU.
set -u
out=gpurun_out/r6i
mkdir -p "$out"
FGI_LIBRARY=$PWD/stl.fusion_amd/lib/libfgi_probe.so FGI_TRACE=1 timeout -k 10 400 python -u profiles/wave_levels.py rmat27 \
    > "$out/probe_rmat27.log" 2>&1 || { echo "probe rc=$?"; tail -20 "$out/probe_rmat27.log"; exit 1; }
grep -E "^\[probe\]|^wave|^\[fgi\] (level|wave)" "$out/probe_rmat27.log" | tail -16
