#!/bin/bash
# Per-level phase probes (make variant-probe; FGI_TRACE=1) of configs[0] and configs[1] on this build.
set -u
out=gpurun_out/r6f
mkdir -p "$out"
for c in layered_1m rmat24; do
  FGI_LIBRARY=$PWD/stl.fusion_amd/lib/libfgi_probe.so FGI_TRACE=1 timeout -k 10 240 python -u profiles/wave_levels.py $c \
      > "$out/probe_$c.log" 2>&1 || { echo "probe $c rc=$?"; tail -20 "$out/probe_$c.log"; exit 1; }
  grep -E "^\[probe\]|^wave|^\[fgi\] (level|wave)" "$out/probe_$c.log" | tail -16
done
# first tail pass: entries 2-3 only (pass1_4, HEAD's behaviour) vs whole lists of <= 8 (libfgi) / <= 12 entries
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6f_ab0 3 --args --config layered_1m -- $L/libfgi_pass1_4.so $L/libfgi.so $L/libfgi_pass1_12.so || exit 1
bash profiles/r5_ab.sh r6f_ab24 2 $L/libfgi_pass1_4.so $L/libfgi.so $L/libfgi_pass1_12.so || exit 1
