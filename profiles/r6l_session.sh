#!/bin/bash
# Tail-scan flush threshold: a wave scans its queued tails once 64 (libfgi) / 128 (tf128) are waiting,
# overlapping their round trips with other waves' runs, instead of only near queue overflow (tf257 =
# HEAD). GPU tests on libfgi, then an A/B on configs[2]'s graph (3.9 M queued per wave), configs[1] and
# configs[0].
set -u
out=gpurun_out/r6l
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6l_ab27 2 --args --config rmat27 -- $L/libfgi_tf257.so $L/libfgi_tf128.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6l_ab24 2 $L/libfgi_tf257.so $L/libfgi_tf128.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6l_ab0 2 --args --config layered_1m -- $L/libfgi_tf257.so $L/libfgi_tf128.so $L/libfgi.so || exit 1
