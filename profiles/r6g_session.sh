#!/bin/bash
# (1) Pull candidates ordered hot-first within each block (libfgi) vs slot order (libfgi_slotorder, HEAD):
#     GPU tests, A/B on configs[1], configs[2]'s graph and configs[0].
# (2) Pull-block granularity (FGI_PULL_TPB: tiles per block; default 13 at configs[1] = 1,280 blocks, one
#     resident round) and the beta rule (FGI_PULL_BETA 12: configs[1]'s level 3 pushes) on configs[1].
set -u
out=gpurun_out/r6g
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
bash profiles/r5_ab.sh r6g_ab24 3 $L/libfgi_slotorder.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6g_ab27 2 --args --config rmat27 -- $L/libfgi_slotorder.so $L/libfgi.so || exit 1
bash profiles/r5_ab.sh r6g_ab0 2 --args --config layered_1m -- $L/libfgi_slotorder.so $L/libfgi.so || exit 1
bash profiles/env_ab.sh r6g_env24 2 "-" "FGI_PULL_TPB=7" "FGI_PULL_TPB=4" "FGI_PULL_BETA=12" || exit 1
