#!/bin/bash
# LDS copy of the hot heads' snapshot in pull blocks: GPU tests on the default build (8 KB), parity
# subsets on the 16 KB / 32 KB variants, then an A/B against HEAD's build on configs[1] and configs[2].
set -u
R=$(pwd)
out=$R/gpurun_out/r5g
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
for v in ldshot4096 ldshot8192; do
  FGI_LIBRARY=$R/$L/libfgi_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_part.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests_$v.log" 2>&1 \
    || { echo "tests $v rc=$?"; tail -30 "$out/tests_$v.log"; exit 1; }
  tail -1 "$out/tests_$v.log"
done
bash profiles/r5_ab.sh r5g_ab24 3 $L/libfgi_base.so $L/libfgi.so $L/libfgi_ldshot4096.so $L/libfgi_ldshot8192.so || exit 1
bash profiles/r5_ab.sh r5g_ab27 1 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi.so $L/libfgi_ldshot4096.so $L/libfgi_ldshot8192.so || exit 1
