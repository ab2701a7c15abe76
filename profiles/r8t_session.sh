#!/bin/bash
# round 4: level groups ending in a host spin on a published sequence word (libfgi) against a
# stream synchronisation + counter copy (libfgi_nospin); the step-gap diagnostic on both; GPU tests
set -u
L=stl.fusion_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py > gpurun_out/r8t_wave_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r8t_wave_tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r5_ab.sh r8t_ab 4 $L/libfgi.so $L/libfgi_nospin.so || exit 1
timeout -k 10 240 python -u profiles/debug/step_gap.py > gpurun_out/r8t_gap_spin.txt 2>&1 || exit 1
FGI_LIBRARY=$PWD/$L/libfgi_nospin.so timeout -k 10 240 python -u profiles/debug/step_gap.py > gpurun_out/r8t_gap_nospin.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r8t_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r8t_gpu_tests.log; exit $rc
