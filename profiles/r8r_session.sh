#!/bin/bash
# round 4: the wave-end event recorded before the final synchronisation (no second round trip when
# a stats struct is passed) vs the previous build (record + event sync after the stream sync);
# then the wave / partition GPU tests on the new build
set -u
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r8r_ab 4 $L/libfgi.so $L/libfgi_oldev.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r8r_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r8r_gpu_tests.log; exit $rc
