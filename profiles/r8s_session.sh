#!/bin/bash
# round 4: the step's host gap (profiles/debug/step_gap.py), default scheduling, then spin (flag 1)
# and blocking sync (flag 4)
set -u
timeout -k 10 240 python -u profiles/debug/step_gap.py > gpurun_out/r8s_gap_default.txt 2>&1 || exit 1
FGI_DIAG_SPIN=1 timeout -k 10 240 python -u profiles/debug/step_gap.py > gpurun_out/r8s_gap_spin.txt 2>&1 || exit 1
FGI_DIAG_SPIN=2 timeout -k 10 240 python -u profiles/debug/step_gap.py > gpurun_out/r8s_gap_yield.txt 2>&1 || exit 1
cat gpurun_out/r8s_gap_*.txt
