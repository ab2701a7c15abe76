#!/bin/bash
# Round-4 HEAD after the spin wait: GPU suite + smoke + bench line (CPU baseline, e2e), then the
# rocprofv3 kernel trace + PMC passes of bench.py (run_profile.sh -> summarize.py)
set -u
bash profiles/r8z_session.sh r9a || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > gpurun_out/r9a/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r9a/smoke.log; exit 1; }
tail -1 gpurun_out/r9a/smoke.log
bash profiles/run_profile.sh r9a --steps 20 --warmup 3 --no-cpu --no-e2e || { echo "profile rc=$?"; exit 1; }
python profiles/summarize.py gpurun_out/prof_r9a r9a --steps 20 > gpurun_out/r9a/summarize.log 2>&1 || { echo "summarize rc=$?"; tail -5 gpurun_out/r9a/summarize.log; }
tail -5 gpurun_out/r9a/summarize.log
