#!/bin/bash
# Round 5: k_roots with the roots' rows requested together with their node words — rocprofv3 kernel-trace
# stats of configs[1] (20 timed steps) for the new build and the previous one (FGI_LIBRARY=libfgi_base.so), twice
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13p; mkdir -p $out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_labels.py tests/test_gpu_part.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $out/parity.log; exit 1; }
tail -1 $out/parity.log
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_base.so; else unset FGI_LIBRARY; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${v}_$k -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --no-secondary --steps 20 --warmup 5 > $out/${v}_$k.json 2> $out/${v}_$k.err || { echo "rocprof rc=$?"; tail -5 $out/${v}_$k.err; exit 1; }
    python3 - <<PY
import csv
rows = list(csv.DictReader(open("$out/${v}_$k/run_kernel_stats.csv")))
d = {r["Name"].split("(")[0].split("<")[0]: float(r["AverageNs"]) / 1000 for r in rows}
print("$v $k", " ".join(f"{k}={d[k]:.2f}" for k in ("k_wave_init", "k_roots", "k_level", "k_collect", "k_final_write") if k in d))
PY
  done
done
