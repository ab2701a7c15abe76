#!/bin/bash
# Round 5: why k_final_count costs ~70 us at configs[2] with labels: kernel trace without labels, then
# one SQ counter pass over k_final_count with labels (a pass of its own, no trace domains).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r11i; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
FGI_LABELS=-1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $out/trace_c2off -o run --output-format csv -- python3 $R/bench.py --config rmat27 --no-secondary --no-cpu --no-e2e --steps 5 --warmup 1 > $out/trace_c2off.json 2> $out/trace_c2off.err || { echo "trace rc=$?"; tail -5 $out/trace_c2off.err; exit 1; }
grep -E "k_final|k_wave_init|k_roots" $out/trace_c2off/run_kernel_stats.csv | cut -c1-200
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "k_final_count" -T -d $out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --config rmat27 --no-secondary --no-cpu --no-e2e --steps 5 --warmup 1 > $out/pmc_sq.json 2> $out/pmc_sq.err || { echo "pmc rc=$?"; tail -5 $out/pmc_sq.err; exit 1; }
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$out/pmc_sq/run_counter_collection.csv")))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, len(v), sum(v) / max(1, len(v)))
print(rows[0].keys() if rows else "no rows")
PY
