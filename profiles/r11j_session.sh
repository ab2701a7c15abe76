#!/bin/bash
# Round 5: k_final_count with hot labels at configs[2] (64K-slot fold tiles): where its waves wait.
# Two counter passes of their own, filtered to the kernel.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r11j; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --config rmat27 --no-secondary --no-cpu --no-e2e --steps 5 --warmup 1"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_final_count" -T -d $out/sq -o run --output-format csv -- $B > $out/sq.json 2> $out/sq.err || { echo "sq rc=$?"; tail -5 $out/sq.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex "k_final_count" -T -d $out/tcc -o run --output-format csv -- $B > $out/tcc.json 2> $out/tcc.err || { echo "tcc rc=$?"; tail -5 $out/tcc.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_final_count" -T -d $out/fetch -o run --output-format csv -- $B > $out/fetch.json 2> $out/fetch.err || { echo "fetch rc=$?"; tail -5 $out/fetch.err; exit 1; }
for d in sq tcc fetch; do
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$out/$d/run_counter_collection.csv")))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print("$d", k, len(v), round(sum(v) / max(1, len(v)), 1))
if rows: print("$d", {k: rows[0][k] for k in ("Grid_Size", "LDS_Block_Size", "VGPR_Count", "SGPR_Count")})
PY
done
