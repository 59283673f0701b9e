#!/bin/bash
# Round profile (run through gpurun from the repo root): per-M screen curve in the
# standalone harness, rocprofv3 kernel trace + stats of bench.py (c4) with the trace-vs-
# bench roofline check, PMC passes of the screen at M = 342, and last (it crashed in round
# 1) one PMC pass on the bench.py process itself.  Output under gpurun_out/prof_<tag>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 "$R/tools/screen_bench" --M 342,320,288,256,224,192,171,128,96,64,32,1 --reps 10 --rounds 5 > "$OUT/screen_curve.txt" 2>&1 || { tail -20 "$OUT/screen_curve.txt"; exit 1; }
cat "$OUT/screen_curve.txt"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o c4 -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" || { tail -20 "$OUT/c4_bench.err"; exit 1; }
python3 "$R/tools/roofline_check.py" "$OUT/c4/c4_kernel_trace.csv" "$OUT/c4_bench.json" > "$OUT/roofline_check.txt"
cat "$OUT/roofline_check.txt"
head -14 "$OUT/c4/c4_kernel_stats.csv"
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc_m342_p$i" -o pmc -- \
        "$R/tools/screen_bench" --M 342 --reps 2 --rounds 1 > "$OUT/pmc_m342_p$i.txt" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc_m342_p$i.txt"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT"/pmc_m342_p*/pmc_counter_collection.csv > "$OUT/pmc_m342.txt"
cat "$OUT/pmc_m342.txt"
echo "=== PMC on the bench.py process (FETCH_SIZE)"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_bench" -o pmc -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_bench.json" 2> "$OUT/pmc_bench.err"
echo "bench under --pmc exit $?"
tail -5 "$OUT/pmc_bench.err"
