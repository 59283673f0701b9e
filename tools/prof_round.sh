#!/bin/bash
# Round profile (run through gpurun from the repo root), output under gpurun_out/prof_<tag>/:
#   1. rocprofv3 kernel trace + stats of bench.py (c4, 2 timed steps) and the trace-vs-bench
#      roofline check (tools/roofline_check.py);
#   2. SQ counter passes on the bench.py process itself (IA_SYNC_EVERY=64: the profiler
#      crashes with thousands of dispatches in flight), summarised per kernel;
#   3. the row-form screen curve over M in the standalone harness (tools/screen_bench).
# HBM traffic of the screen on the bench process: tools/pmc_bench.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o c4 -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" || { tail -20 "$OUT/c4_bench.err"; exit 1; }
python3 "$R/tools/roofline_check.py" "$OUT/c4/c4_kernel_trace.csv" "$OUT/c4_bench.json" > "$OUT/roofline_check.txt"
cat "$OUT/roofline_check.txt"
head -16 "$OUT/c4/c4_kernel_stats.csv" | cut -d, -f1-4
rm -f "$OUT/c4/c4_kernel_trace.csv"   # large; the stats and the check above are kept
export IA_SYNC_EVERY=64
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc_p$i" -o pmc -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_p$i.json" 2> "$OUT/pmc_p$i.err" || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc_p$i.err"; exit 1; }
done
unset IA_SYNC_EVERY
python3 "$R/tools/pmc_summary.py" "$OUT"/pmc_p*/pmc_counter_collection.csv > "$OUT/pmc_bench.txt"
rm -f "$OUT"/pmc_p*/pmc_counter_collection.csv
grep -A17 "k_screen16iILi11" "$OUT/pmc_bench.txt"
timeout -k 10 200 "$R/tools/screen_bench" --M 342,320,288,256,224,192,171,128,96,64,32,1 --reps 10 --rounds 5 > "$OUT/screen_curve.txt" 2>&1 || { tail -20 "$OUT/screen_curve.txt"; exit 1; }
cat "$OUT/screen_curve.txt"
