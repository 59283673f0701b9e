#!/bin/bash
# Round profile of the c4 bench on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of `bench.py` (c4, 1 timed step) and the
#      trace-vs-bench check of the finest level's screen (tools/roofline_check.py)
#   2. PMC passes (SQ/GRBM, LDS/VALU, FETCH_SIZE, WRITE_SIZE separately) of the split-f16
#      screen in the standalone harness tools/screen_bench (no torch in the profiled
#      process) at M = 342 and 256 queries
# Output under gpurun_out/prof_<tag>/; copy the summaries to profiles/.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
make -C "$R/tools" screen_bench > "$OUT/make.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o c4 -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err"
python3 "$R/tools/roofline_check.py" "$OUT/c4/c4_kernel_trace.csv" "$OUT/c4_bench.json" > "$OUT/roofline_check.txt"
echo "kernel trace done"
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
for M in 342 256; do
    i=0
    for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc_m${M}_p$i" -o pmc -- \
            "$R/tools/screen_bench" --M $M --reps 2 --rounds 1 > "$OUT/pmc_m${M}_p$i.txt" 2>&1
    done
    python3 "$R/tools/pmc_summary.py" "$OUT"/pmc_m${M}_p*/pmc_counter_collection.csv > "$OUT/pmc_m$M.txt"
    echo "pmc M=$M done"
done
