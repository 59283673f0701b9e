#!/bin/bash
# Round profile of the c4 bench on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of `bench.py` (c4, 1 timed step)
#   2. PMC passes (FETCH_SIZE, WRITE_SIZE separately) of the production screen variant
#      in the standalone harness tools/screen_bench (no torch in the profiled process)
# Output under gpurun_out/prof_<tag>/; copy the summaries to profiles/.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
make -C "$R/tools" > "$OUT/make.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o c4 -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err"
echo "kernel trace done"
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
        "$R/tools/screen_bench" --M 342 --variants 0x036 --reps 3 --rounds 1 > "$OUT/pmc_$C.txt" 2>&1
    echo "pmc $C done"
done
