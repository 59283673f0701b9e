#!/bin/bash
# HBM traffic of the screen measured on the product process: rocprofv3 PMC passes
# (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass) of `bench.py` (c4, one step),
# summarised per kernel by tools/pmc_traffic.py into gpurun_out/pmc_bench/traffic.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_bench
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# a stream sync every 64 waves: rocprofv3 --pmc crashes with thousands of dispatches in flight
export IA_SYNC_EVERY=${IA_SYNC_EVERY:-64}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o p -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/$C.json" 2> "$OUT/$C.err"
  rc=$?
  echo "$C pass exit $rc"
  if [ $rc -ne 0 ]; then grep -E "SIGSEGV|Abort|rror" "$OUT/$C.err" | head -5; grep -E "^    @" "$OUT/$C.err" | grep -v unknown | head -8; exit 1; fi
done
python3 "$R/tools/pmc_traffic.py" "$OUT/FETCH_SIZE/p_counter_collection.csv" "$OUT/WRITE_SIZE/p_counter_collection.csv" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
