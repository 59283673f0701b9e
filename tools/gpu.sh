#!/bin/bash
# One entry point for the GPU-box tasks of this repo (run it through gpurun), replacing the
# round-1/2 one-off scripts.  Every GPU step runs under its own time limit; output goes to
# gpurun_out/ (merged back by gpurun); a failing step ends the script (set -e semantics).
#
#   tools/gpu.sh tests [PYTEST_K_EXPR]        GPU suite in ONE process (-k filter optional)
#   tools/gpu.sh smoke                        __graft_entry__.smoke()
#   tools/gpu.sh bench TAG [bench.py args]    one bench line -> gpurun_out/bench_TAG.json
#   tools/gpu.sh shardsim TAG G [G ...]       simulated G-shard rank (tools/shard_sim.py)
#   tools/gpu.sh trace TAG -- CMD...          rocprofv3 kernel trace + stats of CMD
#                                             -> gpurun_out/TAG/ (trace csv removed, stats kept)
#   tools/gpu.sh pmc TAG COUNTERS -- CMD...   one rocprofv3 --pmc pass (counters space-separated
#                                             in one argument; respect the per-block limits),
#                                             summarised per kernel (PMC_REGEX filters kernels)
#   tools/gpu.sh traffic TAG -- CMD...        FETCH_SIZE + WRITE_SIZE passes of the screen
#                                             -> gpurun_out/traffic_TAG.json (bench.py reads it
#                                             from profiles/)
#   tools/gpu.sh abknob TAG VAR A B -- CMD... A/B/A/B of an environment knob (CMD prints one line)
#   tools/gpu.sh ablib TAG LIB -- CMD...      A/B/A/B of libia.so against another build (IA_LIB_PATH)
#
# Several tasks in one gpurun call: chain them with && in the gpurun command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
task=$1; shift

split_cmd() {   # everything after "--"
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do shift; done
    shift
    echo "$@"
}

case "$task" in
tests)
    k=()
    [ -n "$1" ] && k=(-k "$1")
    timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread "${k[@]}" \
        > gpurun_out/t_gpu.log 2>&1
    rc=$?
    grep -E "FAILED|ERROR" gpurun_out/t_gpu.log | head -20
    tail -1 gpurun_out/t_gpu.log
    exit $rc ;;
smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail -20 gpurun_out/smoke.log; exit 1; }
    tail -1 gpurun_out/smoke.log ;;
bench)
    tag=$1; shift
    timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
        || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
    python3 - gpurun_out/bench_$tag.json "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']
print('%s: %.0f px/s  %.1f ms/step  frac %.4f (%s %.1f us)  events +%.1f%%  checks %s' % (
    sys.argv[2], d['value'], d['ms_per_step'], r['frac'], r['kernel'], r.get('screen_avg_us', 0),
    100 * d.get('events_pass', {}).get('overhead', 0), d['checks']))
PY
    ;;
shardsim)
    tag=$1; shift
    timeout -k 10 600 python -u tools/shard_sim.py "$@" > gpurun_out/ss_$tag.txt 2>&1 \
        || { tail -20 gpurun_out/ss_$tag.txt; exit 1; }
    cat gpurun_out/ss_$tag.txt ;;
trace)
    tag=$1; shift
    cmd=$(split_cmd "$@")
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$PWD/gpurun_out/$tag" -o run -- $cmd > gpurun_out/$tag.log 2>&1 \
        || { tail -20 gpurun_out/$tag.log; exit 1; }
    python3 tools/trace_summary.py gpurun_out/$tag/run_kernel_trace.csv > gpurun_out/$tag/summary.txt
    cat gpurun_out/$tag/summary.txt
    head -16 gpurun_out/$tag/run_kernel_stats.csv | cut -d, -f1-6
    rm -f gpurun_out/$tag/run_kernel_trace.csv ;;
pmc)
    # counters summarised per kernel on the box (mean per dispatch); the raw csv is dropped
    # unless KEEP_CSV=1.  PMC_REGEX restricts collection to matching kernels.
    tag=$1; counters=$2; shift 2
    cmd=$(split_cmd "$@")
    rx=(); [ -n "$PMC_REGEX" ] && rx=(--kernel-include-regex "$PMC_REGEX")
    timeout -s KILL 600 rocprofv3 --pmc $counters "${rx[@]}" --output-format csv \
        -d "$PWD/gpurun_out/$tag" -o run -- $cmd > gpurun_out/$tag.log 2>&1 \
        || { tail -20 gpurun_out/$tag.log; exit 1; }
    python3 tools/pmc_summary.py gpurun_out/$tag/run_counter_collection.csv > gpurun_out/$tag/summary.txt
    [ "$KEEP_CSV" = 1 ] || rm -f gpurun_out/$tag/run_counter_collection.csv
    grep -A12 -E "k_screen16[ipr]ILi11E" gpurun_out/$tag/summary.txt | head -40
    if grep -qE "k_screen16[ipr]ILi11E" gpurun_out/$tag/summary.txt && grep -q SQ_VALU_MFMA_BUSY gpurun_out/$tag/summary.txt; then
        python3 tools/pmc_sq.py gpurun_out/$tag/summary.txt > gpurun_out/sq_$tag.json
    fi ;;
traffic)
    # HBM bytes per launch of the dominant screen instance on the bench process: separate
    # FETCH_SIZE and WRITE_SIZE passes (MI355X_MICROARCH.md HBM section), a stream sync every
    # 64 waves so the profiler keeps up -> gpurun_out/traffic_TAG.json
    tag=$1; shift
    cmd=$(split_cmd "$@")
    for c in FETCH_SIZE WRITE_SIZE; do
        IA_SYNC_EVERY=64 timeout -s KILL 600 rocprofv3 --pmc $c --kernel-include-regex k_screen16 \
            --output-format csv -d "$PWD/gpurun_out/tr_$tag/$c" -o run -- $cmd \
            > gpurun_out/tr_${tag}_$c.log 2>&1 || { tail -20 gpurun_out/tr_${tag}_$c.log; exit 1; }
    done
    python3 tools/pmc_traffic.py gpurun_out/tr_$tag/FETCH_SIZE/run_counter_collection.csv \
        gpurun_out/tr_$tag/WRITE_SIZE/run_counter_collection.csv > gpurun_out/traffic_$tag.json
    rm -rf gpurun_out/tr_$tag
    cat gpurun_out/traffic_$tag.json ;;
abknob)
    tag=$1; var=$2; va=$3; vb=$4; shift 4
    cmd=$(split_cmd "$@")
    for v in a b a2 b2; do
        val=$va; [ "${v:0:1}" = b ] && val=$vb
        env "$var=$val" timeout -k 10 600 $cmd > gpurun_out/ab_${tag}_$v.txt 2>&1 \
            || { tail -20 gpurun_out/ab_${tag}_$v.txt; exit 1; }
        echo "$v $var=$val: $(tail -1 gpurun_out/ab_${tag}_$v.txt | cut -c1-400)"
    done ;;
ablib)
    tag=$1; lib=$2; shift 2
    cmd=$(split_cmd "$@")
    for v in a b a2 b2; do
        if [ "${v:0:1}" = b ]; then export IA_LIB_PATH=$lib; else unset IA_LIB_PATH; fi
        timeout -k 10 600 $cmd > gpurun_out/ab_${tag}_$v.txt 2>&1 \
            || { tail -20 gpurun_out/ab_${tag}_$v.txt; exit 1; }
        echo "$v: $(tail -1 gpurun_out/ab_${tag}_$v.txt | cut -c1-400)"
    done ;;
*)
    sed -n 2,20p "$0"; exit 2 ;;
esac
