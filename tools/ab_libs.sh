#!/bin/bash
# Bench line per library build, interleaved twice (same box): tools/ab_libs.sh main VARIANT ...
# ("main" = the in-tree libia.so; VARIANT = _ab/libia_VARIANT.so; BENCH_ARGS: extra bench.py args)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
    for v in "$@"; do
        if [ "$v" = main ]; then unset IA_LIB_PATH; else export IA_LIB_PATH=$PWD/_ab/libia_$v.so; fi
        timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err \
            || { tail -5 gpurun_out/abl_$v.err; exit 1; }
        python3 -c "
import json,sys; d=json.loads(open('gpurun_out/abl_$v.json').read().strip().splitlines()[-1])
print('$v', round(d['value']), round(d['ms_per_step'],1), round(d['roofline']['screen_avg_us'],1), d['checks']['checksum'])"
    done
done
