#!/bin/bash
# GPU tests, a short c4 bench and the screen harness (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -3 gpurun_out/t_gpu.log
timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || { tail -20 gpurun_out/b_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_c4.json')); print('c4', round(d['ms_per_step'],1), 'ms/step', round(d['value']), 'px/s', round(d['roofline']['screen_avg_us'],1), 'us', round(d['roofline']['frac'],4), d['checks'])"
timeout -k 10 120 tools/screen_bench --M 342,256,171,64 --reps 3 --rounds 3 > gpurun_out/sb.txt 2>&1 || { tail -20 gpurun_out/sb.txt; exit 1; }
cat gpurun_out/sb.txt
