#!/bin/bash
# GPU tests, the default c4 bench, and the simulated sharded rank times (one GPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || { tail -20 gpurun_out/b_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_c4.json')); print('c4', round(d['ms_per_step'],1), 'ms/step', round(d['roofline']['screen_avg_us'],1), round(d['roofline']['frac'],4), d['checks']['checksum'])"
timeout -k 10 200 python -u tools/shard_sim.py ${SIM:-1 2 4 8} > gpurun_out/ss.txt 2>&1 || { tail -20 gpurun_out/ss.txt; exit 1; }
grep "G=" gpurun_out/ss.txt
