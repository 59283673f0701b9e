#!/bin/bash
# the GPU suite, then 2 bench ranks sharing the GPU on c4 (device-side exchange) vs 1 rank
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
IA_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sd_c4g2.json 2> gpurun_out/sd_c4g2.err || { tail -20 gpurun_out/sd_c4g2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/sd_c4g2.json')); print('c4 2 ranks on one GPU', round(d['value']), round(d['ms_per_step'],1), d['checks'], d['config'].get('exchange'))"
