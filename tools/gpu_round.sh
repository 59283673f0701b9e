#!/bin/bash
# Round check on one GPU: the exchange tests, the whole GPU suite, the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_exchange.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_exch.log 2>&1 || { tail -40 gpurun_out/t_exch.log; exit 1; }
tail -1 gpurun_out/t_exch.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 240 python -u bench.py > gpurun_out/b_def.json 2> gpurun_out/b_def.err || { tail -20 gpurun_out/b_def.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_def.json')); print('c4', round(d['value']), round(d['ms_per_step'],1), 'ms/step frac', round(d['roofline']['frac'],4))"
