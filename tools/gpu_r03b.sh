#!/bin/bash
# round 3: the fused per-wave kernel — rccl parity tests, simulated 8-shard rank, c4 bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k rccl -v --timeout 150 --timeout-method thread > gpurun_out/t_rccl.log 2>&1 || { tail -30 gpurun_out/t_rccl.log; exit 1; }
tail -1 gpurun_out/t_rccl.log
timeout -k 10 400 python -u tools/shard_sim.py 1 8 > gpurun_out/ss.txt 2>&1 || { tail -20 gpurun_out/ss.txt; exit 1; }
cat gpurun_out/ss.txt
IA_XWAVE=0 timeout -k 10 400 python -u tools/shard_sim.py 8 > gpurun_out/ss_old.txt 2>&1 || { tail -20 gpurun_out/ss_old.txt; exit 1; }
cat gpurun_out/ss_old.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || { tail -20 gpurun_out/b_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_c4.json')); print('c4 xw', round(d['value']), round(d['ms_per_step'],1), 'ms/step frac', round(d['roofline']['frac'],4), d['checks'])"
