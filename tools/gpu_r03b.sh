#!/bin/bash
# round 3: fused per-wave kernel + batch path — new tests, rccl tests, shard sim, c4 + c5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xwave.py tests/test_gpu_parity.py -k "rccl or xwave or batch or fused" -v --timeout 150 --timeout-method thread > gpurun_out/t_xw.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" gpurun_out/t_xw.log | tail -30
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/t_xw.log | head -20; exit 1; }
timeout -k 10 400 python -u tools/shard_sim.py 1 8 > gpurun_out/ss.txt 2>&1 || { tail -20 gpurun_out/ss.txt; exit 1; }
cat gpurun_out/ss.txt
IA_XWAVE=0 timeout -k 10 400 python -u tools/shard_sim.py 8 > gpurun_out/ss_old.txt 2>&1 || { tail -20 gpurun_out/ss_old.txt; exit 1; }
cat gpurun_out/ss_old.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || { tail -20 gpurun_out/b_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_c4.json')); print('c4', round(d['value']), round(d['ms_per_step'],1), 'ms/step frac', round(d['roofline']['frac'],4), 'ev', d['events_pass'], d['checks'], d['matcher'])"
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err || { tail -20 gpurun_out/b_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_c5.json')); print('c5', round(d['value']), round(d['ms_per_step'],1), 'ms/step frac', round(d['roofline']['frac'],4), d['checks'], d['config'])"
