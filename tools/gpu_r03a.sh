#!/bin/bash
# round 3, first check of the fused per-wave kernel: smoke, parity + exchange tests, shard sim
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py tests/test_gpu_outputs.py -v --timeout 150 --timeout-method thread > gpurun_out/t_par.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" gpurun_out/t_par.log | tail -60
tail -3 gpurun_out/t_par.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/shard_sim.py 1 8 > gpurun_out/ss.txt 2>&1 || { tail -20 gpurun_out/ss.txt; exit 1; }
cat gpurun_out/ss.txt
