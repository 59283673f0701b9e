#!/bin/bash
# GPU tests (all), then the round profile (tools/prof_round.sh <tag>)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -60 gpurun_out/t_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_gpu.log | tail -2
grep -E "PASSED|FAILED" gpurun_out/t_gpu.log | awk '{print $1}' | sed 's/.*:://' | tr '\n' ' ' | head -c 3000; echo
bash tools/prof_round.sh ${1:-r02}
