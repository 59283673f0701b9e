#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
P=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
for r in 0 1; do
  IA_PEER_TRACE=1 IA_SHARD_MIN_ROWS=0 RANK=$r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$P timeout -k 10 120 python -u tools/exchange_debug.py > gpurun_out/xd_$r.log 2>&1 &
done
wait
cat gpurun_out/xd_0.log gpurun_out/xd_1.log | grep -v amdgpu.ids
