#!/bin/bash
# Same-box A/B of the sharded tail forms on the simulated G = 8 rank (tools/shard_sim.py)
set -o pipefail
for r in 1 2; do
  for T in 0 1; do
    IA_SHARD_TAIL=$T timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/abs_$T.txt 2>&1 || { tail -5 gpurun_out/abs_$T.txt; exit 1; }
    echo "tail $T: $(grep G= gpurun_out/abs_$T.txt)"
  done
done
