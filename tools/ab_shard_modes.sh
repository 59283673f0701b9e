#!/bin/bash
# Same-box A/B of the simulated G = 8 rank (tools/shard_sim.py 8, image-form DB): exact-stage
# form (IA_RESCORE 0 = per-query k_rescore, 1 = work list) x sharded tail (IA_SHARD_TAIL)
set -o pipefail
for r in 1 2; do
  for RM in 0 1; do
    for T in 0 1; do
      IA_RESCORE=$RM IA_SHARD_TAIL=$T timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/absm.txt 2>&1 || { tail -5 gpurun_out/absm.txt; exit 1; }
      echo "IA_RESCORE=$RM IA_SHARD_TAIL=$T: $(grep G= gpurun_out/absm.txt)"
    done
  done
done
