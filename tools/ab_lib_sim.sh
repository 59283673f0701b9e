#!/bin/bash
# A/B/A/B of two libia.so builds (IA_LIB_PATH = the B build) on the simulated 8-shard rank
set -o pipefail
mkdir -p gpurun_out
B=$1
for v in a b a2 b2; do
  if [ ${v:0:1} = b ]; then export IA_LIB_PATH=$B; else unset IA_LIB_PATH; fi
  timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/ab_ss_$v.txt 2>&1 || { tail -20 gpurun_out/ab_ss_$v.txt; exit 1; }
  echo "$v $(grep G= gpurun_out/ab_ss_$v.txt)"
done
