#!/bin/bash
# A/B of HIP-graph capture for small levels (IA_TARGET_CHUNKS default vs 512): per-level c4 times, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for G in 0 512; do
    IA_TARGET_CHUNKS=$G timeout -k 10 120 python -u tools/level_times.py c4 > gpurun_out/tc_$G.txt 2>&1 || { tail -20 gpurun_out/tc_$G.txt; exit 1; }
    echo "chunks $G: $(grep L1 gpurun_out/tc_$G.txt)"
  done
done
