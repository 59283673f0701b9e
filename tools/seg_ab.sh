#!/bin/bash
# A/B of the segment cap (IA_SEG_MAX 512 vs 256): per-level c4 times, interleaved, one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for S in 512 256; do
    IA_SEG_MAX=$S timeout -k 10 120 python -u tools/level_times.py c4 > gpurun_out/seg_$S.txt 2>&1 || { tail -20 gpurun_out/seg_$S.txt; exit 1; }
    echo "seg $S: $(grep L1 gpurun_out/seg_$S.txt)"
  done
done
