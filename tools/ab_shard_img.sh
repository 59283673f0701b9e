#!/bin/bash
# Same-box A/B of the simulated G = 8 rank (tools/shard_sim.py) with the image-form DB
# (IA_DB_IMAGE=1: screen + exact stage from the image form, no row form) and the row form
set -o pipefail
for r in 1 2; do
  for V in 1 0; do
    IA_DB_IMAGE=$V timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/absi_$V.txt 2>&1 || { tail -5 gpurun_out/absi_$V.txt; exit 1; }
    echo "IA_DB_IMAGE=$V: $(grep G= gpurun_out/absi_$V.txt)"
  done
done
