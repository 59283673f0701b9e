#!/bin/bash
# Screen forms at the per-rank DB sizes of the sharded c4 finest level (G = 8, 4, 2:
# A = 724, 1024, 1448 -> 0.52 M, 1.05 M, 2.10 M rows), h16s (0x20007) vs the default (chain-balanced where it applies),
# at two chunk counts.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
make -C "$R/tools" screen_bench > /dev/null
for TC in 1024 512; do
  for A in 724 1024 1448; do
    echo "== chunks $TC A $A"
    IA_TARGET_CHUNKS=$TC timeout -k 10 120 "$R/tools/screen_bench" --A $A --M 342,256,171 --variants 0x20007,0x007 --reps 3 --rounds 3
  done
done
