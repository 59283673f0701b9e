#!/bin/bash
# A/B of the current tree against a second built tree (_ab_old/, a git worktree): GPU tests
# on the current tree, then interleaved c4 per-level times and the simulated 8-shard rank.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
for r in 1 2; do
  for T in . _ab_old; do
    timeout -k 10 120 python -u $T/tools/level_times.py c4 > gpurun_out/lt_ab.txt 2>&1 || { tail -20 gpurun_out/lt_ab.txt; exit 1; }
    echo "$T: $(grep L1 gpurun_out/lt_ab.txt)"
  done
done
for T in . _ab_old; do
  timeout -k 10 120 python -u $T/tools/shard_sim.py 8 > gpurun_out/ss_ab.txt 2>&1 || { tail -20 gpurun_out/ss_ab.txt; exit 1; }
  echo "$T: $(grep G= gpurun_out/ss_ab.txt)"
done
