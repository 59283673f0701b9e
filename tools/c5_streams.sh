#!/bin/bash
# c5 (batch of independent 512x512 jobs): jobs run 1, 4, 8 at a time on their own streams
set -o pipefail
mkdir -p gpurun_out
for JS in "4 1" "4 4" "8 8" "16 8"; do
  set -- $JS
  timeout -k 10 300 python -u bench.py --config c5 --jobs $1 --streams $2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$1_$2.json 2> gpurun_out/c5_$1_$2.err || { tail -20 gpurun_out/c5_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c5_$1_$2.json')); print('jobs $1 streams $2', round(d['value']), 'px/s', round(d['ms_per_step'],1), 'ms/step', d['checks'])"
done
