#!/bin/bash
# Round-end run: GPU tests, the default c4 bench (with the CPU baseline), the rocprof round
# profile (tools/prof_c4.sh), then one bench line per other config.
set -o pipefail
mkdir -p gpurun_out
bash tools/verify_round.sh || exit 1
for C in c1 c3 c5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline > gpurun_out/b_$C.json 2> gpurun_out/b_$C.err || { tail -20 gpurun_out/b_$C.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b_$C.json')); print('$C', round(d['value']), d['unit'], round(d['ms_per_step'],1), 'ms/step')"
done
