#!/bin/bash
# One bench line per non-default config (c1, c2 brute + LSH, c3, c5), N = 1
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { tail -20 gpurun_out/b_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_$tag.json')); print('$tag', round(d['value']), d['unit'], round(d['ms_per_step'],1), 'ms/step', d['checks'])"
}
run c1 --config c1
run c2 --config c2
run c2_lsh --config c2 --matcher lsh
run c3 --config c3
run c5 --config c5
