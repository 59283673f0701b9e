#!/bin/bash
# A/B/A/B on c4 of one environment knob: bash tools/ab_knob.sh VAR VALUE
set -o pipefail
mkdir -p gpurun_out
VAR=$1; VAL=$2
for v in a b a2 b2; do
  if [ ${v:0:1} = b ]; then export $VAR=$VAL; else unset $VAR; fi
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', '$VAR=' + ('$VAL' if '$v'[0] == 'b' else 'default'), round(d['value']), round(d['ms_per_step'],1), 'frac', round(d['roofline']['frac'],4), d['checks']['checksum'])"
done
