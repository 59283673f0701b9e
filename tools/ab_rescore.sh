#!/bin/bash
# A/B/A on c4: the exact stage's form at the 4.19 M-row finest level (IA_RESCORE unset =
# work list above 2^20 rows, 0 = per-query k_rescore everywhere)
set -o pipefail
mkdir -p gpurun_out
for v in def r0 def2 r0b; do
  if [ ${v:0:2} = r0 ]; then export IA_RESCORE=0; else unset IA_RESCORE; fi
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value']), round(d['ms_per_step'],1), 'frac', round(d['roofline']['frac'],4), d['checks']['checksum'])"
done
