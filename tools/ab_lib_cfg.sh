#!/bin/bash
# A/B/A/B of two libia.so builds (IA_LIB_PATH = the B build) on several configs:
#   bash tools/ab_lib_cfg.sh /root/repo/_ab/libia_x.so c3 c5 c4
set -o pipefail
mkdir -p gpurun_out
B=$1; shift
for c in "$@"; do
  for v in a b a2 b2; do
    if [ ${v:0:1} = b ]; then export IA_LIB_PATH=$B; else unset IA_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --config $c --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${c}_$v.json 2> gpurun_out/ab_${c}_$v.err || { tail -20 gpurun_out/ab_${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${c}_$v.json')); print('$c', '$v', 'B' if '$v'[0] == 'b' else 'A', round(d['value']), round(d['ms_per_step'],2), d['checks']['checksum'])"
  done
done
