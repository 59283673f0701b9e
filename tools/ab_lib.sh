#!/bin/bash
# A/B/A/B on c4 of two builds of libia.so (IA_LIB_PATH = the B build), then the simulated
# 8-shard rank with each: bash tools/ab_lib.sh /root/repo/_ab/libia_old.so
set -o pipefail
mkdir -p gpurun_out
B=$1
for v in a b a2 b2; do
  if [ ${v:0:1} = b ]; then export IA_LIB_PATH=$B; else unset IA_LIB_PATH; fi
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', 'B' if '$v'[0] == 'b' else 'A', round(d['value']), round(d['ms_per_step'],1), 'frac', round(d['roofline']['frac'],4), d['checks']['checksum'])"
done
for v in a b; do
  if [ $v = b ]; then export IA_LIB_PATH=$B; else unset IA_LIB_PATH; fi
  timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/ab_ss_$v.txt 2>&1 || { tail -20 gpurun_out/ab_ss_$v.txt; exit 1; }
  echo "$v $(grep G= gpurun_out/ab_ss_$v.txt)"
done
