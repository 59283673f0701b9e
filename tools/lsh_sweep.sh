#!/bin/bash
# c4 with the LSH matcher over a few (tables, hashes, width) settings: speed vs quality
set -o pipefail
mkdir -p gpurun_out
for P in 16,4,1.0 16,4,2.0 32,2,1.0; do
  timeout -k 10 300 python -u bench.py --config c4 --matcher lsh --lsh $P --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lsh_$P.json 2> gpurun_out/lsh_$P.err || { tail -5 gpurun_out/lsh_$P.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/lsh_$P.json')); q=d['lsh_quality']; print('lsh $P: %.1f ms/step %.0f px/s exact %.3f dist ratio %.3f' % (d['ms_per_step'], d['value'], q['exact_frac'], q['mean_dist_ratio']))"
done
