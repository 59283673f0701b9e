#!/bin/bash
# c2 (the reference's own LSH-vs-brute config, 180 x 117, kappa 5): the LSH matcher over a grid
# of (tables, hashes, width x RMS spread) against the exact matcher: px/s, the finest level's
# exact-match fraction and mean matched distance ratio (bench.py lsh_quality)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lshc2_brute.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/lshc2_brute.json').read().strip().splitlines()[-1]); print('brute: %.2f ms/step %.0f px/s' % (d['ms_per_step'], d['value']))"
for P in 16,4,1.0 16,4,2.0 32,2,1.0 32,2,2.0 64,1,1.0 64,1,2.0 16,2,2.0 8,1,4.0 32,1,4.0 16,1,8.0; do
  timeout -k 10 300 python -u bench.py --config c2 --matcher lsh --lsh $P --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lshc2_$P.json 2> gpurun_out/lshc2_$P.err || { tail -5 gpurun_out/lshc2_$P.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/lshc2_$P.json').read().strip().splitlines()[-1]); q=d['lsh_quality']; print('lsh %s: %.2f ms/step %.0f px/s exact %.3f dist ratio %.3f' % ('$P', d['ms_per_step'], d['value'], q['exact_frac'], q['mean_dist_ratio']))"
done
