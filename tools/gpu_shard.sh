#!/bin/bash
# Shard simulation (8 shards, rank 0) with both exchange forms, then a 2-rank c3 bench whose
# ranks share the box's GPU against the 1-rank c3 bench (same checksum).
set -o pipefail
mkdir -p gpurun_out
for K in peer rccl; do
  IA_EXCHANGE=$K timeout -k 10 300 python -u tools/shard_sim.py 1 8 > gpurun_out/ss_$K.txt 2>&1 || { tail -20 gpurun_out/ss_$K.txt; exit 1; }
  grep G= gpurun_out/ss_$K.txt
done
IA_SHARE_GPU=1 IA_SHARD_MIN_ROWS=0 timeout -k 10 300 python -u bench.py --gpus 2 --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_c3_g2.json 2> gpurun_out/b_c3_g2.err || { tail -20 gpurun_out/b_c3_g2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_c3_g1.json 2> gpurun_out/b_c3_g1.err || { tail -20 gpurun_out/b_c3_g1.err; exit 1; }
python3 - <<'PY'
import json
a = json.load(open('gpurun_out/b_c3_g1.json')); b = json.load(open('gpurun_out/b_c3_g2.json'))
print('c3 g1', a['checks']['checksum'], a['value'], 'g2', b['checks']['checksum'], b['value'], 'replicas', b['checks']['replicas_identical'], b['config'].get('exchange'), b['config'].get('parallelism'))
PY
IA_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_c4_g2.json 2> gpurun_out/b_c4_g2.err || { tail -20 gpurun_out/b_c4_g2.err; exit 1; }
python3 -c "import json; b=json.load(open('gpurun_out/b_c4_g2.json')); print('c4 g2 shared', b['checks'], b['value'], b['ms_per_step'], b['config'].get('exchange'))"
