#!/bin/bash
# The exchange tests, then the whole GPU suite, the default bench, the shard simulation
# with both exchange forms and a 2-rank c3 bench whose ranks share the box's GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_exchange.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_exch.log 2>&1 || { tail -40 gpurun_out/t_exch.log; exit 1; }
tail -1 gpurun_out/t_exch.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/b_def.json 2> gpurun_out/b_def.err || { tail -20 gpurun_out/b_def.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_def.json')); print('c4', round(d['value']), round(d['ms_per_step'],1), 'ms/step frac', round(d['roofline']['frac'],4))"
for K in rccl peer; do
  IA_EXCHANGE=$K timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/ss_$K.txt 2>&1 || { tail -20 gpurun_out/ss_$K.txt; exit 1; }
  grep G= gpurun_out/ss_$K.txt
done
IA_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --config c3 --steps 2 --warmup 1 > gpurun_out/b_c3_g2.json 2> gpurun_out/b_c3_g2.err || { tail -20 gpurun_out/b_c3_g2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_c3_g1.json 2> gpurun_out/b_c3_g1.err || { tail -20 gpurun_out/b_c3_g1.err; exit 1; }
python3 - <<'PY'
import json
a = json.load(open('gpurun_out/b_c3_g1.json')); b = json.load(open('gpurun_out/b_c3_g2.json'))
print('c3 g1 checksum', a['checks']['checksum'], 'g2 checksum', b['checks']['checksum'], 'replicas', b['checks']['replicas_identical'], b['config'].get('exchange'))
PY
