#!/bin/bash
# image-form exact stage: split16 / parity / configs tests, then c4 bench (default = image-only DB)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${IMGX_TESTS:-tests/test_gpu_split16.py tests/test_gpu_parity.py tests/test_gpu_configs.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/t_imgx.log 2>&1 || { tail -40 gpurun_out/t_imgx.log; exit 1; }
tail -2 gpurun_out/t_imgx.log
for v in 1 0; do
  IA_DB_IMAGE=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_imgx$v.json 2> gpurun_out/b_imgx$v.err || { tail -20 gpurun_out/b_imgx$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_imgx$v.json')); print('IA_DB_IMAGE=$v', round(d['ms_per_step'],1), 'ms/step', round(d['value']), 'px/s', round(d['roofline']['frac'],4), d['checks'], {k: (round(v['us'],1), round(v['frac'],3)) for k, v in d['hbm_kernels'].items()})"
done
