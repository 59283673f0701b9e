#!/bin/bash
# The exchange tests, then bench ranks sharing the box's GPU over the device-side exchange
# (bench.py --gpus N with IA_SHARE_GPU=1): c3 with every level sharded (2 and 3 ranks) and
# c4 (2 ranks); the 1-rank checksums are c3 131623552.32391898, c4 2452528227.5270057.
# Then the 8-shard rank simulation.  A bench run that ends with a Python error (exit 1) is
# a result; any other failure stops the script.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_exchange.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_exch.log 2>&1 || { tail -40 gpurun_out/t_exch.log; exit 1; }
tail -1 gpurun_out/t_exch.log
run() {
  local tag=$1 n=$2 cfg=$3; shift 3
  env IA_SHARE_GPU=1 "$@" timeout -k 10 200 python -u bench.py --gpus $n --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sd_$tag.json 2> gpurun_out/sd_$tag.err
  local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/sd_$tag.json')); print(round(d['value']), round(d['ms_per_step'],1), d['checks'], d['config'].get('exchange'), d['config'].get('parallelism'))" 2>/dev/null) $(grep -o 'timed out' gpurun_out/sd_$tag.err | head -1)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run c3g2 2 c3 IA_SHARD_MIN_ROWS=0
run c3g3 3 c3 IA_SHARD_MIN_ROWS=0
run c4g2 2 c4
timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/ss_peer_split.txt 2>&1 || { tail -20 gpurun_out/ss_peer_split.txt; exit 1; }
grep G= gpurun_out/ss_peer_split.txt
