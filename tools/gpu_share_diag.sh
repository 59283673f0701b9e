#!/bin/bash
# Ranks sharing the box's GPU over the device-side exchange (bench.py --gpus N with
# IA_SHARE_GPU=1): c3 with every level sharded (2 and 3 ranks) and c4 (2 ranks), each
# against the 1-rank checksum; then the 8-shard rank simulation.  A run that ends with a
# Python error (exit 1) is a result; any other failure stops the script.
mkdir -p gpurun_out
run() {
  local tag=$1 n=$2 cfg=$3; shift 3
  env IA_SHARE_GPU=1 "$@" timeout -k 10 200 python -u bench.py --gpus $n --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sd_$tag.json 2> gpurun_out/sd_$tag.err
  local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/sd_$tag.json')); print(d['value'], d['ms_per_step'], d['checks'], d['config'].get('exchange'), d['config'].get('parallelism'))" 2>/dev/null) $(grep -o 'ia_peer_status failed' gpurun_out/sd_$tag.err | head -1)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run c3g1 1 c3 IA_SHARD_MIN_ROWS=0
run c3g2 2 c3 IA_SHARD_MIN_ROWS=0
run c3g3 3 c3 IA_SHARD_MIN_ROWS=0
run c4g1 1 c4
run c4g2 2 c4
timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/ss_peer_serial.txt 2>&1 || { tail -20 gpurun_out/ss_peer_serial.txt; exit 1; }
grep G= gpurun_out/ss_peer_serial.txt
