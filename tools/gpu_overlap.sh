#!/bin/bash
# Sharded levels overlapping (IA_SHARD_OVERLAP=1) with the split device-side exchange:
# the simulated 8-shard rank both ways, then 2 and 3 bench ranks sharing the GPU.
mkdir -p gpurun_out
for o in 0 1; do
  IA_SHARD_OVERLAP=$o timeout -k 10 300 python -u tools/shard_sim.py 8 > gpurun_out/ss_ov$o.txt 2>&1 || { tail -20 gpurun_out/ss_ov$o.txt; exit 1; }
  echo "overlap=$o $(grep G= gpurun_out/ss_ov$o.txt)"
done
run() {
  local tag=$1 n=$2 cfg=$3; shift 3
  env IA_SHARE_GPU=1 IA_SHARD_OVERLAP=1 "$@" timeout -k 10 200 python -u bench.py --gpus $n --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ov_$tag.json 2> gpurun_out/ov_$tag.err
  local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ov_$tag.json')); print(round(d['value']), round(d['ms_per_step'],1), d['checks']['checksum'], d['config'].get('exchange'))" 2>/dev/null) $(grep -o 'timed out' gpurun_out/ov_$tag.err | head -1)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run c4g2 2 c4
run c3g2 2 c3 IA_SHARD_MIN_ROWS=0
run c3g3 3 c3 IA_SHARD_MIN_ROWS=0
