#!/bin/bash
# Same-box A/B of the level pipeline: off, and the (order, priority) forms; then PMC probes
set -o pipefail
mkdir -p gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$tag.json')); r=d['roofline']; print('$tag', round(d['ms_per_step'],1), 'ms/step', round(d['value']), r['kernel'], round(r['screen_avg_us'],1), round(r['frac'],4), 'finest', round(r['finest_level']['frac'],4), d['checks']['checksum'])"
}
for r in 1 2; do
  run seq IA_PIPELINE=0
  run lazy_noprio IA_PIPE_ORDER=0 IA_PIPE_PRIO=0
  run order_noprio IA_PIPE_ORDER=1 IA_PIPE_PRIO=0
  run lazy_prio IA_PIPE_ORDER=0 IA_PIPE_PRIO=1
  run order_prio IA_PIPE_ORDER=1 IA_PIPE_PRIO=1
done
cd /tmp && export TMPDIR=/tmp
for S in "stack" "bench"; do
  echo "=== pmc FETCH_SIZE probe: $S"
  if [ "$S" = bench ]; then
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcprobe2 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --config c1 > $GRAFT_REPO_ROOT/gpurun_out/pmcprobe.txt 2>&1
  else
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcprobe -o p -- python3 $GRAFT_REPO_ROOT/tools/pmc_probe.py fill clone stack libia > $GRAFT_REPO_ROOT/gpurun_out/pmcprobe.txt 2>&1
  fi
  rc=$?
  grep -E " ok$" $GRAFT_REPO_ROOT/gpurun_out/pmcprobe.txt | tr '\n' ' '; echo "exit $rc"
  if [ $rc -ne 0 ]; then grep -E "SIGSEGV|Abort|rror" $GRAFT_REPO_ROOT/gpurun_out/pmcprobe.txt | head -5; grep -E "^    @" $GRAFT_REPO_ROOT/gpurun_out/pmcprobe.txt | grep -v unknown | head -8; exit 0; fi
done
