#!/bin/bash
# Kernel trace of the simulated 8-shard rank (tools/shard_sim.py 8) on one GPU.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_shard
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g8" -o g8 -- \
    python3 "$R/tools/shard_sim.py" ${1:-8} > "$OUT/g8.txt" 2>&1
cat "$OUT/g8.txt" | grep "G="
python3 - "$OUT/g8/g8_kernel_trace.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the finest level of the last repetition: the last 4093 k_query_wave dispatches onward
qi = [i for i, r in enumerate(rows) if 'k_query_wave' in r['Kernel_Name']]
start = qi[-4093]
sel = rows[start:]
t0, t1 = int(sel[0]['Start_Timestamp']), int(sel[-1]['End_Timestamp'])
busy = collections.Counter(); cnt = collections.Counter()
for r in sel:
    n = r['Kernel_Name'].split('(')[0][:60]
    busy[n] += int(r['End_Timestamp']) - int(r['Start_Timestamp']); cnt[n] += 1
tot = sum(busy.values())
print('finest level span %.1f ms, kernel busy %.1f ms, idle %.1f ms' % ((t1 - t0) / 1e6, tot / 1e6, (t1 - t0 - tot) / 1e6))
for n, b in busy.most_common():
    print('  %-60s %6d  %8.1f us avg  %7.1f ms' % (n, cnt[n], b / cnt[n] / 1e3, b / 1e6))
PY
