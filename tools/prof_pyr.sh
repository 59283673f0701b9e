#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_pyr
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o pyr -- python3 "$R/tools/pyr_bench.py" > "$OUT/log.txt" 2>&1 || { tail -20 "$OUT/log.txt"; exit 1; }
python3 - "$OUT/pyr_kernel_trace.csv" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name'].split('(')[0]
    d[(n, r['Grid_Size_X'], r['Grid_Size_Y'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items()):
    v.sort()
    print('%-24s grid %6s x %-5s n %3d  median %7.1f us' % (k[0][:24], k[1], k[2], len(v), v[len(v) // 2]))
PY
