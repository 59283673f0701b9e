cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ss8 -o ss -- python3 $GRAFT_REPO_ROOT/tools/shard_sim.py 8 > $GRAFT_REPO_ROOT/gpurun_out/ss8.txt 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/ss8.txt; exit 1; }
grep G= $GRAFT_REPO_ROOT/gpurun_out/ss8.txt
head -14 $GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_stats.csv | cut -d, -f1-4
python3 - "$GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_trace.csv" <<'PY'
import csv, sys, collections
import numpy as np
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name']
    if any(k in n for k in ('k_rescore', 'finish_gather', 'k_query_wave', 'copyBuffer', 'k_screen16iILi11')):
        d[n.split('(')[0][:40]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    print(k, len(v), 'p10 %.1f p50 %.1f p90 %.1f us' % tuple(np.percentile(np.array(v), [10, 50, 90])))
PY
rm -f $GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_trace.csv
