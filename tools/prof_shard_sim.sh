# rocprofv3 kernel trace of the simulated 8-shard rank (tools/shard_sim.py 8, levels one at
# a time then pipelined): per-kernel duration percentiles of the per-wave kernels, and the
# idle gaps between consecutive kernels on the finest level's stream.
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ss8 -o ss -- python3 $GRAFT_REPO_ROOT/tools/shard_sim.py 8 > $GRAFT_REPO_ROOT/gpurun_out/ss8.txt 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/ss8.txt; exit 1; }
grep G= $GRAFT_REPO_ROOT/gpurun_out/ss8.txt
head -14 $GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_stats.csv | cut -d, -f1-4
python3 - "$GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_trace.csv" <<'PY'
import csv, sys, collections
import numpy as np
d = collections.defaultdict(list)
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r['Kernel_Name']
    if any(k in n for k in ('k_rescore', 'finish_gather', 'k_peer_finish', 'k_query_wave', 'copyBuffer', 'k_screen16iILi11', 'k_gather', 'k_items', 'k_select')):
        d[n.split('(')[0][:40]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    print(k, len(v), 'p10 %.1f p50 %.1f p90 %.1f us' % tuple(np.percentile(np.array(v), [10, 50, 90])))
# the finest level's waves run one after the other on one queue: gaps between consecutive
# kernels of the k_screen16i<11> .. next k_screen16i<11> period
by_q = collections.defaultdict(list)
for r in rows:
    by_q[r.get('Queue_Id', r.get('Stream_Id', '0'))].append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0][:30]))
for q, ks in by_q.items():
    ks.sort()
    idx = [i for i, k in enumerate(ks) if 'k_screen16iILi11' in k[2]]
    if len(idx) < 100:
        continue
    per = np.diff([ks[i][0] for i in idx]) / 1e3
    gaps = collections.defaultdict(list)
    for a, b in zip(ks[idx[len(idx)//2]:], ks[idx[len(idx)//2] + 1:]):
        pass
    seg = ks[idx[len(idx)//3]: idx[2*len(idx)//3]]
    for a, b in zip(seg, seg[1:]):
        gaps[a[2] + ' -> ' + b[2]].append((b[0] - a[1]) / 1e3)
    print('queue', q, 'screen<11> period p50 %.1f us over %d waves' % (np.median(per), len(per)))
    for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:8]:
        print('  gap', k, len(v), 'p50 %.1f us' % np.median(v))
PY
rm -f $GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_trace.csv
