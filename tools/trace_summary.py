"""Summary of a rocprofv3 kernel trace (tools/gpu.sh trace): per kernel (template arguments
kept, parameters dropped) the launch count, total and p10 / p50 / p90 duration in us; then,
for the queue with the most launches, the median idle gap between consecutive kernels by
(kernel -> next kernel) pair.

usage: python tools/trace_summary.py run_kernel_trace.csv [top]
"""
import collections
import csv
import sys

import numpy as np


def name(k):
    k = k.split('(')[0]
    return k[:60]


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    rows = list(csv.DictReader(open(path)))
    dur = collections.defaultdict(list)
    by_q = collections.defaultdict(list)
    for r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        n = name(r['Kernel_Name'])
        dur[n].append((e - s) / 1e3)
        by_q[r.get('Queue_Id', r.get('Stream_Id', '0'))].append((s, e, n))
    print('%-62s %7s %10s %8s %8s %8s' % ('kernel', 'n', 'total_ms', 'p10_us', 'p50_us', 'p90_us'))
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:top]:
        a = np.array(v)
        p = np.percentile(a, [10, 50, 90])
        print('%-62s %7d %10.2f %8.1f %8.1f %8.1f' % (n, len(a), a.sum() / 1e3, p[0], p[1], p[2]))
    q, ks = max(by_q.items(), key=lambda kv: len(kv[1]))
    ks.sort()
    gaps = collections.defaultdict(list)
    for a, b in zip(ks, ks[1:]):
        gaps[a[2] + ' -> ' + b[2]].append((b[0] - a[1]) / 1e3)
    print('queue %s: %d launches' % (q, len(ks)))
    for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:8]:
        print('  gap %-90s n=%-6d p50 %.2f us' % (k, len(v), float(np.median(v))))


if __name__ == '__main__':
    main()
