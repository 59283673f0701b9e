"""Per hardware queue of a rocprofv3 kernel trace: which kernels it ran, their durations, and
the idle time between consecutive dispatches on it (the dual-queue study).
For the finest level of a c1-style run it also pairs each screen (the widest k_screen16
grids) with the k_xwave that follows it and prints the hand-over times.

usage: python tools/trace_queues.py run_kernel_trace.csv
"""
import collections
import csv
import sys

import numpy as np


def short(k):
    return k.split('(')[0][:48]


def pct(v):
    a = np.asarray(v, dtype=float)
    if a.size == 0:
        return 'n=0'
    p = np.percentile(a, [10, 50, 90])
    return 'n=%-5d p10 %7.1f p50 %7.1f p90 %7.1f mean %7.1f' % (a.size, p[0], p[1], p[2], a.mean())


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = []
    for r in rows:
        ks.append(dict(q=r.get('Queue_Id', '?'), s=int(r['Start_Timestamp']) / 1e3,
                       e=int(r['End_Timestamp']) / 1e3, n=short(r['Kernel_Name']),
                       g=int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0)))
    ks.sort(key=lambda k: k['s'])
    byq = collections.defaultdict(list)
    for k in ks:
        byq[k['q']].append(k)
    for q, v in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        names = collections.Counter(k['n'] for k in v)
        gaps = [b['s'] - a['e'] for a, b in zip(v, v[1:])]
        print('queue %s: %d dispatches; gap %s' % (q, len(v), pct(gaps)))
        for n, c in names.most_common(4):
            print('   %-48s %6d  dur %s' % (n, c, pct([k['e'] - k['s'] for k in v if k['n'] == n])))
    scr = [k for k in ks if 'k_screen16I' in k['n'] or 'k_screen16<' in k['n']]
    if not scr:
        return
    gmax = max(k['g'] for k in scr)
    fs = [k for k in scr if k['g'] == gmax]
    xw = [k for k in ks if 'k_xwave' in k['n']]
    qs = collections.Counter(k['q'] for k in fs).most_common(1)[0][0]
    fs = [k for k in fs if k['q'] == qs]
    # the finest level's fused kernels: the queue most of the k_xwave launches right after a
    # finest screen ran on
    nxt = []
    j = 0
    for k in fs:
        while j < len(xw) and xw[j]['s'] < k['s']:
            j += 1
        cand = [x for x in xw[j:j + 8] if x['e'] > k['e']]
        nxt.append(cand[0] if cand else None)
    qx = collections.Counter(x['q'] for x in nxt if x).most_common(1)[0][0]
    tails = [x for x in xw if x['q'] == qx]
    print('finest screens (grid %d) on queue %s: %d; fused kernels on queue %s: %d' % (gmax, qs, len(fs), qx, len(tails)))
    # pair screen t with the first fused kernel on qx that ENDS after it (the one that waited)
    pairs = []
    j = 0
    for k in fs:
        while j < len(tails) and tails[j]['e'] <= k['e']:
            j += 1
        if j < len(tails):
            pairs.append((k, tails[j]))
    print('screen duration           ', pct([s['e'] - s['s'] for s, _ in pairs]))
    print('fused duration            ', pct([x['e'] - x['s'] for _, x in pairs]))
    print('fused start - screen end  ', pct([x['s'] - s['e'] for s, x in pairs]))
    print('fused end - screen end    ', pct([x['e'] - s['e'] for s, x in pairs]))
    print('next screen start - fused end', pct([b[0]['s'] - a[1]['e'] for a, b in zip(pairs, pairs[1:])]))
    print('screen-to-screen period   ', pct([b[0]['s'] - a[0]['s'] for a, b in zip(pairs, pairs[1:])]))
    # per step (finest screens more than 2 ms apart start a new step): the warmup, the timed
    # steps and bench.py's events pass (HIP events between the kernels) separately
    steps = [[fs[0]]]
    for a, b in zip(fs, fs[1:]):
        if b['s'] - a['s'] > 2000:
            steps.append([])
        steps[-1].append(b)
    for i, st in enumerate(steps):
        per = np.array([b['s'] - a['s'] for a, b in zip(st, st[1:])])
        print('step %d: finest level %.2f ms, %d waves, wave period p50 %.1f us, %d periods > 60 us' %
              (i, (st[-1]['e'] - st[0]['s']) / 1e3, len(st), float(np.median(per)), int((per > 60).sum())))


if __name__ == '__main__':
    main()
