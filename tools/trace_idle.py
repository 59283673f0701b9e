"""GPU idle time in a rocprofv3 kernel trace: the union of all kernel intervals against the
trace's span, and every idle gap longer than a threshold with the kernels on either side
(host-side synchronisations and host work between launches show up as such gaps).

usage: python tools/trace_idle.py run_kernel_trace.csv [min_gap_us=300] [max_listed=40]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0
    nmax = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    ks = sorted((int(r['Start_Timestamp']) / 1e3, int(r['End_Timestamp']) / 1e3,
                 r['Kernel_Name'].split('(')[0][:44]) for r in csv.DictReader(open(path)))
    t0 = ks[0][0]
    busy, gaps = 0.0, []
    cs, ce, last = ks[0][0], ks[0][1], ks[0][2]
    for s, e, n in ks[1:]:
        if s > ce:
            busy += ce - cs
            if s - ce > thr:
                gaps.append(((ce - t0) / 1e3, (s - ce) / 1e3, last, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        if e >= ce:
            last = n
    busy += ce - cs
    span = ce - t0
    print('span %.1f ms, GPU busy %.1f ms (%.1f %%), %d gaps > %.0f us totalling %.1f ms' %
          (span / 1e3, busy / 1e3, 100 * busy / span, len(gaps), thr, sum(g[1] for g in gaps)))
    kinds = collections.Counter((g[2], g[3]) for g in gaps)
    print('gap kinds (before -> after: count, total ms):')
    for (a, b), c in kinds.most_common(12):
        tot = sum(g[1] for g in gaps if (g[2], g[3]) == (a, b))
        print('   %-44s -> %-44s %5d %8.2f' % (a, b, c, tot))
    for g in gaps[:nmax]:
        print('   at %9.2f ms: %7.2f ms idle, %s -> %s' % g)


if __name__ == '__main__':
    main()
