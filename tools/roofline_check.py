"""Cross-check bench.py's roofline against a rocprofv3 kernel trace of the same command.

    python tools/roofline_check.py <kernel_trace.csv> [bench.json]

The trace is split into levels at every k_db_build dispatch (one per level and step); the
levels with the most screen dispatches are the finest level of each step.  Prints the mean
duration of the finest level's screen dispatches (k_screen*), which bench.py's
``roofline.screen_avg_us`` (HIP events around the same launches) must agree with.
"""
import csv
import json
import sys


def main(trace, bench=None):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r['Start_Timestamp']))
    # the dominant screen instance (k_screen16<G> with the most total time)
    tot = {}
    for r in rows:
        n = r['Kernel_Name']
        if 'k_screen16' in n:
            d = tot.setdefault(n, [0, 0])
            d[0] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            d[1] += 1
    if tot:
        dom = max(tot, key=lambda n: tot[n][0])
        print('dominant kernel %s: %d dispatches, mean duration %.1f us'
              % (dom, tot[dom][1], tot[dom][0] / tot[dom][1] / 1e3))
    levels, cur = [], None
    for r in rows:
        name = r['Kernel_Name']
        if 'k_db_build' in name:
            cur = []
            levels.append(cur)
        elif cur is not None and 'k_screen' in name:
            cur.append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    nmax = max(len(l) for l in levels)
    fin = [d for l in levels if len(l) == nmax for d in l]
    print('levels traced: %d; finest level: %d segments x %d screen dispatches; '
          'mean duration %.1f us' % (len(levels), sum(len(l) == nmax for l in levels), nmax,
                                     sum(fin) / len(fin) / 1e3))
    if bench:
        b = json.loads(open(bench).read().strip().splitlines()[-1])
        print('bench.py roofline (%s) screen_avg_us (HIP events): %.1f us'
              % (b['roofline']['kernel'], b['roofline']['screen_avg_us']))


if __name__ == '__main__':
    main(*sys.argv[1:])
