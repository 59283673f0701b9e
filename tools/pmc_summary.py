"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel name, the mean of each
counter over its dispatches, plus the dispatch duration (ns)."""
import csv
import sys
from collections import defaultdict

def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r['Kernel_Name'].split('(')[0]
            acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
            dur[k][(p, r['Dispatch_Id'])] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    for k in acc:
        d = list(dur[k].values())
        print('%s  dispatches %d  mean duration %.1f us' % (k, len(d), sum(d) / len(d) / 1e3))
        for c, v in sorted(acc[k].items()):
            print('   %-28s %.4g' % (c, sum(v) / len(v)))

if __name__ == '__main__':
    main(sys.argv[1:])
