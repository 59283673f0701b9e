"""Per-launch HBM traffic of the screen kernel k_screen16<G> from rocprofv3 PMC passes of
bench.py (tools/gpu.sh traffic): FETCH_SIZE (KB, doubled on gfx950: MI355X_MICROARCH.md
§HBM) + WRITE_SIZE (KB), averaged over the dominant instance's dispatches, as JSON.

    python tools/pmc_traffic.py fetch.csv write.csv"""
import csv
import json
import os
import sys

from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] == counter and 'k_screen16' in r['Kernel_Name']:
            per[r['Kernel_Name']].append((float(r['Counter_Value']),
                                          int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
    return per


def screen_src_sha1():
    import hashlib
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        'image-analogies-python_amd', 'csrc')
    h = hashlib.sha1()
    for f in ('ia_screen16.hip', 'ia_split16.h', 'ia_imgwin.h', 'ia_internal.h', 'ia_screen16r.hip', 'ia_rot16.h'):
        h.update(open(os.path.join(root, f), 'rb').read())
    return h.hexdigest()


def main(fetch_csv, write_csv):
    f, w = load(fetch_csv, 'FETCH_SIZE'), load(write_csv, 'WRITE_SIZE')
    dom = max(f, key=lambda k: sum(d for _, d in f[k]))
    fk = sum(v for v, _ in f[dom]) / len(f[dom])
    wk = sum(v for v, _ in w[dom]) / len(w[dom])
    print(json.dumps({'kernel': dom, 'dispatches': len(f[dom]),
                      'fetch_kb': fk, 'write_kb': wk,
                      'traffic_bytes': (2 * fk + wk) * 1024,
                      'screen_src_sha1': screen_src_sha1(),
                      'note': 'FETCH_SIZE x 2 (gfx950) + WRITE_SIZE, mean per dispatch, from '
                              'PMC passes of bench.py'}, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:3])
