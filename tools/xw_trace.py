"""Phase breakdown of the fused per-wave kernel k_xwave (diagnostic).

Runs a bench.py workload's synthesis (or the simulated G-shard rank of tools/shard_sim.py
with --shards G) twice with IA_XW_TRACE=<level>, reads the phase stamps of the first 8
pixels of every wave of that level (ia_diag_xwave_trace: 100 MHz s_memrealtime) and prints
the median time of each phase over the plateau waves (the most queries) and over all.

usage: python tools/xw_trace.py [--config c4] [--level 5] [--shards G]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PHASES = ['ticket', 'e*', 'candidates', 're-screen', 'rescore(w0)', 'coherence+barrier',
          'exchange', 'update', 'neighbour', 'query build']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c4')
    ap.add_argument('--level', type=int, default=5)
    ap.add_argument('--shards', type=int, default=0)
    args = ap.parse_args()
    os.environ['IA_XW_TRACE'] = str(args.level)
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import bench
    _ia, ia = bench._ia, bench.ia
    job = bench.Job(bench.CONFIGS[args.config], 0, 'cuda:0')
    comm = None
    if args.shards:
        comm = [_ia.exchange(0, 1) for _ in range(job.max_levels)]
    for _ in range(2):
        job.step(comm, 0, args.shards or 1)
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8 * 16, dtype=np.uint64)
    _ia.check(_ia.lib().ia_diag_xwave_trace(buf.ctypes.data_as(ctypes.c_void_p)), 'ia_diag_xwave_trace')
    tr = buf.reshape(4096, 8, 16).astype(np.float64) * 0.01      # us
    have = (tr[:, :, 0] > 0) & (tr[:, :, 7] > 0) & (tr[:, :, 10] > 0)
    waves = np.nonzero(have.any(axis=1))[0]
    npx = have.sum(axis=1)
    plateau = waves[npx[waves] == 8]
    print('%s level %d%s: %d traced waves (%d with 8 traced pixels)' % (
        args.config, args.level, ' G=%d' % args.shards if args.shards else '', len(waves), len(plateau)))
    for name, sel in (('all', waves), ('8-px waves', plateau)):
        d = np.diff(tr[sel][:, :, :11], axis=2)          # (waves, px, 10)
        ok = have[sel]
        print(' %-10s' % name + ''.join(' %s %.2f' % (PHASES[k], np.median(d[:, :, k][ok]))
                                       for k in range(10)))
        tot = (tr[sel][:, :, 10] - tr[sel][:, :, 0])[ok]
        skew = (tr[sel][:, :, 0] - tr[sel][:, :1, 0])[ok]
        print('   start->end p10/p50/p90 %.1f / %.1f / %.1f us; start skew vs ticket-0 block p50 %.2f us'
              % (*np.percentile(tot, [10, 50, 90]), np.median(skew)))
    sub = tr[plateau][have[plateau]]
    def med(a, b):
        ok = (sub[:, a] > 0) & (sub[:, b] > 0)
        return np.median(sub[ok, b] - sub[ok, a]) if ok.any() else float('nan')
    print('   candidates->w0 window landed %.2f, ->w0 re-screen done %.2f, ->w1 coherence issued %.2f, '
          'B3->w2 rescore done %.2f, B3->w1 coherence done %.2f, ->B3 %.2f, ->B4 %.2f' % (
              med(3, 11), med(3, 12), med(3, 13), med(4, 14), med(4, 15), med(3, 4), med(4, 6)))
    print('   stamps 11-15 after the ticket (p50, us): ' + ' '.join(
        '%d:%.2f' % (k, med(1, k)) for k in range(11, 16)))
    for cm in comm or []:
        _ia.lib().ia_comm_destroy(cm)


if __name__ == '__main__':
    main()
