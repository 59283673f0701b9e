"""Phase breakdown of the fused per-wave kernel k_xwave (diagnostic).

Runs a bench.py workload's synthesis (or the simulated G-shard rank of tools/shard_sim.py
with --shards G) twice with IA_XW_TRACE=<level>, reads the phase stamps of every pixel of
every wave of that level (ia_diag_xwave_trace: 100 MHz s_memrealtime; slot 16: the pixel's
candidate segment count) and prints the median time of each phase over the first 8 pixels
of the plateau waves (the most queries) and over all, then the per-wave span (first
pixel's start to last pixel's end) against the slowest pixel's candidate count.

usage: python tools/xw_trace.py [--config c4] [--level 5] [--shards G]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PHASES = ['ticket', 'e*', 'candidates', 're-screen', 'rescore(w0)', 'coherence+barrier',
          'exchange', 'update', 'neighbour', 'query build']


def wave_profile(full):
    """per wave: span = last end - first start over ALL its pixels; the slowest pixel's
    candidate segments; the p50 pixel's start->end"""
    import numpy as np
    st = full[:, :, 0].astype(np.float64) * 0.01
    en = full[:, :, 10].astype(np.float64) * 0.01
    ns = full[:, :, 16].astype(np.int64)
    ok = (full[:, :, 0] > 0) & (full[:, :, 10] > 0)
    npx = ok.sum(1)
    waves = np.nonzero(npx >= max(npx.max() // 2, 1))[0]   # the plateau-ish waves
    if not len(waves):
        return
    span, slow, slow_ns, p50, mx_ns, startsk = [], [], [], [], [], []
    for t in waves:
        o = ok[t]
        s0, e0, n0 = st[t][o], en[t][o], ns[t][o]
        span.append(e0.max() - s0.min())
        j = np.argmax(e0)
        slow.append(e0[j] - s0[j])
        slow_ns.append(n0[j])
        mx_ns.append(n0.max())
        p50.append(np.median(e0 - s0))
        startsk.append(np.percentile(s0 - s0.min(), 90))
    span, slow, slow_ns, p50, mx_ns = map(np.array, (span, slow, slow_ns, p50, mx_ns))
    print('per wave over all pixels (%d waves with >= %d pixels): span p50 %.1f us (p10 %.1f, p90 %.1f); '
          'slowest pixel start->end p50 %.1f us; median pixel %.1f us; start spread p90 %.1f us' % (
              len(waves), max(npx.max() // 2, 1), np.median(span), np.percentile(span, 10),
              np.percentile(span, 90), np.median(slow), np.median(p50), np.median(startsk)))
    allns = ns[ok]
    print('candidate segments per pixel: mean %.3f; per wave max: mean %.2f; the slowest pixel\'s: mean %.2f' % (
        allns.mean(), mx_ns.mean(), slow_ns.mean()))
    for k in range(1, 8):
        sel = slow_ns == k
        if sel.any():
            print('  slowest pixel with %d segments: %4d waves, its start->end p50 %.1f us, span p50 %.1f us' % (
                k, sel.sum(), np.median(slow[sel]), np.median(span[sel])))
    for k in range(1, 8):
        sel = (allns == k)
        if sel.any():
            d = (en - st)[ok][sel]
            print('  pixels with %d segments: %6d, start->end p50 %.1f us' % (k, sel.sum(), np.median(d)))


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
    T, PX, N = 4096, 512, 17
    buf = np.zeros(T * PX * N, dtype=np.uint64)
    _ia.check(_ia.lib().ia_diag_xwave_trace(buf.ctypes.data_as(ctypes.c_void_p)), 'ia_diag_xwave_trace')
    full = buf.reshape(T, PX, N)
    wave_profile(full)
    tr = full[:, :8, :16].astype(np.float64) * 0.01      # us
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
