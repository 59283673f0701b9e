"""Image-form screen timing on c4's finest level (the product's dominant kernel,
k_screen16i<G> in strip order over the 4,194,304-row DB) for each stage schedule
(ia_diag_set_screen_sched), at M queries taken from tests/golden/c4_queries.npz; checks
that every schedule gives the same segment minima bit for bit.

  python tools/screen_img_bench.py [--M 342,256,128] [--reps 20] [--forms s0,s1,pc]
  (s0 / s1: k_screen16i with the tile-major / chain-major stage; pc: k_screen16p)
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'image-analogies-python_amd'))
sys.path.insert(0, ROOT)

import _ia            # noqa: E402
import algorithms     # noqa: E402
import bench          # noqa: E402
import config as cfg  # noqa: E402
import img_preprocess as ip  # noqa: E402

F16_PEAK = 4096.0 * 256 * 2.4e9 / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--M', default='342,256,128')
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--forms', default='s0,s1,pc')
    ap.add_argument('--trace', action='store_true',
                    help='k_screen16p stage stamps (ia_diag_screen_trace) for the last M: per-stage '
                         'phase medians of blocks 0 and 300 in shader cycles')
    args = ap.parse_args()
    Ms = [int(x) for x in args.M.split(',')]
    forms = args.forms.split(',')
    dev = torch.device('cuda', 0)
    job = bench.Job(bench.CONFIGS['c4'], 0, dev)
    A_pyr = ip.gaussian_pyramid_dev(job.A, cfg.n_sm, job.levels)
    Ap_pyr = ip.gaussian_pyramid_dev(job.Ap, cfg.n_sm, job.levels)
    level = job.max_levels - 1
    idx = algorithms.level_index(A_pyr, [Ap_pyr], level)
    assert idx.dbi is not None
    lib = _ia.lib()
    N = idx.nrows
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'c4_queries.npz'))
    Mmax = max(Ms)
    Q = np.asarray(g['q'][:Mmax], dtype=np.float64)
    qrows = lib.ia_diag_qp_rows(Mmax)
    q64 = torch.zeros((Mmax, _ia.IA_DP), dtype=torch.float64, device=dev)
    q64[:, :55] = torch.as_tensor(Q).to(dev)
    qp = torch.zeros((qrows, _ia.IA_DP), dtype=torch.float32, device=dev)
    q16 = torch.zeros((qrows, 256), dtype=torch.float16, device=dev)
    nq = torch.zeros(qrows, dtype=torch.float64, device=dev)
    st = _ia.stream()
    _ia.check(lib.ia_diag_query_rows16(_ia.ptr(q64), Mmax, _ia.ptr(idx.center), _ia.ptr(idx.amax),
                                       _ia.ptr(qp), _ia.ptr(q16), _ia.ptr(nq), st), 'query rows')
    nseg = lib.ia_db_rows_padded(N) // min(lib.ia_db_chunk_rows(N), 512)
    ref = {}
    prev = lib.ia_diag_set_screen_sched(-1)
    prev_pc = lib.ia_diag_set_screen_pc(-1)
    for M in Ms:
        for sc in forms:
            lib.ia_diag_set_screen_sched(1 if sc == 's1' else 0)
            lib.ia_diag_set_screen_pc(1 if sc == 'pc' else 0)
            segmin = torch.full((qrows, nseg), float('nan'), dtype=torch.float32, device=dev)

            def run():
                _ia.check(lib.ia_diag_screen16_image(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.dbi),
                                                     _ia.ptr(q16), M, _ia.ptr(segmin), st), 'screen')
            run()
            torch.cuda.synchronize()
            key = segmin[:M].view(torch.int32).clone()
            same = None
            if M in ref:
                same = bool(torch.equal(ref[M], key))
            else:
                ref[M] = key
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            med = ts[len(ts) // 2]
            pairs = float(M) * N
            print('M %3d %s: median %7.1f us  min %7.1f us  pipe_frac %.3f  frac %.3f  same_minima %s'
                  % (M, sc, med, ts[0], 330 * pairs / (med * 1e-6) / 1e12 / F16_PEAK,
                     110 * pairs / (med * 1e-6) / 1e12 / F16_PEAK, same), flush=True)
    if args.trace:
        lib.ia_diag_set_screen_sched(0)
        lib.ia_diag_set_screen_pc(1)
        tr = torch.zeros(16 * 256, dtype=torch.int64, device=dev)
        _ia.check(lib.ia_diag_screen_trace(_ia.ptr(tr)), 'trace on')
        for M in Ms:
            segmin = torch.empty((qrows, nseg), dtype=torch.float32, device=dev)
            for _ in range(3):
                tr.zero_()
                _ia.check(lib.ia_diag_screen16_image(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.dbi),
                                                     _ia.ptr(q16), M, _ia.ptr(segmin), st), 'screen')
                torch.cuda.synchronize()
            t = tr.view(2, 8, 64, 4).cpu().numpy().astype(np.float64)
            for blk in range(2):
                mf, ex = t[blk, :4], t[blk, 4:]
                ok = (mf[:, 1:63, 0] > 0).all() and (ex[:, 1:62, 0] > 0).all()
                if not ok:
                    print('trace block %d: incomplete' % blk)
                    continue
                s_ = slice(4, 60)
                wait_m = np.median(mf[:, s_, 1] - mf[:, s_, 0])        # MFMA waves at the barrier
                mfma = np.median(mf[:, s_, 3] - mf[:, s_, 1])          # MFMAs + folds + close
                close = 0.0
                period = np.median(np.diff(mf[:, 4:61, 1], axis=1))    # stage period
                wait_x = np.median(ex[:, s_, 1] - ex[:, s_, 0])
                work_x = np.median(ex[:, s_, 2] - ex[:, s_, 1])
                vm_x = np.median(ex[:, s_, 3] - ex[:, s_, 2])
                print('M %3d block %d (cycles, median over stages 4-59): period %.0f | MFMA waves: '
                      'barrier wait %.0f, MFMAs %.0f, close %.0f | expanders: barrier wait %.0f, '
                      'copies+operand %.0f, copy wait %.0f' % (M, 300 * blk, period, wait_m, mfma, close,
                                                              wait_x, work_x, vm_x), flush=True)
                for w in range(4):
                    print('   MFMA wave %d: wait %.0f mfma+close %.0f | expander %d: wait %.0f work %.0f '
                          'copy wait %.0f' % (w, np.median(mf[w, s_, 1] - mf[w, s_, 0]),
                                              np.median(mf[w, s_, 3] - mf[w, s_, 1]), w,
                                              np.median(ex[w, s_, 1] - ex[w, s_, 0]),
                                              np.median(ex[w, s_, 2] - ex[w, s_, 1]),
                                              np.median(ex[w, s_, 3] - ex[w, s_, 2])), flush=True)
        _ia.check(lib.ia_diag_screen_trace(None), 'trace off')
    lib.ia_diag_set_screen_sched(prev)
    lib.ia_diag_set_screen_pc(prev_pc)


if __name__ == '__main__':
    main()
