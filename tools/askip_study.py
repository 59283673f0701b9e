"""CPU study (no GPU): candidate segments per query of the R16 screen's exact stage on c4's
finest database, with the skipped components' bound term taken over ALL rows (A_skip, the
round-5 form) or per segment (A_skip,j = max over segment j's rows), for P = 3 and 11.

Proxy: the screen's segment minima are replaced by the exact fp64 values (the screen is
within eps of them), so the counts are those of a screen with no rounding error and the
bound the exact stage must assume.  Queries: the 512 real finest-level queries captured
from a GPU synthesis (tests/golden/c4_queries.npz).  Segments: 4 scanlines x 128 columns
(the strip order of DESIGN.md §3b, 512 rows).

  global:    candidate j  iff  m_j <= e* + 2 eps(A_skip)
  per seg:   candidate j  iff  m_j - eps_j <= min_i (m_i + eps_i)

usage: python tools/askip_study.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
sys.path.insert(0, ROOT)

import ia_oracle as o  # noqa: E402
import make_config_fixtures as mf  # noqa: E402

U = 2.0 ** -24


def main():
    t0 = time.time()
    A, Aps, B, k, cap, seed = mf.workload('c4')
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, cap=cap, seed=seed)
    As = o.create_index(A_pyr, Ap_list, L)[L - 1]
    H, W = A_pyr[L - 1].shape
    c = np.concatenate([np.full(34, A_pyr[L - 1].mean()), np.full(21, Ap_list[0][L - 1].mean())])
    a = As - c
    del As
    na = np.einsum('ij,ij->i', a, a)
    Amax = np.sqrt(na.max())
    rs = np.random.RandomState(0)
    sub = a[rs.choice(len(a), 65536, replace=False)]
    w, V = np.linalg.eigh(sub.T @ sub / len(sub))
    V = V[:, ::-1]
    rho = a @ V
    print('c4 finest DB %d rows built in %.0f s; A = %.4g' % (len(a), time.time() - t0, Amax))
    # segment of each row: (y // 4, x // 128) of the single A' image
    yy, xx = np.divmod(np.arange(len(a)), W)
    seg = (yy // 4) * (W // 128) + xx // 128
    nseg = seg.max() + 1
    order = np.argsort(seg, kind='stable')
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'c4_queries.npz'))
    Q = g['q'][:int(g['n_captured'])]
    for P in (3, 11):
        skn = np.sqrt((rho[:, P:] ** 2).sum(1))
        ask = skn.max()
        ask_seg = skn[order].reshape(nseg, -1).max(1)
        print('P = %d: A_skip %.4g (%.3f A); per-segment A_skip p10/p50/p90/max %.3f / %.3f / %.3f / %.3f of A_skip'
              % (P, ask, ask / Amax, *np.percentile(ask_seg / ask, [10, 50, 90, 100])))
        cg, cs, cmaxg, cmaxs = [], [], [], []
        for m0 in range(0, len(Q), 32):
            qq = Q[m0:m0 + 32] - c
            E = na[:, None] - 2.0 * (a @ qq.T)
            mseg = E[order].reshape(nseg, -1, len(qq)).min(axis=1)      # nseg x m
            nq = np.sqrt((qq ** 2).sum(1))
            nsk = np.sqrt(((qq @ V)[:, P:] ** 2).sum(1))
            base = U * (360 * Amax * nq + 60 * Amax ** 2)
            eg = base + 2.0 ** -9 * 1.01 * ask * nsk
            es = base[None, :] + 2.0 ** -9 * 1.01 * ask_seg[:, None] * nsk[None, :]
            estar = mseg.min(0)
            ng = (mseg <= estar + 2 * eg).sum(0)
            ub = (mseg + es).min(0)
            ns = (mseg - es <= ub).sum(0)
            cg += list(ng)
            cs += list(ns)
        cg, cs = np.array(cg), np.array(cs)
        print('  candidate segments per query: global mean %.3f (max %d, >=2: %.1f %%)   per segment mean %.3f '
              '(max %d, >=2: %.1f %%)' % (cg.mean(), cg.max(), 100 * (cg >= 2).mean(), cs.mean(), cs.max(),
                                          100 * (cs >= 2).mean()))
        # a wave of 342 pixels ends with its slowest: expected max over 342 queries drawn from each
        for name, arr in (('global', cg), ('per segment', cs)):
            mx = [arr[rs.randint(0, len(arr), 342)].max() for _ in range(200)]
            print('  %-12s expected max over a 342-query wave: %.2f' % (name, np.mean(mx)))


if __name__ == '__main__':
    main()
