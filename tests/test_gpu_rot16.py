"""The rotated split-f16 screen (R16; csrc/ia_rot16.h, ia_screen16r.hip) on
the GPU: its segment minima stay inside the bound eps_R the exact stage relies on (every
block shape of the launcher, input scales 1e-3 / 1 / 1e3), even with the per-segment skip
bound eps_j of k_xstrip; A_skip bounds every row's skipped components and A_skip,j every row of
segment j; and syntheses through it equal the split-f16 image form bit for bit
(the oracle fixtures of c4 / c5 run through it by default)."""
import ctypes
import math

import numpy as np
import pytest
import torch

import ia_oracle as o
from conftest import analogy_inputs
from test_gpu_split16 import U32, Q16_HALVES, _scales, _segment_order, dev

pytestmark = pytest.mark.gpu



def _level(seed, shape, cap, scale=1.0):
    import algorithms
    A, Aps, _ = analogy_inputs(seed, shape, (8, 8), n_ap=1)
    A, Aps = A * scale, [x * scale for x in Aps]
    A_pyr = o.compute_gaussian_pyramid(A, 3, cap=cap)
    Ap_pyr = o.compute_gaussian_pyramid(Aps[0], 3, cap=cap)
    L = len(A_pyr)
    idx = algorithms.level_index([dev(p) for p in A_pyr], [[dev(p) for p in Ap_pyr]], L - 1, rot=True)
    assert idx.dbr is not None, 'the rotated DB applies to a 128-multiple-wide level'
    As = o.create_index(A_pyr, [Ap_pyr], L)[L - 1]
    return idx, As


def _r16_vs_fp64(idx, As, Q, Ms):
    """worst |segmin - exact| / eps_R over (query, segment) for each M of Ms"""
    import _ia
    lib = _ia.lib()
    Mmax, N = max(Ms), len(As)
    qrows = lib.ia_diag_qp_rows(Mmax)
    q64 = torch.zeros((Mmax, _ia.IA_DP), dtype=torch.float64, device='cuda')
    q64[:, :55] = dev(Q[:Mmax])
    npad = lib.ia_db_rows_padded(N)
    seg = min(lib.ia_db_chunk_rows(N), 512)
    nseg = npad // seg
    order = _segment_order(idx, N, npad, seg)
    R16_P = lib.ia_db_rot_components()
    amax, askip = (float(x) for x in idx.amax.cpu().numpy())
    c = idx.center.cpu().numpy()
    a = As - c
    na = np.einsum('ij,ij->i', a, a)
    assert np.sqrt(na.max()) <= amax * (1 + 1e-6)
    V = idx.rot.cpu().numpy()[:56 * 56].reshape(56, 56)[:55, :55].astype(np.float64)
    rho = (a @ V).astype(np.float32).astype(np.float64)
    skn = np.sqrt((rho[:, R16_P:] ** 2).sum(1))
    assert skn.max() <= askip * (1 + 1e-6)
    # per segment (ia_rot16.h r16_askc): A_skip,j bounds the segment's rows, and its code's
    # decoded value A_skip c_j / 255 bounds A_skip,j
    tail = idx.dbr.view(torch.uint8)[npad * lib.ia_db_rot_slots() * 2:]
    ask_seg = tail[:4 * nseg].view(torch.float32).cpu().numpy().astype(np.float64)
    codes = tail[(4 * nseg + 255) // 256 * 256:][:nseg].cpu().numpy().astype(np.float64)
    skp = np.concatenate([skn, np.repeat(skn[-1:], npad - N)])
    assert (skp[order].reshape(nseg, seg).max(1) <= ask_seg).all()
    ask_dec = askip * codes / 255.0
    assert (ask_dec >= ask_seg).all() and (codes <= 255).all()
    assert ask_dec.mean() < 0.9 * askip, 'per-segment bounds tighter than the global one'
    exact = np.empty((Mmax, nseg))
    for m0 in range(0, Mmax, 64):
        E = na[:, None] - 2.0 * (a @ (Q[m0:m0 + 64] - c).T)
        E = np.concatenate([E, np.repeat(E[-1:], npad - N, 0)])
        exact[m0:m0 + 64] = E[order].reshape(nseg, seg, -1).min(axis=1).T
    worst = 0.0
    for M in Ms:
        q16 = torch.zeros((qrows, Q16_HALVES), dtype=torch.float16, device='cuda')
        nq = torch.zeros(qrows, dtype=torch.float64, device='cuda')
        nsk = torch.zeros(qrows, dtype=torch.float64, device='cuda')
        segmin = torch.full((qrows, nseg), float('nan'), dtype=torch.float32, device='cuda')
        _ia.check(lib.ia_diag_screen16r(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.dbr), _ia.ptr(idx.rot),
                                        _ia.ptr(idx.amax), _ia.ptr(idx.center), _ia.ptr(q64), M, _ia.ptr(q16),
                                        _ia.ptr(nq), _ia.ptr(nsk), _ia.ptr(segmin), _ia.stream()),
                  'ia_diag_screen16r')
        torch.cuda.synchronize()
        got = segmin[:M].cpu().numpy().astype(np.float64)
        assert np.isfinite(got).all(), M
        nqs, nsks = nq.cpu().numpy(), nsk.cpu().numpy()
        for m in range(M):
            qq = Q[m] - c
            assert nqs[m] == pytest.approx(float(qq @ qq), rel=1e-12)
            kap = qq @ V
            assert nsks[m] == pytest.approx(float((kap[R16_P:] ** 2).sum()), rel=1e-9, abs=1e-300)
            ea, R, eq = _scales(amax, float(nqs[m]))
            true = np.ldexp(exact[m], ea + eq)
            # eps_j of segment j (the per-segment skip bound k_xstrip uses; <= the global eps_R)
            eps = U32 * (360 * amax * math.sqrt(nqs[m]) + lib.ia_db_rot_eps_a2() * amax * amax) + \
                2.0 ** -9 * 1.01 * ask_dec * math.sqrt(nsks[m])
            worst = max(worst, (np.abs(got[m] - true) / np.ldexp(eps, ea + eq)).max())
    return worst


@pytest.mark.parametrize('scale', [1.0, 1e3, 1e-3])
def test_r16_segment_minima_within_bound(gpu, scale):
    """k_screen16r at query counts hitting every block shape (G = 1..11 tiles, split
    launches) on a 1M-row strip-order level: every segment minimum within eps_R of the fp64
    value, at input scales 1e-3, 1, 1e3."""
    idx, As = _level(45, (1024, 1024), 2, scale)
    rs = np.random.RandomState(7)
    n = len(As)
    Q = np.vstack([As[rs.randint(0, n, 64)],                              # exact rows
                   As[rs.randint(0, n, 64)] + rs.randn(64, 55) * 1e-7 * scale,
                   As[rs.randint(0, n, 300)] + rs.randn(300, 55) * 0.01 * scale,
                   rs.rand(271, 55) * As.max(),                          # far queries
                   np.full((1, 55), As.mean())])
    Ms = [1, 20, 64, 65, 100, 128, 160, 192, 224, 256, 288, 320, 342, 353, 500, 700] if scale == 1.0 \
        else [342, 700]
    worst = _r16_vs_fp64(idx, As, Q, Ms)
    print('r16 screen (scale %g): worst |segmin - exact| / eps_R = %.3g' % (scale, worst))
    assert worst < 1.0


def _synth(shape_A, shape_B, cap, seed, rot_on, monkeypatch, batch=1):
    import _ia
    import image_analogies as ia
    monkeypatch.setenv('IA_DB_ROT', '1' if rot_on else '0')
    A, Aps, B = analogy_inputs(seed, shape_A, shape_B, n_ap=1)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, cap=cap, seed=seed)
    w = _ia.to_dev(o.compute_weights(3, 5, 12, 1))
    d = lambda p: [dev(x) for x in p]  # noqa: E731
    if batch == 1:
        Bp = d(Bp_pyr)
        out = ia.synthesize_dev(d(A_pyr), [d(p) for p in Ap_list], d(B_pyr), Bp, L, 0.5, w)
        return [(Bp[l].cpu().numpy(), s.cpu().numpy(), im.cpu().numpy()) for l, (s, im) in sorted(out.items())]
    jobs = [(d(A_pyr), [d(p) for p in Ap_list], d(B_pyr), d(Bp_pyr)) for _ in range(batch)]
    outs = ia.synthesize_batch_dev(jobs, L, 0.5, w)
    return [[(j[3][l].cpu().numpy(), s.cpu().numpy(), im.cpu().numpy()) for l, (s, im) in sorted(o_.items())]
            for j, o_ in zip(jobs, outs)]


def test_r16_synthesis_equals_image_form(gpu, monkeypatch):
    """A whole synthesis (A 1024^2, B 512^2, 4-level cap: strip levels of 65 k to 1 M rows)
    through the rotated screen equals the split-f16 image form's, B', s and im bit for bit."""
    r = _synth((1024, 1024), (512, 512), 4, 51, True, monkeypatch)
    i = _synth((1024, 1024), (512, 512), 4, 51, False, monkeypatch)
    assert len(r) == len(i)
    for (b0, s0, m0), (b1, s1, m1) in zip(r, i):
        assert np.array_equal(s0, s1) and np.array_equal(m0, m1) and np.array_equal(b0, b1)


def test_r16_batch_equals_image_form(gpu, monkeypatch):
    """A batch of 3 jobs (ia_synth_levels_batch) through the rotated screen equals the image
    form's results."""
    r = _synth((512, 512), (256, 256), 4, 53, True, monkeypatch, batch=3)
    i = _synth((512, 512), (256, 256), 4, 53, False, monkeypatch, batch=3)
    for jr, ji in zip(r, i):
        for (b0, s0, m0), (b1, s1, m1) in zip(jr, ji):
            assert np.array_equal(s0, s1) and np.array_equal(m0, m1) and np.array_equal(b0, b1)


def _segmin_r16(idx, Q, M, N):
    import _ia
    lib = _ia.lib()
    qrows = lib.ia_diag_qp_rows(M)
    q64 = torch.zeros((M, _ia.IA_DP), dtype=torch.float64, device='cuda')
    q64[:, :55] = dev(Q[:M])
    nseg = lib.ia_db_rows_padded(N) // min(lib.ia_db_chunk_rows(N), 512)
    q16 = torch.zeros((qrows, Q16_HALVES), dtype=torch.float16, device='cuda')
    nq = torch.zeros(qrows, dtype=torch.float64, device='cuda')
    nsk = torch.zeros(qrows, dtype=torch.float64, device='cuda')
    segmin = torch.full((qrows, nseg), float('nan'), dtype=torch.float32, device='cuda')
    _ia.check(lib.ia_diag_screen16r(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.dbr), _ia.ptr(idx.rot),
                                    _ia.ptr(idx.amax), _ia.ptr(idx.center), _ia.ptr(q64), M, _ia.ptr(q16),
                                    _ia.ptr(nq), _ia.ptr(nsk), _ia.ptr(segmin), _ia.stream()),
              'ia_diag_screen16r')
    torch.cuda.synchronize()
    return segmin[:M].cpu().numpy()


@pytest.mark.parametrize('shape,cap', [((1024, 1024), 2), ((512, 256), 2), ((2048, 1024), 2)])
def test_r16_wave_form_equals_block_form(gpu, shape, cap):
    """The wave-owned screen (k_screen16w, the default) and the block form (k_screen16r) give
    the same segment minima bit for bit at every block shape (G = 1..11, split launches),
    on levels of 512-row (1 M and 2 M rows) and 256-row (131 k rows) segments."""
    import _ia
    lib = _ia.lib()
    idx, As = _level(45, shape, cap)
    rs = np.random.RandomState(8)
    n = len(As)
    Q = np.vstack([As[rs.randint(0, n, 64)], As[rs.randint(0, n, 300)] + rs.randn(300, 55) * 0.01,
                   rs.rand(336, 55) * As.max()])
    prev = lib.ia_diag_set_r16_form(1)
    try:
        for M in [1, 20, 64, 65, 128, 192, 256, 320, 342, 353, 700]:
            lib.ia_diag_set_r16_form(1)
            w = _segmin_r16(idx, Q, M, n)
            lib.ia_diag_set_r16_form(0)
            b = _segmin_r16(idx, Q, M, n)
            assert np.isfinite(w).all(), M
            assert np.array_equal(w.view(np.uint32), b.view(np.uint32)), M
    finally:
        lib.ia_diag_set_r16_form(prev)


def test_build_rot_refuses_a_non_orthonormal_rotation(gpu):
    """The builders' precondition (include/ia.h): a rotation that is not orthonormal
    to fp32 rounding (here the principal basis scaled by 1 + 1e-4, ||V^T V - I||_F ~ 1.5e-3
    against the budget 2 sqrt(n) 2^-24) is refused with IA_E_ARG, for the luminance builder
    (n = 55) and the 3-channel one (n = 165); the unscaled basis passes both."""
    import _ia
    import algorithms
    lib = _ia.lib()
    idx, _ = _level(73, (128, 128), 2)
    ok = lib.ia_db_build_rot(ctypes.byref(idx.src), idx.row0, idx.nrows, _ia.ptr(idx.center),
                             _ia.ptr(idx.rot), _ia.ptr(idx.amax), _ia.ptr(idx.dbr), _ia.stream())
    assert ok == 0
    bad = idx.rot.clone()
    bad[:56 * 56].view(56, 56)[:55, :55] *= 1.0001
    rc = lib.ia_db_build_rot(ctypes.byref(idx.src), idx.row0, idx.nrows, _ia.ptr(idx.center),
                             _ia.ptr(bad), _ia.ptr(idx.amax), _ia.ptr(idx.dbr), _ia.stream())
    assert rc == _ia.IA_E_ARG and b'not orthonormal' in lib.ia_last_error()
    # 3 channels
    A, Aps, _ = analogy_inputs(74, (40, 36), (8, 8), n_ap=1)
    A3 = np.dstack([A, A ** 2, np.sqrt(A)])
    Ap3 = np.dstack([Aps[0], Aps[0] ** 2, np.sqrt(Aps[0])])
    A_pyr = [dev(p) for p in o.compute_gaussian_pyramid(A3, 3, cap=2)]
    Ap_pyr = [dev(p) for p in o.compute_gaussian_pyramid(Ap3, 3, cap=2)]
    ix3 = algorithms.LevelIndex3(A_pyr[0], A_pyr[1], torch.stack([Ap_pyr[0]]), torch.stack([Ap_pyr[1]]))
    rot = algorithms.rot3_rotation(ix3.db3, ix3.N)
    dbr = algorithms.rot3_apply(ix3.db3, ix3.N, rot)
    assert dbr is not None
    bad3 = rot.clone()
    bad3[:165 * 168].view(165, 168)[:, :165] *= 1.0001
    rc = lib.ia_db3_build_rot(_ia.ptr(ix3.db3), ix3.N, _ia.ptr(bad3), _ia.ptr(dbr), _ia.stream())
    assert rc == _ia.IA_E_ARG and b'not orthonormal' in lib.ia_last_error()
