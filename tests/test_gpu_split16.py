"""The split-f16 screen on the GPU: its segment minima stay inside the
error bound eps16 the exact stage relies on (every block shape of the launcher), and the
matcher / synthesis built on it stay bit-exact with either form of the exact stage."""
import ctypes
import math

import numpy as np
import pytest
import torch

import ia_oracle as o
import ia_oracle_c as oc
from conftest import analogy_inputs

pytestmark = pytest.mark.gpu

U32 = 2.0 ** -24
Q16_HALVES = 128          # split-f16 query row: 16 half8 groups (ia_split16.h Q16_ROW)


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=dtype)


def _ilogb(x):
    return math.frexp(x)[1] - 1


def _scales(amax, nq):
    """Host restatement of split16_db_scale / split16_q_scale (ia_split16.h)."""
    e = _ilogb(amax) if amax > 0 else 0
    e = max(-60, min(60, e))
    ea, R = 13 - e, e + 1
    eq = 15 - R
    if nq > 0:
        eq = min(eq, 12 - _ilogb(math.sqrt(nq)))
    return ea, R, max(eq, -120)


def _index(A, Aps):
    import algorithms
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = [o.compute_gaussian_pyramid(x, 3) for x in Aps]
    L = len(A_pyr)
    idx = algorithms.level_index([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_pyr],
                                 L - 1, rows=True)
    return idx, o.create_index(A_pyr, Ap_pyr, L)[L - 1]


def _queries(As, rs):
    n = len(As)
    return np.vstack([As[rs.randint(0, n, 64)],                              # exact rows
                      As[rs.randint(0, n, 64)] + rs.randn(64, 55) * 1e-7,    # near ties
                      As[rs.randint(0, n, 64)] + rs.randn(64, 55) * 0.02,
                      rs.rand(40, 55) * As.max(),                            # far queries
                      np.full((1, 55), As.mean())])                          # ~ the centre


def _segment_order(idx, N, npad, seg):
    """Local rows in the matcher's segment order (ia_diag_stage_map; ia_internal.h
    stage_lrow): identity for linear chunks, column strips otherwise."""
    import _ia
    m = (ctypes.c_int * 3)()
    _ia.check(_ia.lib().ia_diag_stage_map(idx.row0, N, idx.src.Aw, idx.src.Ah, m), 'ia_diag_stage_map')
    W, nstrip, sc = m[0], m[1], m[2]
    if W == 0:
        return np.arange(npad)
    ch = sc * 128
    out = np.empty(npad, dtype=np.int64)
    for chunk in range(npad // ch):
        sx, yb = chunk % nstrip, chunk // nstrip
        for s in range(sc):
            r0 = (yb * sc + s) * W + sx * 128
            out[chunk * ch + s * 128: chunk * ch + (s + 1) * 128] = np.arange(r0, r0 + 128)
    return out


def _screen_vs_fp64(idx, As, Q, Ms):
    """Run the split-f16 screen on Q[:M] for each M and return the worst
    |segmin - exact| / eps16 over all (query, segment) pairs (exact = fp64 minima of
    |a'|^2 - 2 a'.q' per segment, scaled like the screen)."""
    import _ia
    lib = _ia.lib()
    Mmax, N = max(Ms), len(As)
    qrows = lib.ia_diag_qp_rows(Mmax)
    q64 = torch.zeros((Mmax, _ia.IA_DP), dtype=torch.float64, device='cuda')
    q64[:, :55] = dev(Q[:Mmax])
    qp = torch.zeros((qrows, _ia.IA_DP), dtype=torch.float32, device='cuda')
    q16 = torch.zeros((qrows, Q16_HALVES), dtype=torch.float16, device='cuda')
    nq = torch.zeros(qrows, dtype=torch.float64, device='cuda')
    st = _ia.stream()
    _ia.check(lib.ia_diag_query_rows16(_ia.ptr(q64), Mmax, _ia.ptr(idx.center), _ia.ptr(idx.amax),
                                       _ia.ptr(qp), _ia.ptr(q16), _ia.ptr(nq), st),
              'ia_diag_query_rows16')
    npad = lib.ia_db_rows_padded(N)
    seg = min(lib.ia_db_chunk_rows(N), 512)
    nseg = npad // seg
    order = _segment_order(idx, N, npad, seg)      # rows of segment s: order[s * seg:(s + 1) * seg]
    segmin = torch.empty((qrows, nseg), dtype=torch.float32, device='cuda')
    amax = float(idx.amax[0].item())
    c = idx.center.cpu().numpy()
    a = As - c
    na = np.einsum('ij,ij->i', a, a)
    assert np.sqrt(na.max()) <= amax * (1 + 1e-6)
    nqs = nq.cpu().numpy()
    exact = np.empty((Mmax, nseg))
    for m0 in range(0, Mmax, 64):                                     # fp64, 64 queries at a time
        E = na[:, None] - 2.0 * (a @ (Q[m0:m0 + 64] - c).T)
        E = np.concatenate([E, np.repeat(E[-1:], npad - N, 0)])      # padding repeats the last row
        exact[m0:m0 + 64] = E[order].reshape(nseg, seg, -1).min(axis=1).T
    worst = 0.0
    seg_img = torch.empty_like(segmin)
    for M in Ms:
        segmin.fill_(float('nan'))
        _ia.check(lib.ia_diag_screen16_rows(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.db),
                                            _ia.ptr(q16), M, _ia.ptr(segmin), st),
                  'ia_diag_screen16_rows')
        if idx.dbi is not None:      # the image-form stream: the same minima bit for bit
            seg_img.fill_(float('nan'))
            _ia.check(lib.ia_diag_screen16_image(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.dbi),
                                                 _ia.ptr(q16), M, _ia.ptr(seg_img), st),
                      'ia_diag_screen16_image')
            torch.cuda.synchronize()
            assert torch.equal(seg_img[:M].view(torch.int32), segmin[:M].view(torch.int32)), M
        torch.cuda.synchronize()
        got = segmin[:M].cpu().numpy().astype(np.float64)
        assert np.isfinite(got).all(), M
        for m in range(M):
            qq = Q[m] - c
            assert nqs[m] == pytest.approx(float(qq @ qq), rel=1e-12)
            ea, R, eq = _scales(amax, float(nqs[m]))
            true = np.ldexp(exact[m], ea + eq)
            eps = np.ldexp(U32 * (300 * amax * math.sqrt(nqs[m]) + 50 * amax * amax), ea + eq)
            worst = max(worst, np.abs(got[m] - true).max() / eps)
    return worst


@pytest.mark.parametrize('scale', [1.0, 1e3, 1e-3])
def test_split16_segment_minima_within_bound(gpu, scale):
    A, Aps, _ = analogy_inputs(41, (90, 117), (8, 8), n_ap=2)
    A, Aps = A * scale, [x * scale for x in Aps]
    idx, As = _index(A, Aps)
    Q = _queries(As, np.random.RandomState(2))
    worst = _screen_vs_fp64(idx, As, Q, [len(Q)])
    print('split16 screen: worst |segmin - exact| / eps16 = %.3g' % worst)
    assert worst < 1.0


@pytest.mark.parametrize('sched,pc', [(0, 0), (1, 0), (0, 1)])
def test_split16_screen_every_query_split(gpu, sched, pc):
    """k_screen16 at query counts that hit every block shape (G = 1..11 query tiles, and
    launches of more than 11 tiles split into equal groups) on a 1M-row level (8192-row
    chunks: 16 segments per chunk, many stages): every segment minimum within eps16 of
    the fp64 value, and the image-form stream (k_screen16i) gives the same minima bit for
    bit; for both stage schedules (ia_diag_set_screen_sched: tile-major, chain-major) and
    the producer / consumer strip kernel (ia_diag_set_screen_pc)."""
    import _ia
    prev = _ia.lib().ia_diag_set_screen_sched(sched)
    prev_pc = _ia.lib().ia_diag_set_screen_pc(pc)
    try:
        _every_query_split()
    finally:
        _ia.lib().ia_diag_set_screen_sched(prev)
        _ia.lib().ia_diag_set_screen_pc(prev_pc)


def _every_query_split():
    import algorithms
    A, Aps, _ = analogy_inputs(45, (1024, 1024), (8, 8), n_ap=1)
    A_pyr = o.compute_gaussian_pyramid(A, 3, cap=2)
    Ap_pyr = o.compute_gaussian_pyramid(Aps[0], 3, cap=2)
    L = len(A_pyr)
    idx = algorithms.level_index([dev(p) for p in A_pyr], [[dev(p) for p in Ap_pyr]], L - 1,
                                 rows=True)
    As = o.create_index(A_pyr, [Ap_pyr], L)[L - 1]
    rs = np.random.RandomState(7)
    Q = np.vstack([As[rs.randint(0, len(As), 400)] + rs.randn(400, 55) * 0.01,
                   rs.rand(300, 55)])
    Ms = [1, 20, 64, 65, 100, 128, 160, 192, 224, 256, 288, 320, 342, 353, 500, 700]
    assert idx.dbi is not None                # 1024 wide: the image form applies
    worst = _screen_vs_fp64(idx, As, Q, Ms)
    print('split16 screen (1M rows): worst |segmin - exact| / eps16 = %.3g' % worst)
    assert worst < 1.0


@pytest.mark.parametrize('shape,n_ap,shards', [((64, 96), 2, 1), ((70, 128), 1, 3),
                                               ((33, 32), 3, 2), ((256, 512), 1, 1)])
def test_db_build_tiled_equals_per_row(gpu, shape, n_ap, shards):
    """ia_db_build's LDS-tiled kernels (width and row0 multiples of 32) write the same
    bytes and amax as the per-row gather kernels, for whole levels and for shards whose
    row ranges end mid-tile (padding rows repeat the last real row)."""
    import _ia
    import algorithms
    A, Aps, _ = analogy_inputs(47, shape, (8, 8), n_ap=n_ap)
    A_pyr = [dev(p) for p in o.compute_gaussian_pyramid(A, 3, cap=2)]
    Ap_pyr = [[dev(p) for p in o.compute_gaussian_pyramid(x, 3, cap=2)] for x in Aps]
    L = len(A_pyr) - 1
    N = n_ap * shape[0] * shape[1]
    # shard boundaries on multiples of 32 with a ragged last shard
    cuts = [0] + [((N * r // shards) // 32) * 32 for r in range(1, shards)] + [N]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        got = []
        for form in (1, 0):
            prev = _ia.db_build_form(form)
            try:
                idx = algorithms.level_index(A_pyr, Ap_pyr, L, lambda l, n: (r0, r1 - r0),
                                             rows=True)
                torch.cuda.synchronize()
                got.append((idx.db.cpu().numpy().copy(), float(idx.amax[0].item())))
            finally:
                _ia.db_build_form(prev)
        assert got[0][1] == got[1][1], (r0, r1)
        assert np.array_equal(got[0][0], got[1][0]), (r0, r1)


@pytest.mark.parametrize('scale', [1.0, 1e3, 1e-3])
def test_match_exact(gpu, scale):
    A, Aps, _ = analogy_inputs(42, (70, 101), (8, 8), n_ap=2, flat=(scale == 1.0))
    idx, As = _index(A * scale, [x * scale for x in Aps])
    Q = _queries(As, np.random.RandomState(4))
    gi, gd = idx.match(Q)
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    for q, i, d in zip(Q, gi, gd):
        dd = np.add.reduce((As - q) ** 2, axis=1)
        j = int(np.argmin(dd))
        assert i == j and d == dd[j]


@pytest.fixture
def rescore():
    import _ia
    prev = _ia.rescore_mode()
    yield _ia.rescore_mode
    _ia.rescore_mode(prev)


@pytest.fixture
def graph():
    import _ia
    prev = _ia.graph_mode()
    yield _ia.graph_mode
    _ia.graph_mode(prev)


@pytest.mark.parametrize('image,mode', [(True, 0), (True, 1), (False, -1)])
def test_synthesis_with_image_form_db(gpu, monkeypatch, rescore, image, mode):
    """A 128 x 256 analogy (two A' images; levels of width 256 and 128 take the DB's image
    form, the 64-wide coarsest level the row form): B', s and im equal the oracle's with the
    image form on (no row form built; both forms of the exact stage re-screen from it) and
    off."""
    import image_analogies as ia
    monkeypatch.setenv('IA_DB_IMAGE', '1' if image else '0')
    rescore(mode)
    A, Aps, B = analogy_inputs(48, (128, 256), (64, 128), n_ap=2)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=48, cap=3)
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 1.0, w)
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, 1.0, w)
    for l in ref:
        assert np.array_equal(out[l][0].cpu().numpy(), ref[l][1]), l
        assert np.array_equal(out[l][1].cpu().numpy(), ref[l][2]), l
        assert np.array_equal(Bp_dev[l].cpu().numpy(), ref[l][0]), l


@pytest.mark.parametrize('gmode', [0, 2])
@pytest.mark.parametrize('mode', [0, 1])
def test_synthesis_bit_exact_with_either_exact_stage(gpu, rescore, graph, mode, gmode):
    """Both forms of the exact stage (one workgroup per query with the fused tail, or the
    work list k_select / k_items / k_gather with the tail in k_gather), launched eagerly or
    from a captured HIP graph, give the oracle's B', s and im."""
    import _ia
    import image_analogies as ia
    rescore(mode)
    graph(gmode)
    A, Aps, B = analogy_inputs(46, (52, 67), (44, 47), n_ap=2, flat=True)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=46)
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 2.0, w)
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, 2.0, w)
    for l in ref:
        assert np.array_equal(out[l][0].cpu().numpy(), ref[l][1]), l
        assert np.array_equal(out[l][1].cpu().numpy(), ref[l][2]), l
        assert np.array_equal(Bp_dev[l].cpu().numpy(), ref[l][0]), l
    _ia.check(_ia.lib().ia_release_thread_resources(), 'ia_release_thread_resources')


def test_image_form_alone_equals_image_form_from_rows(gpu):
    """ia_db_build_image without a row form (amax from the value ranges, norm slots from the
    LDS-tiled build's norm pass) writes the same bytes and amax as from ia_db_build's rows;
    the matcher run from it alone (screen + both exact stages) gives the brute-force 1-NN."""
    import _ia
    import algorithms
    A, Aps, _ = analogy_inputs(49, (256, 384), (8, 8), n_ap=2)
    A_pyr = o.compute_gaussian_pyramid(A, 3, cap=2)
    Ap_pyr = [o.compute_gaussian_pyramid(x, 3, cap=2) for x in Aps]
    L = len(A_pyr)
    Ad, Apd = [dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_pyr]
    both = algorithms.level_index(Ad, Apd, L - 1, rows=True)
    alone = algorithms.level_index(Ad, Apd, L - 1)
    assert alone.db is None and alone.dbi is not None and both.db is not None
    # rebuilt into zeroed buffers (the sections' alignment gaps are never written)
    lib = _ia.lib()
    n = lib.ia_db_image_bytes(ctypes.byref(alone.src), 0, alone.nrows) - 65536
    z_rows, z_alone = torch.zeros_like(both.dbi), torch.zeros_like(alone.dbi)
    amax = torch.zeros(1, dtype=torch.float32, device='cuda')
    _ia.check(lib.ia_db_build_image(ctypes.byref(both.src), 0, both.nrows, _ia.ptr(both.center),
                                    _ia.ptr(both.db), _ia.ptr(both.amax), _ia.ptr(z_rows),
                                    _ia.stream()), 'ia_db_build_image')
    _ia.check(lib.ia_db_build_image(ctypes.byref(alone.src), 0, alone.nrows, _ia.ptr(alone.center),
                                    None, _ia.ptr(amax), _ia.ptr(z_alone), _ia.stream()),
              'ia_db_build_image')
    torch.cuda.synchronize()
    assert float(alone.amax[0].item()) == float(both.amax[0].item()) == float(amax.item())
    assert torch.equal(z_alone[:n], z_rows[:n])         # all but the build's scratch
    As = o.create_index(A_pyr, Ap_pyr, L)[L - 1]
    rs = np.random.RandomState(5)
    Q = np.vstack([As[rs.randint(0, len(As), 40)] + rs.randn(40, 55) * 0.003, rs.rand(24, 55)])
    for mode in (0, 1):
        prev = _ia.rescore_mode(mode)
        try:
            i, d = alone.match(Q)
        finally:
            _ia.rescore_mode(prev)
        i, d = i.cpu().numpy(), d.cpu().numpy()
        for qi, q in enumerate(Q):
            dd = np.add.reduce((As - q) ** 2, axis=1)
            j = int(np.argmin(dd))
            assert (d[qi], i[qi]) == (dd[j], j), (mode, qi)


@pytest.mark.parametrize('shape,n_ap,shards,jitter', [((256, 384), 2, 1, False), ((129, 256), 1, 1, False),
                                                      ((130, 128), 3, 3, False), ((64, 512), 1, 2, False),
                                                      ((129, 256), 2, 1, True)])
def test_image_form_fused_build_equals_kernel_chain(gpu, shape, n_ap, shards, jitter):
    """ia_db_build_image's one-pass build (k_db_range_at + k_img_build: windows in registers,
    pads, norm slots and the bound in one sweep) writes the same bytes (pads of every image,
    the shard's norm slots) and the same amax as the range / bound / pad / norm-pass chain,
    for odd heights, several A' images and row shards; jitter: a centre whose features differ
    within A's and A''s groups (the build's general path instead of its squared windows)."""
    import _ia
    import algorithms
    import image_analogies as ia
    A, Aps, _ = analogy_inputs(51, shape, (8, 8), n_ap=n_ap)
    A_pyr = o.compute_gaussian_pyramid(A, 3, cap=2)
    Ap_pyr = [o.compute_gaussian_pyramid(x, 3, cap=2) for x in Aps]
    L = len(A_pyr)
    Ad, Apd = [dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_pyr]
    lib = _ia.lib()
    for r in range(shards):
        idx = algorithms.level_index(Ad, Apd, L - 1, (lambda lv, N: ia.shard_rows(N, r, shards))
                                     if shards > 1 else None)
        if idx.dbi is None:
            continue
        if jitter:
            idx.center += torch.arange(idx.center.numel(), device='cuda', dtype=idx.center.dtype) * 1e-3
        n = lib.ia_db_image_bytes(ctypes.byref(idx.src), idx.row0, idx.nrows) - 65536
        outs = []
        for fused in (0, 1):
            prev = lib.ia_diag_set_img_fused(fused)
            try:
                z = torch.zeros_like(idx.dbi)
                amax = torch.zeros(1, dtype=torch.float32, device='cuda')
                _ia.check(lib.ia_db_build_image(ctypes.byref(idx.src), idx.row0, idx.nrows,
                                                _ia.ptr(idx.center), None, _ia.ptr(amax), _ia.ptr(z),
                                                _ia.stream()), 'ia_db_build_image')
                torch.cuda.synchronize()
                outs.append((z[:n].clone(), float(amax.item())))
            finally:
                lib.ia_diag_set_img_fused(prev)
        assert outs[0][1] == outs[1][1] > 0, (r, outs[0][1], outs[1][1])
        assert torch.equal(outs[0][0], outs[1][0]), r
