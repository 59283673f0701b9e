"""3-channel matching (the reference's convert=False on colour images: config.py:29-42
num_ch = 3, 165-dim rows of channel-interleaved windows, algorithms.py:11-47) on the GPU
against the numpy oracle: the feature arrays, the per-pixel API (exact 1-NN, coherence,
weighted distance), whole-level synthesis (B' in all three channels, s, im and the debug
lists) and image_analogies_main end to end from colour image files."""
import numpy as np
import pytest
import torch

import ia_oracle as o
from conftest import smooth_noise

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=torch.float64)


def colour(seed, shape):
    """A smooth colour image (h, w, 3) in [0, 1]: three differently seeded channels."""
    return np.dstack([smooth_noise(seed + 17 * ch, shape) for ch in range(3)])


def pyr3(img, cap=None):
    """Per-channel oracle pyramids stacked (skimage multichannel=True semantics)."""
    chans = [o.compute_gaussian_pyramid(img[..., ch], 3, cap) for ch in range(3)]
    return [np.dstack([c[l] for c in chans]) for l in range(len(chans[0]))]


def inputs(seed, A_shape, B_shape, n_ap=1, cap=None):
    from scipy.ndimage import gaussian_filter
    A = colour(seed, A_shape)
    Aps = [np.dstack([gaussian_filter(A[..., ch], 1.0 + 0.5 * i) for ch in range(3)])
           for i in range(n_ap)]
    B = colour(seed + 1, B_shape)
    A_pyr, B_pyr = pyr3(A, cap), pyr3(B, cap)
    Ap_list = [pyr3(x, cap) for x in Aps]
    L = min(len(A_pyr), len(B_pyr))
    Bp_pyr = o.initialize_Bp(B_pyr, True, seed + 2)
    return A_pyr, Ap_list, B_pyr, Bp_pyr, L


def test_features3_vs_oracle(gpu):
    import algorithms
    import config as c
    A_pyr, Ap_list, _, _, _ = inputs(81, (37, 45), (20, 20))
    for full in (True, False):
        got = algorithms.compute_feature_array(A_pyr, c, full)
        ref = o.compute_feature_array(A_pyr, full)
        for l in range(1, len(A_pyr)):
            assert got[l].shape == ref[l].shape == (A_pyr[l].shape[0] * A_pyr[l].shape[1],
                                                    102 if full else 63)
            assert np.array_equal(got[l], ref[l]), (l, full)


def test_api3_vs_oracle(gpu):
    """create_index / best_approximate_match / best_coherence_match / compute_distance with
    165-dim rows (the per-pixel API of algorithms.py:50-135)."""
    import algorithms
    import config as c
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = inputs(82, (33, 40), (30, 28), n_ap=2)
    c.max_levels, c.matcher = L, 'brute'
    index, params, As, As_size = algorithms.create_index(A_pyr, Ap_list, c)
    ref_As = o.create_index(A_pyr, Ap_list, L)
    level = L - 1
    assert As_size[level] == ref_As[level].shape
    assert np.array_equal(As[level], ref_As[level])
    rs = np.random.RandomState(3)
    Q = np.vstack([ref_As[level][rs.randint(0, len(ref_As[level]), 20)] +
                   rs.randn(20, 165) * 0.01, rs.rand(10, 165)])
    got = algorithms.best_approximate_match_batch(index[level], Q)
    for q, g in zip(Q, got):
        assert g == o.best_approximate_match(ref_As[level], q)
    w = o.compute_weights(3, 5, 12, 3)
    for i in range(5):
        a = ref_As[level][rs.randint(0, len(ref_As[level]))]
        assert algorithms.compute_distance(a, Q[i], w) == o.compute_distance(a, Q[i], w)
    # coherence: a synthetic s / im history over a 6 x 7 B' patch
    A_h, A_w = Ap_list[0][level].shape[:2]
    H, W = 6, 7
    s = [(int(rs.randint(0, A_h)), int(rs.randint(0, A_w))) for _ in range(H * W)]
    im = [int(rs.randint(0, 2)) for _ in range(H * W)]
    for px in [(3, 4), (2, 0), (5, 6), (0, 3)]:
        q = Q[px[0] + px[1]]
        n = px[0] * W + px[1]
        got = algorithms.best_coherence_match(As[level], (A_h, A_w), q, s[:n], im[:n], px, W, c)
        ref = o.best_coherence_match(ref_As[level], (A_h, A_w), q, s[:n], im[:n], px, W)
        assert tuple(np.asarray(got[0]).tolist()) == tuple(np.asarray(ref[0]).tolist())
        if tuple(np.asarray(ref[0]).tolist()) != (-1, -1):
            assert int(got[1]) == int(ref[1])
            assert tuple(np.asarray(got[2]).tolist()) == tuple(np.asarray(ref[2]).tolist())


@pytest.fixture
def color16():
    """Select the 3-channel matcher (1 split-f16 screen + exact stage, 0 exhaustive fp64)."""
    import _ia
    lib = _ia.lib()
    prev = lib.ia_diag_set_color16(1)
    yield lib.ia_diag_set_color16
    lib.ia_diag_set_color16(prev)


@pytest.mark.parametrize('scale', [1e-3, 1.0, 1e3])
def test_screen3_error_bound(gpu, scale):
    """The colour screen's tile minima (split-f16 MFMA) are within eps3 of
    the exact min over the tile of |a - q|^2 - |q'|^2, at input scales 1e-3 .. 1e3, for
    queries near DB rows (small distances) and far from them."""
    import ctypes
    import _ia
    import algorithms
    A_pyr, Ap_list, _, _, L = inputs(85, (45, 70), (20, 20), n_ap=2)
    lv = L - 1
    sc = lambda p: dev(p * scale)  # noqa: E731
    idx = algorithms.LevelIndex3(sc(A_pyr[lv - 1]), sc(A_pyr[lv]),
                                 torch.stack([sc(p[lv - 1]) for p in Ap_list]),
                                 torch.stack([sc(p[lv]) for p in Ap_list]))
    rows = idx.features().cpu().numpy()
    N = rows.shape[0]
    rs = np.random.RandomState(5)
    Q = np.vstack([rows[rs.randint(0, N, 40)] + rs.randn(40, 165) * 1e-3 * scale,
                   rs.rand(24, 165) * scale, rows[rs.randint(0, N, 6)]])
    M = Q.shape[0]
    nt = (N + 31) // 32
    e = torch.empty((M, nt), dtype=torch.float64, device='cuda')
    eps = torch.empty(M, dtype=torch.float64, device='cuda')
    qn = torch.empty(M, dtype=torch.float64, device='cuda')
    Qd = dev(Q)
    _ia.check(_ia.lib().ia_diag_screen3(_ia.ptr(idx.db3), N, _ia.ptr(Qd), M, _ia.ptr(e),
                                        _ia.ptr(eps), _ia.ptr(qn)), 'ia_diag_screen3')
    torch.cuda.synchronize()
    e, eps, qn = e.cpu().numpy(), eps.cpu().numpy(), qn.cpu().numpy()
    pad = np.vstack([rows, np.repeat(rows[-1:], nt * 32 - N, 0)])
    worst = 0.0
    for m in range(M):
        D = ((pad - Q[m]) ** 2).sum(1) - qn[m]
        x = D.reshape(nt, 32).min(1)
        err = np.abs(e[m] - x).max()
        slack = 1e-12 * (np.abs(x).max() + qn[m])
        assert err <= eps[m] + slack, (m, err, eps[m])
        worst = max(worst, err / eps[m])
    assert worst > 0.0


@pytest.mark.parametrize('scale', [1e-3, 1.0, 1e3])
def test_screen3r_error_bound(gpu, scale):
    """The rotated colour screen's tile minima (R16c, DESIGN.md §4e: 3 principal components
    as f16 pairs, 162 as f16, 11 MFMAs per tile) are within eps_Rc of the exact min over the
    tile of |a - q|^2 - |q'|^2 at input scales 1e-3 .. 1e3, near and far from the rows, and
    A_skip bounds every row's skipped components."""
    import ctypes
    import _ia
    import algorithms
    A_pyr, Ap_list, _, _, L = inputs(85, (45, 70), (20, 20), n_ap=2)
    lv = L - 1
    sc = lambda p: dev(p * scale)  # noqa: E731
    idx = algorithms.LevelIndex3(sc(A_pyr[lv - 1]), sc(A_pyr[lv]),
                                 torch.stack([sc(p[lv - 1]) for p in Ap_list]),
                                 torch.stack([sc(p[lv]) for p in Ap_list])).build_rot()
    rows = idx.features().cpu().numpy()
    N = rows.shape[0]
    P = _ia.lib().ia_db3_rot_components()
    V = idx.rot.cpu().numpy().reshape(165, 168)[:, :165].astype(np.float64)
    c = rows.min(0) * 0.5 + rows.max(0) * 0.5       # the DB's centre (midrange)
    rho = ((rows - c) @ V).astype(np.float32).astype(np.float64)
    ask = ctypes.c_float()
    _ia.check(_ia.lib().ia_diag_db3_askip(_ia.ptr(idx.dbr), N, ctypes.byref(ask)), 'askip')
    assert np.sqrt((rho[:, P:] ** 2).sum(1)).max() <= ask.value * (1 + 1e-6)
    rs = np.random.RandomState(5)
    Q = np.vstack([rows[rs.randint(0, N, 40)] + rs.randn(40, 165) * 1e-3 * scale,
                   rs.rand(24, 165) * scale, rows[rs.randint(0, N, 6)]])
    M = Q.shape[0]
    nt = (N + 31) // 32
    e = torch.empty((M, nt), dtype=torch.float64, device='cuda')
    eps = torch.empty(M, dtype=torch.float64, device='cuda')
    qn = torch.empty(M, dtype=torch.float64, device='cuda')
    Qd = dev(Q)
    _ia.check(_ia.lib().ia_diag_screen3r(_ia.ptr(idx.db3), _ia.ptr(idx.dbr), _ia.ptr(idx.rot), N, _ia.ptr(Qd),
                                         M, _ia.ptr(e), _ia.ptr(eps), _ia.ptr(qn)), 'ia_diag_screen3r')
    torch.cuda.synchronize()
    e, eps, qn = e.cpu().numpy(), eps.cpu().numpy(), qn.cpu().numpy()
    pad = np.vstack([rows, np.repeat(rows[-1:], nt * 32 - N, 0)])
    worst = 0.0
    for m in range(M):
        assert qn[m] == pytest.approx(float(((Q[m] - c) ** 2).sum()), rel=1e-12)
        D = ((pad - Q[m]) ** 2).sum(1) - qn[m]
        x = D.reshape(nt, 32).min(1)
        err = np.abs(e[m] - x).max()
        slack = 1e-12 * (np.abs(x).max() + qn[m])
        assert err <= eps[m] + slack, (m, err, eps[m])
        worst = max(worst, err / eps[m])
    print('R16c screen (scale %g): worst |tile min - exact| / eps = %.3g' % (scale, worst))
    assert worst > 0.0


@pytest.mark.parametrize('pipeline', [True, False])
@pytest.mark.parametrize('matcher', [1, 0])
@pytest.mark.parametrize('n_ap,k', [(1, 1.0), (2, 25.0)])
def test_synthesis3_vs_oracle(gpu, color16, n_ap, k, matcher, pipeline):
    """Whole-level 3-channel synthesis: B' (all channels), s, im and the debug lists equal
    the oracle's scanline run (image_analogies.py:130-240 with num_ch = 3), with the
    split-f16 screen + exact stage (1) and the exhaustive fp64 search (0), the levels
    pipelined (ia_synth_levels3) or one at a time (ia_synth_level3)."""
    import image_analogies as ia
    color16(matcher)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = inputs(83 + n_ap, (36, 44), (30, 34), n_ap=n_ap)
    w = o.compute_weights(3, 5, 12, 3)
    As = o.create_index(A_pyr, Ap_list, L)
    Bp_ref = [b.copy() for b in Bp_pyr]
    ref = {}
    for level in range(1, L):
        dbg = {}
        s, im = o.synthesize_level(level, L, A_pyr, Ap_list, B_pyr, Bp_ref, As[level], w, k,
                                   debug=dbg)
        ref[level] = (s, im, dbg)
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, k, w, debug=True, pipeline=pipeline)
    for level in range(1, L):
        s, im, dbg = out[level]
        rs, rim, rd = ref[level]
        assert np.array_equal(s.cpu().numpy(), rs), level
        assert np.array_equal(im.cpu().numpy(), rim), level
        assert np.array_equal(Bp_dev[level].cpu().numpy(), Bp_ref[level]), level
        rec = ia.debug_record(s, im, dbg, Bp_ref[level].shape[:2])
        for key in ('sa', 'sc', 'rstars'):
            assert rec[key] == rd[key], (level, key)
        assert np.array_equal(rec['app_dist'], rd['app_dist']), level
        assert np.array_equal(rec['coh_dist'], rd['coh_dist']), level


def test_synthesis3_split_larger_vs_oracle(gpu, color16):
    """A larger 3-channel synthesis on the split-f16 screen (A 72 x 90, two A' images, B
    60 x 66, every level): s, im and B' equal the oracle's, and the exact stage's work stays
    small (candidate tiles per query, no query scanning every tile)."""
    import ctypes
    import _ia
    import image_analogies as ia
    color16(1)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = inputs(88, (72, 90), (60, 66), n_ap=2)
    w = o.compute_weights(3, 5, 12, 3)
    As = o.create_index(A_pyr, Ap_list, L)
    Bp_ref = [b.copy() for b in Bp_pyr]
    ref = {l: o.synthesize_level(l, L, A_pyr, Ap_list, B_pyr, Bp_ref, As[l], w, 2.0)
           for l in range(1, L)}
    st = (ctypes.c_ulonglong * 2)()
    _ia.check(_ia.lib().ia_diag_color16_stats(st), 'stats')
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, 2.0, w)
    _ia.check(_ia.lib().ia_diag_color16_stats(st), 'stats')
    for level in range(1, L):
        s, im = out[level]
        assert np.array_equal(s.cpu().numpy(), ref[level][0]), level
        assert np.array_equal(im.cpu().numpy(), ref[level][1]), level
        assert np.array_equal(Bp_dev[level].cpu().numpy(), Bp_ref[level]), level
    queries = sum(B_pyr[l].shape[0] * B_pyr[l].shape[1] for l in range(1, L))
    print('candidate tiles per query %.3f, full scans %d' % (st[0] / queries, st[1]))
    assert st[1] == 0 and st[0] < 8 * queries


@pytest.mark.parametrize('rot', ['1', '0'])
def test_synthesis3_screen_forms_vs_oracle(gpu, color16, monkeypatch, rot):
    """The colour synthesis through the rotated screen (R16c, IA_DB_ROT=1, the default) and
    the split-f16 one (IA_DB_ROT=0): both equal the oracle (A 72 x 90, two A' images, every
    level), with few candidate tiles per query and no full scans."""
    import ctypes
    import _ia
    import image_analogies as ia
    color16(1)
    monkeypatch.setenv('IA_DB_ROT', rot)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = inputs(89, (72, 90), (60, 66), n_ap=2)
    w = o.compute_weights(3, 5, 12, 3)
    As = o.create_index(A_pyr, Ap_list, L)
    Bp_ref = [b.copy() for b in Bp_pyr]
    ref = {l: o.synthesize_level(l, L, A_pyr, Ap_list, B_pyr, Bp_ref, As[l], w, 5.0)
           for l in range(1, L)}
    st = (ctypes.c_ulonglong * 2)()
    _ia.check(_ia.lib().ia_diag_color16_stats(st), 'stats')
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, 5.0, w)
    _ia.check(_ia.lib().ia_diag_color16_stats(st), 'stats')
    for level in range(1, L):
        s, im = out[level]
        assert np.array_equal(s.cpu().numpy(), ref[level][0]), level
        assert np.array_equal(im.cpu().numpy(), ref[level][1]), level
        assert np.array_equal(Bp_dev[level].cpu().numpy(), Bp_ref[level]), level
    queries = sum(B_pyr[l].shape[0] * B_pyr[l].shape[1] for l in range(1, L))
    print('IA_DB_ROT=%s: candidate tiles per query %.3f, full scans %d' % (rot, st[0] / queries, st[1]))
    assert st[1] == 0 and st[0] < 8 * queries


def test_main_convert_false_colour_vs_oracle(gpu, tmp_path):
    """image_analogies_main with the reference's default config (convert=False) on colour
    image files: every level's colour output (each pixel its source's A' colour,
    image_analogies.py:216-217) equals the oracle's."""
    import matplotlib.pyplot as plt
    from PIL import Image
    import config as c
    import image_analogies as ia
    from scipy.ndimage import gaussian_filter
    A = colour(91, (32, 40))
    Ap = np.dstack([gaussian_filter(A[..., ch], 1.2) for ch in range(3)])
    B = colour(92, (30, 36))
    files = {}
    for name, img in (('A', A), ('Ap', Ap), ('B', B)):
        files[name] = str(tmp_path / (name + '.png'))
        Image.fromarray(np.clip(np.round(img * 255), 0, 255).astype(np.uint8), 'RGB').save(files[name])
    c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k, c.seed = False, False, True, 1, 2.0, 9
    c.levels, c.matcher = None, 'brute'
    out_dir = str(tmp_path / 'out') + '/'
    out = {}
    ia.image_analogies_main(files['A'], [files['Ap']], files['B'], out_dir, c, outputs=out)
    dec = {n: plt.imread(p)[..., :3].astype(np.float64) for n, p in files.items()}
    sc = lambda x: 255. if np.max(x) > 1 else 1.0  # noqa: E731
    A_pyr = pyr3(dec['A'] / sc(dec['A']))
    Ap_list = [pyr3(dec['Ap'] / sc(dec['Ap'][0]))]
    B_pyr = pyr3(dec['B'] / sc(dec['B']))
    L = min(len(A_pyr), len(B_pyr))
    Bp_pyr = o.initialize_Bp(B_pyr, True, 9)
    As = o.create_index(A_pyr, Ap_list, L)
    w = o.compute_weights(3, 5, 12, 3)
    assert sorted(out) == list(range(1, L))
    for level in range(1, L):
        s, im = o.synthesize_level(level, L, A_pyr, Ap_list, B_pyr, Bp_pyr, As[level], w, 2.0)
        H, W = Bp_pyr[level].shape[:2]
        ref = np.array([Ap_list[i][level][r, cc] for (r, cc), i in zip(s, im)]).reshape(H, W, 3)
        assert np.array_equal(out[level]['s'], s) and np.array_equal(out[level]['im'], im), level
        assert np.array_equal(out[level]['color'], ref), level
        assert np.array_equal((out[level]['color'] * 255).astype(np.uint8),
                              (ref * 255).astype(np.uint8)), level


@pytest.mark.timeout(300)
@pytest.mark.parametrize('name', ['c1rgb', 'c3rgb'])
def test_colour_config_full_size_vs_oracle(gpu, name):
    """3-channel matching (the reference's default convert=False: num_ch = 3, 165-dim rows)
    at the BASELINE sizes: c1 (180 x 117, kappa 0.5, every level) and c3 (362 x 638, kappa
    25, 5-level cap, every level, the finest 231 k pixels against 231 k rows): s, im and the
    B' hash of every level equal the C oracle's full scanline run
    (tests/golden/<name>_oracle.npz, make_config_fixtures.py colour_workload)."""
    import hashlib
    import os
    import sys
    import image_analogies as ia
    from conftest import ROOT, golden
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import make_config_fixtures as mcf
    g = golden(name + '_oracle.npz')
    A_pyr, Ap_list, B_pyr, Bp_pyr, L, k = mcf.colour_workload(name)
    assert L == int(g['max_levels'])
    w = o.compute_weights(3, 5, 12, 3)
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, k, w)
    torch.cuda.synchronize()
    assert sorted(out) == list(range(1, L))
    for level in range(1, L):
        s, im = out[level][0], out[level][1]
        assert np.array_equal(s.cpu().numpy(), g['s%d' % level].astype(np.int32)), level
        assert np.array_equal(im.cpu().numpy(), g['im%d' % level].astype(np.int32)), level
        bp = np.ascontiguousarray(Bp_dev[level].cpu().numpy(), dtype=np.float64)
        assert hashlib.sha256(bp.tobytes()).hexdigest() == str(g['bp_sha%d' % level]), level
