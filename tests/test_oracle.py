"""Pin the CPU oracle against the reference: golden vectors produced by the reference's
own modules (tests/golden/make_golden.py), the KATs of the reference's tests
(algorithms_test.py, config_test.py, img_preprocess_test.py), and C-vs-numpy oracle
agreement.  CPU only."""
import numpy as np
import pytest

import ia_oracle as o
import ia_oracle_c as oc
from conftest import analogy_inputs, golden


# ---- config.py ----------------------------------------------------------------------------

def test_weights_match_reference_goldens():
    g = golden()
    g310 = golden('ref_weights_py310.npz')
    for ch, key in ((1, 'ch1'), (3, 'ch3')):
        w = o.compute_weights(3, 5, 12, ch)
        # reference config.py under this interpreter's numpy: bit-exact
        assert np.array_equal(w, g310[key])
        # under the skimage-era numpy 1.26.4: np.exp differs by <= 1 ulp
        assert np.allclose(w, g['weights_%s' % key], rtol=1e-15, atol=0)


def test_compute_weights_kat():
    """config_test.py:5-62 restated."""
    for ch in (1, 3):
        gs = o.matlab_style_gauss2D((3, 3), 0.5)
        gl = o.matlab_style_gauss2D((5, 5), 1)
        w_sm = np.repeat(((1. / 9) * gs).flatten(), ch)
        w_lg = np.repeat(((1. / 25) * gl).flatten(), ch)
        w_half = np.repeat(((1. / 12) * gl.flatten()[:12]), ch)
        assert len(w_sm) == 9 * ch and len(w_lg) == 25 * ch and len(w_half) == 12 * ch
        assert np.isclose(np.sum(w_sm), ch / 9.)
        assert np.isclose(np.sum(w_lg), ch / 25.)
        assert np.sum(w_half) < ch * 0.5 / 12
        assert np.allclose(o.compute_weights(3, 5, 12, ch), np.hstack([w_sm, w_lg, w_sm, w_half]))


# ---- img_preprocess.py -------------------------------------------------------------------------

def test_yiq_rgb_match_reference():
    g = golden()
    assert np.array_equal(o.convert_to_YIQ(g['yiq_in']), g['yiq_out'])
    assert np.array_equal(o.convert_to_RGB(g['yiq_out']), g['rgb_out'])
    assert np.array_equal(o.convert_to_YIQ(g['yiq_u8_in'] / 255.), g['yiq_u8_out'])


def test_yiq_einsum_order():
    """The kernels' per-channel order (m0*x0 + m2*x2) + m1*x1 is numpy's einsum order."""
    x = np.random.RandomState(3).rand(31, 17, 3)
    e = o.convert_to_YIQ(x)
    for i in range(3):
        m = o.YIQ_M[i]
        assert np.array_equal(e[..., i], (m[0] * x[..., 0] + m[2] * x[..., 2]) + m[1] * x[..., 1])


def test_converts_roundtrip():
    """img_preprocess_test.py:6-13."""
    img = np.random.RandomState(0xba5eba11).rand(25, 25, 3)
    assert np.allclose(o.convert_to_RGB(o.convert_to_YIQ(img)), img, atol=0.05)
    for img in (np.ones((25, 25, 3)), np.zeros((25, 25, 3))):
        assert np.allclose(o.convert_to_RGB(o.convert_to_YIQ(img)), img)


def test_remap_luminance_matches_reference():
    g = golden()
    a, ap = o.remap_luminance(g['remap_A'], [g['remap_Ap']], g['remap_B'])
    assert np.array_equal(a, g['remap_A_out']) and np.array_equal(ap[0], g['remap_Ap_out'])
    # img_preprocess_test.py:16-26 intent (the reference test passes a bare array)
    B = g['remap_B']
    for X in (a, ap[0]):
        assert np.isclose(np.mean(B), np.mean(X), atol=0.05)
        assert np.isclose(np.std(B), np.std(X), atol=0.05)


@pytest.mark.parametrize('k', range(9))
def test_pyramid_bit_exact_vs_skimage(k):
    """img_preprocess.py:47-63 -> skimage 0.18.3 pyramid_gaussian, every level bit-exact."""
    g = golden()
    img = g['pyr%d_in' % k]
    n = int(g['pyr%d_n' % k])
    pyr = o.compute_gaussian_pyramid(img, 3)
    assert len(pyr) == n
    for l in range(n):
        assert np.array_equal(pyr[l], g['pyr%d_l%d' % (k, l)]), (k, l)


def test_initialize_Bp():
    """img_preprocess_test.py:29-42 intent, seeded."""
    img = np.random.RandomState(0xba5eba11).rand(25, 40)
    pyr = o.compute_gaussian_pyramid(img, 3)
    for a, b in zip(pyr, o.initialize_Bp(pyr, init_rand=False)):
        assert np.array_equal(a, b)
    for a, b in zip(pyr, o.initialize_Bp(pyr, init_rand=True, seed=5)):
        assert not np.allclose(a, b)
    r1 = o.initialize_Bp(pyr, True, seed=5)
    r2 = o.initialize_Bp(pyr, True, seed=5)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r2))


# ---- algorithms.py KATs (algorithms_test.py:10-115) --------------------------------------------

SM_0 = np.array([[0, 0, 0.5], [0, 0, 0.5], [0.5, 0.5, 0.5]])
LG_0 = np.array([[0.3, 0.3, 0.3, 0.3, 0.3],
                 [0.3, 1, 1, 0.3, 0.3],
                 [0.3, 1, 1, 0.3, 0.3],
                 [0.3, 0.3, 0.3, 0.3, 0.3],
                 [0.3, 0.3, 0.3, 0.3, 0.3]])


def kat_images():
    sm = 0.5 * np.ones((4, 5)); sm[0, 0] = 0
    lg = 0.3 * np.ones((7, 10)); lg[0, 0] = 1
    return sm, lg


def test_compute_feature_array_kat():
    sm, lg = kat_images()
    feat = o.compute_feature_array([sm, lg], True)
    assert len(feat) == 2 and feat[0] == []
    assert feat[1].shape == (70, 34)
    assert np.allclose(feat[1][0], np.hstack([SM_0.flatten(), LG_0.flatten()]))
    feat = o.compute_feature_array([sm, lg], False)
    assert feat[1].shape == (70, 21)
    assert np.allclose(feat[1][0], np.hstack([SM_0.flatten(), LG_0.flatten()[:12]]))


def test_extract_pixel_feature_kat():
    sm, lg = kat_images()
    assert np.allclose(o.extract_pixel_feature(sm, lg, (0, 0), True),
                       np.hstack([SM_0.flatten(), LG_0.flatten()]))
    assert np.allclose(o.extract_pixel_feature(sm, lg, (0, 0), False),
                       np.hstack([SM_0.flatten(), LG_0.flatten()[:12]]))
    # the index-map form equals explicit symmetric padding (algorithms.py:81-84)
    psm, plg = o.pad_img_pair(sm, lg)
    for r in range(7):
        for c in range(10):
            ref = np.hstack([psm[r // 2:r // 2 + 3, c // 2:c // 2 + 3].flatten(),
                             plg[r:r + 5, c:c + 5].flatten()])
            assert np.array_equal(o.extract_pixel_feature(sm, lg, (r, c), True), ref)


def test_best_coherence_match_property():
    """algorithms_test.py:158-207 restated with the current signature: with B = A and
    s(q - (1,1)) = q - (1,1), coherence must return exactly q."""
    A, Aps, _ = analogy_inputs(7, (40, 52), (8, 8))
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = o.compute_gaussian_pyramid(Aps[0], 3)
    As = o.create_index(A_pyr, [Ap_pyr], len(A_pyr))[-1]
    imh, imw = A.shape
    rs = np.random.RandomState(1)
    for row, col in [(1, 1), (1, imw - 1), (imh - 1, 1), (imh - 1, imw - 1), (imh // 2, imw // 2)]:
        num_px = row * imw + col
        s = [(int(a), int(b)) for a, b in zip(rs.randint(0, imh, num_px), rs.randint(0, imw, num_px))]
        s[(row - 1) * imw + col - 1] = (row - 1, col - 1)
        im = [0] * num_px
        q = As[row * imw + col]
        p, i, r_star = o.best_coherence_match(As, (imh, imw), q, s, im, (row, col), imw)
        assert p == (row, col) and i == 0


def test_brute_force_is_first_min():
    rs = np.random.RandomState(2)
    As = rs.rand(500, 55)
    As[300] = As[100]       # exact duplicate: the lower row must win
    assert o.best_approximate_match(As, As[100] + 1e-9) == 100


# ---- C oracle == numpy oracle (end to end) -------------------------------------------------------

@pytest.mark.parametrize('case', [
    dict(seed=0, A=(30, 40), B=(28, 33), n_ap=1, k=0.5, flat=False),
    dict(seed=3, A=(26, 21), B=(17, 30), n_ap=2, k=5.0, flat=False),
    dict(seed=5, A=(24, 24), B=(24, 24), n_ap=1, k=2.0, flat=True),
])
def test_c_oracle_equals_numpy_oracle(case):
    A, Aps, B = analogy_inputs(case['seed'], case['A'], case['B'], case['n_ap'], case['flat'])
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=case['seed'])
    Bp2 = [b.copy() for b in Bp_pyr]
    r1 = o.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, case['k'])
    r2 = oc.synthesize(A_pyr, Ap_list, B_pyr, Bp2, L, case['k'], o.compute_weights(3, 5, 12, 1))
    assert set(r1) == set(r2) == set(range(1, L))
    for l in r1:
        for a, b in zip(r1[l], r2[l]):
            assert np.array_equal(a, b), l


def _colour_inputs(seed, A_shape, B_shape, n_ap):
    """3-channel analogy pyramids (per-channel, skimage multichannel semantics)."""
    from scipy.ndimage import gaussian_filter
    from conftest import smooth_noise
    A = np.dstack([smooth_noise(seed + 17 * ch, A_shape) for ch in range(3)])
    Aps = [np.dstack([gaussian_filter(A[..., ch], 1.0 + 0.5 * i) for ch in range(3)]) for i in range(n_ap)]
    B = np.dstack([smooth_noise(seed + 1 + 17 * ch, B_shape) for ch in range(3)])

    def pyr3(img):
        chans = [o.compute_gaussian_pyramid(img[..., ch], 3) for ch in range(3)]
        return [np.dstack([c[l] for c in chans]) for l in range(len(chans[0]))]
    A_pyr, B_pyr = pyr3(A), pyr3(B)
    Ap_list = [pyr3(x) for x in Aps]
    L = min(len(A_pyr), len(B_pyr))
    return A_pyr, Ap_list, B_pyr, o.initialize_Bp(B_pyr, True, seed + 2), L


@pytest.mark.parametrize('seed,A,B,n_ap,k', [(11, (30, 40), (20, 26), 1, 0.5), (12, (24, 22), (18, 20), 2, 25.0)])
def test_c_oracle_colour_equals_numpy_oracle(seed, A, B, n_ap, k):
    """The C oracle's 3-channel form (num_ch = 3, config.py:29-42: 165-dim rows, every
    channel of B' updated) equals the numpy oracle end to end, with the scan and with the
    projection index."""
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = _colour_inputs(seed, A, B, n_ap)
    w = o.compute_weights(3, 5, 12, 3)
    r1 = o.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, k)
    for indexed in (False, True):
        r2 = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, k, w, indexed=indexed)
        assert set(r1) == set(r2) == set(range(1, L))
        for l in r1:
            for a, b in zip(r1[l], r2[l]):
                assert np.array_equal(a, b), (l, indexed)


# ---- LSH restatement (this build's definition, no reference code) -------

def test_lsh_keys_kat():
    """One table, one axis-aligned projection, b = 0, w = 1: key = floor(x0) * golden."""
    proj = np.zeros((1, 56), np.float32)
    proj[0, 0] = 1.0
    X = np.zeros((4, 55), np.float32)
    X[:, 0] = [0.5, 1.5, -0.5, 7.0]
    keys = o.lsh_hash_keys(X, proj, 1, 1, 1.0)[:, 0]
    want = [(h * 0x9E3779B1) & 0x7fffffff for h in (0, 1, 0xffffffff, 7)]
    assert [o.lsh_bits(n) for n in (1, 2, 3, 1024, 1025, 1 << 40)] == [2, 2, 3, 11, 12, 30]
    assert keys.tolist() == want


def test_lsh_single_bucket_is_bruteforce():
    """A bucket wider than the data holds every row: with N <= cap the LSH matcher is the
    exact first-minimum brute force."""
    rs = np.random.RandomState(0)
    As = rs.rand(30, 55)
    proj = np.zeros((2, 56), np.float32)
    proj[:, :55] = rs.randn(2, 55)
    proj[:, 55] = 5e5      # offset b = w / 2 keeps every |p . x| << w in bucket 0
    Q = np.vstack([As[:5], rs.rand(20, 55)])
    idx, dist = o.lsh_match(As, As.mean(0), proj, 1, 2, 1e6, Q)
    for q, i, d in zip(Q, idx, dist):
        dd = np.add.reduce((As - q) ** 2, axis=1)
        assert i == np.argmin(dd) and d == dd.min()


def test_lsh_recall_on_perturbed_rows():
    """Sanity of the definition: near-duplicate queries find their row (or an equally
    close one) in most cases with the default 16 x 4 tables."""
    A, Aps, _ = analogy_inputs(4, (40, 50), (8, 8))
    pyr = o.compute_gaussian_pyramid(A, 3)
    ppyr = o.compute_gaussian_pyramid(Aps[0], 3)
    As = o.create_index(pyr, [ppyr], len(pyr))[-1]
    c = As.mean(0)
    rs = np.random.RandomState(1)
    sigma = np.sqrt(((As - c) ** 2).mean())
    P = np.zeros((64, 56), np.float32)
    P[:, :55] = rs.standard_normal((64, 55))
    P[:, 55] = rs.uniform(0, sigma, 64)
    rows = rs.randint(0, len(As), 200)
    Q = As[rows] + rs.randn(200, 55) * 1e-3 * sigma
    idx, dist = o.lsh_match(As, c, P, 16, 4, sigma, Q)
    exact = np.array([np.add.reduce((As - q) ** 2, axis=1).min() for q in Q])
    assert np.all(dist >= exact)
    assert np.mean(dist == exact) > 0.9


def test_c3_fixture_reproduces_coarse_levels():
    """tests/golden/c3_oracle.npz (make_config_fixtures.py c3) re-derived here for its
    three coarsest synthesized levels from bench.py's c3 inputs."""
    import hashlib
    import sys
    import ia_oracle_c as oc
    from conftest import ROOT
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    g = golden('c3_oracle.npz')
    conf = bench.CONFIGS['c3']
    A, Ap, B = bench.make_inputs(conf, 0)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, [Ap], B, cap=conf['levels'], seed=2)
    assert L == int(g['max_levels'])
    out = oc.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, conf['k'],
                        o.compute_weights(3, 5, 12, 1), levels=[1, 2, 3])
    for l, (bp, s, im) in out.items():
        assert np.array_equal(s, g['s%d' % l]) and np.array_equal(im, g['im%d' % l])
        assert hashlib.sha256(bp.tobytes()).hexdigest() == str(g['bp_sha%d' % l])


@pytest.mark.parametrize('full', [True, False])
def test_level_features_3ch_match_extract_patches_2d(full):
    """The oracle's 3-channel feature rows equal the reference's construction
    (algorithms.py:11-47): symmetric np.pad, sklearn extract_patches_2d, flatten, the
    c.num_ch * c.n_half cut of the fine half, coarse patch at (row // 2) * ceil(w / 2) +
    col // 2."""
    from sklearn.feature_extraction.image import extract_patches_2d
    rs = np.random.RandomState(5)
    lg = rs.rand(9, 12, 3)
    sm = rs.rand(5, 6, 3)
    pad = lambda x, p: np.pad(x, ((p, p), (p, p), (0, 0)), mode='symmetric')  # noqa: E731
    psm = extract_patches_2d(pad(sm, 1), (3, 3))
    plg = extract_patches_2d(pad(lg, 2), (5, 5))
    plg = plg.reshape(plg.shape[0], -1)
    if not full:
        plg = plg[:, :3 * 12]
    h, w = lg.shape[:2]
    ref = np.vstack([np.hstack([psm[(r // 2) * int(np.ceil(w / 2.)) + c // 2].flatten(),
                                plg[r * w + c].flatten()])
                     for r in range(h) for c in range(w)])
    got = o.level_features(sm, lg, full)
    assert got.shape == ref.shape and np.array_equal(got, ref)


# ---- the projection index the full-size fixtures were generated through ------------------

def _fixture_module():
    import os
    import sys
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
    if here not in sys.path:
        sys.path.insert(0, here)
    import make_config_fixtures as mf
    return mf


def test_oracle_index_equals_scan_at_c4_scale():
    """c4_full.npz was generated through the oracle's projection index.  On
    c4's finest level (4,194,304 rows, bench.py's seed-0 inputs) the index must return the
    brute-force scan's row and distance for every committed c4 query (512 captured from a
    GPU synthesis + 64 near-ties; c4_queries.npz holds the scan's answers,
    make_config_fixtures.make_c4), at P = 1 and P = 4 projections (~20 s on 8 threads)."""
    mf = _fixture_module()
    prev = oc.set_threads(8)
    try:
        A, Aps, B, k, cap, seed = mf.workload('c4')
        A_pyr = o.compute_gaussian_pyramid(A, 3, cap)
        Ap_pyr = o.compute_gaussian_pyramid(Aps[0], 3, cap)
        db = oc.LevelDB(len(A_pyr) - 1, A_pyr, [Ap_pyr])
        assert db.N == 4194304
        f = golden('c4_queries.npz')
        for P in (1, 4):
            ix = db.index(P)
            idx, d = ix.nn(f['q'])
            del ix
            assert np.array_equal(idx, f['idx']), P
            assert np.array_equal(d, f['dist']), P
    finally:
        oc.set_threads(prev)


def test_colour_index_equals_scan_165_dims():
    """the index's rounding margin for 165-dim rows.  Random rows, exact
    duplicates, 1e-12 near-ties and nudged rows of a 3-channel level: index == scan."""
    rs = np.random.RandomState(11)
    mf = _fixture_module()
    A_pyr, Ap_list, B_pyr, Bp_pyr, L, k = mf.colour_workload('c1rgb')
    db = oc.LevelDB(L - 1, A_pyr, Ap_list)
    assert db.D == 165
    N = db.N
    Q = np.vstack([db.rows[rs.randint(0, N, 16)], db.rows[rs.randint(0, N, 16)] + 1e-12,
                   db.rows[rs.randint(0, N, 16)] + rs.randn(16, 165) * 1e-3, rs.rand(8, 165)])
    i0, d0 = db.scan(Q)
    for P in (1, 4):
        i1, d1 = db.index(P).nn(Q)
        assert np.array_equal(i0, i1) and np.array_equal(d0, d1), P


def test_colour_fixture_equals_brute_force_scan():
    """c1rgb_oracle.npz (generated through the projection index) re-derived with the
    brute-force scan at every level: s, im and the B' hash (~60 s on 8 threads)."""
    mf = _fixture_module()
    prev = oc.set_threads(8)
    try:
        A_pyr, Ap_list, B_pyr, Bp_pyr, L, k = mf.colour_workload('c1rgb')
        w = o.compute_weights(3, 5, 12, 3)
        out = oc.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, k, w, indexed=False)
    finally:
        oc.set_threads(prev)
    f = golden('c1rgb_oracle.npz')
    assert sorted(out) == list(range(1, int(f['max_levels'])))
    for l, (bp, s, im) in out.items():
        assert np.array_equal(s.astype(np.int16), f['s%d' % l]), l
        assert np.array_equal(im.astype(np.uint8), f['im%d' % l]), l
        assert mf.bp_hash(bp) == str(f['bp_sha%d' % l]), l
