"""HIP path vs the oracle, on the GPU.  Every comparison is bit-exact: the kernels
reproduce the reference's fp64 operation order, and the matcher's fp32 screen only
selects candidates that are then scored in fp64 exactly like the oracle."""
import numpy as np
import pytest
import torch

import ia_oracle as o
import ia_oracle_c as oc
from conftest import analogy_inputs, golden

pytestmark = pytest.mark.gpu


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=dtype)


# ---- a1-a4 ------------------------------------------------------------------------------------

def test_yiq_kernels_match_reference(gpu):
    import img_preprocess as ip
    g = golden()
    assert np.array_equal(ip.convert_to_YIQ(g['yiq_in']), g['yiq_out'])
    assert np.array_equal(ip.convert_to_RGB(g['yiq_out']), g['rgb_out'])
    yiq, y = ip.rgb_to_yiq_dev(dev(g['yiq_u8_in'], torch.uint8), 255.)
    assert np.array_equal(yiq.cpu().numpy(), g['yiq_u8_out'])
    assert np.array_equal(y.cpu().numpy(), g['yiq_u8_out'][..., 0])
    f32 = (g['yiq_in'] * 0.999).astype(np.float32)
    _, y = ip.rgb_to_yiq_dev(dev(f32, torch.float32), 1.0)
    assert np.array_equal(y.cpu().numpy(), o.convert_to_YIQ(f32.astype(np.float64))[..., 0])


def test_remap_and_compress_match_reference(gpu):
    import img_preprocess as ip
    g = golden()
    a, ap = ip.remap_luminance(g['remap_A'], [g['remap_Ap']], g['remap_B'])
    assert np.array_equal(a, g['remap_A_out']) and np.array_equal(ap[0], g['remap_Ap_out'])
    A, B = g['remap_A'], g['remap_B']
    for w in (1, 0.3, 0.5):
        a2, b2 = ip.compress_values(A, B, w)
        ra, rb = o.compress_values(A, B, w)
        assert np.array_equal(a2, ra) and np.array_equal(b2, rb)


# ---- a5 pyramid -----------------------------------------------------------------------------------

@pytest.mark.parametrize('k', range(9))
def test_pyramid_kernel_bit_exact_vs_skimage(gpu, k):
    import img_preprocess as ip
    g = golden()
    pyr = ip.compute_gaussian_pyramid(g['pyr%d_in' % k], 3)
    n = int(g['pyr%d_n' % k])
    assert len(pyr) == n
    for l in range(n):
        assert np.array_equal(pyr[l], g['pyr%d_l%d' % (k, l)]), (k, l)


@pytest.mark.parametrize('shape,cap', [((300, 517), None), ((1024, 1024), 5), ((2, 9), None),
                                       ((5, 300), None)])
def test_pyramid_kernel_vs_oracle_large(gpu, shape, cap):
    import img_preprocess as ip
    img = np.random.RandomState(sum(shape)).rand(*shape)
    if min(shape) <= 3:
        # below min_size: one reduce step directly
        a = ip.pyramid_reduce_dev(dev(img)).cpu().numpy()
        assert np.array_equal(a, o.pyramid_reduce(img))
        return
    pyr = ip.compute_gaussian_pyramid(img, 3, cap)
    ref = o.compute_gaussian_pyramid(img, 3, cap)
    assert len(pyr) == len(ref)
    for a, b in zip(pyr, ref):
        assert np.array_equal(a, b)


@pytest.mark.parametrize('shape', [(2048, 2048), (96, 130), (8, 4), (517, 300), (33, 1000), (4, 5),
                                   (2, 2), (3, 255), (257, 124)])
@pytest.mark.parametrize('kind', ['noise', 'flat'])
def test_pyramid_streaming_form_equals_tiled(gpu, shape, kind):
    """k_pyr_wave (one LDS-free pass, waves of 28 output columns x 16 rows, the clip from
    per-wave partials) writes the same level as the tiled k_pyr_reduce + k_pyr_clip, bit for
    bit, and the oracle's; 'flat' images (saturated regions) exercise the clip itself."""
    import _ia
    import img_preprocess as ip
    rs = np.random.RandomState(sum(shape))
    img = rs.rand(*shape)
    if kind == 'flat':
        img = np.minimum(1.0, img * 3.0)          # ~2/3 of the pixels exactly 1.0
    x = dev(img)
    outs = []
    for form, oh in [(0, 0), (1, 0)]:
        prev = _ia.pyr_form(form, oh if oh else 16)
        try:
            outs.append(ip.pyramid_reduce_dev(x).cpu().numpy())
        finally:
            _ia.pyr_form(prev, 16)
    for o_ in outs[1:]:
        assert np.array_equal(o_.view(np.int64), outs[0].view(np.int64))
    if max(shape) <= 600:
        assert np.array_equal(outs[1], o.pyramid_reduce(img))


# ---- a9 features ---------------------------------------------------------------------------------

def test_feature_kernel_kat_and_oracle(gpu):
    import algorithms
    import config as c
    sm = 0.5 * np.ones((4, 5)); sm[0, 0] = 0
    lg = 0.3 * np.ones((7, 10)); lg[0, 0] = 1
    c.num_ch, c.padding_sm, c.padding_lg, c.weights = c.setup_vars(lg)
    for full in (True, False):
        f = algorithms.compute_feature_array([sm, lg], c, full)
        assert f[0] == [] and np.array_equal(f[1], o.compute_feature_array([sm, lg], full)[1])
    img = np.random.RandomState(4).rand(37, 53)
    pyr = o.compute_gaussian_pyramid(img, 3)
    for full in (True, False):
        f = algorithms.compute_feature_array(pyr, c, full)
        r = o.compute_feature_array(pyr, full)
        for l in range(1, len(pyr)):
            assert np.array_equal(f[l], r[l])


# ---- a10/a11 matcher ----------------------------------------------------------------------------

def _index(A, Aps):
    import algorithms
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = [o.compute_gaussian_pyramid(x, 3) for x in Aps]
    L = len(A_pyr)
    idx = algorithms.level_index([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_pyr], L - 1)
    As = o.create_index(A_pyr, Ap_pyr, L)[L - 1]
    return idx, As


@pytest.mark.parametrize('flat', [False, True])
def test_match_batch_equals_bruteforce(gpu, flat):
    A, Aps, _ = analogy_inputs(21, (96, 131), (8, 8), n_ap=2, flat=flat)
    idx, As = _index(A, Aps)
    rs = np.random.RandomState(3)
    Q = np.vstack([As[rs.randint(0, len(As), 200)],                       # exact rows
                   As[rs.randint(0, len(As), 200)] + rs.randn(200, 55) * 1e-7,  # near ties
                   rs.rand(300, 55)])                                     # far queries
    gi, gd = idx.match(Q)
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    for q, i, d in zip(Q, gi, gd):
        dd = np.add.reduce((As - q) ** 2, axis=1)
        j = int(np.argmin(dd))
        assert i == j and d == dd[j]


def test_best_approximate_match_api(gpu):
    import algorithms
    import config as c
    A, Aps, _ = analogy_inputs(8, (40, 44), (8, 8))
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = [o.compute_gaussian_pyramid(Aps[0], 3)]
    c.max_levels = len(A_pyr)
    flann, params, As, As_size = algorithms.create_index(A_pyr, Ap_pyr, c)
    Ar = o.create_index(A_pyr, Ap_pyr, len(A_pyr))
    L = len(A_pyr) - 1
    assert As_size[L] == Ar[L].shape and np.array_equal(As[L], Ar[L])
    q = Ar[L][17] * 0.97
    assert algorithms.best_approximate_match(flann[L], params[L], q) == o.best_approximate_match(Ar[L], q)


def test_coherence_and_distance_api(gpu):
    import algorithms
    import config as c
    A, Aps, _ = analogy_inputs(9, (30, 36), (8, 8))
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = o.compute_gaussian_pyramid(Aps[0], 3)
    As = o.create_index(A_pyr, [Ap_pyr], len(A_pyr))[-1]
    imh, imw = A.shape
    c.num_ch, c.padding_sm, c.padding_lg, c.weights = c.setup_vars(A)
    rs = np.random.RandomState(5)
    for row, col in [(1, 1), (3, imw - 1), (imh - 1, 2), (imh // 2, imw // 2), (0, 5)]:
        n = row * imw + col
        s = [(int(a), int(b)) for a, b in zip(rs.randint(0, imh, n), rs.randint(0, imw, n))]
        im = [0] * n
        q = As[rs.randint(0, len(As))] + rs.randn(55) * 0.01
        p, i, r = algorithms.best_coherence_match(As, (imh, imw), q, s, im, (row, col), imw, c)
        pr, ir, rr = o.best_coherence_match(As, (imh, imw), q, s, im, (row, col), imw)
        assert tuple(p) == tuple(pr) and i == ir
        d = algorithms.compute_distance(As[5], q, c.weights)
        assert d == o.compute_distance(As[5], q, c.weights)


# ---- a12-a15 level synthesis -----------------------------------------------------------------------

def _run_both(A, Aps, B, k, seed, cap=None):
    import image_analogies as ia
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed, cap=cap)
    Bp_dev = [dev(b) for b in Bp_pyr]
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, k, w)
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, k, w)
    return ref, out, Bp_dev


@pytest.mark.parametrize('case', [
    dict(seed=0, A=(30, 40), B=(28, 33), n_ap=1, k=0.5, flat=False),
    dict(seed=3, A=(26, 21), B=(17, 30), n_ap=2, k=5.0, flat=False),
    dict(seed=5, A=(24, 24), B=(24, 24), n_ap=1, k=2.0, flat=True),
    dict(seed=6, A=(45, 30), B=(45, 30), n_ap=1, k=0.5, flat=False),
    dict(seed=7, A=(64, 96), B=(50, 61), n_ap=3, k=1.0, flat=False),
    dict(seed=8, A=(117, 180), B=(117, 180), n_ap=1, k=25.0, flat=False),
])
def test_synthesis_bit_exact_vs_oracle(gpu, case):
    A, Aps, B = analogy_inputs(case['seed'], case['A'], case['B'], case['n_ap'], case['flat'])
    ref, out, Bp_dev = _run_both(A, Aps, B, case['k'], case['seed'])
    assert set(ref) == set(out)
    for l in ref:
        Bp, s, im = ref[l]
        assert np.array_equal(out[l][0].cpu().numpy(), s), l
        assert np.array_equal(out[l][1].cpu().numpy(), im), l
        assert np.array_equal(Bp_dev[l].cpu().numpy(), Bp), l


def test_full_pipeline_from_uint8_images(gpu, tmp_path):
    """image_analogies_main end to end (YIQ convert, pyramids, all levels) vs the oracle
    pipeline on the same decoded pixels; JPEG-free PNG inputs keep the pixels exact."""
    import matplotlib.pyplot as plt
    import config as c
    import image_analogies as ia
    rs = np.random.RandomState(12)
    A, Aps, B = analogy_inputs(12, (45, 60), (40, 52))
    to_rgb = lambda x: np.dstack([x, x * 0.8 + 0.1, 1 - x])  # noqa: E731
    files = {}
    for name, img in (('A', A), ('Ap', Aps[0]), ('B', B)):
        files[name] = str(tmp_path / (name + '.png'))
        plt.imsave(files[name], to_rgb(img))
    c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k, c.seed = True, False, True, 1, 0.5, 3
    c.levels = None
    out_dir = str(tmp_path / 'out') + '/'
    Bp = ia.image_analogies_main(files['A'], [files['Ap']], files['B'], out_dir, c)
    # oracle on the same decoded inputs
    dec = {k: plt.imread(v)[..., :3] for k, v in files.items()}
    scale = lambda x: 255. if np.max(x) > 1 else 1.0  # noqa: E731
    Ay = o.convert_to_YIQ(dec['A'] / scale(dec['A']))[..., 0]
    By = o.convert_to_YIQ(dec['B'] / scale(dec['B']))[..., 0]
    Apy = o.convert_to_YIQ(dec['Ap'] / scale(dec['Ap'][0]))[..., 0]
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(Ay, [Apy], By, seed=3)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, 0.5, o.compute_weights(3, 5, 12, 1))
    for l in range(1, L):
        assert np.array_equal(Bp[l], ref[l][0]), l
    assert (tmp_path / 'out' / 'level_1_color.jpg').exists()


def test_synthesis_through_rccl_exchange(gpu):
    """The multi-GPU path (DB shard + RCCL all-gather of per-rank winners + replicated
    finish) with a 1-rank communicator on the box's single GPU: same kernels and the
    same ncclAllGather call as the 2/4/8-GPU run, result must equal the oracle."""
    import ctypes
    import _ia
    import image_analogies as ia
    buf = ctypes.create_string_buffer(128)
    _ia.check(_ia.lib().ia_comm_unique_id(buf), 'ia_comm_unique_id')
    comm = ctypes.c_void_p()
    _ia.check(_ia.lib().ia_comm_init(buf.raw, 1, 0, ctypes.byref(comm)), 'ia_comm_init')
    try:
        assert _ia.lib().ia_comm_nranks(comm) == 1
        A, Aps, B = analogy_inputs(31, (40, 52), (33, 47), n_ap=2)
        A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=31)
        w = o.compute_weights(3, 5, 12, 1)
        ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 1.0, w)
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 1.0, w, comm=comm, rank=0,
                                nranks=1)
        for l in ref:
            assert np.array_equal(out[l][0].cpu().numpy(), ref[l][1]), l
            assert np.array_equal(out[l][1].cpu().numpy(), ref[l][2]), l
            assert np.array_equal(Bp_dev[l].cpu().numpy(), ref[l][0]), l
    finally:
        _ia.check(_ia.lib().ia_comm_destroy(comm), 'ia_comm_destroy')


def test_pipelined_sharded_levels_through_rccl(gpu):
    """Every level sharded (1-rank communicators, one per level) AND pipelined
    (ia_synth_levels: each level's RCCL exchange on its own stream): the oracle's B', s, im."""
    import ctypes
    import _ia
    import image_analogies as ia
    comms = []
    try:
        A, Aps, B = analogy_inputs(32, (44, 50), (37, 45), n_ap=2)
        A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=32)
        for _ in range(1, L):
            buf = ctypes.create_string_buffer(128)
            _ia.check(_ia.lib().ia_comm_unique_id(buf), 'ia_comm_unique_id')
            cm = ctypes.c_void_p()
            _ia.check(_ia.lib().ia_comm_init(buf.raw, 1, 0, ctypes.byref(cm)), 'ia_comm_init')
            comms.append(cm)
        w = o.compute_weights(3, 5, 12, 1)
        ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 0.7, w)
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 0.7, w, comm=comms, rank=0,
                                nranks=1, pipeline=True)
        for l in ref:
            assert np.array_equal(out[l][0].cpu().numpy(), ref[l][1]), l
            assert np.array_equal(out[l][1].cpu().numpy(), ref[l][2]), l
            assert np.array_equal(Bp_dev[l].cpu().numpy(), ref[l][0]), l
    finally:
        torch.cuda.synchronize()
        for cm in comms:
            _ia.check(_ia.lib().ia_comm_destroy(cm), 'ia_comm_destroy')


@pytest.mark.parametrize('seed', [51, 52])
def test_pipelined_levels_equal_sequential(gpu, seed):
    """ia_synth_levels (levels overlapped, each on its own stream) gives bitwise the same
    B', s, im as one level at a time, and both equal the oracle."""
    import image_analogies as ia
    A, Aps, B = analogy_inputs(seed, (70, 83), (66, 90), n_ap=2, flat=(seed == 52))
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed)
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 1.0, w)
    outs = []
    for pipe in (False, True):
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 1.0, w, pipeline=pipe)
        outs.append({l: (out[l][0].cpu().numpy(), out[l][1].cpu().numpy(),
                         Bp_dev[l].cpu().numpy()) for l in out})
    for l in ref:
        for o_ in outs:
            assert np.array_equal(o_[l][0], ref[l][1]), l
            assert np.array_equal(o_[l][1], ref[l][2]), l
            assert np.array_equal(o_[l][2], ref[l][0]), l


def test_back_to_back_pipelined_calls_match_oracle(gpu):
    """Two pipelined calls queued with no host sync between them (every level index built
    first, so the second ia_synth_levels enters while the first runs): the second waits for
    the first on the host (IA_PIPE_DRAIN) and reuses its streams and events; both equal the
    oracle bit for bit."""
    import algorithms
    import image_analogies as ia
    w = o.compute_weights(3, 5, 12, 1)
    runs = []
    for seed in (61, 62):
        A, Aps, B = analogy_inputs(seed, (64, 77), (60, 84), n_ap=2, flat=(seed == 62))
        A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed)
        ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 1.0, w)
        Ad, Apd, Bd = [dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list], [dev(p) for p in B_pyr]
        Bp_dev = [dev(b) for b in Bp_pyr]
        wd = dev(w)
        calls = [ia._LevelCall(l, L, algorithms.level_index(Ad, Apd, l), Bd[l - 1], Bd[l],
                               Bp_dev[l - 1], Bp_dev[l], wd, 1.0)
                 for l in range(1, L)]
        runs.append((ref, calls, Bp_dev, (Ad, Apd, Bd, wd)))
    torch.cuda.synchronize()
    outs = [ia.synthesize_levels_dev(calls) for _, calls, _, _ in runs]   # no sync between
    torch.cuda.synchronize()
    for (ref, calls, Bp_dev, _), out in zip(runs, outs):
        for i, l in enumerate(range(1, len(calls) + 1)):
            assert np.array_equal(out[i][0].cpu().numpy(), ref[l][1]), l
            assert np.array_equal(out[i][1].cpu().numpy(), ref[l][2]), l
            assert np.array_equal(Bp_dev[l].cpu().numpy(), ref[l][0]), l


def test_sharded_level_index_rows(gpu):
    """Per-rank shards: each rank's exact local winner, combined with the lexicographic
    (distance, row) rule, equals the global exact winner (the rule k_finish applies to the
    all-gathered winners)."""
    import algorithms
    from image_analogies import shard_rows
    A, Aps, _ = analogy_inputs(33, (70, 90), (8, 8), n_ap=2, flat=True)
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = [o.compute_gaussian_pyramid(x, 3) for x in Aps]
    L = len(A_pyr)
    As = o.create_index(A_pyr, Ap_pyr, L)[L - 1]
    N = len(As)
    rs = np.random.RandomState(8)
    Q = np.vstack([As[rs.randint(0, N, 60)], rs.rand(40, 55)])
    Ad = [dev(p) for p in A_pyr]
    Apd = [[dev(p) for p in q] for q in Ap_pyr]
    for G in (2, 3, 8):
        per = []
        for r in range(G):
            idx = algorithms.level_index(Ad, Apd, L - 1, lambda lv, n: shard_rows(n, r, G))
            i, d = idx.match(Q)
            per.append((d.cpu().numpy(), i.cpu().numpy()))
        for qi, q in enumerate(Q):
            win = min((per[r][0][qi], per[r][1][qi]) for r in range(G))
            dd = np.add.reduce((As - q) ** 2, axis=1)
            j = int(np.argmin(dd))
            assert win == (dd[j], j)


def test_concurrent_jobs_on_streams_match_oracle(gpu):
    """bench.py c5 drives libia from several host threads, one HIP stream each: jobs
    synthesised concurrently that way give the oracle's result, job by job."""
    from concurrent.futures import ThreadPoolExecutor
    import image_analogies as ia
    w = o.compute_weights(3, 5, 12, 1)
    jobs = []
    for j in range(3):
        A, Aps, B = analogy_inputs(50 + j, (36, 44), (30, 41), n_ap=1)
        A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=50 + j)
        ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 0.5, w)
        jobs.append((A_pyr, Ap_list, B_pyr, Bp_pyr, L, ref))
    main = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in jobs]

    def run(i):
        A_pyr, Ap_list, B_pyr, Bp_pyr, L, _ = jobs[i]
        streams[i].wait_stream(main)
        with torch.cuda.stream(streams[i]):
            out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                    [dev(p) for p in B_pyr], [dev(b) for b in Bp_pyr], L, 0.5, w)
            res = {l: (s.cpu().numpy(), im.cpu().numpy()) for l, (s, im) in out.items()}
        return res

    with ThreadPoolExecutor(len(jobs)) as pool:
        outs = list(pool.map(run, range(len(jobs))))
    for (_, _, _, _, _, ref), out in zip(jobs, outs):
        for l in ref:
            assert np.array_equal(out[l][0], ref[l][1]), l
            assert np.array_equal(out[l][1], ref[l][2]), l


@pytest.mark.parametrize('G,image', [(2, False), (3, False), (2, True)])
def test_sharded_reduction_with_the_real_kernels(gpu, G, image):
    # (the in-process shard path always uses the ShardRec tail: exact stage MODE 2 +
    # k_finish; the RCCL tests above run the default IA_SHARD_TAIL=0 form)
    """The sharded path's per-wave reduction run by the product kernels on one GPU: every
    level's database split into G shards (each built from its own rows, its own amax);
    per wave each shard's exact stage writes its (distance, row, weighted distance)
    records and k_finish reduces them as after the RCCL exchange
    (ia_diag_synth_level_shards).  Flat regions put exact ties across shard boundaries.
    image: 128-wide levels whose shards are whole chunks, so every shard runs from the
    image form alone (no row form), as a c4 rank does."""
    import ctypes
    import _ia
    import algorithms
    import image_analogies as ia
    if image:
        A, Aps, B = analogy_inputs(35, (128, 256), (64, 128), n_ap=2, flat=True)
    else:
        A, Aps, B = analogy_inputs(34, (46, 57), (41, 49), n_ap=2, flat=True)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=34)
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, 3.0, w)
    A_d = [dev(p) for p in A_pyr]
    Ap_d = [[dev(p) for p in q] for q in Ap_list]
    B_d = [dev(p) for p in B_pyr]
    Bp_d = [dev(b) for b in Bp_pyr]
    wd = dev(w)
    image_levels = 0
    for level in range(1, L):
        full = algorithms.level_index(A_d, Ap_d, level)
        shards = [algorithms.level_index(A_d, Ap_d, level,
                                         lambda lv, n, r=r: ia.shard_rows(n, r, G))
                  for r in range(G)]
        image_only = all(x.db is None and x.dbi is not None for x in shards)
        image_levels += image_only
        call = ia._LevelCall(level, L, full, B_d[level - 1], B_d[level], Bp_d[level - 1],
                             Bp_d[level], wd, 3.0)
        arr = (_ia.IaShardDb * G)(*[_ia.IaShardDb(_ia.ptr(x.db).value, x.row0, x.nrows,
                                                  _ia.ptr(x.amax).value, x.dbi_ptr())
                                    for x in shards])
        _ia.check(_ia.lib().ia_diag_synth_level_shards(ctypes.byref(call.args), arr, G,
                                                        _ia.stream()),
                  'ia_diag_synth_level_shards')
        s, im = call.result()
        assert np.array_equal(s.cpu().numpy(), ref[level][1]), level
        assert np.array_equal(im.cpu().numpy(), ref[level][2]), level
        assert np.array_equal(Bp_d[level].cpu().numpy(), ref[level][0]), level
    assert image_levels >= (1 if image else 0), image_levels
