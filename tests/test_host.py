"""Host-side logic of the product, CPU only: C-ABI exports, config parity, the skimage
coefficient fit, the skewed-wavefront schedule, and the multi-rank sharding/exchange rule
(gloo, world_size 2)."""
import ctypes
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ia_oracle as o
from conftest import analogy_inputs, golden


def test_libia_loads_and_exports_every_declared_symbol():
    import _ia
    lib = ctypes.CDLL(_ia.LIB_PATH)
    names = _ia.declared_symbols('all')      # include/ia.h + include/ia_diag.h
    assert len(names) >= 29
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    bound = set(_ia._SIGS)                                  # every ia.h entry is bound;
    assert bound >= set(_ia.declared_symbols())             # extra ones are ia_diag.h's
    assert bound <= set(names)
    assert _ia.lib().ia_version() == 1


def test_product_config_matches_reference():
    import config as c
    g310 = golden('ref_weights_py310.npz')
    assert np.array_equal(c.compute_weights(3, 5, 12, 1), g310['ch1'])
    assert np.array_equal(c.compute_weights(3, 5, 12, 3), g310['ch3'])
    num_ch, psm, plg, w = c.setup_vars(np.zeros((7, 9)))
    assert (num_ch, psm, plg) == (1, 1, 2) and w.shape == (55,)
    num_ch, psm, plg, w = c.setup_vars(np.zeros((7, 9, 3)))
    assert num_ch == 3 and w.shape == (165,)
    assert (c.n_half, c.pad_sm, c.pad_lg) == (12, 1, 2)


def test_resize_coeffs_equal_skimage_fit():
    """The product's host restatement of skimage's AffineTransform fit gives the same
    coefficients as the oracle (which reproduces skimage's pyramids bit for bit)."""
    import img_preprocess as ip
    for H in range(2, 80):
        for W in (H, H + 1, 2 * H + 3, max(2, H // 3)):
            out = ((H + 1) // 2, (W + 1) // 2)
            assert ip.resize_coeffs((H, W), out) == o.affine_coeffs((H, W), out), (H, W)
    for shp in [(2048, 2048), (1024, 1024), (362, 638), (117, 180)]:
        out = ((shp[0] + 1) // 2, (shp[1] + 1) // 2)
        assert ip.resize_coeffs(shp, out) == o.affine_coeffs(shp, out)


def test_num_layers_and_index_maps():
    import img_preprocess as ip
    for h, w in [(180, 117), (362, 638), (2048, 2048), (4, 4), (25, 40)]:
        assert ip.num_layers(h, w, 3) == o.pyramid_num_layers(h, w, 3)
        assert ip.num_layers(h, w, 3, 5) == o.pyramid_num_layers(h, w, 3, 5)
    h, w = 7, 11
    ix = np.arange(3 * h * w)
    (px, img) = ip.Ap_ix2px(ix, h, w)
    assert np.array_equal(ip.Ap_px2ix(px, img, h, w), ix)
    assert np.array_equal(ip.px2ix(ip.ix2px(ix[:h * w], w), w), ix[:h * w])


# ---- skewed wavefront t = x + 3y ---------------------------------------------------------------

def wave_rows(t, H, W):
    """y range of wave t — the formula of ia_synth_level's loop (ia_synth.hip)."""
    lo_num = t - (W - 1)
    y_lo = (lo_num + 2) // 3 if lo_num > 0 else 0
    y_hi = min(t // 3, H - 1)
    return y_lo, y_hi


def read_set(y, x, H, W):
    """Every B' fine-level position the query of (y, x) reads (image_analogies.py:166-168,
    symmetric padding) plus the coherence window's s/im positions (algorithms.py:101-106)."""
    pts = set()
    for t in range(12):
        pts.add((int(o.sym_index(y + t // 5 - 2, H)), int(o.sym_index(x + t % 5 - 2, W))))
    for rr in range(max(0, y - 2), y + 1):
        for cc in range(max(0, x - 2), min(W, x + 3)):
            if rr * W + cc < y * W + x:
                pts.add((rr, cc))
    return pts


@pytest.mark.parametrize('skew,ok', [(3, True), (2, False)])
def test_wavefront_reads_equal_scanline_reads(skew, ok):
    """For every H <= 23, W <= 30: a position read by q was written before q in scanline
    order  <=>  its wave index is smaller.  Skew 3 holds everywhere, skew 2 does not."""
    all_ok = True
    for H in range(1, 24):
        for W in range(1, 31):
            for y in range(H):
                for x in range(W):
                    for (py, px) in read_set(y, x, H, W):
                        before = py * W + px < y * W + x
                        if before != (px + skew * py < x + skew * y):
                            all_ok = False
    assert all_ok == ok


def test_wave_rows_cover_every_pixel_once():
    for H in range(1, 20):
        for W in range(1, 25):
            seen = np.zeros((H, W), int)
            for t in range((W - 1) + 3 * (H - 1) + 1):
                y_lo, y_hi = wave_rows(t, H, W)
                for y in range(y_lo, y_hi + 1):
                    x = t - 3 * y
                    assert 0 <= x < W
                    seen[y, x] += 1
            assert (seen == 1).all()


def test_wavefront_synthesis_equals_scanline_oracle():
    """The oracle run wave by wave (all queries of a wave read the state before the wave
    writes) produces the scanline oracle's B', s and im exactly."""
    A, Aps, B = analogy_inputs(11, (22, 27), (19, 24), n_ap=2)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=4)
    Bp_w = [b.copy() for b in Bp_pyr]
    ref = o.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, 1.0)
    w = o.compute_weights(3, 5, 12, 1)
    As = o.create_index(A_pyr, Ap_list, L)
    for level in range(1, L):
        H, W = Bp_w[level].shape
        Ah, Aw = Ap_list[0][level].shape
        Bf = o.level_features(B_pyr[level - 1], B_pyr[level], True)
        f = o.kappa_factor(level, L, 1.0)
        s = np.zeros((H * W, 2), np.int64)
        im = np.zeros(H * W, np.int64)
        for t in range((W - 1) + 3 * (H - 1) + 1):
            y_lo, y_hi = wave_rows(t, H, W)
            snap = Bp_w[level].copy()
            upd = []
            for y in range(y_lo, y_hi + 1):
                x = t - 3 * y
                q = np.hstack([Bf[y * W + x], o.extract_pixel_feature(Bp_w[level - 1], snap, (y, x), False)])
                app = o.best_approximate_match(As[level], q)
                p, i = o.Ap_ix2px(app, Ah, Aw)
                if (y, x) != (0, 0):
                    sl = [tuple(v) for v in s]
                    pc, ic, _ = o.best_coherence_match(As[level], (Ah, Aw), q, sl, list(im), (y, x), W)
                    if pc != (-1, -1):
                        da = o.compute_distance(As[level][app], q, w)
                        dc = o.compute_distance(As[level][o.Ap_px2ix(pc, ic, Ah, Aw)], q, w)
                        if dc <= da * f:
                            p, i = pc, ic
                upd.append((y, x, p, i))
            for y, x, p, i in upd:
                Bp_w[level][y, x] = Ap_list[i][level][p[0], p[1]]
                s[y * W + x] = p
                im[y * W + x] = i
        assert np.array_equal(Bp_w[level], ref[level][0])
        assert np.array_equal(s, ref[level][1]) and np.array_equal(im, ref[level][2])


# ---- sharded database: per-rank exact winners + lexicographic min (gloo, 2 ranks) -------------

def _shard_worker(rank, world, port, N, Q, As, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from image_analogies import shard_rows
    r0, nr = shard_rows(N, rank, world)
    d = np.add.reduce((As[r0:r0 + nr][None, :, :] - Q[:, None, :]) ** 2, axis=2)
    loc = np.argmin(d, axis=1)
    mine = torch.tensor(np.stack([d[np.arange(len(Q)), loc], (loc + r0).astype(np.float64)], 1))
    allw = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allw, mine)                      # the RCCL all-gather of ia_comm.hip
    best = []
    for qi in range(len(Q)):
        cands = sorted((float(a[qi, 0]), int(a[qi, 1])) for a in allw)
        best.append(cands[0][1])                     # (distance, lowest row) minimum
    out[rank] = best
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_exchange_equals_global_argmin(world):
    rs = np.random.RandomState(9)
    N = 1001
    As = np.round(rs.rand(N, 55) * 8) / 8      # coarse values: many exact ties across shards
    Q = As[rs.randint(0, N, 40)] + (rs.rand(40, 55) < 0.1) / 8
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + rs.randint(0, 2000)
    mp.spawn(_shard_worker, args=(world, port, N, Q, As, out), nprocs=world, join=True)
    ref = [o.best_approximate_match(As, q) for q in Q]
    for r in range(world):
        assert out[r] == ref
    from image_analogies import shard_rows
    spans = [shard_rows(N, r, world) for r in range(world)]
    assert spans[0][0] == 0 and sum(n for _, n in spans) == N
    assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_branch_free_symmetric_index_equals_period_map():
    """ia_common.h symi2 (three selects, used by every feature gather) equals the
    period-2n symmetric map on its domain i in [-2, n + 1], n >= 1."""
    def symi2(i, n):
        i = -1 - i if i < 0 else i
        i = 2 * n - 1 - i if i >= n else i
        return -1 - i if i < 0 else i
    for n in range(1, 12):
        for i in range(-2, n + 2):
            assert symi2(i, n) == o.sym_index(i, n), (i, n)


def test_shard_level_policy(monkeypatch):
    """Levels below IA_SHARD_MIN_ROWS run replicated on every rank; a 1-rank communicator
    always takes the exchange path; c4's level databases: only the 1 M and 4 M-row levels
    are sharded by default."""
    from image_analogies import level_rows, shard_level
    monkeypatch.delenv('IA_SHARD_MIN_ROWS', raising=False)
    c4 = [128 * 128, 256 * 256, 512 * 512, 1024 * 1024, 2048 * 2048]
    assert [shard_level(n, 8) for n in c4] == [False, False, False, True, True]
    assert all(shard_level(n, 1) for n in c4)
    monkeypatch.setenv('IA_SHARD_MIN_ROWS', '0')
    assert all(shard_level(n, 4) for n in c4)
    pyr = [[np.zeros((2, 3)), np.zeros((4, 6))], [np.zeros((2, 3)), np.zeros((4, 6))]]
    assert level_rows(pyr, 1) == 2 * 24


def test_bench_launcher_starts_the_requested_ranks():
    """`bench.py --gpus 2` without torch.distributed.run's environment starts 2 rank
    processes itself (torch.distributed.run as a child); every rank checks its world size
    against --gpus.  --dry-run: the ranks meet over gloo without touching a GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2',
                          '--dry-run'], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(line) == 1, out.stdout
    rec = json.loads(line[0])
    assert rec['n_gpus'] == 2 and rec['rank_sum'] == 1.0
    # a world that does not match --gpus is refused
    env2 = dict(env, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    bad = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2',
                          '--dry-run'], capture_output=True, text=True, env=env2, timeout=300)
    assert bad.returncode != 0 and 'world size 1 != --gpus 2' in bad.stderr


def test_threaded_oracle_scan_equals_serial():
    """The oracle's 1-NN scan split over threads (row blocks combined in row order) gives
    the serial scan's rows and distances, ties included."""
    import ia_oracle_c as oc
    rs = np.random.RandomState(3)
    A, Aps, B = analogy_inputs(61, (70, 90), (40, 52), n_ap=2, flat=True)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=61)
    job = oc.LevelJob(L - 1, A_pyr, Ap_list, B_pyr, Bp_pyr, o.compute_weights(3, 5, 12, 1), 1.5)
    db = job.build_db()
    N = 2 * A_pyr[L - 1].size
    As = np.ctypeslib.as_array(db, shape=(N * 55,)).reshape(N, 55)
    Q = np.vstack([As[rs.randint(0, N, 40)], As[rs.randint(0, N, 40)] + 1e-9, rs.rand(20, 55)])
    try:
        oc.set_threads(1)
        i1, d1 = oc.nn_batch(db, N, Q)
        serial = [oc.lib().ia_oracle_nn(db, N, oc._d(np.ascontiguousarray(q)), None) for q in Q]
        oc.set_threads(5)
        i5, d5 = oc.nn_batch(db, N, Q)
        par = [oc.lib().ia_oracle_nn(db, N, oc._d(np.ascontiguousarray(q)), None) for q in Q]
    finally:
        oc.set_threads(1)
    ref = [int(np.argmin(np.add.reduce((As - q) ** 2, axis=1))) for q in Q]
    assert list(i1) == ref == serial == par and list(i5) == ref
    assert np.array_equal(d1, d5)


# ---- device-side exchange setup: agreed fallback to RCCL (gloo, 2 ranks, fake library) ---------

class _FakeLib:
    """Stands in for libia.so's exchange entries: rank `bad` fails at step `where` (no
    usable receive box, cannot map a peer's box, or wrong records in the stress waves)."""
    def __init__(self, rank, bad, where, log):
        self.rank, self.bad, self.where, self.log = rank, bad, where, log

    def _fails(self, step):
        return self.rank == self.bad and self.where == step

    def ia_peer_create(self, world, rank, mcap, h, hd):
        self.log.append('peer_create')
        return -4 if self._fails('create') else 0

    def ia_peer_connect(self, h, handles):
        self.log.append('peer_connect')
        return 7 if self._fails('connect') else 0

    def ia_peer_check(self, h, st):
        self.log.append('peer_check')
        return 0

    def ia_diag_peer_stress(self, h, nwaves, M, bad, st):
        self.log.append('peer_stress')
        bad._obj.value = 3 if self._fails('stress') else 0
        return 0

    def ia_comm_destroy(self, h):
        self.log.append('destroy')
        return 0

    def ia_peer_mem_kind(self, h):
        return 0

    def ia_last_error(self):
        return b'hipIpcOpenMemHandle: invalid argument'

    def ia_comm_unique_id(self, buf):
        self.log.append('unique_id')
        return 0

    def ia_comm_init(self, uid, world, rank, h):
        self.log.append('comm_init')
        return 0


def _fallback_worker(rank, world, port, bad, where, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ.pop('IA_EXCHANGE', None)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import _ia
    log = []
    fake = _FakeLib(rank, bad, where, log)
    _ia.lib = lambda: fake
    _ia.stream = lambda: None
    torch.cuda.synchronize = lambda *a: None
    _ia.exchange(rank, world)
    out[rank] = (log, _ia.exchange_kind())
    dist.destroy_process_group()


@pytest.mark.parametrize('bad,where', [(-1, None), (1, 'connect'), (1, 'create'), (0, 'stress')])
def test_peer_exchange_setup_falls_back_to_rccl_on_every_rank(bad, where):
    """_ia.exchange: when one rank has no usable receive box, cannot map the others' boxes
    or sees wrong records in the stress waves, every rank (not only the failing one) drops
    the device-side exchange and builds the RCCL one, so the ranks never disagree on the
    per-wave protocol; with every rank fine, no RCCL setup."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    port = 31500 + np.random.RandomState(bad + 5 + len(where or '')).randint(0, 2000)
    mp.spawn(_fallback_worker, args=(world, port, bad, where, out), nprocs=world, join=True)
    rccl = lambda r: (['unique_id'] if r == 0 else []) + ['comm_init']  # noqa: E731
    for r in range(world):
        log, kind = out[r]
        if bad < 0:
            assert log == ['peer_create', 'peer_connect', 'peer_check', 'peer_stress'] and kind == 'peer'
            continue
        assert kind == 'peer->rccl'
        if where == 'create':
            # the failing rank never got a box; the other destroys its own
            assert log == ['peer_create'] + ([] if r == bad else ['destroy']) + rccl(r)
        elif where == 'connect':
            assert log[:2] == ['peer_create', 'peer_connect'] and 'peer_check' not in log
            assert log[2:] == ['destroy'] + rccl(r)
        else:
            assert log == ['peer_create', 'peer_connect', 'peer_check', 'peer_stress', 'destroy'] + rccl(r)


def _symi2(i, n):
    i = -1 - i if i < 0 else i
    i = 2 * n - 1 - i if i >= n else i
    return -1 - i if i < 0 else i


@pytest.mark.parametrize('h,w', [(8, 128), (9, 256), (64, 384), (2048, 2048)])
def test_strip_windows_hold_every_reflected_sample(h, w):
    """k_xstrip's LDS windows (ia_xwave.hip): for every candidate segment position (nst
    scanlines of a 128-pixel strip, edges included) every sample of every pixel's 55
    features sits in the window at base + fixed offset, holding the reflected image value
    (rows reflected when filled, edge pieces rewritten with symi2 of their columns)."""
    hs, ws = (h + 1) // 2, (w + 1) // 2
    for nst in (1, 2, 4):
        ys = sorted({0, nst, h - nst - (h % nst), h // 2 // nst * nst} - {-1})
        for y0 in [y for y in ys if 0 <= y <= h - nst]:
            for x0 in range(0, w, 128):
                # what each window slot holds: (image row, image col) of its plane
                def fine(r, c, nrows, clamp_row):
                    assert 0 <= r < nrows and 0 <= c < 136
                    R, C = y0 - 2 + r, x0 - 4 + c
                    return _symi2(min(R, clamp_row), h), _symi2(min(max(C, -2), w + 1), w)

                def coarse(r, c):
                    assert 0 <= r < 4 and 0 <= c < 68
                    R, C = (y0 >> 1) - 1 + r, (x0 >> 1) - 2 + c
                    return (_symi2(min(R, ((y0 + nst - 1) >> 1) + 1), hs),
                            _symi2(min(max(C, -2), ws + 1), ws))
                for y in range(y0, y0 + nst):
                    for x in range(x0, x0 + 128, 17):
                        for dy in range(-2, 3):
                            for dx in range(-2, 3):
                                want = (_symi2(y + dy, h), _symi2(x + dx, w))
                                assert fine(y - y0 + 2 + dy, x - x0 + 4 + dx, 8, y0 + nst + 1) == want
                                if dy < 0 or (dy == 0 and dx <= 0):   # A' fine half + the pixel
                                    assert fine(y - y0 + 2 + dy, x - x0 + 4 + dx, 6, y0 + nst - 1) == want
                        for dy in range(-1, 2):
                            for dx in range(-1, 2):
                                want = (_symi2((y >> 1) + dy, hs), _symi2((x >> 1) + dx, ws))
                                assert coarse((y >> 1) - (y0 >> 1) + 1 + dy,
                                              (x >> 1) - (x0 >> 1) + 2 + dx) == want


def test_hot_kernels_do_not_spill():
    """The build's kernel resource reports (csrc/_build/*.res, -Rpass-analysis=kernel-
    resource-usage): the hot path's kernels (screens, the fused strip kernel, pyramid, YIQ,
    DB build) use no scratch memory: a spill there (e.g. G = 11 of the screen at 249 of
    256 VGPRs) costs 2.5x silently."""
    import glob
    import re
    res = glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'image-analogies-python_amd', 'csrc', '_build', '*.res'))
    if not res:
        pytest.skip('no resource reports (build with make -C image-analogies-python_amd/csrc)')
    import hashlib
    hot = ('k_screen16', 'k_xstrip', 'k_pyr_wave', 'k_db_build_t', 'k_rgb_to_yiq', 'k_img_pad')
    # k_xwave (the fused kernel of non-strip levels: c1-c3) has no VGPR spill; its 96 B of
    # scratch is the by-value argument of the cold row-list overflow path (row_rec, noinline)
    no_vgpr_spill = ('k_xwave',)
    seen, bad, stale = 0, [], []
    for f in res:
        text = open(f).read()
        src = os.path.join(os.path.dirname(os.path.dirname(f)), os.path.basename(f)[:-4] + '.hip')
        m = re.search(r'source-sha1: ([0-9a-f]{40})', text)
        if not m or hashlib.sha1(open(src, 'rb').read()).hexdigest() != m.group(1):
            stale.append(os.path.basename(f))
            continue
        name = None
        for line in text.splitlines():
            m = re.search(r'Function Name: (\S+)', line)
            if m:
                name = m.group(1)
                continue
            m = re.search(r'ScratchSize \[bytes/lane\]: (\d+)', line)
            # (the batch form k_xstrip<true, ...> is built for 4 workgroups per CU and spills
            # 17 VGPRs there: measured faster than unspilled at 3 per CU, c5 +2.3-3.6 % on one
            # box, profiles/r06_c5_xstrip_occupancy_ab.txt; the single-job form is checked)
            if m and name and 'k_xstripILb1E' in name:
                continue
            if m and name and any(h in name for h in hot):
                seen += 1
                if int(m.group(1)) != 0:
                    bad.append((name, int(m.group(1))))
            m = re.search(r'VGPRs Spill: (\d+)', line)
            if m and name and any(h in name for h in no_vgpr_spill):
                seen += 1
                if int(m.group(1)) != 0:
                    bad.append((name, 'VGPR spill', int(m.group(1))))
    if stale:
        pytest.skip('resource reports older than their sources (rebuild): %s' % stale)
    assert seen > 20, seen
    assert not bad, bad


def test_oracle_index_equals_scan():
    """The oracle's projection index (ia_oracle_c.Index, used to generate full-size fixtures)
    returns the brute-force scan's row and distance for every query, exact duplicates and
    1e-12 near-ties included, and the indexed synthesis equals the scanning one."""
    import ia_oracle_c as oc
    rs = np.random.RandomState(7)
    A, Aps, B = analogy_inputs(62, (70, 90), (40, 52), n_ap=2, flat=True)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=62)
    db = oc.LevelDB(L - 1, A_pyr, Ap_list)
    N = db.N
    Q = np.vstack([db.rows[rs.randint(0, N, 30)], db.rows[rs.randint(0, N, 30)] + 1e-12,
                   db.rows[rs.randint(0, N, 30)] + rs.randn(30, 55) * 1e-3, rs.rand(10, 55)])
    i0, d0 = db.nn(Q)
    for P in (1, 4):
        i1, d1 = db.index(P).nn(Q)
        assert np.array_equal(i0, i1) and np.array_equal(d0, d1)
    w = o.compute_weights(3, 5, 12, 1)
    outs = []
    for indexed in (False, True):
        bp = [b.copy() for b in Bp_pyr]
        outs.append(oc.synthesize(A_pyr, Ap_list, B_pyr, bp, L, 0.5, w, indexed=indexed))
    for l in outs[0]:
        for a, b in zip(outs[0][l], outs[1][l]):
            assert np.array_equal(a, b), l


def test_chunk_target_is_per_thread():
    """a batch's chunk target (ia_set_chunk_target) must not reach another
    thread's DB builds and syntheses (their layouts derive from it)."""
    import threading
    import _ia
    lib = _ia.lib()
    N = 262144
    base = lib.ia_db_chunk_rows(N)
    prev = lib.ia_set_chunk_target(64)
    try:
        mine = lib.ia_db_chunk_rows(N)
        other = []
        th = threading.Thread(target=lambda: other.append(lib.ia_db_chunk_rows(N)))
        th.start()
        th.join()
        assert mine > base and other == [base]
    finally:
        lib.ia_set_chunk_target(prev)
    assert lib.ia_db_chunk_rows(N) == base


def test_residency_rule_refuses_the_known_starvation():
    """The forward-progress rule for sharded levels over the device-side exchange
    (image_analogies.residency_ok / sharded_schedule): workgroups of the fused
    kernel that wait for other ranks must leave a CU for the screens.  The configuration
    that timed out in round 4 (commit 1efae07: the producer / consumer screen, ~94 KB of LDS
    and 256 VGPRs, beside 2 ranks' waiting k_xstrip workgroups on one GPU) is refused; the
    production c4 layout (one rank per GPU, the finest and the 1 M-row level sharded and
    pipelined, the rotated screen) pipelines; 2 ranks sharing a GPU serialize the sharded
    levels; 3 are refused."""
    import image_analogies as ia
    c4 = [(1024, 1024), (512, 512)]
    fused_r16, screen_r16 = (36864, 135), (60416, 158)
    fused_r4, screen_pc = (36864, 148), (96 * 1024, 256)
    ok, j = ia.residency_ok(2 * ia.wave_max_queries(1024, 1024), fused_r4, screen_pc)
    assert not ok and j == 1
    with pytest.raises(RuntimeError, match='forward progress'):
        ia.sharded_schedule(c4, True, 2, fused_r4, screen_pc)
    assert ia.sharded_schedule(c4, True, 1, fused_r16, screen_r16) is True
    assert ia.sharded_schedule(c4, True, 2, fused_r16, screen_r16) is False
    with pytest.raises(RuntimeError, match='forward progress'):
        ia.sharded_schedule(c4, True, 3, fused_r16, screen_r16)
    # the pigeonhole bound itself: cus * (jmax + 1) waiting workgroups can fill every CU
    ok, j = ia.residency_ok(256 * 3 - 1, fused_r16, screen_r16)
    assert ok and j == 2
    assert not ia.residency_ok(256 * 3, fused_r16, screen_r16)[0]


def test_pass_check_classifies_a_cascade_as_an_exchange_failure(monkeypatch):
    """A dead or slow peer also trips the fused kernel's neighbour-decision waits (the same
    10 s limit): with both error words set, bench.pass_check raises ExchangeTimeout (the one
    error its RCCL fallback handles), not ScheduleFault; the neighbour fault alone still
    raises ScheduleFault (a fake lib reports the words; no GPU)."""
    import _ia
    import bench

    class FakeLib:
        def __init__(self, peer, sched):
            self.peer, self.sched = peer, sched

        def ia_peer_mem_kind(self, comm):
            return 0

        def ia_peer_status(self, comm):
            return self.peer

        def ia_sched_status(self, clear):
            return self.sched

        def ia_last_error(self):
            return b'a wait timed out'

    monkeypatch.setattr(bench.torch.cuda, 'synchronize', lambda *a: None)
    monkeypatch.setattr(_ia, 'lib', lambda: FakeLib(_ia.IA_E_TIMEOUT, _ia.IA_E_SCHED))
    with pytest.raises(_ia.ExchangeTimeout):
        bench.pass_check([object()])
    monkeypatch.setattr(_ia, 'lib', lambda: FakeLib(0, _ia.IA_E_SCHED))
    with pytest.raises(_ia.ScheduleFault):
        bench.pass_check([object()])
    monkeypatch.setattr(_ia, 'lib', lambda: FakeLib(0, 0))
    bench.pass_check([object()])


def test_residency_rule_takes_each_levels_own_kernels():
    """the rule must take every sharded level's own fused kernel.  A non-strip
    level runs k_xwave (2 workgroups per CU: ~52 KB of LDS, ~252 VGPRs), so a CU beside a
    screen holds at most one waiting workgroup of it (j_max 1), not the strip kernel's two:
    2 ranks sharing one GPU on a ~1000-px-wide sharded level (2 x 335 waiting workgroups)
    are admitted with k_xstrip's resources and refused with k_xwave's; a strip level plus a
    k_xwave level are pipelined only if the worst of both fits."""
    import image_analogies as ia
    xstrip, xwave, screen = (36864, 135), (52224, 252), (60416, 158)
    lvl = [(1000, 1000)]
    assert ia.residency_ok(2 * ia.wave_max_queries(1000, 1000), xstrip, screen)[0]
    assert ia.sharded_schedule(lvl, True, 2, [xstrip], [screen]) is True
    ok, j = ia.residency_ok(2 * ia.wave_max_queries(1000, 1000), xwave, screen)
    assert not ok and j == 1
    with pytest.raises(RuntimeError, match='forward progress'):
        ia.sharded_schedule(lvl, True, 2, [xwave], [screen])
    # one rank per GPU: c4's finest (strip) level beside a k_xwave level of 172 queries
    two = [(1024, 1024), (512, 512)]
    assert ia.sharded_schedule(two, True, 1, [xstrip, xstrip], [screen, screen]) is True
    assert ia.sharded_schedule(two, True, 1, [xstrip, xwave], [screen, screen]) is False


# ---- multi-GPU from the package API (gloo, 2 ranks; the device calls are faked) -------------

def test_rank_jobs_partition_and_bench_seeds():
    """image_analogies.rank_jobs splits n jobs over ranks as j = rank (mod world): disjoint,
    complete, and bench.py's c5 job seeds (1000 + 3 (rank + world i)) are its indices."""
    import image_analogies as ia
    for n, world in ((32 * 8, 8), (7, 3), (2, 4), (0, 2)):
        parts = [ia.rank_jobs(n, r, world) for r in range(world)]
        flat = sorted(j for p in parts for j in p)
        assert flat == list(range(n))
        for r, p in enumerate(parts):
            assert all(j % world == r for j in p)
    assert [1000 + 3 * j for j in ia.rank_jobs(16, 1, 4)] == [1000 + 3 * (1 + 4 * i) for i in range(4)]
    with pytest.raises(ValueError):
        ia.rank_jobs(4, 2, 2)


class _Shape:
    def __init__(self, *shape):
        self.shape = shape


def _api_worker(rank, world, port, tmp, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import _ia
    import image_analogies as ia
    log = {'batch': [], 'single': [], 'dev': [], 'exch': 0, 'destroyed': 0, 'main': []}
    # synthesize_jobs: the whole job list; this rank's entries are callables, the others None
    jobs = [(lambda j=j: ('job', j, None, None)) if j % world == rank else None for j in range(7)]

    def fake_batch(ins, L, ks, w, prof=False, debug=False, check=True):
        log['batch'].append(([x[1] for x in ins], list(ks)))
        return [{'job': x[1]} for x in ins]

    def fake_dev(A_pyr, Ap, B_pyr, Bp, L, k, w, comm=None, rank=0, nranks=1, **kw):
        if A_pyr == 'job':
            log['single'].append((Ap, k))
            return {'job': Ap}
        log['dev'].append((None if comm is None else len(comm), rank, nranks))
        return {l: (None, None) for l in range(1, L)}
    ia.synthesize_batch_dev = fake_batch
    ia.synthesize_dev = fake_dev
    ks = [0.5 * j for j in range(7)]
    res = ia.synthesize_jobs(jobs, 4, ks, None, rank, world, batch=2)
    out['jobs%d' % rank] = (sorted(res), log['batch'], log['single'])
    # image_analogies_main(comm='auto'): one exchange per sharded level, the device calls
    # with this rank's place, files written by rank 0 only
    import config as c

    class FakeLib:
        def ia_comm_destroy(self, h):
            log['destroyed'] += 1
            return 0
    _ia.lib = lambda: FakeLib()
    _ia.to_dev = lambda x: x
    _ia.exchange_status = lambda cm: None

    def fake_exchange(r, wsz, kind=None):
        assert (r, wsz) == (rank, world)
        log['exch'] += 1
        return object()
    _ia.exchange = fake_exchange
    torch.cuda.synchronize = lambda *a: None
    ia._read = lambda f: np.zeros((4, 4))
    Ap_pyr = [_Shape(2, 2), _Shape(256, 256), _Shape(768, 768), _Shape(1024, 1024)]

    class Lvl:
        def __init__(self, n):
            self.shape = (n, n)

        def cpu(self):
            return self

        def numpy(self):
            return np.zeros(self.shape)

    def fake_setup(A, Aps, B, cc):
        cc.max_levels = 4
        cc.weights = np.ones(55)
        return None, [Ap_pyr], None, [Lvl(2), Lvl(256), Lvl(512), Lvl(1024)], None
    ia.setup_dev = fake_setup
    ia.color_output = lambda *a: np.zeros((2, 2, 3))
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    plt.imsave = lambda path, im: open(path, 'w').close()
    path = os.path.join(tmp, 'run%d/' % 0)
    ia.image_analogies_main('A.jpg', ['Ap.jpg'], 'B.jpg', path, c, comm='auto')
    out['main%d' % rank] = (log['dev'], log['exch'], log['destroyed'])
    # multi_main: the serial script loop spread over the ranks, overrides applied per run
    runs = [('A%d' % j, ['Ap%d' % j], 'B%d' % j, os.path.join(tmp, 'm%d/' % j), {'k': j + 0.5})
            for j in range(5)]

    def fake_main(A, Aps, B, p, cc, debug=False, rank=None, nranks=None, **kw):
        log['main'].append((A, cc.k, rank, nranks))
        return A
    ia.image_analogies_main = fake_main
    got = ia.multi_main(runs, c)
    out['multi%d' % rank] = (sorted(got), log['main'])
    dist.destroy_process_group()


def test_multi_gpu_package_entry_points_gloo(tmp_path):
    """multi-GPU reachable from the drop-in API, driven over a gloo world of 2
    (device calls faked, no GPU): synthesize_jobs runs rank r's jobs j = r (mod 2) in
    batches with their own kappas; image_analogies_main(comm='auto') makes one exchange per
    sharded level (c4-like shapes: the two levels of >= 2^19 rows), passes each rank's place
    to the synthesis, releases the exchanges, and only rank 0 writes the outputs;
    multi_main spreads the script's runs likewise with each run's config overrides."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    port = 33500 + np.random.RandomState(17).randint(0, 1000)
    mp.spawn(_api_worker, args=(world, port, str(tmp_path), out), nprocs=world, join=True)
    ks = [0.5 * j for j in range(7)]
    for r in range(world):
        mine, batches, singles = out['jobs%d' % r]
        assert mine == [j for j in range(7) if j % world == r]
        flat = [j for b, _ in batches for j in b] + [j for j, _ in singles]
        assert sorted(flat) == mine
        assert all(len(b) <= 2 for b, _ in batches)
        for b, kk in batches:
            assert kk == [ks[j] for j in b]
        dev, nexch, ndestroyed = out['main%d' % r]
        assert dev == [(2, r, world)] and nexch == 2 and ndestroyed == 2
        got, calls = out['multi%d' % r]
        assert got == [j for j in range(5) if j % world == r]
        assert [(a, k) for a, k, _, _ in calls] == [('A%d' % j, j + 0.5) for j in got]
        assert all(rk == 0 and nr == 1 for _, _, rk, nr in calls)
    assert os.path.exists(os.path.join(str(tmp_path), 'run0', 'metadata.txt'))
