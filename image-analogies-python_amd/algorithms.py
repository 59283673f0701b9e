"""Feature construction and matching — drop-in for the reference's ``algorithms`` module
(reference algorithms.py:1-135), computed by libia.so.

    compute_feature_array   ia_level_features_f64 (a9)
    create_index            per level: resident fp64 source pyramids + the split-f16
                            screening database (ia_db_build, a10); returns
                            (index handles, params, As, As_size) like the reference
    best_approximate_match  ia_match_batch on one query (a11) — EXACT 1-NN, where the
                            reference asks FLANN's randomized kd-tree
    best_coherence_match    candidate bookkeeping as the reference + ia_coherence_pick (a13)
    compute_distance        ia_wdist_batch (a14)

The synthesis path (image_analogies.py) does not call the per-pixel functions: it runs
whole levels on device through ``ia_synth_level``.
"""
import ctypes

import numpy as np
import torch

import _ia


# ---- features -----------------------------------------------------------------------------

def level_features_dev(sm, lg, full_feat):
    """One level of compute_feature_array on device: (h*w, 34 or 21) fp64."""
    hs, ws = sm.shape
    h, w = lg.shape
    out = torch.empty((h * w, 34 if full_feat else 21), dtype=torch.float64, device=lg.device)
    _ia.check(_ia.lib().ia_level_features_f64(_ia.ptr(sm), hs, ws, _ia.ptr(lg), h, w,
                                              1 if full_feat else 0, _ia.ptr(out),
                                              _ia.stream()), 'ia_level_features_f64')
    return out


def level_features3_dev(sm, lg, full_feat):
    """One level of compute_feature_array for 3-channel images (h, w, 3): (h*w, 102 or
    63) fp64, windows flattened (row, col, channel)."""
    hs, ws = sm.shape[:2]
    h, w = lg.shape[:2]
    out = torch.empty((h * w, 102 if full_feat else 63), dtype=torch.float64, device=lg.device)
    _ia.check(_ia.lib().ia_level_features3_f64(_ia.ptr(sm.contiguous()), hs, ws,
                                               _ia.ptr(lg.contiguous()), h, w,
                                               1 if full_feat else 0, _ia.ptr(out),
                                               _ia.stream()), 'ia_level_features3_f64')
    return out


def compute_feature_array(im_pyr, c, full_feat):
    """Per-level [3x3 coarse | 5x5 (or half) fine] neighbourhood rows
    (algorithms.py:11-47), 1 or 3 channels; entry 0 is an empty placeholder as in the
    reference."""
    dev = [_ia.to_dev(p) for p in im_pyr]
    fn = level_features3_dev if dev[0].dim() == 3 else level_features_dev
    feats = [[]]
    for level in range(1, len(im_pyr)):
        feats.append(fn(dev[level - 1], dev[level], full_feat).cpu().numpy())
    return feats


# ---- the level database (index) ---------------------------------------------------------------

def lsh_projections(tables, hashes, width, seed=0):
    """E2LSH parameters (host): (tables*hashes, 56) float32 rows, p ~ N(0, I_55) in
    elements 0..54 and the offset b ~ U[0, width) in element 55."""
    rs = np.random.RandomState(seed)
    n = int(tables) * int(hashes)
    P = np.zeros((n, _ia.IA_DP), dtype=np.float32)
    P[:, :55] = rs.standard_normal((n, 55))
    P[:, 55] = rs.uniform(0.0, width, n)
    return P


def lsh_params(c):
    """LSH settings from the config namespace (None unless c.matcher == 'lsh')."""
    if getattr(c, 'matcher', 'brute') != 'lsh':
        return None
    return dict(tables=getattr(c, 'lsh_tables', 16), hashes=getattr(c, 'lsh_hashes', 4),
                width=getattr(c, 'lsh_width', 1.0), seed=getattr(c, 'lsh_seed', 0))


class LevelIndex:
    """Device-resident As[level] for rows [row0, row0 + nrows) (a shard when sharded).

    Holds the fp64 A / A' pyramid levels (the exact rescore gathers features straight
    from them) and the split-f16 screening database: its image form (ia_db_build_image, one
    split pair per pixel) where the level allows it, else the 224-B rows of ia_db_build.  Centre = the means
    of A (34 A dims) and of the A' images (21 A' dims): any centre is exact for the
    distances; centring only tightens the screen's error bound.
    """

    def __init__(self, A_sm, A_lg, Ap_sm, Ap_lg, row0=0, nrows=None, rows=None, rot=False):
        self.A_sm, self.A_lg = A_sm.contiguous(), A_lg.contiguous()
        self.Ap_sm, self.Ap_lg = Ap_sm.contiguous(), Ap_lg.contiguous()
        self.src = _ia.src_level(self.A_sm, self.A_lg, self.Ap_sm, self.Ap_lg)
        self.N = int(Ap_lg.shape[0] * Ap_lg.shape[1] * Ap_lg.shape[2])
        self.row0 = int(row0)
        self.nrows = self.N - self.row0 if nrows is None else int(nrows)
        self.shape = (self.N, 55)
        dev = A_lg.device
        lib = _ia.lib()
        st = _ia.stream()
        mA = _ia.mean_dev(self.A_lg)
        mAp = _ia.mean_dev(self.Ap_lg)
        self.center = torch.empty(55, dtype=torch.float64, device=dev)
        _ia.check(lib.ia_center_fill(_ia.ptr(self.center), mA, mAp, st), 'ia_center_fill')
        self.amax = torch.zeros(2, dtype=torch.float32, device=dev)   # {A, A_skip (R16)}
        # the image form where it applies: the matcher then reads only it, and
        # the 224-B rows are built only on request (rows=True: tests, the row-form bench leg)
        ibytes = (lib.ia_db_image_bytes(ctypes.byref(self.src), self.row0, self.nrows)
                  if _ia.db_image_enabled() else 0)
        self.db = self.dbi = None
        if rows or not ibytes:
            nbytes = lib.ia_db_bytes(self.nrows)      # split-f16 rows, 224 B each
            self.db = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            _ia.check(lib.ia_db_build(ctypes.byref(self.src), self.row0, self.nrows,
                                      _ia.ptr(self.center), _ia.ptr(self.db), _ia.ptr(self.amax),
                                      st), 'ia_db_build')
        if ibytes:
            self.dbi = torch.empty(ibytes, dtype=torch.uint8, device=dev)
            _ia.check(lib.ia_db_build_image(ctypes.byref(self.src), self.row0, self.nrows,
                                            _ia.ptr(self.center), _ia.ptr(self.db),
                                            _ia.ptr(self.amax), _ia.ptr(self.dbi), st),
                      'ia_db_build_image')
        self.lsh = None
        self.dbr = self.rot = None
        if rot and lib.ia_db_rot_applies(ctypes.byref(self.src), self.row0, self.nrows):
            self.build_rot()

    def build_rot(self):
        """The rotated split DB of the synthesis screen (R16): the covariance
        of ~64 k sampled centred rows on device (ia_db_cov), its eigenvectors on the host
        (55 x 55; any orthonormal basis keeps the matcher exact, the principal one keeps its
        bound tight), then ia_db_build_rot (amax[1] = A_skip)."""
        lib, st, dev = _ia.lib(), _ia.stream(), self.A_lg.device
        cov = torch.empty(lib.ia_db_cov_bytes() // 8, dtype=torch.float64, device=dev)
        _ia.check(lib.ia_db_cov(ctypes.byref(self.src), self.row0, self.nrows,
                                _ia.ptr(self.center), _ia.ptr(cov), st), 'ia_db_cov')
        C = cov[:56 * 56].view(56, 56)[:55, :55].cpu().numpy()
        w, V = _eigh(C)
        V = V[:, ::-1]                       # components by decreasing variance
        R = np.zeros(_ia.R16_ROT_FLOATS, dtype=np.float32)
        R[:56 * 56].reshape(56, 56)[:55, :55] = V.astype(np.float32)
        self.rot_var = w[::-1].copy()
        self.rot = torch.as_tensor(R).to(dev)
        self.dbr = torch.empty(lib.ia_db_rot_bytes(self.nrows), dtype=torch.uint8, device=dev)
        _ia.check(lib.ia_db_build_rot(ctypes.byref(self.src), self.row0, self.nrows,
                                      _ia.ptr(self.center), _ia.ptr(self.rot), _ia.ptr(self.amax),
                                      _ia.ptr(self.dbr), st), 'ia_db_build_rot')
        return self

    def dbi_ptr(self):
        return _ia.ptr(self.dbi).value if self.dbi is not None else None

    def build_lsh(self, tables=16, hashes=4, width=1.0, seed=0):
        """Switch this index to the approximate LSH matcher (c.matcher = 'lsh', SURVEY
        §8(f)1): ``tables`` x ``hashes`` Gaussian projections drawn from
        RandomState(seed), bucket width ``width`` x the RMS per-dimension spread of the
        centred rows (estimated from the A / A' pixel variances)."""
        dev = self.A_lg.device
        L, k = int(tables), int(hashes)
        if not (1 <= L and 1 <= k and L * k <= 64):
            raise ValueError('LSH needs 1 <= tables * hashes <= 64')
        var = (34 * _ia.var_f64(self.A_lg) + 21 * _ia.var_f64(self.Ap_lg)) / 55.0
        w = float(width) * max(np.sqrt(var), 1e-6)
        self.lsh_proj_host = lsh_projections(L, k, w, seed)
        self.lsh_proj = torch.as_tensor(self.lsh_proj_host).to(dev)
        lib = _ia.lib()
        self.lsh_mem = _ia.workspace(lib.ia_lsh_bytes(self.nrows, L))
        h = _ia.IaLsh()
        h.mem, h.proj, h.L, h.k, h.w = (_ia.ptr(self.lsh_mem).value, _ia.ptr(self.lsh_proj).value,
                                        L, k, w)
        _ia.check(lib.ia_lsh_build(ctypes.byref(self.src), self.row0, self.nrows,
                                   _ia.ptr(self.center), ctypes.byref(h), _ia.stream()),
                  'ia_lsh_build')
        self.lsh = h
        return self

    def lsh_ptr(self):
        return ctypes.pointer(self.lsh) if self.lsh is not None else None

    def match(self, Q, exact=None):
        """1-NN rows (global index, fp64 distance) of queries Q (M x 55): exact, or from
        the LSH buckets when build_lsh() was called (``exact=True`` forces exact)."""
        dev = self.A_lg.device
        Q = torch.as_tensor(Q, dtype=torch.float64)
        if Q.dim() == 1:
            Q = Q[None]
        M = Q.shape[0]
        q = torch.zeros((M, _ia.IA_DP), dtype=torch.float64, device=dev)
        q[:, :55] = Q.to(dev)
        idx = torch.empty(M, dtype=torch.int64, device=dev)
        dist = torch.empty(M, dtype=torch.float64, device=dev)
        ws = _ia.workspace(_ia.lib().ia_match_workspace_bytes(M, self.nrows))
        a = _ia.IaMatchArgs()
        a.src = self.src
        a.db, a.row0, a.nrows = _ia.ptr(self.db).value, self.row0, self.nrows
        a.center, a.amax, a.q64, a.M = (_ia.ptr(self.center).value, _ia.ptr(self.amax).value,
                                        _ia.ptr(q).value, M)
        a.idx, a.dist, a.workspace = _ia.ptr(idx).value, _ia.ptr(dist).value, _ia.ptr(ws).value
        a.dbi = self.dbi_ptr()
        if not exact and self.lsh is not None:
            a.lsh = self.lsh_ptr()
        _ia.check(_ia.lib().ia_match_batch(ctypes.byref(a), _ia.stream()), 'ia_match_batch')
        return idx, dist

    def features(self):
        """The full fp64 As[level] matrix (N x 55), materialised on demand."""
        A = level_features_dev(self.A_sm, self.A_lg, True)
        rows = [torch.cat([A, level_features_dev(self.Ap_sm[i], self.Ap_lg[i], False)], 1)
                for i in range(self.Ap_lg.shape[0])]
        return torch.cat(rows, 0)


def _eigh(C):
    """np.linalg.eigh of a small covariance (55 or 165 square) on ONE BLAS thread: the
    threaded LAPACK is slower at this size (165: 3.8-4.6 vs 5.7-6.0 ms on 8 threads, more
    with 16 busy ones)."""
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:   # (the pin is only a speed-up)
        return np.linalg.eigh(C)
    with threadpool_limits(1):
        return np.linalg.eigh(C)


def rot3_rotation(db3, N):
    """The rotation of the 3-channel screen (R16c) from an ia_db3_build buffer:
    the covariance of ~64 k sampled rows around their mean (ia_db3_cov, on device), its
    eigenvectors on the host (165 x 165; one device sync).  Any orthonormal basis keeps the
    matcher exact; the principal one keeps the bound tight."""
    lib, st = _ia.lib(), _ia.stream()
    cov = torch.empty(lib.ia_db3_cov_bytes() // 8, dtype=torch.float64, device=db3.device)
    _ia.check(lib.ia_db3_cov(_ia.ptr(db3), N, _ia.ptr(cov), st), 'ia_db3_cov')
    w, V = _eigh(cov[:165 * 168].view(165, 168)[:, :165].cpu().numpy())
    R = np.zeros(lib.ia_db3_rot_floats(), dtype=np.float32)
    R.reshape(165, 168)[:, :165] = V[:, ::-1]
    return torch.as_tensor(R).to(db3.device)


def rot3_apply(db3, N, rot):
    """The rotated split DB of one level under rotation rot (ia_db3_build_rot)."""
    lib, st = _ia.lib(), _ia.stream()
    dbr = torch.empty(lib.ia_db3_rot_bytes(N), dtype=torch.uint8, device=db3.device)
    _ia.check(lib.ia_db3_build_rot(_ia.ptr(db3), N, _ia.ptr(rot), _ia.ptr(dbr), st), 'ia_db3_build_rot')
    return dbr


def rot3_build(db3, N):
    """The rotated split DB of the 3-channel screen from one level's own principal directions.
    Returns (rot, dbr)."""
    rot = rot3_rotation(db3, N)
    return rot, rot3_apply(db3, N, rot)


class LevelIndex3:
    """As[level] for 3-channel images (num_ch = 3): the materialised fp64 rows
    [A full | A'_i half], 165 values each (ia_db3_build, which also builds the split-f16
    rows of the synthesis screen after them), searched exhaustively in fp64
    (ia_match3_batch) — exact like LevelIndex."""

    def __init__(self, A_sm, A_lg, Ap_sm, Ap_lg):
        self.A_sm, self.A_lg = A_sm.contiguous(), A_lg.contiguous()
        self.Ap_sm, self.Ap_lg = Ap_sm.contiguous(), Ap_lg.contiguous()
        src = _ia.IaSrcLevel()
        src.A_sm, src.A_lg, src.Ap_sm, src.Ap_lg = (_ia.ptr(self.A_sm).value, _ia.ptr(self.A_lg).value,
                                                    _ia.ptr(self.Ap_sm).value, _ia.ptr(self.Ap_lg).value)
        src.A_hs, src.A_ws = self.A_sm.shape[:2]
        src.Ah, src.Aw = self.A_lg.shape[:2]
        src.nAp = self.Ap_lg.shape[0]
        self.src = src
        self.N = int(src.nAp * src.Ah * src.Aw)
        self.shape = (self.N, 165)
        lib = _ia.lib()
        self.db3 = torch.empty(lib.ia_db3_bytes(self.N) // 8, dtype=torch.float64,
                               device=A_lg.device)
        _ia.check(lib.ia_db3_build(ctypes.byref(src), 0, self.N, _ia.ptr(self.db3), _ia.stream()),
                  'ia_db3_build')
        self.lsh = None
        self.rot = self.dbr = None

    def build_rot(self):
        """The rotated split DB of the synthesis screen (R16c, rot3_build)."""
        self.rot, self.dbr = rot3_build(self.db3, self.N)
        return self

    def match(self, Q, exact=None):
        """1-NN rows (global index, fp64 distance) of queries Q (M x 165)."""
        dev = self.A_lg.device
        Q = torch.as_tensor(Q, dtype=torch.float64)
        if Q.dim() == 1:
            Q = Q[None]
        Q = Q.to(dev).contiguous()
        M = Q.shape[0]
        idx = torch.empty(M, dtype=torch.int64, device=dev)
        dist = torch.empty(M, dtype=torch.float64, device=dev)
        ws = _ia.workspace(_ia.lib().ia_match3_workspace_bytes(M, self.N))
        _ia.check(_ia.lib().ia_match3_batch(_ia.ptr(self.db3), self.N, _ia.ptr(Q), M, _ia.ptr(idx),
                                            _ia.ptr(dist), _ia.ptr(ws), _ia.stream()),
                  'ia_match3_batch')
        return idx, dist

    def features(self):
        """The full fp64 As[level] matrix (N x 165)."""
        return self.db3[:self.N * 168].view(self.N, 168)[:, :165]


class _LazyAs(list):
    """``As`` of the reference: As[level] is the (N, 55) (3 channels: 165) fp64 feature matrix.  Levels are
    materialised from the device index only when a caller indexes them."""

    def __init__(self, index):
        super().__init__([[] for _ in index])
        self._index = index

    def __getitem__(self, level):
        cur = super().__getitem__(level)
        if isinstance(cur, list) and self._index[level] is not None:
            cur = self._index[level].features().cpu().numpy()
            super().__setitem__(level, cur)
        return cur


def level_index(A_pyr, Ap_pyr_list, level, row_range=None, lsh=None, rows=None, rot=None):
    """Device index of one level from device pyramids.  row_range(level, N) ->
    (row0, nrows) selects this rank's shard of the rows; lsh (dict of build_lsh
    arguments) switches it to the LSH matcher; rows=True keeps the row form next to the
    image form; rot (default: the exact matcher on a level or shard of at least
    _ia.rot_min_rows() rows) also builds the synthesis screen's rotated DB (R16)."""
    Ap_sm = torch.stack([p[level - 1] for p in Ap_pyr_list])
    Ap_lg = torch.stack([p[level] for p in Ap_pyr_list])
    N = Ap_lg.shape[0] * Ap_lg.shape[1] * Ap_lg.shape[2]
    r0, nr = (0, N) if row_range is None else row_range(level, N)
    if rot is None:
        rot = lsh is None and _ia.db_rot_enabled() and nr >= _ia.rot_min_rows()
    index = LevelIndex(A_pyr[level - 1], A_pyr[level], Ap_sm, Ap_lg, r0, nr, rows=rows, rot=rot)
    if lsh is not None:
        index.build_lsh(**lsh)
    return index


def create_index_dev(A_pyr, Ap_pyr_list, max_levels, row_range=None, lsh=None):
    """Device index per level 1..max_levels-1 (entry 0 unused)."""
    return [None] + [level_index(A_pyr, Ap_pyr_list, l, row_range, lsh)
                     for l in range(1, max_levels)]


def create_index(A_pyr, Ap_pyr_list, c):
    """Per-level database of [A full | A'_i half] rows (algorithms.py:50-70).  Returns
    (index, params, As, As_size) in the reference's shape: ``index[level]`` replaces the
    FLANN object, ``params[level]`` describes it, ``As`` materialises lazily."""
    dev = _ia.require_device()
    A_dev = [_ia.to_dev(p) for p in A_pyr]
    Ap_dev = [[_ia.to_dev(p) for p in pyr] for pyr in Ap_pyr_list]
    lsh = lsh_params(c)
    if A_dev[0].dim() == 3:      # 3 channels: materialised rows, exact search
        if lsh is not None:
            raise NotImplementedError('3-channel matching runs with the exact matcher only')
        index = [None] + [LevelIndex3(A_dev[l - 1], A_dev[l],
                                      torch.stack([p[l - 1] for p in Ap_dev]),
                                      torch.stack([p[l] for p in Ap_dev]))
                          for l in range(1, c.max_levels)]
    else:
        index = create_index_dev(A_dev, Ap_dev, c.max_levels, lsh=lsh)
    if lsh is None:
        desc = {'algorithm': 'brute', 'exact': True, 'device': str(dev)}
    else:
        desc = dict(lsh, algorithm='lsh', exact=False, device=str(dev))
    params = [[]] + [dict(desc) for _ in range(1, c.max_levels)]
    As_size = [[]] + [index[l].shape for l in range(1, c.max_levels)]
    return index, params, _LazyAs(index), As_size


def best_approximate_match(flann, params, BBp_feat):
    """Nearest database row of one query (algorithms.py:73-75) — exact."""
    idx, _ = flann.match(np.asarray(BBp_feat, dtype=np.float64)[None])
    return int(idx[0].item())


def best_approximate_match_batch(flann, Q):
    """Batched form: nearest rows of M queries (M x 55) -> int64 numpy array."""
    idx, _ = flann.match(np.asarray(Q, dtype=np.float64))
    return idx.cpu().numpy()


# ---- per-pixel helpers ---------------------------------------------------------------------------

def extract_pixel_feature(padded_pair, px, c, full_feat):
    """Feature of one pixel from a padded (coarse, fine) pair (algorithms.py:78-89)."""
    im_sm_padded, im_lg_padded = padded_pair
    row, col = int(px[0]), int(px[1])
    rs, cs = row // 2, col // 2
    f = np.concatenate([
        im_sm_padded[rs:rs + 2 * c.pad_sm + 1, cs:cs + 2 * c.pad_sm + 1].ravel(),
        im_lg_padded[row:row + 2 * c.pad_lg + 1, col:col + 2 * c.pad_lg + 1].ravel()])
    return f if full_feat else f[:c.num_ch * (c.n_sm * c.n_sm + c.n_half)]


def best_coherence_match(As, A_shape, BBp_feat, s, im, px, Bp_w, c):
    """Coherence candidate p = s(r*) + (q - r*) over the causal 5x5 half window
    (algorithms.py:92-130); the distance argmin runs on device."""
    assert len(s) >= 1
    A_h, A_w = A_shape
    row, col = int(px[0]), int(px[1])
    q_ix = row * Bp_w + col
    cands, rows = [], []
    for rr in range(max(0, row - c.pad_lg), row + 1):
        for cc in range(max(0, col - c.pad_lg), min(Bp_w, col + c.pad_lg + 1)):
            r_ix = rr * Bp_w + cc
            if r_ix >= q_ix:
                continue
            pr = (int(s[r_ix][0]) + row - rr, int(s[r_ix][1]) + col - cc)
            if 0 <= pr[0] < A_h and 0 <= pr[1] < A_w:
                img = int(im[r_ix])
                cands.append(((rr, cc), img))
                rows.append(((A_h * img) + pr[0]) * A_w + pr[1])
    if not cands:
        return (-1, -1), 0, (0, 0)
    feats = _ia.to_dev(np.asarray(As[np.array(rows)], dtype=np.float64))
    q = _ia.to_dev(np.asarray(BBp_feat, dtype=np.float64))
    out = torch.empty(1, dtype=torch.int32, device=q.device)
    pick = _ia.lib().ia_coherence_pick3 if feats.shape[1] == 165 else _ia.lib().ia_coherence_pick
    _ia.check(pick(_ia.ptr(feats), len(rows), _ia.ptr(q), _ia.ptr(out), _ia.stream()),
              'ia_coherence_pick')
    (rr, cc), img = cands[int(out.item())]
    sr = s[rr * Bp_w + cc]
    return np.array([int(sr[0]) + row - rr, int(sr[1]) + col - cc]), img, np.array([rr, cc])


def compute_distance(AAp_p, BBp_q, weights):
    """Weighted squared distance |(a - q) * w|^2 (algorithms.py:133-135)."""
    assert AAp_p.shape == BBp_q.shape == weights.shape
    a, q, w = (_ia.to_dev(np.asarray(x, dtype=np.float64)) for x in (AAp_p, BBp_q, weights))
    out = torch.empty(1, dtype=torch.float64, device=a.device)
    fn = _ia.lib().ia_wdist3_batch if a.numel() == 165 else _ia.lib().ia_wdist_batch
    _ia.check(fn(_ia.ptr(a), _ia.ptr(q), _ia.ptr(w), 1, _ia.ptr(out), _ia.stream()),
              'ia_wdist_batch')
    return float(out.item())
