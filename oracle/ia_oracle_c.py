"""ctypes binding of the C oracle (oracle/ia_oracle.c) — TEST INFRASTRUCTURE ONLY.

Used by tests/ (as the fast checker) and by bench.py's cpu_baseline leg.  Builds
``oracle/_build/libia_oracle.so`` with ``make -C oracle`` on first use if missing.
"""
import ctypes
import os
import subprocess
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, '_build', 'libia_oracle.so')
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


class IaOracleLevel(ctypes.Structure):
    _fields_ = [
        ('A_sm', _dp), ('A_lg', _dp), ('Ap_sm', _dp), ('Ap_lg', _dp),
        ('A_hs', ctypes.c_int), ('A_ws', ctypes.c_int), ('Ah', ctypes.c_int),
        ('Aw', ctypes.c_int), ('nAp', ctypes.c_int),
        ('B_sm', _dp), ('B_lg', _dp),
        ('B_hs', ctypes.c_int), ('B_ws', ctypes.c_int), ('H', ctypes.c_int),
        ('W', ctypes.c_int),
        ('Bp_sm', _dp), ('Bp_lg', _dp), ('weights', _dp),
        ('kappa_factor', ctypes.c_double),
        ('s', _ip), ('im', _ip), ('max_pixels', ctypes.c_long), ('nch', ctypes.c_int),
    ]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(['make', '-s', '-C', _HERE])
        _lib = ctypes.CDLL(_LIB)
        _lib.ia_oracle_synth_level.restype = ctypes.c_long
        _lib.ia_oracle_synth_level.argtypes = [ctypes.POINTER(IaOracleLevel), _dp]
        _lib.ia_oracle_build_db.restype = _dp
        _lib.ia_oracle_build_db.argtypes = [ctypes.POINTER(IaOracleLevel)]
        _lib.ia_oracle_free.argtypes = [ctypes.c_void_p]
        _lib.ia_oracle_nn.restype = ctypes.c_long
        _lib.ia_oracle_nn.argtypes = [_dp, ctypes.c_long, _dp, _dp]
        _lib.ia_oracle_set_threads.argtypes = [ctypes.c_int]
        _lib.ia_oracle_threads.restype = ctypes.c_int
        _lib.ia_oracle_nn_batch.argtypes = [_dp, ctypes.c_long, _dp, ctypes.c_long,
                                            ctypes.POINTER(ctypes.c_long), _dp]
        _lib.ia_oracle_index_build2.restype = ctypes.c_void_p
        _lib.ia_oracle_index_build2.argtypes = [_dp, ctypes.c_long, ctypes.c_int, _dp, ctypes.c_int]
        _lib.ia_oracle_index_free.argtypes = [ctypes.c_void_p]
        _lib.ia_oracle_index_nn_batch.argtypes = [ctypes.c_void_p, _dp, _dp, ctypes.c_long,
                                                  ctypes.POINTER(ctypes.c_long), _dp]
        _lib.ia_oracle_nn_n_batch.argtypes = [_dp, ctypes.c_long, ctypes.c_int, _dp, ctypes.c_long,
                                              ctypes.POINTER(ctypes.c_long), _dp]
        _lib.ia_oracle_synth_level_ix.restype = ctypes.c_long
        _lib.ia_oracle_synth_level_ix.argtypes = [ctypes.POINTER(IaOracleLevel), _dp,
                                                  ctypes.c_void_p]
    return _lib


def set_threads(n):
    """Threads of the oracle's 1-NN scan (1 = serial; 0 = OMP_NUM_THREADS).  Any count
    gives the serial scan's result (row blocks combined in row order).  Returns the count
    in effect."""
    lib().ia_oracle_set_threads(int(n))
    return lib().ia_oracle_threads()


def nn_batch(db_ptr, N, Q):
    """Exact 1-NN (first minimum of the pairwise-8 squared distance) of the rows of Q
    (M x 55) over an oracle database (ia_oracle_build_db) -> (idx int64, dist fp64)."""
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    M = Q.shape[0]
    idx = np.empty(M, np.int64)
    d = np.empty(M, np.float64)
    lib().ia_oracle_nn_batch(db_ptr, N, _d(Q), M, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_long)),
                             _d(d))
    return idx, d


def _d(a):
    return a.ctypes.data_as(_dp)


class LevelJob:
    """Holds contiguous copies of one level's inputs and the ctypes descriptor."""

    def __init__(self, level, A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, weights, kappa_factor,
                 max_pixels=-1):
        c = np.ascontiguousarray
        self.A_sm, self.A_lg = c(A_pyr[level - 1], np.float64), c(A_pyr[level], np.float64)
        self.Ap_sm = c(np.stack([p[level - 1] for p in Ap_pyr_list]), np.float64)
        self.Ap_lg = c(np.stack([p[level] for p in Ap_pyr_list]), np.float64)
        self.B_sm, self.B_lg = c(B_pyr[level - 1], np.float64), c(B_pyr[level], np.float64)
        self.Bp_sm = c(Bp_pyr[level - 1], np.float64)
        self.Bp_lg = np.array(Bp_pyr[level], dtype=np.float64, order='C')
        self.w = c(weights, np.float64)
        H, W = self.B_lg.shape[:2]
        self.nch = self.B_lg.shape[2] if self.B_lg.ndim == 3 else 1
        self.D = 55 * self.nch
        self.s = np.zeros((H * W, 2), np.int32)
        self.im = np.zeros(H * W, np.int32)
        L = IaOracleLevel()
        L.A_sm, L.A_lg, L.Ap_sm, L.Ap_lg = _d(self.A_sm), _d(self.A_lg), _d(self.Ap_sm), _d(self.Ap_lg)
        L.A_hs, L.A_ws = self.A_sm.shape[:2]
        L.Ah, L.Aw = self.A_lg.shape[:2]
        L.nAp = len(Ap_pyr_list)
        L.B_sm, L.B_lg = _d(self.B_sm), _d(self.B_lg)
        L.B_hs, L.B_ws = self.B_sm.shape[:2]
        L.H, L.W = H, W
        L.Bp_sm, L.Bp_lg, L.weights = _d(self.Bp_sm), _d(self.Bp_lg), _d(self.w)
        L.kappa_factor = kappa_factor
        L.s = self.s.ctypes.data_as(_ip)
        L.im = self.im.ctypes.data_as(_ip)
        L.max_pixels = max_pixels
        L.nch = self.nch
        self.L = L
        self.db = None

    def build_db(self):
        if self.db is None:
            self.db = lib().ia_oracle_build_db(ctypes.byref(self.L))
        return self.db

    def run(self, use_db=True, index=None):
        db = self.build_db() if use_db or index is not None else None
        if index is not None:
            n = lib().ia_oracle_synth_level_ix(ctypes.byref(self.L), db, index.ptr)
        else:
            n = lib().ia_oracle_synth_level(ctypes.byref(self.L), db)
        if n == -2:
            raise ValueError('oracle index built for another row length')
        if n < 0:
            raise MemoryError('oracle db allocation failed')
        return n

    def __del__(self):
        if self.db is not None and _lib is not None:
            _lib.ia_oracle_free(self.db)
            self.db = None


def synthesize(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, max_levels, k, weights, levels=None,
               indexed=False):
    """All levels (scanline order) with the C oracle; updates Bp_pyr in place.
    Returns {level: (Bp_level, s, im)} like ia_oracle.synthesize.  indexed=True finds each
    1-NN through a projection index (Index: the brute force's exact answer, faster on
    large databases; fixture generation)."""
    out = {}
    for level in range(1, max_levels):
        if levels is not None and level not in levels:
            continue
        f = 1 + (2.0 ** (level - max_levels)) * k
        job = LevelJob(level, A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, weights, f)
        if indexed:
            db = job.build_db()
            N = job.A_lg.shape[0] * job.A_lg.shape[1] * job.Ap_lg.shape[0]
            rows = np.ctypeslib.as_array(db, shape=(N * job.D,)).reshape(N, job.D)
            t0 = time.time()
            job.run(index=Index(db, rows))
            print('oracle level %d (%d x %d px, %d rows): %.1f s' % (
                level, job.L.H, job.L.W, N, time.time() - t0), flush=True)
        else:
            job.run()
        Bp_pyr[level] = job.Bp_lg.reshape(Bp_pyr[level].shape)
        out[level] = (Bp_pyr[level].copy(), job.s.copy(), job.im.copy())
    return out


class LevelDB:
    """The oracle's As[level] (algorithms.py:50-70: [A full | A'_i half] rows, fp64) built
    by the C oracle; ``rows`` is a numpy view (N x 55) valid while this object lives."""

    def __init__(self, level, A_pyr, Ap_pyr_list):
        dummy = [np.zeros((2, 2))] * (level + 1)
        C = A_pyr[level].shape[2] if A_pyr[level].ndim == 3 else 1
        if C > 1:
            dummy = [np.zeros((2, 2, C))] * (level + 1)
        self._job = LevelJob(level, A_pyr, Ap_pyr_list, dummy, dummy, np.zeros(55 * C), 1.0)
        self.ptr = self._job.build_db()
        self.D = 55 * C
        self.N = A_pyr[level].shape[0] * A_pyr[level].shape[1] * len(Ap_pyr_list)
        self.rows = np.ctypeslib.as_array(self.ptr, shape=(self.N * self.D,)).reshape(self.N, self.D)

    def nn(self, Q):
        """Exact 1-NN rows and distances of Q (M x 55; 165-dim rows: through the index)."""
        if self.D != 55:
            return self.index().nn(Q)
        return nn_batch(self.ptr, self.N, Q)

    def scan(self, Q):
        """Exact 1-NN by the brute-force scan, any row length (no index)."""
        Q = np.ascontiguousarray(Q, dtype=np.float64)
        M = Q.shape[0]
        idx = np.empty(M, np.int64)
        d = np.empty(M, np.float64)
        lib().ia_oracle_nn_n_batch(self.ptr, self.N, self.D, _d(Q), M,
                                   idx.ctypes.data_as(ctypes.POINTER(ctypes.c_long)), _d(d))
        return idx, d

    def index(self, P=4):
        """An exact projection Index over these rows (same answers as nn, faster)."""
        return Index(self.ptr, self.rows, P)


class Index:
    """Exact 1-NN index over an oracle database (ia_oracle_index_build): rows sorted by
    their first principal projection, pruned by a Bessel lower bound over P principal
    directions with rounding margins.  Returns the brute-force scan's (row, distance)
    exactly (tests/test_oracle.py checks it, ties included).  Test infrastructure only:
    it makes full-size fixtures affordable; the CPU baseline keeps the scan."""

    def __init__(self, db_ptr, rows, P=4, sample=200000):
        N = rows.shape[0]
        step = max(1, N // sample)
        sub = np.asarray(rows[::step], dtype=np.float64)
        if len(sub) > 1:
            C = np.cov((sub - sub.mean(0)).T)
            _, V = np.linalg.eigh(C)
            V = V[:, ::-1][:, :P].T.copy()
        else:
            V = np.eye(rows.shape[1])[:P]
        V, _ = np.linalg.qr(V.T)          # re-orthonormalise
        V = np.ascontiguousarray(V.T[:P], dtype=np.float64)
        self.P = V.shape[0]
        self.V = V
        self.db = db_ptr
        self.N = N
        self.D = rows.shape[1]
        self.ptr = lib().ia_oracle_index_build2(db_ptr, N, self.D, _d(V), self.P)
        if not self.ptr:
            raise MemoryError('oracle index allocation failed')

    def nn(self, Q):
        Q = np.ascontiguousarray(Q, dtype=np.float64)
        M = Q.shape[0]
        idx = np.empty(M, np.int64)
        d = np.empty(M, np.float64)
        lib().ia_oracle_index_nn_batch(self.ptr, self.db, _d(Q), M,
                                       idx.ctypes.data_as(ctypes.POINTER(ctypes.c_long)), _d(d))
        return idx, d

    def __del__(self):
        if getattr(self, 'ptr', None) and _lib is not None:
            _lib.ia_oracle_index_free(self.ptr)
            self.ptr = None
