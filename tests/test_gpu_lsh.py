"""LSH matcher: the HIP tables and queries against the oracle's
restatement of the same definition (oracle/ia_oracle.py LshIndex).  There is no
reference LSH code, so these pin the HIP path to this build's own definition (parity
unpinned against any reference); the exact matcher stays the default."""
import numpy as np
import pytest
import torch

import ia_oracle as o
from conftest import analogy_inputs

pytestmark = pytest.mark.gpu


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype)


def _oracle_lsh(index, As):
    h = index.lsh
    return o.LshIndex(As, index.center.cpu().numpy(), index.lsh_proj_host, h.L, h.k,
                      np.float32(h.w))


@pytest.mark.parametrize('params', [dict(tables=16, hashes=4, width=1.0, seed=0),
                                    dict(tables=8, hashes=2, width=0.5, seed=3),
                                    dict(tables=1, hashes=8, width=4.0, seed=1)])
def test_lsh_match_vs_oracle(gpu, params):
    import algorithms
    A, Aps, _ = analogy_inputs(21, (96, 131), (8, 8), n_ap=2)
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = [o.compute_gaussian_pyramid(x, 3) for x in Aps]
    L = len(A_pyr) - 1
    index = algorithms.level_index([dev(p) for p in A_pyr],
                                   [[dev(p) for p in q] for q in Ap_pyr], L, lsh=params)
    As = o.create_index(A_pyr, Ap_pyr, L + 1)[L]
    rs = np.random.RandomState(4)
    Q = np.vstack([As[rs.randint(0, len(As), 300)],
                   As[rs.randint(0, len(As), 300)] + rs.randn(300, 55) * 0.01,
                   rs.rand(100, 55)])
    gi, gd = index.match(Q)
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    ri, rd = _oracle_lsh(index, As).match(Q)
    same = gi == ri
    # bucket keys agree except for fp32 double-rounding ties of the emulated FMA chain
    assert same.mean() >= 0.99, same.mean()
    assert np.array_equal(gd[same], rd[same])
    # approximate, never better than exact; the exact path is still reachable
    ei, ed = index.match(Q, exact=True)
    ed = ed.cpu().numpy()
    assert np.all(gd >= ed)
    bd = np.array([np.add.reduce((As - q) ** 2, axis=1).min() for q in Q])
    assert np.array_equal(ed, bd)


def test_lsh_synthesis_vs_oracle(gpu):
    """Whole levels with c.matcher = 'lsh': the wavefront + LSH path against the scanline
    oracle driven by the same tables."""
    import algorithms
    import image_analogies as ia
    A, Aps, B = analogy_inputs(2, (30, 40), (28, 33), n_ap=2)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=2)
    w = o.compute_weights(3, 5, 12, 1)
    A_d = [dev(p) for p in A_pyr]
    Ap_d = [[dev(p) for p in q] for q in Ap_list]
    B_d = [dev(p) for p in B_pyr]
    Bp_d = [dev(b) for b in Bp_pyr]
    Bp_ref = [b.copy() for b in Bp_pyr]
    As = o.create_index(A_pyr, Ap_list, L)
    params = dict(tables=8, hashes=3, width=1.0, seed=7)
    for level in range(1, L):
        index = algorithms.level_index(A_d, Ap_d, level, lsh=params)
        s, im = ia.synthesize_level_dev(level, L, index, B_d[level - 1], B_d[level],
                                        Bp_d[level - 1], Bp_d[level], dev(w), 1.0)
        lsh = _oracle_lsh(index, As[level])
        rs_, rim = o.synthesize_level(level, L, A_pyr, Ap_list, B_pyr, Bp_ref, As[level], w,
                                      1.0, matcher=lambda q: lsh.match(q)[0][0])
        assert np.array_equal(s.cpu().numpy(), rs_), level
        assert np.array_equal(im.cpu().numpy(), rim), level
        assert np.array_equal(Bp_d[level].cpu().numpy(), Bp_ref[level]), level


def test_lsh_api_create_index(gpu):
    """create_index honours c.matcher = 'lsh' (params describe the tables)."""
    import algorithms
    import config as c
    A, Aps, _ = analogy_inputs(8, (40, 44), (8, 8))
    A_pyr = o.compute_gaussian_pyramid(A, 3)
    Ap_pyr = [o.compute_gaussian_pyramid(Aps[0], 3)]
    c.max_levels = len(A_pyr)
    old = c.matcher
    try:
        c.matcher = 'lsh'
        flann, params, As, _ = algorithms.create_index(A_pyr, Ap_pyr, c)
    finally:
        c.matcher = old
    L = len(A_pyr) - 1
    assert params[L]['algorithm'] == 'lsh' and not params[L]['exact']
    assert (params[L]['tables'], params[L]['hashes']) == (c.lsh_tables, c.lsh_hashes)
    q = As[L][17] * 0.98
    i = algorithms.best_approximate_match(flann[L], params[L], q)
    assert i == _oracle_lsh(flann[L], As[L]).match(q)[0][0]
