"""Golden fixtures of the BASELINE configs, computed HERE (CPU) by the C oracle
(oracle/ia_oracle.c: the reference's scanline loop, image_analogies.py:130-220, with the
exact brute-force matcher, algorithms.py:73-75 restated):

  c3_oracle.npz   config c3 at full size (362x638 A = A' blur, B, kappa 25, 5-level cap,
                  bench.py's seeded synthetic inputs): per synthesized level the index
                  maps s, im and the SHA-256 of B' (float64 bytes, C order).
  c4_queries.npz  config c4's finest level (A = A' 2048x2048, 4,194,304 database rows):
                  fp64 queries captured from a GPU synthesis (tools/capture_c4_queries.py,
                  committed as c4_queries_in.npz) plus synthetic near-ties, with the
                  oracle's exact 1-NN row and distance over the full database.
  c4_levels.npz   config c4 (job seed 0) with every level below the finest synthesized
                  in full by the oracle (levels 1-3: up to 512x512 B' pixels against the
                  1,048,576-row database): s, im and the SHA-256 of B' per level.
  c5_job.npz      config c5's first job (512x512, seed 1000 = bench.py's rank 0 job 0),
                  every level in full (349,184 B' pixels; 262,144 rows at the finest level).
  c4_full.npz     config c4 (job seed 0) with EVERY level in full, the finest included
                  (1,048,576 B' pixels against the 4,194,304-row database): s, im and the
                  SHA-256 of B' per level.  The 1-NN goes through the oracle's projection
                  index (ia_oracle_c.Index: the brute-force scan's exact answer; pinned to
                  the scan on small DBs and, at this level's full 4,194,304 rows, to
                  c4_queries.npz's brute-force answers by tests/test_oracle.py
                  ::test_oracle_index_equals_scan_at_c4_scale), which makes the run minutes
                  instead of a day.

  c1rgb_oracle.npz  3-channel matching (convert=False, the reference's default: num_ch = 3,
                  165-dim rows) at the c1 size (180 x 117 colour A = A' blur, B; kappa 0.5):
                  every level in full (colour_workload: the pyramids are the oracle's per
                  channel, skimage multichannel semantics).
  c3rgb_oracle.npz  the same at the c3 size (362 x 638 colour, kappa 25, 5-level cap): the
                  synthesized levels s1..s5, the finest included.  Both colour fixtures go
                  through the projection index; c1rgb is re-derived by the brute-force scan
                  in tests/test_oracle.py::test_colour_fixture_equals_brute_force_scan.

Usage:  python tests/golden/make_config_fixtures.py c3|c4|c4levels|c4full|c5|c1rgb|c3rgb [threads]
The inputs are rebuilt from bench.py's workload definitions, so the GPU tests regenerate
them identically on the box.
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, ROOT)

import ia_oracle as o      # noqa: E402
import ia_oracle_c as oc   # noqa: E402


def workload(name, job_seed=0):
    """(A, [A'], B, kappa, levels cap, B' init seed) of a bench.py config (bench.Job)."""
    import bench
    conf = bench.CONFIGS[name]
    A, Ap, B = bench.make_inputs(conf, job_seed)
    return A, [Ap], B, conf['k'], conf['levels'], job_seed + 2


def bp_hash(x):
    return hashlib.sha256(np.ascontiguousarray(x, dtype=np.float64).tobytes()).hexdigest()


def full_run(name, fname, job_seed=0, skip_finest=False, indexed=False):
    """The oracle's scanline run of a config's levels -> per-level s, im, B' hash."""
    A, Aps, B, k, cap, seed = workload(name, job_seed)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, cap=cap, seed=seed)
    w = o.compute_weights(3, 5, 12, 1)
    levels = range(1, L - 1) if skip_finest else None
    t0 = time.time()
    out = oc.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, k, w, levels=levels, indexed=indexed)
    print('%s oracle: %d levels in %.1f s' % (name, len(out), time.time() - t0))
    rec = {'max_levels': np.int32(L), 'job_seed': np.int32(job_seed)}
    for l, (bp, s, im) in out.items():
        rec['s%d' % l] = s.astype(np.int16)
        rec['im%d' % l] = im.astype(np.uint8)
        rec['bp_sha%d' % l] = np.array(bp_hash(bp))
        rec['bp_sum%d' % l] = np.float64(bp.sum())
    np.savez_compressed(os.path.join(HERE, fname), **rec)


def make_c3():
    full_run('c3', 'c3_oracle.npz')


def make_c4levels():
    full_run('c4', 'c4_levels.npz', skip_finest=True)


def make_c4full():
    full_run('c4', 'c4_full.npz', indexed=True)


COLOUR = {   # name: (A = B shape, kappa, level cap, seed)
    'c1rgb': ((180, 117), 0.5, None, 7),
    'c3rgb': ((362, 638), 25.0, 5, 10),
}


def colour_workload(name):
    """3-channel inputs of a colour config: smooth colour noise A (channel ch seeded
    seed + 17 ch), A' = gaussian_filter(A, 1.5) per channel, B (seed + 1), the oracle's
    per-channel pyramids, B' init RandomState(seed + 2).  Returns (A_pyr, [Ap_pyr], B_pyr,
    Bp_pyr, L, kappa)."""
    from scipy.ndimage import gaussian_filter
    import bench
    shape, k, cap, seed = COLOUR[name]
    A = np.dstack([bench.smooth_noise(seed + 17 * ch, shape) for ch in range(3)])
    Ap = np.dstack([gaussian_filter(A[..., ch], 1.5) for ch in range(3)])
    B = np.dstack([bench.smooth_noise(seed + 1 + 17 * ch, shape) for ch in range(3)])

    def pyr3(img):
        chans = [o.compute_gaussian_pyramid(img[..., ch], 3, cap) for ch in range(3)]
        return [np.dstack([c[l] for c in chans]) for l in range(len(chans[0]))]
    A_pyr, Ap_pyr, B_pyr = pyr3(A), pyr3(Ap), pyr3(B)
    L = min(len(A_pyr), len(B_pyr))
    return A_pyr, [Ap_pyr], B_pyr, o.initialize_Bp(B_pyr, True, seed + 2), L, k


def colour_run(name, skip_finest=False):
    A_pyr, Ap_list, B_pyr, Bp_pyr, L, k = colour_workload(name)
    w = o.compute_weights(3, 5, 12, 3)
    levels = range(1, L - 1) if skip_finest else None
    t0 = time.time()
    out = oc.synthesize(A_pyr, Ap_list, B_pyr, Bp_pyr, L, k, w, levels=levels, indexed=True)
    print('%s oracle: %d levels in %.1f s' % (name, len(out), time.time() - t0))
    rec = {'max_levels': np.int32(L)}
    for l, (bp, s, im) in out.items():
        rec['s%d' % l] = s.astype(np.int16)
        rec['im%d' % l] = im.astype(np.uint8)
        rec['bp_sha%d' % l] = np.array(bp_hash(bp))
    np.savez_compressed(os.path.join(HERE, name + '_oracle.npz'), **rec)


def make_c5():
    full_run('c5', 'c5_job.npz', job_seed=1000)


def make_c4():
    A, Aps, B, k, cap, seed = workload('c4')
    A_pyr = o.compute_gaussian_pyramid(A, 3, cap)
    Ap_pyr = o.compute_gaussian_pyramid(Aps[0], 3, cap)
    level = len(A_pyr) - 1
    cap_in = np.load(os.path.join(HERE, 'c4_queries_in.npz'))
    Q = cap_in['q']
    rs = np.random.RandomState(44)
    db = oc.LevelDB(level, A_pyr, [Ap_pyr])
    As = db.rows
    N = db.N
    # near ties: exact database rows, and rows nudged by 1 ulp-scale noise
    rows = rs.randint(0, N, 32)
    Qt = np.vstack([As[rows], As[rows[:32]] + rs.randn(32, 55) * 1e-12])
    Qall = np.vstack([Q, Qt])
    t0 = time.time()
    idx, d = db.nn(Qall)
    print('c4 oracle: %d queries over %d rows in %.1f s' % (len(Qall), N, time.time() - t0))
    np.savez_compressed(os.path.join(HERE, 'c4_queries.npz'), q=Qall, idx=idx, dist=d,
                        pixels=cap_in['pixels'], n_captured=np.int32(len(Q)))


if __name__ == '__main__':
    if len(sys.argv) > 2:
        oc.set_threads(int(sys.argv[2]))
    {'c3': make_c3, 'c4': make_c4, 'c4levels': make_c4levels, 'c4full': make_c4full,
     'c5': make_c5, 'c1rgb': lambda: colour_run('c1rgb'),
     'c3rgb': lambda: colour_run('c3rgb')}[sys.argv[1]]()
