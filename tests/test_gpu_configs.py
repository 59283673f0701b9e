"""Parity at the BASELINE configs' own sizes (bench.py's workload definitions, seeded):

  c3  362x638, kappa 25, 5-level cap: every level's s / im / B' bit-exact against the C
      oracle's full scanline run (tests/golden/c3_oracle.npz, make_config_fixtures.py c3)
  c4  A = A' 2048x2048 x B 1024x1024: (1) the matcher over the 4,194,304-row finest
      database against the oracle's exact 1-NN of 500+ queries captured from a GPU
      synthesis plus near-ties (tests/golden/c4_queries.npz); (2) the whole synthesis,
      EVERY level (the finest: 1024 x 1024 pixels x 4,194,304 rows) bit-exact against the
      oracle's full scanline run (tests/golden/c4_full.npz, make_config_fixtures.py
      c4full), through both screens (rotated R16 and split-f16); B' == A'[im][s]
  c5  one whole 512x512 job (seed 1000), alone and inside a batch, bit-exact against the
      oracle's full run (tests/golden/c5_job.npz)
  c2  180x117, kappa 5, LSH matcher: every level bit-exact against the oracle's scanline
      loop driven by the same LSH tables (oracle LshIndex)
"""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

import ia_oracle as o
import ia_oracle_c as oc
from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _bench():
    import bench
    return bench


def _job(name, **kw):
    bench = _bench()
    return bench.Job(bench.CONFIGS[name], 0, torch.device('cuda', 0), **kw)


def _pyr(job, img):
    import config as cfg
    import img_preprocess as ip
    return ip.gaussian_pyramid_dev(img, cfg.n_sm, job.levels)


def _threads():
    env = os.environ.get('OMP_NUM_THREADS', '')
    return max(1, min(16, int(env) if env.isdigit() else (os.cpu_count() or 1)))


def test_c3_full_size_bit_exact_vs_oracle(gpu):
    g = golden('c3_oracle.npz')
    job = _job('c3')
    out = job.step()
    torch.cuda.synchronize()
    assert job.max_levels == int(g['max_levels'])
    assert sorted(out) == list(range(1, job.max_levels))
    for l, (s, im) in out.items():
        assert np.array_equal(s.cpu().numpy(), g['s%d' % l].astype(np.int32)), l
        assert np.array_equal(im.cpu().numpy(), g['im%d' % l].astype(np.int32)), l
        bp = job.Bp[l].cpu().numpy()
        assert hashlib.sha256(np.ascontiguousarray(bp).tobytes()).hexdigest() == str(g['bp_sha%d' % l]), l


def test_c4_matcher_vs_oracle_fixture(gpu):
    """The exact matcher over c4's full finest database (4,194,304 rows) against the
    oracle's brute force, bit-exact in row and distance."""
    import algorithms
    g = golden('c4_queries.npz')
    job = _job('c4')
    level = job.max_levels - 1
    A_pyr, Ap_pyr = _pyr(job, job.A), _pyr(job, job.Ap)
    index = algorithms.level_index(A_pyr, [Ap_pyr], level)
    assert index.N == 4194304
    gi, gd = index.match(g['q'])
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    bad = np.nonzero((gi != g['idx']) | (gd != g['dist']))[0]
    assert len(bad) == 0, (len(bad), bad[:10])


@pytest.mark.parametrize('G', [2, 8])
def test_c4_matcher_sharded_reduction_vs_oracle_fixture(gpu, G):
    """The sharded DB of c4's finest level (algorithms.py:63-69 rows split contiguously over
    G ranks, each shard with its own split scale): every shard's exact winners, reduced
    with the exchange's lexicographic (distance, lowest row) rule, equal the oracle's brute
    force over all 4,194,304 rows (tests/golden/c4_queries.npz)."""
    import algorithms
    import image_analogies as ia
    g = golden('c4_queries.npz')
    job = _job('c4')
    level = job.max_levels - 1
    A_pyr, Ap_pyr = _pyr(job, job.A), _pyr(job, job.Ap)
    best_d = np.full(len(g['q']), np.inf)
    best_i = np.full(len(g['q']), np.iinfo(np.int64).max)
    for r in range(G):
        index = algorithms.level_index(A_pyr, [Ap_pyr], level,
                                       lambda lv, N: ia.shard_rows(N, r, G))
        si, sd = index.match(g['q'])
        si, sd = si.cpu().numpy(), sd.cpu().numpy()
        assert np.all((si >= index.row0) & (si < index.row0 + index.nrows))
        take = (sd < best_d) | ((sd == best_d) & (si < best_i))
        best_d = np.where(take, sd, best_d)
        best_i = np.where(take, si, best_i)
    bad = np.nonzero((best_i != g['idx']) | (best_d != g['dist']))[0]
    assert len(bad) == 0, (len(bad), bad[:10])


@pytest.mark.timeout(600)
@pytest.mark.parametrize('rot', ['1', '0'])
def test_c4_full_synthesis_vs_oracle(gpu, rot, monkeypatch):
    """c4 whole (job seed 0): EVERY level bit-exact against the oracle's full scanline run,
    the finest included (1024 x 1024 B' pixels against the 4,194,304-row database:
    tests/golden/c4_full.npz, s / im / B' hash per level), through the rotated split screen
    (R16, IA_DB_ROT=1) and the split-f16 image form (0); B' == A'[im][s] at every pixel."""
    monkeypatch.setenv('IA_DB_ROT', rot)
    g = golden('c4_full.npz')
    job = _job('c4')
    out = job.step()
    torch.cuda.synchronize()
    assert job.max_levels == int(g['max_levels'])
    assert sorted(out) == list(range(1, job.max_levels))
    Ap_pyr = _pyr(job, job.Ap)
    for l, (s, im) in out.items():
        src = Ap_pyr[l]
        assert torch.equal(job.Bp[l].flatten(), src[s[:, 0].long(), s[:, 1].long()]), l
        assert np.array_equal(im.cpu().numpy(), g['im%d' % l].astype(np.int32)), l
        sg = s.cpu().numpy()
        want = g['s%d' % l].astype(np.int32)
        bad = np.nonzero((sg != want).any(axis=1))[0]
        assert len(bad) == 0, (l, len(bad), bad[:5])
        bp = job.Bp[l].cpu().numpy()
        assert hashlib.sha256(np.ascontiguousarray(bp).tobytes()).hexdigest() == str(g['bp_sha%d' % l]), l


def _c5_check(g, out, Bp):
    assert sorted(out) == list(range(1, int(g['max_levels'])))
    for l, r in out.items():
        s, im = r[0], r[1]
        assert np.array_equal(s.cpu().numpy(), g['s%d' % l].astype(np.int32)), l
        assert np.array_equal(im.cpu().numpy(), g['im%d' % l].astype(np.int32)), l
        bp = Bp[l].cpu().numpy()
        assert hashlib.sha256(np.ascontiguousarray(bp).tobytes()).hexdigest() == str(g['bp_sha%d' % l]), l


def test_c5_job_full_size_bit_exact_vs_oracle(gpu):
    """c5's first job (512 x 512, seed 1000 = bench.py's rank 0 job 0, 349,184 B' pixels)
    synthesised alone: every level's s / im / B' bit-exact against the oracle's whole
    scanline run (tests/golden/c5_job.npz)."""
    bench = _bench()
    g = golden('c5_job.npz')
    job = bench.Job(bench.CONFIGS['c5'], int(g['job_seed']), torch.device('cuda', 0))
    assert job.max_levels == int(g['max_levels'])
    out = job.step()
    torch.cuda.synchronize()
    _c5_check(g, out, job.Bp)


def test_c5_job_in_a_batch_bit_exact_vs_oracle(gpu):
    """The same job as the first of a 3-job batch (ia_synth_levels_batch: one screen and one
    fused launch per wave serve all three, bench.py's c5 form): bit-exact against the
    oracle's whole run."""
    import image_analogies as ia
    bench = _bench()
    g = golden('c5_job.npz')
    dev = torch.device('cuda', 0)
    jobs = [bench.Job(bench.CONFIGS['c5'], int(g['job_seed']) + 3 * j, dev) for j in range(3)]
    ins = [jb.prepare() for jb in jobs]
    outs = ia.synthesize_batch_dev(ins, jobs[0].max_levels, [jb.k for jb in jobs], jobs[0].weights)
    torch.cuda.synchronize()
    _c5_check(g, outs[0], jobs[0].Bp)


def test_c2_lsh_full_size_vs_oracle(gpu):
    """c2 (180x117, kappa 5) with c.matcher = 'lsh' (bench.py --matcher lsh defaults):
    every level's s / im / B' equal the oracle's scanline loop driven by the same tables."""
    import algorithms
    import image_analogies as ia
    lsh = dict(tables=16, hashes=4, width=1.0, seed=0)
    job = _job('c2', lsh=lsh)
    A_d, Ap_d, B_d = _pyr(job, job.A), _pyr(job, job.Ap), _pyr(job, job.B)
    A_pyr = [p.cpu().numpy() for p in A_d]
    Ap_list = [[p.cpu().numpy() for p in Ap_d]]
    B_pyr = [p.cpu().numpy() for p in B_d]
    Bp_d = [x.clone() for x in job.Bp_init]
    Bp_ref = [x.cpu().numpy() for x in job.Bp_init]
    w = o.compute_weights(3, 5, 12, 1)
    As = o.create_index(A_pyr, Ap_list, job.max_levels)
    for level in range(1, job.max_levels):
        index = algorithms.level_index(A_d, [Ap_d], level, lsh=lsh)
        s, im = ia.synthesize_level_dev(level, job.max_levels, index, B_d[level - 1], B_d[level],
                                        Bp_d[level - 1], Bp_d[level], job.weights, job.k)
        h = index.lsh
        table = o.LshIndex(As[level], index.center.cpu().numpy(), index.lsh_proj_host, h.L, h.k,
                           np.float32(h.w))
        rs_, rim = o.synthesize_level(level, job.max_levels, A_pyr, Ap_list, B_pyr, Bp_ref,
                                      As[level], w, job.k, matcher=lambda q: table.match(q)[0][0])
        assert np.array_equal(s.cpu().numpy(), rs_), level
        assert np.array_equal(im.cpu().numpy(), rim), level
        assert np.array_equal(Bp_d[level].cpu().numpy(), Bp_ref[level]), level
