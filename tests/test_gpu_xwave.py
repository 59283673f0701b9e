"""The fused per-wave kernel (k_xwave: exact stage, device-side exchange, per-pixel tail
and the next wave's query rows in one launch) and the batched multi-job
path built on it (ia_synth_levels_batch, the multi_script workload of SURVEY §8(e)),
against the scanline C oracle (reference image_analogies.py:130-220 restated)."""
import numpy as np
import pytest
import torch

import ia_oracle as o
import ia_oracle_c as oc
from conftest import analogy_inputs

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=torch.float64)


def oracle_case(seed, A_shape, B_shape, n_ap, k, flat=False, cap=None):
    A, Aps, B = analogy_inputs(seed, A_shape, B_shape, n_ap, flat)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed, cap=cap)
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, k, w)
    return (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref


def assert_equal_oracle(out, Bp_dev, ref):
    assert set(ref) == set(out)
    for l in ref:
        Bp, s, im = ref[l]
        assert np.array_equal(out[l][0].cpu().numpy(), s), l
        assert np.array_equal(out[l][1].cpu().numpy(), im), l
        assert np.array_equal(Bp_dev[l].cpu().numpy(), Bp), l


@pytest.mark.parametrize('xw', [1, 0])
def test_fused_and_separate_kernels_match_oracle(gpu, xw):
    """The same synthesis with the fused per-wave kernel (default) and with the separate
    kernels it replaces (query build, k_rescore, tail): both bit-exact vs the oracle."""
    import _ia
    import image_analogies as ia
    (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref = oracle_case(61, (44, 57), (37, 49), 2, 1.5)
    prev = _ia.xwave(xw)
    try:
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 1.5, w)
        assert_equal_oracle(out, Bp_dev, ref)
    finally:
        _ia.xwave(prev)


@pytest.mark.parametrize('xw', [2, 1])
def test_fused_kernel_image_form_level(gpu, xw):
    """A finest level whose DB runs in its image form (width 256), flat regions for exact
    ties (many candidate segments per query): the strip form k_xstrip (xw 2: every row of
    the candidate segments rescored in fp64 from LDS windows, 128-row segments) and k_xwave
    (xw 1: fp32 re-screen of DMA'd split windows), both bit-exact vs the oracle."""
    import _ia
    import image_analogies as ia
    (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref = oracle_case(62, (256, 256), (40, 52), 1, 0.5,
                                                             flat=True, cap=3)
    assert A_pyr[-1].shape == (256, 256)       # the finest level's DB is 65,536 rows wide 256
    prev = _ia.xwave(xw)
    try:
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 0.5, w)
        assert_equal_oracle(out, Bp_dev, ref)
    finally:
        _ia.xwave(prev)


def test_strip_kernel_512_two_images_matches_oracle(gpu):
    """k_xstrip on 512-row segments (4 scanlines of a 128-pixel strip: A 512 x 512, two A'
    images, 524,288 rows) and 256-row segments (the 256 x 256 level): the reflected LDS
    windows at the images' four edges, segments in both A' images, vs the oracle."""
    import image_analogies as ia
    (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref = oracle_case(63, (512, 512), (40, 32), 2, 2.0, cap=3)
    assert A_pyr[-1].shape == (512, 512)
    Bp_dev = [dev(b) for b in Bp_pyr]
    out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                            [dev(p) for p in B_pyr], Bp_dev, L, 2.0, w)
    assert_equal_oracle(out, Bp_dev, ref)


def test_strip_kernel_equals_xwave_large(gpu):
    """A 1024 x 1024 (1,048,576 rows, 512-row segments), B 96 x 128: B', s, im and every
    debug record of the strip form equal k_xwave's (itself pinned to the oracle above)."""
    import _ia
    import image_analogies as ia
    A, Aps, B = analogy_inputs(64, (1024, 1024), (96, 128), 1)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=64, cap=2)
    w = o.compute_weights(3, 5, 12, 1)
    res = {}
    for xw in (2, 1):
        prev = _ia.xwave(xw)
        try:
            Bp_dev = [dev(b) for b in Bp_pyr]
            out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                    [dev(p) for p in B_pyr], Bp_dev, L, 1.0, w, debug=True)
            res[xw] = (out, Bp_dev)
        finally:
            _ia.xwave(prev)
    (o2, b2), (o1, b1) = res[2], res[1]
    for l in o1:
        assert torch.equal(b2[l], b1[l]), l
        assert torch.equal(o2[l][0], o1[l][0]) and torch.equal(o2[l][1], o1[l][1]), l
        for x, y in zip(o2[l][2], o1[l][2]):
            assert torch.equal(x, y), l


@pytest.mark.parametrize('A_shape,B_shape,cap', [((36, 44), (30, 41), None), ((256, 256), (33, 47), 3)])
def test_batch_jobs_match_oracle(gpu, A_shape, B_shape, cap):
    """Three independent jobs (different images, B' inits and kappas; identical shapes)
    synthesised as ONE batch (each wave's screen and fused kernel serve all three): every
    job equals its own oracle run, debug records included in the result set."""
    import image_analogies as ia
    jobs, refs, ks = [], [], [0.5, 5.0, 25.0]
    for j, k in enumerate(ks):
        (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref = oracle_case(70 + j, A_shape, B_shape, 1, k, cap=cap)
        jobs.append(([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                     [dev(p) for p in B_pyr], [dev(b) for b in Bp_pyr]))
        refs.append(ref)
    outs = ia.synthesize_batch_dev(jobs, L, ks, w)
    for (_, _, _, Bp_dev), out, ref in zip(jobs, outs, refs):
        assert_equal_oracle(out, Bp_dev, ref)


def test_batch_debug_records_equal_single(gpu):
    """The batch path's per-pixel debug records (p_app, p_coh, r*, distances) equal the
    single-job path's."""
    import image_analogies as ia
    jobs, singles = [], []
    for j in range(2):
        (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), _ = oracle_case(80 + j, (30, 38), (27, 35), 1, 2.0)
        mk = lambda: ([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],  # noqa: E731
                      [dev(p) for p in B_pyr], [dev(b) for b in Bp_pyr])
        jobs.append(mk())
        a, ap, b, bp = mk()
        singles.append(ia.synthesize_dev(a, ap, b, bp, L, 2.0, w, debug=True))
    outs = ia.synthesize_batch_dev(jobs, L, 2.0, w, debug=True)
    for out, single in zip(outs, singles):
        for l in single:
            for x, y in zip(out[l][2], single[l][2]):
                assert torch.equal(x, y), l
            assert torch.equal(out[l][0], single[l][0]) and torch.equal(out[l][1], single[l][1])
