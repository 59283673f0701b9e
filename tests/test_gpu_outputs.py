"""Colour reconstruction and debug export of image_analogies_main
against the oracle, end to end from image files:

  convert=True   B' luminance + B's I/Q pyramid -> RGB (img_preprocess.py:16-22 via
                 image_analogies.py:255-258), clipped to [0, 1]
  convert=False  each pixel copies its source's value in the A' colour pyramid
                 (image_analogies.py:216-217)
  debug=True     sa / sc / rstars / s / im and the d_app / d_coh maps of every level
                 (image_analogies.py:141-159, 222-253)

The RGB image handed to plt.imsave must equal the oracle's bit for bit (so its uint8 form
(x * 255).astype(uint8), what plt.imsave stores, is equal too: "B' pixels within 1/255").
"""
import os
import pickle

import numpy as np
import pytest

import ia_oracle as o
from conftest import analogy_inputs

pytestmark = pytest.mark.gpu


def _write_png(path, img, mode):
    from PIL import Image
    Image.fromarray(np.clip(np.round(img * 255), 0, 255).astype(np.uint8), mode).save(path)


def _oracle_run(Ay, Apy, By, seed, k, color_level_fn):
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(Ay, [Apy], By, seed=seed)
    As = o.create_index(A_pyr, Ap_list, L)
    w = o.compute_weights(3, 5, 12, 1)
    res = {}
    for level in range(1, L):
        dbg = {}
        s, im = o.synthesize_level(level, L, A_pyr, Ap_list, B_pyr, Bp_pyr, As[level], w, k,
                                   debug=dbg)
        res[level] = dict(s=s, im=im, dbg=dbg, color=color_level_fn(level, Bp_pyr, s, im, Ap_list))
    return res, L


def _check(out, ref, L):
    assert sorted(out) == list(range(1, L))
    for level in range(1, L):
        g, r = out[level], ref[level]
        assert np.array_equal(g['s'], r['s']) and np.array_equal(g['im'], r['im']), level
        assert g['color'].shape == r['color'].shape
        assert np.array_equal(g['color'], r['color']), level
        assert np.array_equal((g['color'] * 255).astype(np.uint8),
                              (r['color'] * 255).astype(np.uint8)), level
        d, rd = g['debug'], r['dbg']
        for key in ('sa', 'sc', 'rstars'):
            assert d[key] == rd[key], (level, key)
        assert np.array_equal(d['app_dist'], rd['app_dist']), level
        assert np.array_equal(d['coh_dist'], rd['coh_dist']), level


@pytest.mark.parametrize('seed,k', [(71, 0.5), (72, 25.0)])
def test_color_convert_true_and_debug_vs_oracle(gpu, tmp_path, seed, k):
    import matplotlib.pyplot as plt
    import config as c
    import image_analogies as ia
    A, Aps, B = analogy_inputs(seed, (36, 47), (33, 40))
    to_rgb = lambda x: np.dstack([x, 0.3 + 0.5 * x * x, 1 - x])  # noqa: E731
    files = {}
    for name, img in (('A', A), ('Ap', Aps[0]), ('B', B)):
        files[name] = str(tmp_path / (name + '.png'))
        _write_png(files[name], to_rgb(img), 'RGB')
    c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k, c.seed = True, False, True, 1, k, seed
    c.levels, c.matcher = None, 'brute'
    out_dir = str(tmp_path / 'out') + '/'
    out = {}
    ia.image_analogies_main(files['A'], [files['Ap']], files['B'], out_dir, c, debug=True,
                            outputs=out)
    dec = {n: plt.imread(p)[..., :3].astype(np.float64) for n, p in files.items()}
    sc = lambda x: 255. if np.max(x) > 1 else 1.0  # noqa: E731
    B_yiq = o.convert_to_YIQ(dec['B'] / sc(dec['B']))
    color_pyr = o.compute_gaussian_pyramid(B_yiq, 3)

    def color(level, Bp_pyr, s, im, Ap_list):
        rgb = o.convert_to_RGB(np.dstack([Bp_pyr[level], color_pyr[level][:, :, 1:]]))
        return np.clip(rgb, 0, 1)
    ref, L = _oracle_run(o.convert_to_YIQ(dec['A'] / sc(dec['A']))[..., 0],
                         o.convert_to_YIQ(dec['Ap'] / sc(dec['Ap'][0]))[..., 0],
                         B_yiq[..., 0], seed, k, color)
    _check(out, ref, L)
    # the debug files the reference writes
    for level in range(1, L):
        with open(out_dir + '%d_srcs.pickle' % level, 'rb') as f:
            sa, scl, rstars, s, im = pickle.load(f)
        assert sa == ref[level]['dbg']['sa'] and scl == ref[level]['dbg']['sc']
        assert [tuple(x) for x in ref[level]['s']] == s and list(ref[level]['im']) == im
        for n in ('psrc', 'appdist', 'cohdist', 'output', 'imgsrc'):
            assert os.path.exists(out_dir + '%d_%s.eps' % (level, n))
    assert os.path.exists(out_dir + 'level_%d_color.jpg' % (L - 1))


def test_color_convert_false_vs_oracle(gpu, tmp_path):
    """convert=False on greyscale images: each output pixel is its source's A' value."""
    import matplotlib.pyplot as plt
    import config as c
    import image_analogies as ia
    A, Aps, B = analogy_inputs(73, (30, 41), (34, 38))
    files = {}
    for name, img in (('A', A), ('Ap', Aps[0]), ('B', B)):
        files[name] = str(tmp_path / (name + '.png'))
        _write_png(files[name], img, 'L')
    c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k, c.seed = False, False, True, 1, 1.0, 5
    c.levels, c.matcher = None, 'brute'
    out_dir = str(tmp_path / 'out') + '/'
    out = {}
    ia.image_analogies_main(files['A'], [files['Ap']], files['B'], out_dir, c, debug=True,
                            outputs=out)
    dec = {n: plt.imread(p).astype(np.float64) for n, p in files.items()}
    assert dec['A'].ndim == 2
    sc = lambda x: 255. if np.max(x) > 1 else 1.0  # noqa: E731

    def color(level, Bp_pyr, s, im, Ap_list):
        H, W = Bp_pyr[level].shape
        v = np.array([Ap_list[i][level][r, cc] for (r, cc), i in zip(s, im)]).reshape(H, W)
        return np.repeat(v[..., None], 3, axis=2)
    ref, L = _oracle_run(dec['A'] / sc(dec['A']), dec['Ap'] / sc(dec['Ap'][0]),
                         dec['B'] / sc(dec['B']), 5, 1.0, color)
    _check(out, ref, L)
