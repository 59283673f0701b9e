"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run with the image's Python 3.9 environment, which has the reference's third-party
stack (numpy 1.26.4, scipy 1.7.1, scikit-image 0.18.3):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

It imports the reference's own ``config.py`` and ``img_preprocess.py`` from
/root/reference (read-only; nothing is copied) and records their OUTPUTS on seeded
inputs.  Only data is written (``ref_golden.npz``, allow_pickle=False).  The reference's
``algorithms.py`` / ``image_analogies.py`` are Python-2 sources (SyntaxError under 3.x)
and need pyflann, so they cannot be imported; their behaviour is pinned by the KATs of
``algorithms_test.py`` (transcribed in tests/test_oracle.py) instead.
"""
import os
import sys
import warnings

import numpy as np

warnings.filterwarnings('ignore')
REF = '/root/reference'
sys.path.insert(0, REF)

import config as ref_config            # noqa: E402  (reference config.py)
import img_preprocess as ref_ip        # noqa: E402  (reference img_preprocess.py)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ref_golden.npz')

# shapes exercised: the reference test image (25x40, img_preprocess_test.py:31),
# config-1 crop (180x117 -> (117, 180) rows x cols), pyramid levels of it, odd sizes,
# and tiny images that hit the multi-reflection boundary paths.
PYR_SHAPES = [(25, 40), (117, 180), (45, 30), (23, 15), (30, 45), (7, 9), (4, 4),
              (64, 64), (33, 70)]


def main():
    g = {}
    # config.py:68-79 (int n_half, as config_test.py:7,37 passes)
    g['weights_ch1'] = ref_config.compute_weights(3, 5, 12, 1)
    g['weights_ch3'] = ref_config.compute_weights(3, 5, 12, 3)
    g['gauss_sm'] = ref_config.matlab_style_gauss2D((3, 3), 0.5)
    g['gauss_lg'] = ref_config.matlab_style_gauss2D((5, 5), 1)

    # img_preprocess.py:6-22 on a seeded image (img_preprocess_test.py:7 seed)
    rs = np.random.RandomState(0xba5eba11)
    rgb = rs.rand(25, 25, 3)
    g['yiq_in'] = rgb
    g['yiq_out'] = ref_ip.convert_to_YIQ(rgb)
    g['rgb_out'] = ref_ip.convert_to_RGB(g['yiq_out'])
    u8 = rs.randint(0, 256, size=(13, 17, 3)).astype(np.uint8)
    g['yiq_u8_in'] = u8
    g['yiq_u8_out'] = ref_ip.convert_to_YIQ(u8 / 255.)

    # img_preprocess.py:25-40 (list of A' as the function expects)
    A = rs.rand(25, 25); Ap = rs.rand(25, 25); B = rs.rand(30, 30)
    Ar, Apr = ref_ip.remap_luminance(A, [Ap], B)
    g['remap_A'], g['remap_Ap'], g['remap_B'] = A, Ap, B
    g['remap_A_out'], g['remap_Ap_out'] = Ar, Apr[0]

    # img_preprocess.py:47-63 -> skimage pyramid_gaussian, all levels
    for k, shp in enumerate(PYR_SHAPES):
        img = rs.rand(*shp)
        pyr = ref_ip.compute_gaussian_pyramid(img, 3) if min(shp) > 3 else \
            list(reversed(list(__import__('skimage.transform', fromlist=['x'])
                               .pyramid_gaussian(img, max_layer=2))))
        g['pyr%d_in' % k] = img
        g['pyr%d_n' % k] = np.array(len(pyr))
        for l, lvl in enumerate(pyr):
            g['pyr%d_l%d' % (k, l)] = lvl

    np.savez_compressed(OUT, **g)
    print('wrote', OUT, 'keys', len(g))


if __name__ == '__main__':
    main()
