"""Shared test setup: import paths, the `gpu` marker, synthetic inputs.

`-m "not gpu"` tests run on CPU (oracle vs golden vectors, host logic, C-ABI exports,
gloo multi-process logic); `-m gpu` tests call the HIP library and compare with the
oracle (tests/ is the only place besides smoke()/bench's cpu_baseline that may use
oracle/)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'image-analogies-python_amd')
ORACLE = os.path.join(ROOT, 'oracle')
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP (MI355X) device')


def golden(name='ref_golden.npz'):
    return np.load(os.path.join(GOLDEN, name))


def smooth_noise(seed, shape, sigma=2.0):
    """SURVEY §8(d) synthetic image: gaussian-filtered uniform noise rescaled to [0, 1]."""
    from scipy.ndimage import gaussian_filter
    x = gaussian_filter(np.random.RandomState(seed).rand(*shape), sigma)
    return (x - x.min()) / (x.max() - x.min())


def analogy_inputs(seed, A_shape, B_shape, n_ap=1, flat=False):
    """(A, [A'...], B) luminance images: A' = blur(A) (a filter analogy).  flat=True
    clamps the brightest quarter of every image to a constant (exact feature ties)."""
    from scipy.ndimage import gaussian_filter
    A = smooth_noise(seed, A_shape)
    B = smooth_noise(seed + 1, B_shape)
    Aps = [gaussian_filter(A, 1.0 + 0.5 * i) for i in range(n_ap)]
    if flat:
        A = np.minimum(A, 0.75)
        B = np.minimum(B, 0.75)
        Aps = [np.minimum(x, 0.6) for x in Aps]
    return A, Aps, B


@pytest.fixture(scope='session')
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import _ia
    _ia.lib()
    return torch.device('cuda', 0)
