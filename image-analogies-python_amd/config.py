"""Run parameters — drop-in for the reference's ``config`` module (reference
config.py:7-79): the module itself is the mutable parameter namespace ``c`` that
``image_analogies_main`` and the batch scripts read and assign.

Names and meanings follow the reference.  ``n_half`` and the paddings are plain ints
(the reference derives them with ``np.floor`` and gets floats, which numpy >= 1.12 no
longer accepts as indices).  Fields added by this build:

    levels   cap on pyramid halvings (skimage ``max_layer``); None = reference rule
    seed     seed of the B' random initialisation (the reference draws unseeded)
    matcher  'brute': exact 1-NN (split-f16 MFMA screen + fp64 rescore), the default;
             'lsh': approximate E2LSH matcher with
             lsh_tables x lsh_hashes projections, bucket width lsh_width (in units of
             the rows' RMS per-dimension spread) and projection seed lsh_seed
"""
import numpy as np

# -- reference parameters (config.py:7-20) -------------------------------------------
convert = False     # YIQ: match on luminance, colour from B (else colour from A')
remap_lum = False   # remap A / A' luminance statistics onto B's
init_rand = True    # B' starts as uniform noise (else as B's own pyramid)
if remap_lum:
    assert convert

AB_weight = 1       # weight of the A/B features relative to A'/B'
k = 0.5             # coherence parameter kappa
n_sm, n_lg = 3, 5   # coarse / fine neighbourhood sizes
n_half = n_lg * n_lg // 2
pad_sm, pad_lg = n_sm // 2, n_lg // 2

# -- filled in by setup_vars / img_setup (config.py:22-26) ---------------------------
num_ch = None
max_levels = None
padding_sm = None
padding_lg = None
weights = None

# -- additions -------------------------------------------------------------------------
levels = None
seed = 0
matcher = 'brute'
lsh_tables = 16
lsh_hashes = 4
lsh_width = 1.0
lsh_seed = 0


def setup_vars(img):
    """(num_ch, padding_sm, padding_lg, weights) for an image of 2 or 3 dims
    (config.py:29-42)."""
    assert img.ndim in (2, 3)
    ch = img.shape[2] if img.ndim == 3 else 1
    if ch == 1:
        pads = (int(pad_sm), int(pad_lg))
    else:
        pads = tuple(((p, p), (p, p), (0, 0)) for p in (pad_sm, pad_lg))
    return ch, pads[0], pads[1], compute_weights(n_sm, n_lg, n_half, ch)


def save_metadata(out_path, names, vars):
    """Write ``name: value`` lines to <out_path>metadata.txt (config.py:45-49)."""
    lines = ['%s: %s\n' % (n, v) for n, v in zip(names, vars)]
    with open(out_path + 'metadata.txt', 'w') as f:
        f.writelines(lines)


def matlab_style_gauss2D(shape=(3, 3), sigma=0.5):
    """MATLAB ``fspecial('gaussian', shape, sigma)`` (config.py:52-65): exp of the
    squared radius over 2 sigma^2, tiny tails zeroed, normalised to sum 1."""
    half_r, half_c = (shape[0] - 1.) / 2., (shape[1] - 1.) / 2.
    yy = np.arange(-half_r, half_r + 1)[:, None]
    xx = np.arange(-half_c, half_c + 1)[None, :]
    g = np.exp(-(xx * xx + yy * yy) / (2. * sigma * sigma))
    g[g < np.finfo(g.dtype).eps * g.max()] = 0
    total = g.sum()
    return g / total if total != 0 else g


def compute_weights(n_sm, n_lg, n_half, num_ch):
    """Per-feature weights of the kappa distance (config.py:68-79):
    [coarse A/B | fine A/B | coarse A'/B' | half-fine A'/B'], each Gaussian mask
    normalised by its sample count, channels interleaved per pixel."""
    n_half = int(n_half)
    sm = np.repeat(matlab_style_gauss2D((n_sm, n_sm), 0.5).ravel(), num_ch)
    lg = np.repeat(matlab_style_gauss2D((n_lg, n_lg), 1).ravel(), num_ch)
    parts = [(1. / (n_sm * n_sm)) * sm,
             (1. / (n_lg * n_lg)) * lg,
             (1. / (n_sm * n_sm)) * sm,
             (1. / n_half) * lg[:n_half * num_ch]]
    return np.concatenate(parts)
