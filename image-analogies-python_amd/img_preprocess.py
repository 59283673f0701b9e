"""Image preprocessing — drop-in for the reference's ``img_preprocess`` module
(reference img_preprocess.py:1-113), computed by the HIP kernels of libia.so.

Public functions keep the reference's names, arguments and numpy-in / numpy-out
contract.  The ``*_dev`` variants take and return device tensors and are what the
synthesis path uses (inputs stay resident in HBM).

    convert_to_YIQ / convert_to_RGB   ia_rgb_to_yiq / ia_yiq_to_rgb   (a1, a2)
    remap_luminance / compress_values ia_axpb_f64 (host computes mean/std scalars, a3/a4)
    compute_gaussian_pyramid          ia_pyr_reduce_f64 per level          (a5)
    initialize_Bp                     host RandomState in the reference's draw order (a6)
    pad_img_pair, px2ix, ix2px, Ap_ix2px, Ap_px2ix   index bookkeeping (a7, a8)
"""
import ctypes
import math

import numpy as np
import torch

import _ia

# scipy.ndimage Gaussian taps for skimage pyramid_reduce's sigma = 2*2/6 (radius 3),
# fixed to the values of the skimage 0.18.3 / numpy 1.26.4 environment the reference
# goldens come from (numpy 2.x computes tap 2 one ulp lower).  (w0, w1, w2, w3).
PYR_TAPS = (
    float.fromhex('0x1.324af5ad1bf73p-1'),
    float.fromhex('0x1.8dc13f0096171p-3'),
    float.fromhex('0x1.b38896102b1bcp-8'),
    float.fromhex('0x1.921e9614385a4p-16'),
)


def _dtype_code(a):
    if a.dtype == np.uint8 or a.dtype == torch.uint8:
        return 0
    if a.dtype == np.float32 or a.dtype == torch.float32:
        return 1
    if a.dtype == np.float64 or a.dtype == torch.float64:
        return 2
    raise TypeError('unsupported image dtype %s' % (a.dtype,))


# ---- colour ---------------------------------------------------------------------------

def rgb_to_yiq_dev(src, div=1.0, want_yiq=True):
    """Device (H, W, 3) uint8/float -> (yiq (H, W, 3) or None, Y (H, W)) fp64, with the
    reference's scaling ``src / div`` fused in (image_analogies.py:32-50)."""
    dev = _ia.require_device()
    src = src.contiguous()
    H, W = src.shape[:2]
    y = torch.empty((H, W), dtype=torch.float64, device=dev)
    yiq = torch.empty((H, W, 3), dtype=torch.float64, device=dev) if want_yiq else None
    _ia.check(_ia.lib().ia_rgb_to_yiq(_ia.ptr(src), _dtype_code(src), H * W, float(div),
                                      _ia.ptr(yiq), _ia.ptr(y), _ia.stream()),
              'ia_rgb_to_yiq')
    return yiq, y


def convert_to_YIQ(img):
    """RGB -> YIQ (img_preprocess.py:6-13)."""
    assert 0 <= np.max(img) <= 1
    yiq, _ = rgb_to_yiq_dev(torch.as_tensor(np.ascontiguousarray(img)).to(_ia.require_device()))
    return yiq.cpu().numpy()


def convert_to_RGB(img):
    """YIQ -> RGB (img_preprocess.py:16-22)."""
    x = _ia.to_dev(img)
    out = torch.empty_like(x)
    _ia.check(_ia.lib().ia_yiq_to_rgb(_ia.ptr(x), x.shape[0] * x.shape[1], _ia.ptr(out),
                                      _ia.stream()), 'ia_yiq_to_rgb')
    return out.cpu().numpy()


def scale_dev(src, div):
    """Device image / div in fp64 (image_analogies.py:51-56, convert=False path)."""
    dev = _ia.require_device()
    src = src.contiguous()
    out = torch.empty(src.shape, dtype=torch.float64, device=dev)
    _ia.check(_ia.lib().ia_scale_to_f64(_ia.ptr(src), _dtype_code(src), src.numel(), float(div),
                                        _ia.ptr(out), _ia.stream()), 'ia_scale_to_f64')
    return out


# ---- luminance remap / compression ----------------------------------------------------

def _axpb_dev(x, mode, a, m=0.0, b=0.0):
    out = torch.empty_like(x)
    _ia.check(_ia.lib().ia_axpb_f64(_ia.ptr(x), x.numel(), mode, float(a), float(m), float(b),
                                    _ia.ptr(out), _ia.stream()), 'ia_axpb_f64')
    return out


def remap_stats(A, B):
    """(s_B / s_A, m_A, m_B) with numpy's own reductions, as the reference computes them
    (img_preprocess.py:29-32)."""
    A = np.asarray(A); B = np.asarray(B)
    return np.std(B) / np.std(A), np.mean(A), np.mean(B)


def remap_luminance_dev(A, Ap_list, B):
    """Device form: tensors in, tensors out; statistics from host copies."""
    ratio, m_A, m_B = remap_stats(A.cpu().numpy(), B.cpu().numpy())
    f = lambda X: _axpb_dev(X, 1, ratio, m_A, m_B)  # noqa: E731
    return f(A), [f(Ap) for Ap in Ap_list]


def remap_luminance(A, Ap_list, B):
    """Match A / A' luminance mean and std to B (img_preprocess.py:25-40)."""
    assert len(A.shape) == len(Ap_list[0].shape) == len(B.shape) == 2
    A2, Ap2 = remap_luminance_dev(_ia.to_dev(A), [_ia.to_dev(x) for x in Ap_list], _ia.to_dev(B))
    return A2.cpu().numpy(), [x.cpu().numpy() for x in Ap2]


def compress_values_dev(A, B, ratio):
    return _axpb_dev(A, 0, ratio), _axpb_dev(B, 0, ratio)


def compress_values(A, B, ratio):
    """Scale A and B (not A') by AB_weight (img_preprocess.py:43-44)."""
    A2, B2 = compress_values_dev(_ia.to_dev(A), _ia.to_dev(B), ratio)
    return A2.cpu().numpy(), B2.cpu().numpy()


# ---- Gaussian pyramid -------------------------------------------------------------------

def num_layers(h, w, min_size, cap=None):
    """Halvings until the short side is <= min_size (img_preprocess.py:48-54), optionally
    capped (config ``levels``)."""
    n, size = 0, min(h, w)
    while size > min_size:
        size //= 2
        n += 1
    return n if cap is None else min(n, int(cap))


def _normalize_points(p):
    """skimage _center_and_normalize_points: similarity transform to zero mean and
    RMS distance sqrt(2)."""
    centroid = np.mean(p, axis=0)
    rms = np.sqrt(np.sum((p - centroid) ** 2) / p.shape[0])
    f = np.sqrt(2) / rms
    T = np.array([[f, 0, -f * centroid[0]], [0, f, -f * centroid[1]], [0, 0, 1]])
    ph = (T @ np.vstack([p.T, np.ones((p.shape[0]),)])).T
    out = ph[:, :2]
    out[:, 0] /= ph[:, 2]
    out[:, 1] /= ph[:, 2]
    return T, out


def resize_coeffs(in_shape, out_shape):
    """(sx, tx, sy, ty) of the sampling map ``src = s * dst + t`` that skimage 0.18.3's
    ``resize`` uses inside pyramid_reduce: an AffineTransform least-squares fit (SVD) to
    three output corners mapped with ``f * (x + 0.5) - 0.5``, shear terms then zeroed.
    The fit is reproduced step for step (pixel-centre formula alone differs by ulps)."""
    rows, cols = out_shape
    if rows == 1 and cols == 1:
        return 1.0, in_shape[1] / 2.0 - 0.5, 1.0, in_shape[0] / 2.0 - 0.5
    fr, fc = np.asarray(in_shape, dtype=float) / np.asarray(out_shape, dtype=float)
    src = np.array([[0, 0], [0, rows - 1], [cols - 1, rows - 1]])
    dst = np.empty(src.shape, dtype=np.double)
    dst[:, 0] = fc * (src[:, 0] + 0.5) - 0.5
    dst[:, 1] = fr * (src[:, 1] + 0.5) - 0.5
    Ts, s = _normalize_points(src)
    Td, d = _normalize_points(dst)
    M = np.zeros((6, 7))
    M[:3, 0], M[:3, 1], M[:3, 2] = s[:, 0], s[:, 1], 1
    M[3:, 3], M[3:, 4], M[3:, 5] = s[:, 0], s[:, 1], 1
    M[:3, 6], M[3:, 6] = d[:, 0], d[:, 1]
    V = np.linalg.svd(M)[2]
    Hm = np.zeros((3, 3))
    Hm.flat[[0, 1, 2, 3, 4, 5, 8]] = -V[-1, :-1] / V[-1, -1]
    Hm[2, 2] = 1
    Hm = np.linalg.inv(Td) @ Hm @ Ts
    return float(Hm[0, 0]), float(Hm[0, 2]), float(Hm[1, 1]), float(Hm[1, 2])


def pyramid_reduce_dev(img):
    """One skimage pyramid_reduce(downscale=2) step on device (fp64)."""
    H, W = img.shape
    h, w = (H + 1) // 2, (W + 1) // 2
    out = torch.empty((h, w), dtype=torch.float64, device=img.device)
    ws = _ia.workspace(_ia.lib().ia_pyr_workspace_bytes(H, W))
    coef = (ctypes.c_double * 4)(*resize_coeffs((H, W), (h, w)))
    taps = (ctypes.c_double * 4)(*PYR_TAPS)
    _ia.check(_ia.lib().ia_pyr_reduce_f64(_ia.ptr(img), H, W, _ia.ptr(out), h, w, coef, taps,
                                          _ia.ptr(ws), _ia.stream()), 'ia_pyr_reduce_f64')
    return out


def gaussian_pyramid_dev(img, min_size, cap=None):
    """Device pyramid, smallest level first (img_preprocess.py:47-63).  A 3-D image is
    reduced per channel (skimage ``multichannel=True`` semantics)."""
    img = img.to(torch.float64).contiguous()
    if img.dim() == 3:
        chans = [gaussian_pyramid_dev(img[..., k].contiguous(), min_size, cap)
                 for k in range(img.shape[2])]
        return [torch.stack([c[l] for c in chans], dim=-1) for l in range(len(chans[0]))]
    n = num_layers(img.shape[0], img.shape[1], min_size, cap)
    pyr = [img]
    for _ in range(n):
        nxt = pyramid_reduce_dev(pyr[-1])
        if tuple(nxt.shape) == tuple(pyr[-1].shape):
            break   # skimage stops once the size no longer changes
        pyr.append(nxt)
    pyr.reverse()
    assert min(pyr[1].shape[:2]) > min_size
    assert min(pyr[1].shape[:2]) <= min(pyr[-1].shape[:2])
    return pyr


def compute_gaussian_pyramid(img, min_size, levels=None):
    """Gaussian pyramid as a smallest-first list of numpy arrays (img_preprocess.py:47-63)."""
    return [p.cpu().numpy() for p in gaussian_pyramid_dev(_ia.to_dev(img), min_size, levels)]


# ---- B' initialisation -----------------------------------------------------------------

def initialize_Bp(B_pyr, init_rand=True, seed=None):
    """B' pyramid start (img_preprocess.py:66-78): uniform noise drawn level by level,
    smallest first (seeded RandomState when ``seed`` is given), or a copy of B's levels."""
    rng = np.random if seed is None else np.random.RandomState(seed)
    if not init_rand:
        return [np.array(np.asarray(lvl), copy=True) for lvl in B_pyr]
    return [rng.rand(int(np.prod(lvl.shape))).reshape(tuple(lvl.shape)) for lvl in B_pyr]


# ---- padding and index maps -----------------------------------------------------------

def pad_img_pair(img_sm, img_lg, c):
    """Symmetric padding of a (coarse, fine) pair (img_preprocess.py:81-83)."""
    return [np.pad(img_sm, c.padding_sm, mode='symmetric'),
            np.pad(img_lg, c.padding_lg, mode='symmetric')]


def px2ix(pxs, w):
    """(row, col) -> flat index (img_preprocess.py:85-87)."""
    return (np.asarray(pxs[0]) * w + np.asarray(pxs[1])).astype(int)


def ix2px(ixs, w):
    """flat index -> [rows, cols] (img_preprocess.py:90-93)."""
    ixs = np.asarray(ixs)
    return np.array([ixs // w, ixs % w])


def Ap_ix2px(ixs, h, w):
    """Row of the stacked A' database -> ((row, col), image number)
    (img_preprocess.py:96-101)."""
    ixs = np.asarray(ixs)
    img_nums = (ixs // w) // h
    return ix2px(ixs - img_nums * h * w, w), img_nums


def Ap_px2ix(pxs, img_nums, h, w):
    """((row, col), image number) -> row of the stacked database (img_preprocess.py:104-106)."""
    return (((h * np.asarray(img_nums)) + np.asarray(pxs[0])) * w + np.asarray(pxs[1])).astype(int)


def savefig_noborder(fileName, fig):
    """Save the current figure without axes or border (img_preprocess.py:109-113)."""
    import matplotlib.pyplot as plt
    plt.axis('off')
    fig.axes.get_xaxis().set_visible(False)
    fig.axes.get_yaxis().set_visible(False)
    plt.savefig(fileName, bbox_inches='tight', pad_inches=0)
