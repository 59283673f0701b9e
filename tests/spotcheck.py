"""Per-pixel re-derivation of the reference's decision from a finished synthesis — the
size-independent parity check used at BASELINE sizes the oracle cannot synthesise whole
(c4: 1,048,576 finest-level pixels x 4,194,304 database rows).

For a B' pixel q = (y, x) of level l, the reference (image_analogies.py:161-220) built
its query from B (static), the finished coarse level B'[l-1], and the fine level B'[l] as
it stood when q was visited: final values at pixels before q in scanline order, the
initial values elsewhere (the symmetric padding reads both).  Given a device run's final
B'[l], its initial B'[l] and its s / im maps, this module rebuilds that query exactly,
takes the oracle's exact 1-NN (ia_oracle_c.nn_batch), the oracle's coherence candidate
over the device's own earlier s / im (algorithms.py:92-130) and the kappa test
(algorithms.py:133-135, image_analogies.py:200-211), and returns the (row, col, image)
the reference would have written at q.  Test infrastructure only (uses oracle/).
"""
import numpy as np

import ia_oracle as o


def query_at(B_sm, B_lg, Bp_sm, Bp_final, Bp_init, y, x):
    """The 55-dim query of pixel (y, x) at the moment the scanline loop visited it."""
    H, W = B_lg.shape
    full = o.extract_pixel_feature(B_sm, B_lg, (y, x), True)                  # 9 + 25
    coarse = o.extract_pixel_feature(Bp_sm, Bp_final, (y, x), False)[:9]     # final B'[l-1]
    qi = y * W + x
    fine = []
    for t in range(o.N_HALF):
        yy = int(o.sym_index(np.array([y + t // 5 - 2]), H)[0])
        xx = int(o.sym_index(np.array([x + t % 5 - 2]), W)[0])
        fine.append(Bp_final[yy, xx] if yy * W + xx < qi else Bp_init[yy, xx])
    return np.concatenate([full, coarse, np.array(fine)])


def queries(B_pyr, Bp_final_pyr, Bp_init_lvl, level, pixels):
    return np.vstack([query_at(B_pyr[level - 1], B_pyr[level], Bp_final_pyr[level - 1],
                               Bp_final_pyr[level], Bp_init_lvl, y, x) for y, x in pixels])


def decide(As, A_shape, q, app_row, s, im, y, x, W, weights, kappa_factor):
    """(row, col, image) the reference writes at (y, x): the exact match app_row, or the
    coherence candidate when it passes the kappa test (s, im: the run's maps)."""
    A_h, A_w = A_shape
    (pr, pc), pimg = o.Ap_ix2px(int(app_row), A_h, A_w)
    if y == 0 and x == 0:
        return pr, pc, pimg
    p_coh, i_coh, _ = o.best_coherence_match(As, A_shape, q, s, im, (y, x), W)
    if tuple(p_coh) == (-1, -1):
        return pr, pc, pimg
    d_app = o.compute_distance(As[int(app_row)], q, weights)
    d_coh = o.compute_distance(As[o.Ap_px2ix(p_coh, i_coh, A_h, A_w)], q, weights)
    if d_coh <= d_app * kappa_factor:
        return int(p_coh[0]), int(p_coh[1]), int(i_coh)
    return pr, pc, pimg


def sample_pixels(H, W, rng, n_rand=256, full_rows=(), border_step=0):
    """Border, corner and interior pixels of an H x W level (deterministic given rng);
    full_rows: whole scanlines added; border_step > 0: every border_step-th pixel of the
    four borders (plus the two pixels next to each corner) added."""
    rows = sorted({0, 1, 2, 3, H // 2, H - 3, H - 2, H - 1})
    cols = sorted({0, 1, 2, 3, W // 3, W // 2, W - 3, W - 2, W - 1})
    px = [(y, x) for y in rows for x in cols if 0 <= y < H and 0 <= x < W]
    px += [(int(y), int(x)) for y, x in zip(rng.randint(0, H, n_rand), rng.randint(0, W, n_rand))]
    for y in full_rows:
        px += [(y, x) for x in range(W)]
    if border_step:
        px += [(y, x) for y in (0, H - 1) for x in list(range(0, W, border_step)) + [1, W - 2]]
        px += [(y, x) for x in (0, W - 1) for y in list(range(0, H, border_step)) + [1, H - 2]]
    return sorted(set(px))
