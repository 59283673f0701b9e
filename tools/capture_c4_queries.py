"""Capture real c4 finest-level queries from a GPU synthesis (run on the GPU box):
bench.py's c4 job, one step, then the exact query the scanline loop would have formed at
each sampled pixel (query_at below: final B' before the pixel, initial B' after it).  Writes gpurun_out/c4_queries_in.npz {q (M x 55), pixels (M x 2)}; the oracle
answers are computed on the CPU by tests/golden/make_config_fixtures.py c4."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle')):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402
import img_preprocess as ip  # noqa: E402
import config as cfg  # noqa: E402
import ia_oracle as o  # noqa: E402


def query_at(B_sm, B_lg, Bp_sm, Bp_final, Bp_init, y, x):
    """The 55-dim query of pixel (y, x) at the moment the reference's scanline loop
    (image_analogies.py:161-168) visited it: final values before it, initial ones after."""
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


def sample_pixels(H, W, rng, n_rand):
    """Border, corner and interior pixels of an H x W level, plus n_rand random ones."""
    rows = sorted({0, 1, 2, 3, H // 2, H - 3, H - 2, H - 1})
    cols = sorted({0, 1, 2, 3, W // 3, W // 2, W - 3, W - 2, W - 1})
    px = [(y, x) for y in rows for x in cols if 0 <= y < H and 0 <= x < W]
    px += [(int(y), int(x)) for y, x in zip(rng.randint(0, H, n_rand), rng.randint(0, W, n_rand))]
    return sorted(set(px))


def main():
    torch.cuda.set_device(0)
    job = bench.Job(bench.CONFIGS['c4'], 0, torch.device('cuda', 0))
    job.step()
    torch.cuda.synchronize()
    level = job.max_levels - 1
    B_pyr = [p.cpu().numpy() for p in ip.gaussian_pyramid_dev(job.B, cfg.n_sm, job.levels)]
    Bp = [p.cpu().numpy() for p in job.Bp]
    init = job.Bp_init[level].cpu().numpy()
    H, W = B_pyr[level].shape
    px = sample_pixels(H, W, np.random.RandomState(2024), n_rand=440)
    Q = np.vstack([query_at(B_pyr[level - 1], B_pyr[level], Bp[level - 1], Bp[level], init, y, x)
                   for y, x in px])
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, 'gpurun_out', 'c4_queries_in.npz'), q=Q,
                        pixels=np.array(px, dtype=np.int32))
    print('captured %d queries at level %d (%dx%d)' % (len(Q), level, H, W))


if __name__ == '__main__':
    main()
