"""Capture real c4 finest-level queries from a GPU synthesis (run on the GPU box):
bench.py's c4 job, one step, then the exact query the scanline loop would have formed at
each sampled pixel (tests/spotcheck.py query_at: final B' before the pixel, initial B'
after it).  Writes gpurun_out/c4_queries_in.npz {q (M x 55), pixels (M x 2)}; the oracle
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
import spotcheck  # noqa: E402


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
    px = spotcheck.sample_pixels(H, W, np.random.RandomState(2024), n_rand=440)
    Q = spotcheck.queries(B_pyr, Bp, init, level, px)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, 'gpurun_out', 'c4_queries_in.npz'), q=Q,
                        pixels=np.array(px, dtype=np.int32))
    print('captured %d queries at level %d (%dx%d)' % (len(Q), level, H, W))


if __name__ == '__main__':
    main()
