"""Throughput of 3-channel matching (the reference's default convert=False on colour images:
config.py:29-42 num_ch = 3, 165-dim rows, algorithms.py:11-47) on one GPU, next to the
luminance path on the same images (their Y channel): B' pixels per second of whole
syntheses (device pyramids, B' reset, every level), inputs resident in HBM.

usage: python tools/colour_bench.py [H W] [steps]      (default 180 117 (c1 size), 3 steps)
       COLOUR_PIPE=0: the colour levels one at a time (default: pipelined, ia_synth_levels3)
       COLOUR_ONLY=1: the 3-channel run alone (kernel traces of it)
Also reports the colour exact stage's candidate tiles per query (ia_diag_color16_stats) and a
B' checksum (equal with and without the pipeline).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

ip, cfg, ia = bench.ip, bench.cfg, bench.ia


def main():
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (180, 117)
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    from scipy.ndimage import gaussian_filter
    dev = 'cuda:0'
    A = np.dstack([bench.smooth_noise(7 + 17 * c, (H, W)) for c in range(3)])
    Ap = np.dstack([gaussian_filter(A[..., c], 1.5) for c in range(3)])
    B = np.dstack([bench.smooth_noise(8 + 17 * c, (H, W)) for c in range(3)])
    w = torch.as_tensor(cfg.compute_weights(3, 5, 12, 3)).to(dev)
    w1 = torch.as_tensor(cfg.compute_weights(3, 5, 12, 1)).to(dev)
    import ctypes
    import _ia
    pipe = os.environ.get('COLOUR_PIPE', '1') != '0'
    out = {'size': [H, W], 'pipeline': pipe}
    runs = {'rgb': (A, Ap, B, w), 'luminance': (A[..., 0], Ap[..., 0], B[..., 0], w1)}
    if os.environ.get('COLOUR_ONLY', '0') != '0':
        del runs['luminance']
    for name, (a, ap, b, ww) in runs.items():
        a, ap, b = (torch.as_tensor(x).to(dev) for x in (a, ap, b))
        nB = ip.num_layers(H, W, cfg.n_sm, None)
        L = nB + 1
        shapes = [b.shape]
        for _ in range(nB):
            shapes.append(tuple([(shapes[-1][0] + 1) // 2, (shapes[-1][1] + 1) // 2] + list(b.shape[2:])))
        shapes.reverse()
        init = [torch.as_tensor(x).to(dev)
                for x in ip.initialize_Bp([np.empty(s) for s in shapes], True, 9)]
        Bp = [x.clone() for x in init]
        pixels = sum(s[0] * s[1] for s in shapes[1:L])

        def step():
            A_pyr = ip.gaussian_pyramid_dev(a, cfg.n_sm)
            Ap_pyr = ip.gaussian_pyramid_dev(ap, cfg.n_sm)
            B_pyr = ip.gaussian_pyramid_dev(b, cfg.n_sm)
            for d, s in zip(Bp, init):
                d.copy_(s)
            ia.synthesize_dev(A_pyr, [Ap_pyr], B_pyr, Bp, L, 0.5, ww, pipeline=pipe)

        st = (ctypes.c_ulonglong * 2)()
        _ia.check(_ia.lib().ia_diag_color16_stats(st), 'stats')   # (reads and clears)
        step()
        torch.cuda.synchronize()
        _ia.check(_ia.lib().ia_diag_color16_stats(st), 'stats')
        cand = (st[0] / pixels, int(st[1]))
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        out[name] = {'ms_per_step': dt * 1e3, 'px_per_s': pixels / dt, 'pixels': pixels,
                     'bp_checksum': float(sum(float(x.sum()) for x in Bp[1:L]))}
        if name == 'rgb':
            out[name]['candidate_tiles_per_query'], out[name]['full_scans'] = cand
    if 'luminance' in out:
        out['rgb_vs_luminance_slowdown'] = out['luminance']['px_per_s'] / out['rgb']['px_per_s']
    print(json.dumps(out))


if __name__ == '__main__':
    main()
