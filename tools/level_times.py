"""Per-level wall time of the c4 synthesis (diagnostic): each level run alone between
torch.cuda.synchronize() calls, twice (the second is reported), under the current IA_*
environment.  Usage: python tools/level_times.py [config]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

conf = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c4']
job = bench.Job(conf, 1234, 'cuda:0')
ip, cfg, ia = bench.ip, bench.cfg, bench.ia
A_pyr = ip.gaussian_pyramid_dev(job.A, cfg.n_sm, job.levels)
Ap_pyr = ip.gaussian_pyramid_dev(job.Ap, cfg.n_sm, job.levels)
B_pyr = ip.gaussian_pyramid_dev(job.B, cfg.n_sm, job.levels)
res = {}
for rep in range(2):
    for level in range(1, job.max_levels):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ia.synthesize_dev(A_pyr, [Ap_pyr], B_pyr, job.Bp, job.max_levels, job.k, job.weights,
                          levels={level})
        torch.cuda.synchronize()
        res[level] = (time.perf_counter() - t0) * 1e3
print(' '.join('L%d %.1f ms' % (l, t) for l, t in sorted(res.items())),
      'env', {k: v for k, v in os.environ.items() if k.startswith('IA_')}, flush=True)
