"""Kernel-boundary gaps of the c4 synthesis (diagnostic, run under rocprofv3 --kernel-trace):
mode 'pipe' = bench.py's step (levels pipelined on their streams), mode 'finest' = the finest
level alone on one stream (the coarse levels synthesised first, untraced region marked by a
sync).  Compare the gap rows of tools/trace_summary.py between the two.
Usage: python tools/gap_probe.py pipe|finest [config]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

mode = sys.argv[1]
conf = bench.CONFIGS[sys.argv[2] if len(sys.argv) > 2 else 'c4']
job = bench.Job(conf, 0, 'cuda:0')
ip, cfg, ia = bench.ip, bench.cfg, bench.ia
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode == 'pipe':
        job.step()
    else:
        A_pyr, Ap_list, B_pyr, Bp = job.prepare()
        L = job.max_levels
        ia.synthesize_dev(A_pyr, Ap_list, B_pyr, Bp, L, job.k, job.weights, levels=set(range(1, L - 1)))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ia.synthesize_dev(A_pyr, Ap_list, B_pyr, Bp, L, job.k, job.weights, levels={L - 1},
                          pipeline=False)
    torch.cuda.synchronize()
    print('%s rep %d: %.1f ms' % (mode, rep, (time.perf_counter() - t0) * 1e3), flush=True)
