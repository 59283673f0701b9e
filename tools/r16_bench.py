"""Timing of the rotated screen (R16, k_screen16r<G>) on c4's finest level: the product's
dominant kernel over the 4,194,304-row rotated DB at M queries from
tests/golden/c4_queries.npz, HIP events around reps launches (IA_LIB_PATH selects a variant
build, tools/build_variant.sh).  Prints per M: mean us per launch, algorithmic frac of the
f16 peak (110 flop per pair), pipe frac (160 f16 flop issued per pair), DB GB/s.

  python tools/r16_bench.py [--M 342,256,128] [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'image-analogies-python_amd'))
sys.path.insert(0, ROOT)

import _ia            # noqa: E402
import algorithms     # noqa: E402
import bench          # noqa: E402
import config as cfg  # noqa: E402
import img_preprocess as ip  # noqa: E402

F16_PEAK = 4096.0 * 256 * 2.4e9 / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--M', default='342,256,128')
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--sleep', type=int, default=0, help='GPU cycles of idle spin after each launch '
                    '(torch.cuda._sleep: the product\'s gaps between screens); not counted')
    args = ap.parse_args()
    Ms = [int(x) for x in args.M.split(',')]
    dev = torch.device('cuda', 0)
    job = bench.Job(bench.CONFIGS['c4'], 0, dev)
    A_pyr = ip.gaussian_pyramid_dev(job.A, cfg.n_sm, job.levels)
    Ap_pyr = ip.gaussian_pyramid_dev(job.Ap, cfg.n_sm, job.levels)
    level = job.max_levels - 1
    idx = algorithms.level_index(A_pyr, [Ap_pyr], level, rot=True)
    assert idx.dbr is not None
    lib = _ia.lib()
    N = idx.nrows
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'c4_queries.npz'))
    Mmax = max(Ms)
    qrows = lib.ia_diag_qp_rows(Mmax)
    q64 = torch.zeros((Mmax, _ia.IA_DP), dtype=torch.float64, device=dev)
    q64[:, :55] = torch.as_tensor(np.asarray(g['q'][:Mmax], dtype=np.float64)).to(dev)
    q16 = torch.zeros((qrows, 128), dtype=torch.float16, device=dev)
    nq = torch.zeros(qrows, dtype=torch.float64, device=dev)
    nsk = torch.zeros(qrows, dtype=torch.float64, device=dev)
    nseg = lib.ia_db_rows_padded(N) // min(lib.ia_db_chunk_rows(N), 512)
    segmin = torch.zeros((qrows, nseg), dtype=torch.float32, device=dev)
    st = _ia.stream()
    out = []
    for M in Ms:
        def run():
            _ia.check(lib.ia_diag_screen16r(ctypes.byref(idx.src), idx.row0, N, _ia.ptr(idx.dbr), _ia.ptr(idx.rot),
                                            _ia.ptr(idx.amax), _ia.ptr(idx.center), _ia.ptr(q64), M, _ia.ptr(q16),
                                            _ia.ptr(nq), _ia.ptr(nsk), _ia.ptr(segmin), st), 'screen16r')
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if args.sleep:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for a, b in ev:
                a.record()
                run()
                b.record()
                torch.cuda._sleep(args.sleep)
            torch.cuda.synchronize()
            us = sum(a.elapsed_time(b) for a, b in ev) * 1e3 / args.reps
        else:
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
        pairs = M * N
        out.append({'M': M, 'us': round(us, 1), 'frac': 110 * pairs / (us * 1e-6) / 1e12 / F16_PEAK,
                    'pipe_frac': 2 * lib.ia_db_rot_slots() * pairs / (us * 1e-6) / 1e12 / F16_PEAK,
                    'P': lib.ia_db_rot_components(),
                    'db_gbs': lib.ia_db_rot_bytes(N) / (us * 1e-6) / 1e9,
                    'sleep': args.sleep, 'lib': os.environ.get('IA_LIB_PATH', 'libia.so')})
        print(json.dumps(out[-1]), flush=True)


if __name__ == '__main__':
    main()
