"""Per-rank cost of the sharded c4 synthesis, simulated on one GPU (diagnostic).

Runs the synthesis as rank `r` of G database shards (each level's rows
`shard_rows(N, r, G)`), with a 1-rank exchange (IA_EXCHANGE: rccl — unfused exact stage,
all-gather, k_finish_gather; peer [default] — the exact stage's kernel publishes to and
collects from its own box and finishes the pixel): the per-wave path is the sharded one,
but the exchange moves one shard's winners only, so the time excludes the real xGMI
latency.  The
winners are this shard's, so B' differs from the real result: timing only.
Per level wall time between torch.cuda.synchronize() calls (levels one at a time), and the
whole step with the levels pipelined (ia_synth_levels, one communicator per sharded
level); second repetition reported.

Usage: python tools/shard_sim.py G [G ...]        (G = 1 runs the sharded path unsharded)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

ip, cfg, ia, _ia = bench.ip, bench.cfg, bench.ia, bench._ia


def one_rank_comm():
    return _ia.exchange(0, 1)


def main():
    gs = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    job = bench.Job(bench.CONFIGS['c4'], 0, 'cuda:0')
    A_pyr = ip.gaussian_pyramid_dev(job.A, cfg.n_sm, job.levels)
    Ap_pyr = ip.gaussian_pyramid_dev(job.Ap, cfg.n_sm, job.levels)
    B_pyr = ip.gaussian_pyramid_dev(job.B, cfg.n_sm, job.levels)
    comms = [one_rank_comm() for _ in range(job.max_levels)]
    for G in gs:
        res = {}
        for rep in range(2):
            for level in range(1, job.max_levels):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ia.synthesize_dev(A_pyr, [Ap_pyr], B_pyr, job.Bp, job.max_levels, job.k,
                                  job.weights, comm=comms[0], rank=0, nranks=G, levels={level},
                                  pipeline=False)
                torch.cuda.synchronize()
                res[level] = (time.perf_counter() - t0) * 1e3
        tot = sum(res.values())
        pipe = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ia.synthesize_dev(A_pyr, [Ap_pyr], B_pyr, job.Bp, job.max_levels, job.k, job.weights,
                              comm=comms, rank=0, nranks=G, pipeline=True)
            torch.cuda.synchronize()
            pipe.append((time.perf_counter() - t0) * 1e3)
        print('[%s] G=%d rank0 %.1f ms/step (levels one at a time: ' % (_ia.exchange_kind(), G, tot) +
              ' '.join('L%d %.1f' % (l, t) for l, t in sorted(res.items())) +
              '); pipelined %.1f ms/step' % min(pipe[1:]), flush=True)
    for cm in comms:
        _ia.exchange_status(cm)
        _ia.lib().ia_comm_destroy(cm)


if __name__ == '__main__':
    main()
