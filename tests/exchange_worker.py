"""One rank of a multi-process sharded synthesis (tests/test_gpu_exchange.py).

Started by the test as a child process per rank (RANK, WORLD_SIZE, MASTER_ADDR/PORT in
the environment, gloo rendezvous); every rank runs on the device named by IA_TEST_DEVICE
(the test box has one GPU, so all ranks share cuda:0 — the device-side exchange's boxes
are then IPC-mapped between processes of one GPU, the same protocol as over xGMI).
Every level with a DB of >= IA_SHARD_MIN_ROWS rows is sharded; each rank writes its
per-level (B', s, im) to <out>/rank<r>.npz for the parent to compare with the oracle.

usage: exchange_worker.py OUT SEED AH AW BH BW NAP KAPPA KIND PIPELINE
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import conftest  # noqa: E402  (import paths: package + oracle)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ia_oracle as o  # noqa: E402


def main():
    out_dir, seed, Ah, Aw, Bh, Bw, nap, kappa, kind, pipe = sys.argv[1:11]
    seed, Ah, Aw, Bh, Bw, nap = map(int, (seed, Ah, Aw, Bh, Bw, nap))
    kappa = float(kappa)
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo')
    torch.cuda.set_device(int(os.environ.get('IA_TEST_DEVICE', '0')))
    import _ia
    import image_analogies as ia
    A, Aps, B = conftest.analogy_inputs(seed, (Ah, Aw), (Bh, Bw), n_ap=nap)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed)
    w = o.compute_weights(3, 5, 12, 1)

    def dev(a):
        return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=torch.float64)
    comms = [_ia.exchange(rank, world, kind) for _ in range(1, L)]
    try:
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, kappa, w, comm=comms,
                                rank=rank, nranks=world, pipeline=(pipe == '1'))
        torch.cuda.synchronize()
        for cm in comms:
            _ia.exchange_status(cm)
        res = {}
        for l in out:
            res['s%d' % l] = out[l][0].cpu().numpy()
            res['im%d' % l] = out[l][1].cpu().numpy()
            res['bp%d' % l] = Bp_dev[l].cpu().numpy()
        np.savez(os.path.join(out_dir, 'rank%d.npz' % rank), **res)
    finally:
        torch.cuda.synchronize()
        for cm in comms:
            _ia.check(_ia.lib().ia_comm_destroy(cm), 'ia_comm_destroy')
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
