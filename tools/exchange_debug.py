"""Debug: one rank of a 2-rank peer-exchange synthesis on one GPU vs the same synthesis
unsharded in-process (debug records compared pixel by pixel).  Run as `python tools/exchange_debug.py` on the GPU box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import conftest  # noqa: E402
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import ia_oracle as o  # noqa: E402


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo')
    torch.cuda.set_device(0)
    import _ia
    import image_analogies as ia
    seed = 43
    A, Aps, B = conftest.analogy_inputs(seed, (52, 61), (41, 50), n_ap=2)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed)
    w = o.compute_weights(3, 5, 12, 1)

    def dev(a):
        return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=torch.float64)
    cm = _ia.exchange(rank, world, 'peer')
    for nw, M in ((50, 1), (200, 64), (100, 343)):
        bad = ctypes.c_int(-1)
        _ia.check(_ia.lib().ia_diag_peer_stress(cm, nw, M, ctypes.byref(bad), _ia.stream()),
                  'ia_diag_peer_stress')
        print('rank', rank, 'stress', nw, 'waves x', M, 'queries: bad', bad.value, flush=True)
    _ia.exchange_status(cm)
    _ia.lib().ia_comm_destroy(cm)
    res = []
    for sharded in (True, False):
        comms = [_ia.exchange(rank, world, 'peer')] if sharded else None
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 0.9, w, comm=comms,
                                rank=rank if sharded else 0, nranks=world if sharded else 1,
                                levels={1}, pipeline=False, debug=True)
        torch.cuda.synchronize()
        if comms:
            _ia.exchange_status(comms[0])
            bad = ctypes.c_int(-1)
            rc = _ia.lib().ia_diag_peer_stress(comms[0], 4, 8, ctypes.byref(bad), _ia.stream())
            st = _ia.lib().ia_peer_status(comms[0])
            print('rank', rank, 'stress after the synthesis: rc', rc, 'bad', bad.value, 'status', st, flush=True)
            tr = np.zeros(1024 * 8 * 12, dtype=np.uint64)
            _ia.check(_ia.lib().ia_diag_peer_trace(comms[0], tr.ctypes.data_as(ctypes.c_void_p)), 'trace')
            tr = tr.reshape(1024, 8, 12)
            for e in range(1, 8):
                t = tr[e, 0]
                f = lambda x: float(np.array([x], dtype=np.uint64).view(np.float64)[0])
                print('rank', rank, 'epoch', e, 'own (%.6g, %d) got (%.6g, %d) raw' % (f(t[0]), t[1], f(t[2]), t[3]),
                      ' '.join('%016x' % x for x in t[4:10]), flush=True)
        s, im, (dpx, dd) = out[1]
        res.append((s.cpu().numpy(), im.cpu().numpy(), dpx.cpu().numpy(), dd.cpu().numpy()))
    (s1, i1, p1, d1), (s0, i0, p0, d0) = res
    bad = np.nonzero((s1 != s0).any(1) | (i1 != i0))[0]
    print('rank', rank, 'mismatching pixels', len(bad), 'of', len(s0), flush=True)
    for q in bad[:4]:
        print(' px', q, 'sharded s', s1[q], i1[q], 'dbg', p1[q], d1[q], '| unsharded s', s0[q], i0[q],
              'dbg', p0[q], d0[q], flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
