"""The sharded synthesis's per-wave exchange on the GPU: the device-side
form (IPC-mapped receive boxes written and read by the exact stage's kernel, ia.h
ia_peer_*) against the oracle, in one process (a 1-rank exchange) and across 2 and 3
rank processes sharing the box's GPU; and the RCCL form (1 rank) for the same inputs."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

import ia_oracle as o
import ia_oracle_c as oc
from conftest import analogy_inputs

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to('cuda', dtype=torch.float64)


def oracle_run(seed, A_shape, B_shape, nap, kappa):
    A, Aps, B = analogy_inputs(seed, A_shape, B_shape, n_ap=nap)
    A_pyr, Ap_list, B_pyr, Bp_pyr, L = o.setup_luminance(A, Aps, B, seed=seed)
    w = o.compute_weights(3, 5, 12, 1)
    ref = oc.synthesize(A_pyr, Ap_list, B_pyr, [b.copy() for b in Bp_pyr], L, kappa, w)
    return (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref


@pytest.mark.parametrize('kind,pipeline', [('peer', False), ('peer', True), ('rccl', True)])
def test_one_rank_exchange_matches_oracle(gpu, kind, pipeline):
    """Every level sharded over a 1-rank exchange (one per level; pipelined or one level at
    a time): the oracle's B', s, im bit for bit."""
    import _ia
    import image_analogies as ia
    (A_pyr, Ap_list, B_pyr, Bp_pyr, L, w), ref = oracle_run(41, (46, 54), (39, 47), 2, 0.8)
    comms = [_ia.exchange(0, 1, kind) for _ in range(1, L)]
    try:
        if kind == 'peer':
            assert _ia.lib().ia_peer_mem_kind(comms[0]) in (0, 1, 2)
        Bp_dev = [dev(b) for b in Bp_pyr]
        out = ia.synthesize_dev([dev(p) for p in A_pyr], [[dev(p) for p in q] for q in Ap_list],
                                [dev(p) for p in B_pyr], Bp_dev, L, 0.8, w, comm=comms,
                                rank=0, nranks=1, pipeline=pipeline)
        torch.cuda.synchronize()
        for cm in comms:
            _ia.exchange_status(cm)
        for l in ref:
            assert np.array_equal(out[l][0].cpu().numpy(), ref[l][1]), l
            assert np.array_equal(out[l][1].cpu().numpy(), ref[l][2]), l
            assert np.array_equal(Bp_dev[l].cpu().numpy(), ref[l][0]), l
    finally:
        torch.cuda.synchronize()
        for cm in comms:
            _ia.check(_ia.lib().ia_comm_destroy(cm), 'ia_comm_destroy')


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(('127.0.0.1', 0))
        return sk.getsockname()[1]


def run_ranks(world, argv, timeout=100):
    """Start `world` exchange_worker.py processes (gloo rendezvous, all on cuda:0)."""
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), IA_TEST_DEVICE='0',
                   IA_SHARD_MIN_ROWS='0', IA_SHARE_GPU='1')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.join(HERE, 'exchange_worker.py')]
                                      + [str(a) for a in argv], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0].decode(errors='replace'))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, txt in zip(procs, outs):
        assert p.returncode == 0, txt[-3000:]


@pytest.mark.parametrize('world,pipeline', [(2, 1), (3, 0)])
def test_ranks_on_one_gpu_peer_exchange_match_oracle(gpu, world, pipeline):
    """`world` rank processes, every level's DB sharded over them (ragged shards at 3),
    exchanging through each other's IPC-mapped boxes on the box's one GPU: every rank's
    B', s, im equal the oracle's."""
    seed, A_shape, B_shape, nap, kappa = 43, (52, 61), (41, 50), 2, 0.9
    _, ref = oracle_run(seed, A_shape, B_shape, nap, kappa)
    with tempfile.TemporaryDirectory() as td:
        run_ranks(world, [td, seed, A_shape[0], A_shape[1], B_shape[0], B_shape[1], nap, kappa,
                          'peer', pipeline])
        for r in range(world):
            got = np.load(os.path.join(td, 'rank%d.npz' % r))
            for l in ref:
                assert np.array_equal(got['s%d' % l], ref[l][1]), (r, l)
                assert np.array_equal(got['im%d' % l], ref[l][2]), (r, l)
                assert np.array_equal(got['bp%d' % l], ref[l][0]), (r, l)
