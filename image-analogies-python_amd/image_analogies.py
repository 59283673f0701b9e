"""Image Analogies driver — drop-in for the reference's ``image_analogies`` module
(reference image_analogies.py:17-268), running the whole B' synthesis on an MI355X.

``image_analogies_main(A_fname, Ap_fname_list, B_fname, out_path, c, debug=False)`` keeps
the reference's signature, parameters (``config`` module as ``c``), outputs
(``level_%d_color.jpg`` per level and ``<name>.jpg``, ``metadata.txt``) and printed timings.
Underneath, every level is synthesised by ``ia_synth_level`` (skewed wavefront,
exact matcher, or the LSH matcher with ``c.matcher = 'lsh'``) with the pyramids, databases and index maps resident in HBM.

``synthesize_dev`` is the device-level entry used by bench.py and the parity tests:
device pyramids in, per-level (s, im) index maps out, B' pyramid updated in place;
with ``comm`` it shards the databases of the large levels over the ranks (RCCL all-gather
per wave) and synthesises the small ones on every rank alone (``shard_level``).
"""
import ctypes
import os
import sys
import time
import warnings

import numpy as np
import torch

import _ia
import algorithms
import img_preprocess as ip
from config import save_metadata, setup_vars


def kappa_factor(level, max_levels, k):
    """1 + 2**(level - max_levels) * kappa (image_analogies.py:206)."""
    return 1 + (2.0 ** (level - max_levels)) * k


def shard_rows(N, rank, nranks):
    """Contiguous row range of one rank: [N*r/G, N*(r+1)/G)."""
    r0 = N * rank // nranks
    return r0, N * (rank + 1) // nranks - r0


def shard_min_rows():
    """Smallest level database (rows) that is sharded over the ranks (IA_SHARD_MIN_ROWS,
    default 2**19).  Below it every rank synthesises the level alone from its replicated
    state with the fused single-GPU path: a sharded rank still pays the whole per-wave
    fixed cost (query gather, exact stage, tail) plus one RCCL all-gather per wave, which
    on c4's 64-256 px levels exceeds the screen time sharding saves."""
    return int(os.environ.get('IA_SHARD_MIN_ROWS', 1 << 19))


def shard_level(N, nranks):
    """True when a level with an N-row database is sharded over nranks ranks.  A 1-rank
    communicator always takes the exchange path (that is how the RCCL path is tested on
    one GPU)."""
    return nranks == 1 or N >= shard_min_rows()


def level_rows(Ap_pyr_list, level):
    """Rows of a level's database: n_A' x H x W of A' at that level (algorithms.py:63-67)."""
    return sum(p[level].shape[0] * p[level].shape[1] for p in Ap_pyr_list)


class _LevelCall:
    """Arguments (IaSynthArgs) and outputs of one level's device synthesis; keeps every
    buffer the call reads alive until the caller drops it."""

    def __init__(self, level, max_levels, index, B_sm, B_lg, Bp_sm, Bp_lg, weights, k,
                 comm=None, prof=False, eager=False, debug=False):
        dev = B_lg.device
        H, W = B_lg.shape
        self.index = index
        self.s = torch.empty((H * W, 2), dtype=torch.int32, device=dev)
        self.im = torch.empty(H * W, dtype=torch.int32, device=dev)
        self.dbg = None
        if debug:
            self.dbg = (torch.zeros((H * W, 7), dtype=torch.int32, device=dev),
                        torch.zeros((H * W, 2), dtype=torch.float64, device=dev))
        nranks = _ia.lib().ia_comm_nranks(comm) if comm else 1
        self.ws = _ia.workspace(_ia.lib().ia_synth_workspace_bytes(H, W, index.nrows, nranks))
        a = _ia.IaSynthArgs()
        a.src = index.src
        a.db, a.row0, a.nrows, a.N_total = _ia.ptr(index.db).value, index.row0, index.nrows, index.N
        a.dbi = index.dbi_ptr()
        if getattr(index, 'dbr', None) is not None:
            a.dbr, a.rot = _ia.ptr(index.dbr).value, _ia.ptr(index.rot).value
        a.center, a.amax = _ia.ptr(index.center).value, _ia.ptr(index.amax).value
        a.B_sm, a.B_lg = _ia.ptr(B_sm).value, _ia.ptr(B_lg).value
        a.B_hs, a.B_ws = B_sm.shape
        a.H, a.W = H, W
        a.Bp_sm, a.Bp_lg = _ia.ptr(Bp_sm).value, _ia.ptr(Bp_lg).value
        a.weights = _ia.ptr(weights).value
        self.keep = (weights, B_sm, B_lg, Bp_sm, Bp_lg)   # read by every wave: alive with the call
        a.kappa_factor = kappa_factor(level, max_levels, k)
        a.s, a.im = _ia.ptr(self.s).value, _ia.ptr(self.im).value
        a.workspace = _ia.ptr(self.ws).value
        a.comm = comm
        a.lsh = index.lsh_ptr()
        a.flags = (_ia.IA_SYNTH_EAGER if eager else 0) | (_ia.IA_SYNTH_PROF if prof else 0)
        a.tag = level
        if debug:
            a.dbg_px, a.dbg_dist = _ia.ptr(self.dbg[0]).value, _ia.ptr(self.dbg[1]).value
        self.args = a

    def result(self):
        if self.dbg is not None:
            return self.s, self.im, self.dbg
        return self.s, self.im


def synthesize_level_dev(level, max_levels, index, B_sm, B_lg, Bp_sm, Bp_lg, weights, k,
                         comm=None, prof=False, eager=False, debug=False):
    """One level on device: Bp_lg updated in place; returns (s (H*W, 2), im (H*W,)) int32,
    plus with debug=True the per-pixel debug record (dbg_px (H*W, 7) int32, dbg_dist
    (H*W, 2) fp64; include/ia.h).  prof=True: record this level into the open profile
    (_ia.prof_begin / prof_end; no synchronisation).  eager=True: never capture the
    level's wave loop into a HIP graph."""
    call = _LevelCall(level, max_levels, index, B_sm, B_lg, Bp_sm, Bp_lg, weights, k, comm,
                      prof, eager, debug)
    _ia.check(_ia.lib().ia_synth_level(ctypes.byref(call.args), _ia.stream()), 'ia_synth_level')
    return call.result()


def synthesize_levels_dev(calls):
    """Consecutive levels (a list of _LevelCall, coarse to fine) synthesised together by
    ia_synth_levels: each level on its own stream, running behind the level below as far
    as its coarse windows allow (include/ia.h).  Same results as one level at a time."""
    arr = (_ia.IaSynthArgs * len(calls))(*[c.args for c in calls])
    _ia.check(_ia.lib().ia_synth_levels(arr, len(calls), _ia.stream()), 'ia_synth_levels')
    return [c.result() for c in calls]


def wave_max_queries(H, W):
    """Most pixels of one wave of an H x W level (t = x + 3y), + 1 as ia_synth.hip's."""
    return min(H, (W + 2) // 3) + 1


def residency_ok(waiters, fused, screen, cus=256, lds_per_cu=160 * 1024, vgprs_per_simd=512, gran=8):
    """Forward progress of sharded levels over the device-side exchange.
    A fused workgroup that waits for other ranks' records holds its CU's LDS and one wave's
    VGPRs on each SIMD (256 threads) while it waits; the screens that produce those records
    (another level's, or another rank's on a shared GPU) must still find a CU.  A CU holding
    j waiting workgroups still fits a screen block (also one wave per SIMD) while
    j * fused_lds + screen_lds <= lds_per_cu and j * fused_vgprs + screen_vgprs <=
    vgprs_per_simd (VGPRs in granules of 8).  If fewer than cus * (jmax + 1) workgroups can
    wait at once, some CU holds at most jmax of them (pigeonhole): a screen block always fits.
    fused / screen: (LDS bytes per workgroup, VGPRs per lane).  Returns (ok, jmax)."""
    rnd = lambda v: -(-int(v) // gran) * gran  # noqa: E731
    j_lds = (lds_per_cu - int(screen[0])) // max(1, int(fused[0]))
    j_vgpr = (vgprs_per_simd - rnd(screen[1])) // max(1, rnd(fused[1]))
    jmax = max(-1, min(j_lds, j_vgpr))
    return waiters < cus * (jmax + 1), jmax


def level_resources(call):
    """(waiting kernel, screen) resources, each (LDS bytes per workgroup, VGPRs per lane), of
    the kernels a level's synthesis launches per wave, as ia_synth_level decides them from
    the level's arguments (ia_level_resources): the fused kernel's form (k_xstrip, or k_xwave
    on image-form or row-form levels) and the rotated or split-f16 screen (one
    global choice under-counted k_xwave levels)."""
    out = (ctypes.c_int * 4)()
    _ia.check(_ia.lib().ia_level_resources(ctypes.byref(call.args), out), 'ia_level_resources')
    return (out[0], out[1]), (out[2], out[3])


def sharded_schedule(level_shapes, pipeline, ranks_on_gpu, fused, screen, cus=256):
    """The pipelining of a run's sharded levels (shapes H x W of their B' levels) that the
    forward-progress rule (residency_ok) allows: pipeline as asked if every sharded level's
    waiting workgroups together fit the rule, else one level at a time if one level's do;
    raises if not even one level fits (e.g. too many ranks sharing one GPU).  fused / screen:
    one (LDS, VGPRs) pair for every level, or one pair per level (level_resources); the
    pipelined check takes the worst of each over the levels."""
    ms = [wave_max_queries(H, W) for H, W in level_shapes]
    if not ms:
        return pipeline
    per = lambda x: list(x) if x and isinstance(x[0], (tuple, list)) else [x] * len(ms)  # noqa: E731
    fl, sl = per(fused), per(screen)
    worst = lambda xs: (max(x[0] for x in xs), max(x[1] for x in xs))  # noqa: E731
    if pipeline and residency_ok(ranks_on_gpu * sum(ms), worst(fl), worst(sl), cus)[0]:
        return True
    for m, f, sc in zip(ms, fl, sl):
        ok, jmax = residency_ok(ranks_on_gpu * m, f, sc, cus)
        if not ok:
            raise RuntimeError('sharded synthesis refused: %d waiting workgroups per GPU (%d ranks x %d '
                               'queries) with at most %d per CU beside a screen block cannot guarantee '
                               'forward progress (DESIGN.md §7)' % (ranks_on_gpu * m, ranks_on_gpu,
                                                                     m, jmax))
    return False


def pipeline_default():
    """Levels run pipelined by default (IA_PIPELINE=0: one level at a time)."""
    return os.environ.get('IA_PIPELINE', '1') != '0'


def _src_level3(A_sm, A_lg, Ap_sm, Ap_lg):
    """IaSrcLevel over 3-channel device tensors (A_*: (h, w, 3); Ap_*: (nAp, h, w, 3))."""
    src = _ia.IaSrcLevel()
    src.A_sm, src.A_lg, src.Ap_sm, src.Ap_lg = (_ia.ptr(A_sm).value, _ia.ptr(A_lg).value,
                                                _ia.ptr(Ap_sm).value, _ia.ptr(Ap_lg).value)
    src.A_hs, src.A_ws = A_sm.shape[:2]
    src.Ah, src.Aw = A_lg.shape[:2]
    src.nAp = Ap_lg.shape[0]
    return src


def synthesize3_dev(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, max_levels, k, weights, levels=None,
                    debug=False, pipeline=None):
    """3-channel synthesis (num_ch = 3: convert=False on colour images, 165-dim rows): per
    level the materialised fp64 database (ia_db3_build), and by default (IA_DB_ROT) its
    rotated split-f16 form (R16c, DESIGN.md §4e: ia_db3_build_rot under ONE rotation for all
    levels, the finest level's principal directions, IA_ROT3_SHARED); per wave the rotated
    screen k_screen3r and the fused k_exact3<true> (exact fp64 rescore of the candidate
    tiles in the oracle's order, the coherence / kappa tail, the 3-channel B' update and the
    next wave's rotated query rows).  IA_DB_ROT=0: the split-f16 screen k_screen3 and the
    unfused exact stage (§4c).  pipeline (default pipeline_default()): the levels run
    concurrently (ia_synth_levels3), else one after the other (ia_synth_level3); the same
    results.  Same return value as synthesize_dev."""
    lib = _ia.lib()
    st = _ia.stream()
    weights = weights if torch.is_tensor(weights) else _ia.to_dev(weights)
    if pipeline is None:
        pipeline = pipeline_default()
    out, args, keep, done = {}, [], [], []
    todo = [l for l in range(1, max_levels) if levels is None or l in levels]
    built = {}
    for level in todo:
        A_sm, A_lg = A_pyr[level - 1].contiguous(), A_pyr[level].contiguous()
        Ap_sm = torch.stack([p[level - 1] for p in Ap_pyr_list]).contiguous()
        Ap_lg = torch.stack([p[level] for p in Ap_pyr_list]).contiguous()
        src = _src_level3(A_sm, A_lg, Ap_sm, Ap_lg)
        N = src.nAp * src.Ah * src.Aw
        db3 = torch.empty(lib.ia_db3_bytes(N) // 8, dtype=torch.float64, device=A_lg.device)
        _ia.check(lib.ia_db3_build(ctypes.byref(src), 0, N, _ia.ptr(db3), st), 'ia_db3_build')
        built[level] = (A_sm, A_lg, Ap_sm, Ap_lg, src, N, db3)
    # the rotated split screen (R16c), bit-identical results: one rotation for every level,
    # the principal directions of the finest level's rows (IA_ROT3_SHARED, default 1: one
    # device sync and one 165 x 165 eigh per call instead of one per level; the coarser
    # levels' rows have nearly the same principal directions, and any orthonormal basis keeps
    # the matcher exact); 0: each level its own
    shared = None
    if _ia.db_rot_enabled() and todo and os.environ.get('IA_ROT3_SHARED', '1') != '0':
        _, _, _, _, _, Nf, db3f = built[todo[-1]]
        shared = algorithms.rot3_rotation(db3f, Nf)
    for level in todo:
        A_sm, A_lg, Ap_sm, Ap_lg, src, N, db3 = built[level]
        dev = A_lg.device
        rot = dbr = None
        if shared is not None:
            rot, dbr = shared, algorithms.rot3_apply(db3, N, shared)
        elif _ia.db_rot_enabled():
            rot, dbr = algorithms.rot3_build(db3, N)
        B_sm, B_lg = B_pyr[level - 1].contiguous(), B_pyr[level].contiguous()
        Bp_sm, Bp_lg = Bp_pyr[level - 1], Bp_pyr[level]
        assert Bp_lg.is_contiguous() and Bp_sm.is_contiguous()
        H, W = B_lg.shape[:2]
        s = torch.empty((H * W, 2), dtype=torch.int32, device=dev)
        im = torch.empty(H * W, dtype=torch.int32, device=dev)
        dbg = None
        if debug:
            dbg = (torch.zeros((H * W, 7), dtype=torch.int32, device=dev),
                   torch.zeros((H * W, 2), dtype=torch.float64, device=dev))
        ws = _ia.workspace(lib.ia_synth3_workspace_bytes(H, W, N))
        a = _ia.IaSynthArgs()
        a.src = src
        a.db, a.row0, a.nrows, a.N_total = _ia.ptr(db3).value, 0, N, N
        a.B_sm, a.B_lg = _ia.ptr(B_sm).value, _ia.ptr(B_lg).value
        a.B_hs, a.B_ws = B_sm.shape[:2]
        a.H, a.W = H, W
        a.Bp_sm, a.Bp_lg = _ia.ptr(Bp_sm).value, _ia.ptr(Bp_lg).value
        a.weights = _ia.ptr(weights).value
        a.kappa_factor = kappa_factor(level, max_levels, k)
        a.s, a.im, a.workspace = _ia.ptr(s).value, _ia.ptr(im).value, _ia.ptr(ws).value
        if rot is not None:
            a.dbr, a.rot = _ia.ptr(dbr).value, _ia.ptr(rot).value
        if dbg is not None:
            a.dbg_px, a.dbg_dist = _ia.ptr(dbg[0]).value, _ia.ptr(dbg[1]).value
        done.append((a, (A_sm, A_lg, Ap_sm, Ap_lg, B_sm, B_lg, db3, ws, rot, dbr)))
        if not pipeline:
            _ia.check(lib.ia_synth_level3(ctypes.byref(a), st), 'ia_synth_level3')
        else:
            args.append(a)
            keep.append((A_sm, A_lg, Ap_sm, Ap_lg, B_sm, B_lg, db3, ws, rot, dbr))
        out[level] = (s, im) if dbg is None else (s, im, dbg)
    if args:
        # consecutive runs of levels go through one pipelined call each
        lv = sorted(out)
        i = 0
        while i < len(args):
            j = i + 1
            while j < len(args) and lv[j] == lv[j - 1] + 1:
                j += 1
            arr = (_ia.IaSynthArgs * (j - i))(*args[i:j])
            _ia.check(lib.ia_synth_levels3(arr, j - i, st), 'ia_synth_levels3')
            i = j
        # the level streams are joined into st: buffers freed after this return are reused
        # only by work queued on st behind that join (the caching allocator's stream order)
        del keep
    if done:
        # a decision wait of the fused colour tail that timed out leaves wrong pixels: raise
        arr = (_ia.IaSynthArgs * len(done))(*[x[0] for x in done])
        _ia.check(lib.ia_synth3_status(arr, len(done), st), 'ia_synth3_status')
    return out


def synthesize_dev(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, max_levels, k, weights,
                   comm=None, rank=0, nranks=1, prof=False, levels=None, lsh=None, eager=False,
                   pipeline=None, debug=False, check=True):
    """Synthesise levels 1..max_levels-1 (image_analogies.py:119-220) from device
    pyramids.  Bp_pyr (list of device tensors) is updated in place.  lsh: None (exact
    matcher) or LevelIndex.build_lsh arguments (approximate matcher).  comm: one
    communicator, or a list (one per sharded level, needed when sharded levels run
    pipelined).  pipeline: run the levels concurrently (ia_synth_levels; default
    pipeline_default()), else one after the other.  check: synchronise at the end and raise
    if a wait inside the device schedule timed out (ia_synth_status: the results would be
    wrong) -- a blocking call (one stream sync and one small copy per level, every level's
    workspace kept alive until then); check=False returns as soon as the work is queued,
    and the caller checks later (_ia.sched_status(), as bench.py does once per timed pass);
    a later pipelined call of the same thread then waits for it to end before it enqueues
    (IA_PIPE_DRAIN).  Returns {level: (s, im[, debug])} device tensors."""
    if B_pyr[-1].dim() == 3:     # 3-channel matching (num_ch = 3)
        if comm is not None or nranks > 1 or lsh is not None:
            raise NotImplementedError('3-channel matching runs on one GPU with the exact matcher')
        return synthesize3_dev(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, max_levels, k, weights,
                               levels=levels, debug=debug,
                               pipeline=False if eager else pipeline)
    w = weights if torch.is_tensor(weights) else _ia.to_dev(weights)
    if pipeline is None:
        pipeline = pipeline_default() and not eager
    todo = [l for l in range(1, max_levels) if levels is None or l in levels]
    comms = list(comm) if isinstance(comm, (list, tuple)) else None
    sharded = [l for l in todo            # (the LSH matcher runs unsharded, replicated)
               if comm is not None and lsh is None and
               shard_level(level_rows(Ap_pyr_list, l), nranks)]
    if pipeline and len(sharded) > 1 and (comms is None or len(comms) < len(sharded)):
        # one exchange cannot serve two levels running at once (their records would share
        # the exchange's box cells): levels one at a time then
        pipeline = False
    # (a 1-rank exchange never waits on another rank: each workgroup publishes its record
    # before it collects its own, so the forward-progress rule only binds for nranks > 1)
    peer_rule = (sharded and comm is not None and nranks > 1 and _ia.exchange_kind() == 'peer'
                 and torch.cuda.is_available())
    out = {}
    t_start = time.time()
    calls = []
    done = []

    def make_call(level):
        lcomm, row_range = None, None
        if level in sharded:
            # one exchange per sharded level; fewer only with the levels one at a time
            lcomm = comms[min(sharded.index(level), len(comms) - 1)] if comms else comm
            row_range = lambda level, N: shard_rows(N, rank, nranks)  # noqa: E731
        index = algorithms.level_index(A_pyr, Ap_pyr_list, level, row_range, lsh)
        return _LevelCall(level, max_levels, index, B_pyr[level - 1], B_pyr[level],
                          Bp_pyr[level - 1], Bp_pyr[level], w, k, lcomm, prof, eager, debug)
    early = {}
    if peer_rule:
        # fused workgroups that wait for other ranks must leave room for the screens: the
        # rule takes each sharded level's own kernels (its DB form and rotation decide them)
        for level in sharded:
            early[level] = make_call(level)
        res = [level_resources(early[l]) for l in sharded]
        share = nranks if os.environ.get('IA_SHARE_GPU', '0') == '1' else 1
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        pipeline = sharded_schedule([tuple(B_pyr[l].shape[:2]) for l in sharded], pipeline, share,
                                    [r[0] for r in res], [r[1] for r in res], cus)
        if os.environ.get('IA_VERBOSE'):
            print('[ia] sharded levels %s: kernels %s, pipelined %s' % (sharded, res, pipeline),
                  file=sys.stderr, flush=True)
    for level in todo:
        call = early.pop(level, None) or make_call(level)
        if pipeline:
            calls.append((level, call))
            continue
        _ia.check(_ia.lib().ia_synth_level(ctypes.byref(call.args), _ia.stream()),
                  'ia_synth_level')
        out[level] = call.result()
        done.append(call)
        del call
        if os.environ.get('IA_VERBOSE'):
            torch.cuda.synchronize()
            print('[ia] level %d/%d done %.3f s' % (level, max_levels - 1, time.time() - t_start),
                  file=sys.stderr, flush=True)
    # runs of consecutive levels go to ia_synth_levels together
    i = 0
    while i < len(calls):
        j = i + 1
        while j < len(calls) and calls[j][0] == calls[j - 1][0] + 1:
            j += 1
        res = synthesize_levels_dev([c for _, c in calls[i:j]])
        for (level, _), r in zip(calls[i:j], res):
            out[level] = r
        i = j
    done += [c for _, c in calls]
    if check and done:
        # waits inside the device schedule (a neighbour's decision, another rank's records)
        # that timed out leave wrong pixels: raise instead of returning them
        arr = (_ia.IaSynthArgs * len(done))(*[c.args for c in done])
        _ia.check(_ia.lib().ia_synth_status(arr, len(done), _ia.stream()), 'ia_synth_status')
    return out


def synthesize_batch_dev(jobs, max_levels, k, weights, prof=False, debug=False, check=True):
    """K independent analogies of identical shapes in ONE set of launches per wave (the
    multi_script batch, multi_script.py:13-32: each run an image_analogies_main of its own;
    SURVEY §8(e) config 5).  jobs: list of (A_pyr, Ap_pyr_list, B_pyr, Bp_pyr) device
    pyramids (Bp_pyr updated in place); k: one kappa or one per job.  Every level of every
    job is synthesised exactly as synthesize_dev would (exact matcher, one GPU); each wave's
    screen and fused kernel serve all K jobs at once (ia_synth_levels_batch), so the batch
    costs about one job's per-wave launch latency.  Returns one {level: (s, im[, debug])}
    dict per job."""
    K = len(jobs)
    if K == 0:
        return []
    ks = list(k) if isinstance(k, (list, tuple)) else [k] * K
    w = weights if torch.is_tensor(weights) else _ia.to_dev(weights)
    if any(j[2][-1].dim() == 3 for j in jobs):
        raise NotImplementedError('batches run 1-channel (luminance) matching')
    levels = list(range(1, max_levels))
    calls = []          # level-major: calls[j * K + job]
    # K databases per launch: fewer, longer chunks per database (the screen's workgroups
    # amortise their prologue; c5: +11% on one box), restored before returning
    lib = _ia.lib()
    target = int(os.environ.get('IA_BATCH_CHUNKS', 0)) or max(64, 512 // K)
    prev = lib.ia_set_chunk_target(target)
    try:
        for level in levels:
            for (A_pyr, Ap_list, B_pyr, Bp_pyr), kj in zip(jobs, ks):
                index = algorithms.level_index(A_pyr, Ap_list, level, None, None)
                calls.append(_LevelCall(level, max_levels, index, B_pyr[level - 1], B_pyr[level],
                                        Bp_pyr[level - 1], Bp_pyr[level], w, kj, None, prof, False,
                                        debug))
        arr = (_ia.IaSynthArgs * len(calls))(*[c.args for c in calls])
        _ia.check(lib.ia_synth_levels_batch(arr, len(levels), K, _ia.stream()),
                  'ia_synth_levels_batch')
        if check:   # (the workspaces' layout follows the chunk target: checked under it)
            _ia.check(lib.ia_synth_status(arr, len(calls), _ia.stream()), 'ia_synth_status')
    finally:
        lib.ia_set_chunk_target(prev)
    return [{level: calls[j * K + q].result() for j, level in enumerate(levels)}
            for q in range(K)]


# ---- multi-GPU: one process per GPU ------------------------------------------

def dist_world():
    """(rank, world size) of the initialised torch.distributed group, else (0, 1)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def rank_jobs(n_jobs, rank, world):
    """Indices of the independent analogies one rank runs when n_jobs of them (the
    multi_script loop, multi_script.py:13-32, which runs them one after the other in one
    process) are spread over `world` ranks: j = rank (mod world).  No collective: each rank's
    results are its own (weak scaling)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('rank %d of world %d' % (rank, world))
    return list(range(rank, n_jobs, world))


def sharded_level_count(Ap_pyr_list, max_levels, world):
    """Levels 1..max_levels-1 whose database is sharded over `world` ranks (shard_level)."""
    return sum(shard_level(level_rows(Ap_pyr_list, l), world) for l in range(1, max_levels))


def level_exchanges(Ap_pyr_list, max_levels, rank, world, kind=None):
    """The `comm` of a DB-sharded synthesis (synthesize_dev): one exchange per sharded level
    (pipelined sharded levels each need their own), over the initialised torch.distributed
    group.  Every rank calls it at the same point with pyramids of the same shapes.
    kind: None (IA_EXCHANGE: the device-side exchange, RCCL as the agreed fallback) or
    'rccl'.  Release with release_exchanges."""
    n = sharded_level_count(Ap_pyr_list, max_levels, world)
    return [_ia.exchange(rank, world, kind) for _ in range(max(n, 1))]


def release_exchanges(comms):
    """Check (a device-side wait that timed out raises) and destroy level_exchanges' objects."""
    try:
        for cm in comms or []:
            _ia.exchange_status(cm)
    finally:
        for cm in comms or []:
            _ia.lib().ia_comm_destroy(cm)


def synthesize_jobs(jobs, max_levels, k, weights, rank=0, world=1, batch=0, prof=False,
                    debug=False, check=True):
    """Independent analogies of identical shapes spread over ranks (SURVEY §8(e) config 5,
    multi_script.py:13-32): this rank synthesises jobs[j] for j in rank_jobs(len(jobs),
    rank, world), `batch` of them per set of launches (synthesize_batch_dev; 0 = all of this
    rank's jobs in one batch, 1 = one synthesize_dev call per job), one GPU per rank, no
    collective.  jobs: the WHOLE job list, (A_pyr, Ap_pyr_list, B_pyr, Bp_pyr) device
    pyramids per job (Bp_pyr updated in place); entries of other ranks' jobs are never read
    and may be None (or a callable returning the tuple, called only for this rank's jobs).
    k: one kappa or one per job (whole list).  Returns {j: {level: (s, im[, debug])}} for this
    rank's jobs."""
    mine = rank_jobs(len(jobs), rank, world)
    ks = list(k) if isinstance(k, (list, tuple)) else [k] * len(jobs)
    if len(ks) != len(jobs):
        raise ValueError('synthesize_jobs: %d kappas for %d jobs' % (len(ks), len(jobs)))
    step = batch if batch and batch > 0 else max(1, len(mine))
    out = {}
    for g0 in range(0, len(mine), step):
        group = mine[g0:g0 + step]
        ins = [jobs[j]() if callable(jobs[j]) else jobs[j] for j in group]
        if len(group) == 1:
            A_pyr, Ap_list, B_pyr, Bp_pyr = ins[0]
            res = [synthesize_dev(A_pyr, Ap_list, B_pyr, Bp_pyr, max_levels, ks[group[0]], weights,
                                  prof=prof, debug=debug, check=check)]
        else:
            res = synthesize_batch_dev(ins, max_levels, [ks[j] for j in group], weights, prof=prof,
                                       debug=debug, check=check)
        out.update(zip(group, res))
    return out


# ---- setup (image_analogies.py:17-94) ------------------------------------------------------

def _read(fname):
    """Decode an image file (host; file I/O is outside the device path).  An alpha
    channel (RGBA PNG) is dropped — the reference's 3x3 YIQ einsum would reject it."""
    import matplotlib.pyplot as plt
    img = plt.imread(fname)
    return img[..., :3] if img.ndim == 3 and img.shape[2] == 4 else img


def setup_dev(A_orig, Ap_orig_list, B_orig, c):
    """Numeric part of img_setup on device, from already-decoded images.
    Returns device (A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list) and sets c.*."""
    assert len(A_orig.shape) == len(B_orig.shape)
    if not c.convert and np.ndim(A_orig) == 3:
        if c.remap_lum:
            raise ValueError('remap_lum requires convert (config.py:11-12)')
        if getattr(c, 'matcher', 'brute') != 'brute':
            raise NotImplementedError('3-channel matching runs with the exact matcher only')
    dev = _ia.require_device()
    for Ap in Ap_orig_list:
        assert A_orig.shape == Ap.shape
    # scale to [0, 1]; the A' scale comes from the first row of the LAST A'
    # (image_analogies.py:32-37 reads Ap_orig[0] after the loading loop)
    scales = [255. if np.max(x) > 1.0 else 1.0
              for x in (A_orig, B_orig, Ap_orig_list[-1][0])]
    up = lambda x: torch.as_tensor(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    color_B = None
    if c.convert:
        _, A = ip.rgb_to_yiq_dev(up(A_orig), scales[0], want_yiq=False)
        B_yiq, B = ip.rgb_to_yiq_dev(up(B_orig), scales[1], want_yiq=True)
        Ap_list = [ip.rgb_to_yiq_dev(up(x), scales[2], want_yiq=False)[1] for x in Ap_orig_list]
        color_B = B_yiq
    else:
        A = ip.scale_dev(up(A_orig), scales[0])
        B = ip.scale_dev(up(B_orig), scales[1])
        Ap_list = [ip.scale_dev(up(x), scales[2]) for x in Ap_orig_list]
    if c.remap_lum:
        A, Ap_list = ip.remap_luminance_dev(A, Ap_list, B)
    levels = getattr(c, 'levels', None)
    B_orig_pyr = None if c.init_rand else ip.gaussian_pyramid_dev(B, c.n_sm, levels)
    A, B = ip.compress_values_dev(A, B, c.AB_weight)
    c.num_ch, c.padding_sm, c.padding_lg, c.weights = setup_vars(A)
    A_pyr = ip.gaussian_pyramid_dev(A, c.n_sm, levels)
    B_pyr = ip.gaussian_pyramid_dev(B, c.n_sm, levels)
    Ap_pyr_list = [ip.gaussian_pyramid_dev(Ap, c.n_sm, levels) for Ap in Ap_list]
    if c.convert:
        color_pyr_list = [ip.gaussian_pyramid_dev(color_B, c.n_sm, levels)]
    else:
        color_pyr_list = Ap_pyr_list
    if len(A_pyr) != len(B_pyr):
        c.max_levels = min(len(A_pyr), len(B_pyr))
        warnings.warn('Warning: input images are very different sizes! The minimum number of '
                      'levels will be used.')
    else:
        c.max_levels = len(B_pyr)
    init = ip.initialize_Bp([p.cpu() for p in (B_pyr if c.init_rand else B_orig_pyr)],
                            c.init_rand, getattr(c, 'seed', None))
    Bp_pyr = [torch.as_tensor(np.ascontiguousarray(x)).to(dev) for x in init]
    return A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list


def img_setup(A_fname, Ap_fname_list, B_fname, out_path, c):
    """Read, convert, remap, compress and build pyramids (image_analogies.py:17-94).
    Returns numpy pyramids like the reference."""
    if not os.path.exists(out_path):
        os.makedirs(out_path)
    A_orig, B_orig = _read(A_fname), _read(B_fname)
    Ap_orig_list = [_read(f) for f in Ap_fname_list]
    dev_out = setup_dev(A_orig, Ap_orig_list, B_orig, c)
    to_np = lambda pyr: [p.cpu().numpy() for p in pyr]  # noqa: E731
    A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list = dev_out
    return (to_np(A_pyr), [to_np(p) for p in Ap_pyr_list], to_np(B_pyr), to_np(Bp_pyr),
            [to_np(p) for p in color_pyr_list], c)


def color_output(level, Bp_lvl, s, im, color_pyr_list, c):
    """Colour image of a level (image_analogies.py:216-217, 255-258), on device
    (ia_color_output): with convert, Y from B' and I/Q from B's pyramid (the reference takes
    color_pyr_list[i] with the LAST pixel's i; there is one colour pyramid then), clipped;
    otherwise the A' colour of each pixel's source.  Returns (H, W, 3) numpy."""
    H, W = Bp_lvl.shape[:2]
    out = torch.empty((H, W, 3), dtype=torch.float64, device=Bp_lvl.device)
    if c.convert:
        yiq = color_pyr_list[0][level].contiguous()
        _ia.check(_ia.lib().ia_color_output(_ia.ptr(Bp_lvl.contiguous()), _ia.ptr(yiq), None, None, None,
                                            0, 0, 0, H * W, _ia.ptr(out), _ia.stream()), 'ia_color_output')
        return out.cpu().numpy()
    base = color_pyr_list[0][level]                                   # (h, w[, 3])
    ah, aw = base.shape[:2]
    C = 3 if base.dim() == 3 else 1
    src = (base if len(color_pyr_list) == 1 else
           torch.stack([p[level] for p in color_pyr_list])).contiguous()  # (nAp, h, w[, 3])
    _ia.check(_ia.lib().ia_color_output(None, None, _ia.ptr(s.contiguous()), _ia.ptr(im.contiguous()), _ia.ptr(src),
                                        int(ah), int(aw), C, H * W, _ia.ptr(out), _ia.stream()), 'ia_color_output')
    return out.cpu().numpy()


def debug_record(s, im, dbg, shape):
    """The reference's per-level debug structures (image_analogies.py:141-159, 222-247)
    from a level's device debug record: the lists sa, sc, rstars, s, im (its pickle) and
    the maps p_src (colour code), app_dist, coh_dist, img_src."""
    H, W = shape
    s = s.cpu().numpy()
    im = im.cpu().numpy()
    px = dbg[0].cpu().numpy()
    dd = dbg[1].cpu().numpy()
    sa = [(int(r), int(c)) for r, c in px[:, 0:2]]
    sc = [(int(r), int(c)) for r, c in px[:, 2:4]]
    rstars = [(int(r), int(c)) for r, c in px[:, 4:6]]
    has = px[:, 6].astype(bool)
    app_color, coh_color, err_color = np.array([1, 0, 0]), np.array([1, 1, 0]), np.array([0, 0, 0])
    p_src = np.empty((H * W, 3))
    is_coh = np.all(s == px[:, 2:4], axis=1)            # np.allclose(p, p_coh)
    is_app = np.all(s == px[:, 0:2], axis=1)
    p_src[has & is_coh] = coh_color
    p_src[has & ~is_coh & is_app] = app_color
    p_src[~has] = err_color
    if np.any(has & ~is_coh & ~is_app):
        raise RuntimeError('debug record: a pixel took neither p_app nor p_coh')
    with np.errstate(invalid='ignore', divide='ignore'):
        img_src = (im.astype(np.float64) / np.max(im)).reshape(H, W)
    return {'sa': sa, 'sc': sc, 'rstars': rstars,
            's': [(int(r), int(c)) for r, c in s], 'im': [int(i) for i in im],
            'p_src': p_src.reshape(H, W, 3), 'app_dist': dd[:, 0].reshape(H, W),
            'coh_dist': dd[:, 1].reshape(H, W), 'img_src': img_src}


def save_debug(out_path, level, rec, Bp_level):
    """image_analogies.py:242-253: the per-level maps as borderless .eps images and the
    [sa, sc, rstars, s, im] lists (pickle, as the reference; also .npz arrays)."""
    import pickle
    import matplotlib.pyplot as plt
    paths = ['%d_psrc.eps' % level, '%d_appdist.eps' % level, '%d_cohdist.eps' % level,
             '%d_output.eps' % level, '%d_imgsrc.eps' % level]
    maps = [rec['p_src'], rec['app_dist'], rec['coh_dist'], Bp_level, rec['img_src']]
    for path, var in zip(paths, maps):
        fig = plt.imshow(var, interpolation='nearest', cmap='gray')
        ip.savefig_noborder(out_path + path, fig)
        plt.close()
    with open(out_path + '%d_srcs.pickle' % level, 'wb') as f:
        pickle.dump([rec['sa'], rec['sc'], rec['rstars'], rec['s'], rec['im']], f)
    np.savez(out_path + '%d_srcs.npz' % level, sa=np.array(rec['sa'], np.int32),
             sc=np.array(rec['sc'], np.int32), rstars=np.array(rec['rstars'], np.int32),
             s=np.array(rec['s'], np.int32), im=np.array(rec['im'], np.int32),
             app_dist=rec['app_dist'], coh_dist=rec['coh_dist'])


def image_analogies_main(A_fname, Ap_fname_list, B_fname, out_path, c, debug=False,
                         outputs=None, comm=None, rank=None, nranks=None):
    """Full run (image_analogies.py:97-268): setup, per-level synthesis on device, colour
    output images.  debug=True also writes the reference's debug structures per level
    (save_debug).  outputs (dict, optional) receives per level {'color': the RGB image
    before plt.imsave, 's', 'im', and with debug 'debug': debug_record(...)}.  Returns the
    B' pyramid (numpy).

    Multi-GPU (one process per GPU): comm='auto' shards the databases of the
    large levels over the initialised torch.distributed group (every rank calls this with
    the same files and config; rank / nranks default to the group's): one exchange per
    sharded level (level_exchanges), released before returning.  comm may also be
    exchanges the caller made (then pass rank and nranks).  Every rank ends with the same
    B' (the exchange is deterministic); only rank 0 writes the output files and prints.
    To spread independent runs over GPUs instead (the multi_script loop) use multi_main."""
    import matplotlib.pyplot as plt
    r0, w0 = dist_world()
    rank = r0 if rank is None else rank
    nranks = (w0 if comm is not None else 1) if nranks is None else nranks
    lead = rank == 0
    say = print if lead else (lambda *a, **kw: None)
    begin_time = start_time = time.time()
    if lead and not os.path.exists(out_path):
        os.makedirs(out_path)
    A_orig, B_orig = _read(A_fname), _read(B_fname)
    Ap_orig_list = [_read(f) for f in Ap_fname_list]
    A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list = setup_dev(A_orig, Ap_orig_list,
                                                                  B_orig, c)
    names = ['A_fname', 'Ap_fname_list', 'B_fname', 'c.convert', 'c.remap_lum', 'c.init_rand',
             'c.AB_weight', 'c.k']
    vals = [A_fname, Ap_fname_list, B_fname, c.convert, c.remap_lum, c.init_rand, c.AB_weight,
            c.k]
    if lead:
        save_metadata(out_path, names, vals)
    torch.cuda.synchronize()
    say('Environment Setup: %f' % (time.time() - start_time))
    weights = _ia.to_dev(c.weights)
    own = None
    if isinstance(comm, str):
        if comm != 'auto':
            raise ValueError("comm must be None, 'auto' or exchange objects")
        own = comm = level_exchanges(Ap_pyr_list, c.max_levels, rank, nranks) if nranks > 1 else None
    # all levels on device, pipelined (ia_synth_levels); then each level's outputs
    start_time = time.time()
    say('Computing levels 1 to %d' % (c.max_levels - 1))
    try:
        res = synthesize_dev(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, c.max_levels, c.k, weights,
                             comm=comm, rank=rank, nranks=nranks if comm is not None else 1,
                             lsh=algorithms.lsh_params(c), debug=debug)
        torch.cuda.synchronize()
    finally:
        if own:
            release_exchanges(own)
    say('Synthesis time: %f' % (time.time() - start_time))
    if not lead:
        return [p.cpu().numpy() for p in Bp_pyr]
    for level in range(1, c.max_levels):
        s, im = res[level][0], res[level][1]
        color_im_out = color_output(level, Bp_pyr[level], s, im, color_pyr_list, c)
        rec = None
        if debug:
            rec = debug_record(s, im, res[level][2], Bp_pyr[level].shape[:2])
            save_debug(out_path, level, rec, Bp_pyr[level].cpu().numpy())
        if outputs is not None:
            outputs[level] = {'color': color_im_out, 's': s.cpu().numpy(), 'im': im.cpu().numpy()}
            if rec is not None:
                outputs[level]['debug'] = rec
        plt.imsave(out_path + 'level_%d_color.jpg' % level, color_im_out)
        plt.imsave(out_path + out_path.split('/')[-2] + '.jpg', color_im_out)
    print('Total time: %f' % (time.time() - begin_time))
    return [p.cpu().numpy() for p in Bp_pyr]


def multi_main(runs, c, debug=False, rank=None, world=None):
    """The reference's batch scripts (multi_script.py:13-32, multi_script_2.py:31-40: a
    serial loop of image_analogies_main calls, each with its own files and kappa) spread over
    GPUs, one process per GPU: this rank runs runs[j] for j in rank_jobs(len(runs), rank,
    world) (rank / world default to the initialised torch.distributed group's; (0, 1)
    without one), each on its own GPU alone.  runs: (A_fname, Ap_fname_list, B_fname,
    out_path[, overrides]) tuples; overrides is a dict of config fields set on `c` before
    the run (multi_script.py:31 sets c.k so).  Returns {j: B' pyramid} of this rank's runs."""
    r0, w0 = dist_world()
    rank = r0 if rank is None else rank
    world = w0 if world is None else world
    out = {}
    for j in rank_jobs(len(runs), rank, world):
        A_fname, Ap_fname_list, B_fname, out_path = runs[j][:4]
        for key, val in (runs[j][4] if len(runs[j]) > 4 else {}).items():
            setattr(c, key, val)
        out[j] = image_analogies_main(A_fname, Ap_fname_list, B_fname, out_path, c, debug=debug,
                                      rank=0, nranks=1)
    return out
