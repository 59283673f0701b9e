"""Benchmark: B' synthesis throughput (B' pixels/s) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4]

One STEP = the whole hot path over one synthetic analogy, from the luminance images
resident in HBM to B' and the (s, im) index maps in HBM: Gaussian pyramids of A, A', B
(5-level cap), per level the fp32 screening database, then the wavefront synthesis of
every level (query build, MFMA screen, exact fp64 rescore, coherence + kappa, update).
B' restarts from the same random initialisation each step.

Workloads (BASELINE.json configs):
    c1  180x117 A/A'/B, kappa 0.5           c2  same, kappa 5
    c3  362x638, kappa 25, 5-level cap      c4  A = A' 2048x2048, B 1024x1024, 5-level cap
    c5  independent 512x512 jobs (multi_script batch), --jobs per GPU
Default: c4 — the configuration the metric and its 1/2/4/8-GPU scaling are quoted on.
With N > 1 (one process per GPU) c4 shards the databases of its large levels over the
ranks with one RCCL all-gather per wave (strong scaling); c5 spreads jobs (weak scaling,
no collective).  `--gpus N` launched without torch.distributed.run's environment starts
the N rank processes itself (torch.distributed.run as a child, before any GPU call in
this process); every rank checks that the world size equals --gpus.  rank 0 prints ONE
JSON line.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'image-analogies-python_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _ia  # noqa: E402
import config as cfg  # noqa: E402
import image_analogies as ia  # noqa: E402
import img_preprocess as ip  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
# f16 MFMA dense peak: 32x32x16 = 32768 flop / 32 cycles / SIMD -> 4096 flop/clk/CU x 256 CU
# x 2.4 GHz (MI355X_MICROARCH.md: ~2.5 PF dense)
F16_MFMA_PEAK_TFLOPS = 4096 * 256 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
# HBM traffic of one launch of the dominant screen instance (k_screen16<11>, the c4 finest
# level's plateau waves: 321-342 queries x 4,194,304 rows), from rocprofv3 PMC passes of
# bench.py itself (tools/gpu.sh traffic: FETCH_SIZE x 2 on gfx950 + WRITE_SIZE,
# MI355X_MICROARCH.md §HBM; counters cannot be read from inside the measured process).
# The file records a hash of the screen's sources; a file from other sources is stale and
# the bench then reports traffic null.
SCREEN_PMC_FILE = os.path.join(ROOT, 'profiles', 'r06_screen_traffic_bench_pmc.json')
SCREEN_SRCS = ('ia_screen16.hip', 'ia_split16.h', 'ia_imgwin.h', 'ia_internal.h', 'ia_screen16r.hip',
               'ia_rot16.h')


def screen_src_sha1():
    import hashlib
    h = hashlib.sha1()
    for f in SCREEN_SRCS:
        h.update(open(os.path.join(ROOT, 'image-analogies-python_amd', 'csrc', f), 'rb').read())
    return h.hexdigest()


def screen_pmc():
    if not os.path.exists(SCREEN_PMC_FILE):
        return None
    d = json.load(open(SCREEN_PMC_FILE))
    if d.get('screen_src_sha1') != screen_src_sha1():
        return None
    return {'bytes': d['traffic_bytes'], 'kernel': d['kernel'], 'dispatches': d['dispatches'],
            'source': os.path.relpath(SCREEN_PMC_FILE, ROOT)}

SCREEN_SQ_FILE = os.path.join(ROOT, 'profiles', 'r06_screen_sq_pmc.json')


def screen_sq():
    """MFMA-busy fraction, held clock and wait share of the dominant screen instance
    (tools/pmc_sq.py over a PMC pass of bench.py), if the file matches the screen's sources."""
    if not os.path.exists(SCREEN_SQ_FILE):
        return None
    d = json.load(open(SCREEN_SQ_FILE))
    if d.get('screen_src_sha1') != screen_src_sha1():
        return None
    return {k: d[k] for k in ('mfma_busy', 'clock_ghz', 'wait_inst_share',
                              'lds_bank_conflict_share', 'mean_us')} | {
        'source': os.path.relpath(SCREEN_SQ_FILE, ROOT)}


CONFIGS = {
    'c1': dict(A=(180, 117), B=(180, 117), k=0.5, levels=None, name='shore-crop 180x117 filter analogy, brute force'),
    'c2': dict(A=(180, 117), B=(180, 117), k=5.0, levels=None, name='freud-crop 180x117 kappa=5'),
    'c3': dict(A=(362, 638), B=(362, 638), k=25.0, levels=5, name='texture transfer 362x638 kappa=25, 5-level'),
    'c4': dict(A=(2048, 2048), B=(1024, 1024), k=0.5, levels=5, name='A/A\' 2048x2048 x B 1024x1024, 5-level, DB sharded'),
    'c5': dict(A=(512, 512), B=(512, 512), k=0.5, levels=5, name='independent 512x512 analogies (multi_script batch)'),
}


def smooth_noise(seed, shape, sigma=2.0):
    from scipy.ndimage import gaussian_filter
    x = gaussian_filter(np.random.RandomState(seed).rand(*shape), sigma)
    return (x - x.min()) / (x.max() - x.min())


def make_inputs(conf, seed):
    """SURVEY §8(d) synthetic blur-filter analogy: A smooth noise, A' = blur(A), B noise."""
    from scipy.ndimage import gaussian_filter
    A = smooth_noise(seed, conf['A'])
    Ap = gaussian_filter(A, 1.5)
    B = smooth_noise(seed + 1, conf['B'])
    return A, Ap, B


def pass_check(comm):
    """After a pass: raise ExchangeTimeout if another rank's records never came over a
    device-side exchange, else ScheduleFault if a neighbour-decision wait timed out (a fault
    of the fused kernel).  The exchange is checked FIRST: a dead or slow peer also trips the
    neighbour waits (the same 10 s limit), and such a cascade is an exchange failure, the
    one error the RCCL fallback handles."""
    torch.cuda.synchronize()
    for cm in comm or []:
        _ia.exchange_status(cm)
    _ia.sched_status()


class Job:
    """One analogy with its inputs resident in HBM."""

    def __init__(self, conf, seed, dev, lsh=None):
        A, Ap, B = make_inputs(conf, seed)
        self.seed = seed
        self.lsh = lsh
        self.A, self.Ap, self.B = (torch.as_tensor(x).to(dev) for x in (A, Ap, B))
        self.k, self.levels = conf['k'], conf['levels']
        nB = ip.num_layers(B.shape[0], B.shape[1], cfg.n_sm, self.levels)
        nA = ip.num_layers(A.shape[0], A.shape[1], cfg.n_sm, self.levels)
        self.max_levels = min(nA, nB) + 1
        shapes = [B.shape]
        for _ in range(nB):
            shapes.append(((shapes[-1][0] + 1) // 2, (shapes[-1][1] + 1) // 2))
        shapes.reverse()
        init = ip.initialize_Bp([np.empty(s) for s in shapes], True, seed + 2)
        self.Bp_init = [torch.as_tensor(x).to(dev) for x in init]
        self.Bp = [x.clone() for x in self.Bp_init]
        self.weights = torch.as_tensor(cfg.compute_weights(3, 5, 12, 1)).to(dev)
        self.pixels = sum(s[0] * s[1] for s in shapes[1:self.max_levels])
        self.waves = sum(_ia.waves(*s) for s in shapes[1:self.max_levels])

    def step(self, comm=None, rank=0, nranks=1, prof=False, eager=False, check=True):
        A_pyr = ip.gaussian_pyramid_dev(self.A, cfg.n_sm, self.levels)
        Ap_pyr = ip.gaussian_pyramid_dev(self.Ap, cfg.n_sm, self.levels)
        B_pyr = ip.gaussian_pyramid_dev(self.B, cfg.n_sm, self.levels)
        self.Ap_pyr_last = Ap_pyr
        for dst, src in zip(self.Bp, self.Bp_init):
            dst.copy_(src)
        return ia.synthesize_dev(A_pyr, [Ap_pyr], B_pyr, self.Bp, self.max_levels, self.k,
                                 self.weights, comm=comm, rank=rank, nranks=nranks, prof=prof,
                                 lsh=self.lsh, eager=eager, check=check)

    def prepare(self):
        """Pyramids and the B' reset of one step (the batch path's per-job part)."""
        A_pyr = ip.gaussian_pyramid_dev(self.A, cfg.n_sm, self.levels)
        Ap_pyr = ip.gaussian_pyramid_dev(self.Ap, cfg.n_sm, self.levels)
        B_pyr = ip.gaussian_pyramid_dev(self.B, cfg.n_sm, self.levels)
        self.Ap_pyr_last = Ap_pyr
        for dst, src in zip(self.Bp, self.Bp_init):
            dst.copy_(src)
        return A_pyr, [Ap_pyr], B_pyr, self.Bp

    def lsh_quality(self):
        """LSH vs exact on the same queries: the finest level's B / B' features (B' as
        this job's last synthesis left it), matched by both matchers over one index."""
        import algorithms
        A_pyr = ip.gaussian_pyramid_dev(self.A, cfg.n_sm, self.levels)
        Ap_pyr = ip.gaussian_pyramid_dev(self.Ap, cfg.n_sm, self.levels)
        B_pyr = ip.gaussian_pyramid_dev(self.B, cfg.n_sm, self.levels)
        level = self.max_levels - 1
        index = algorithms.level_index(A_pyr, [Ap_pyr], level, lsh=self.lsh)
        Q = torch.cat([algorithms.level_features_dev(B_pyr[level - 1], B_pyr[level], True),
                       algorithms.level_features_dev(self.Bp[level - 1], self.Bp[level], False)],
                      1)
        li, ld = index.match(Q)
        ei, ed = index.match(Q, exact=True)
        return {'queries': int(Q.shape[0]), 'level': level,
                'exact_frac': float((ld == ed).double().mean().item()),
                'mean_dist_lsh': float(ld.mean().item()),
                'mean_dist_exact': float(ed.mean().item()),
                'mean_dist_ratio': float(ld.mean().item() / max(ed.mean().item(), 1e-300)),
                'params': dict(self.lsh)}

    def sharded_levels(self, nranks):
        """Levels whose database is sharded over nranks ranks (image_analogies.shard_level)."""
        def shapes(img):
            n = ip.num_layers(img.shape[0], img.shape[1], cfg.n_sm, self.levels)
            out = [tuple(img.shape)]
            for _ in range(n):
                out.append(((out[-1][0] + 1) // 2, (out[-1][1] + 1) // 2))
            return out[::-1]
        al = shapes(self.A)
        return sum(ia.shard_level(al[l][0] * al[l][1], nranks) for l in range(1, self.max_levels))

    def algorithmic_pairs(self):
        """sum over synthesized levels of q_l * N_l (the matcher's (query, row) pairs);
        pyramids are aligned from the coarse end as in image_analogies.py:82-86."""
        def shapes(img):
            n = ip.num_layers(img.shape[0], img.shape[1], cfg.n_sm, self.levels)
            out = [tuple(img.shape)]
            for _ in range(n):
                out.append(((out[-1][0] + 1) // 2, (out[-1][1] + 1) // 2))
            return out[::-1]
        bl, al = shapes(self.B), shapes(self.A)
        return sum(bl[l][0] * bl[l][1] * al[l][0] * al[l][1] for l in range(1, self.max_levels))


def wave_spacing(prof, level):
    """Mean / median per-wave spacing of one level from the events pass (us)."""
    recs = [p for p in prof if p['level'] == level and len(p.get('tail_ms', [])) > 1]
    if not recs:
        return None
    scr = np.concatenate([p['launch_ms'] for p in recs]) * 1e3
    tail = np.concatenate([p['tail_ms'] for p in recs]) * 1e3
    gap = np.concatenate([p['gap_ms'][:-1] for p in recs]) * 1e3
    return {'waves': int(len(scr)),
            'screen_mean': float(scr.mean()), 'screen_p50': float(np.median(scr)),
            'fused_tail_mean': float(tail.mean()), 'fused_tail_p50': float(np.median(tail)),
            'gap_to_next_screen_mean': float(gap.mean()), 'gap_to_next_screen_p50': float(np.median(gap)),
            'period_mean': float((scr.sum() + tail.sum() + gap.sum()) / len(scr))}


def cpu_threads():
    """Host threads of the all-cores CPU baseline: OMP_NUM_THREADS when set (the GPU box
    sets it to the box's CPU share), else every CPU of this process's affinity mask."""
    env = os.environ.get('OMP_NUM_THREADS')
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(job, seconds=10.0):
    """The C oracle (scanline synthesis with the exact brute-force matcher)
    timed on a bounded sample of the same workload: the first pixels of the FINEST level
    in scanline order against its full database, extrapolated to the whole job by (query,
    row) pair count.  Two legs in the same run: 1 thread, and all host threads (the 1-NN
    scan split over rows, same result).  ~`seconds` of CPU work per leg."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import ia_oracle_c as oc
    A_pyr = [p.cpu().numpy() for p in ip.gaussian_pyramid_dev(job.A, cfg.n_sm, job.levels)]
    Ap_pyr = [p.cpu().numpy() for p in ip.gaussian_pyramid_dev(job.Ap, cfg.n_sm, job.levels)]
    B_pyr = [p.cpu().numpy() for p in ip.gaussian_pyramid_dev(job.B, cfg.n_sm, job.levels)]
    Bp_pyr = [p.cpu().numpy() for p in job.Bp_init]
    level = job.max_levels - 1
    w = cfg.compute_weights(3, 5, 12, 1)
    N = A_pyr[level].size
    f = ia.kappa_factor(level, job.max_levels, job.k)
    H, W = B_pyr[level].shape
    probe = oc.LevelJob(level, A_pyr, [Ap_pyr], B_pyr, Bp_pyr, w, f, max_pixels=2)
    db = probe.build_db()

    def leg(threads):
        got = oc.set_threads(threads)
        probe.L.max_pixels = 2
        t0 = time.perf_counter()
        probe.run()
        per_px = max((time.perf_counter() - t0) / 2, 1e-6)
        npx = int(max(2, min(H * W, seconds / per_px)))
        job_s = oc.LevelJob(level, A_pyr, [Ap_pyr], B_pyr, Bp_pyr, w, f, max_pixels=npx)
        job_s.db = db
        t0 = time.perf_counter()
        try:
            job_s.run()
        finally:
            job_s.db = None       # owned by probe
        dt = time.perf_counter() - t0
        value = npx * N / dt * job.pixels / job.algorithmic_pairs()
        return {'value': value, 'unit': "B' pixels/s", 'cores': got, 'kind': 'port',
                'sample': '%d B\' pixels (scanline) of the finest level (%dx%d) against its '
                          'full %d-row database, %.1f s on %d thread(s) (host reports %d CPUs); '
                          'extrapolated to the whole job by (query,row) pairs'
                          % (npx, H, W, N, dt, got, os.cpu_count())}
    one = leg(1)
    allc = leg(cpu_threads())
    oc.set_threads(1)
    allc['single_core'] = one
    return allc


def hbm_kernels(dev, reps=20):
    """Achieved HBM rate of the bandwidth-bound kernels: each C-ABI entry
    timed with HIP events on the stream it launches on (10 back-to-back calls per
    measurement, per call), median of `reps`, against
    algorithmic bytes (every input element read once, every output written once):
      yiq        ia_rgb_to_yiq, 2048x2048 uint8 RGB -> YIQ + Y fp64: 3 + 32 B/px
      pyr_reduce ia_pyr_reduce_f64 (one-pass k_pyr_wave + k_pyr_clip_p),
                 2048^2 -> 1024^2 fp64: 8 B per input + 8 B per output pixel
      db_build   ia_db_build (k_db_range + k_db_bound + LDS-tiled k_db_build_t), the c4
                 finest level, 4,194,304 rows: 224 B written per row (split-f16 rows) + the
                 fp64 pyramids read once (A, A' fine: 8 B per row each; coarse: 8 B per 4
                 rows each)
      db_image   ia_db_build_image without a row form (what the product builds where the
                 image form applies: the range pass k_db_range_at + the one-pass build
                 k_img_build), same level: the fp64 pyramids read once (20 B per row) + the padded
                 u32 split pairs (A, A' fine: 4 B per row each; coarse: 4 B per 4 rows each)
                 and the norm slots (4 B per row) written once: 34 B per row
    """
    import algorithms
    st = torch.cuda.current_stream(dev)

    def timed(fn, batch=10):
        # `batch` back-to-back calls between the two events (as the product issues them: a
        # pyramid's levels, the levels' DB builds), per call: the host's launch latency is
        # not in the window (a lone call between two events measures ~5 us of it)
        fn()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(batch):
                fn()
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3 / batch)
        ts.sort()
        return ts[len(ts) // 2]

    out = {}

    def put(name, sec, nbytes, what):
        gbs = nbytes / sec / 1e9
        out[name] = {'us': sec * 1e6, 'bytes': nbytes, 'GB/s': gbs, 'frac': gbs / HBM_PEAK_GBS,
                     'what': what}

    # buffers and host arguments prepared outside the timed region: only the C entry's
    # launches are timed
    lib = _ia.lib()
    H = W = 2048
    rgb = torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device=dev)
    yiq = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
    y = torch.empty((H, W), dtype=torch.float64, device=dev)

    def to_yiq():
        _ia.check(lib.ia_rgb_to_yiq(_ia.ptr(rgb), ip._dtype_code(rgb), H * W, 255.0,
                                    _ia.ptr(yiq), _ia.ptr(y), _ia.stream()), 'ia_rgb_to_yiq')
    put('yiq', timed(to_yiq), H * W * (3 + 32), 'ia_rgb_to_yiq 2048x2048 u8 -> YIQ + Y fp64')
    img = torch.rand((H, W), dtype=torch.float64, device=dev)
    sm = torch.empty((1024, 1024), dtype=torch.float64, device=dev)
    ws = _ia.workspace(lib.ia_pyr_workspace_bytes(H, W))
    coef = (ctypes.c_double * 4)(*ip.resize_coeffs((H, W), (1024, 1024)))
    taps = (ctypes.c_double * 4)(*ip.PYR_TAPS)

    def reduce():
        _ia.check(lib.ia_pyr_reduce_f64(_ia.ptr(img), H, W, _ia.ptr(sm), 1024, 1024, coef, taps,
                                        _ia.ptr(ws), _ia.stream()), 'ia_pyr_reduce_f64')
    put('pyr_reduce', timed(reduce), 8 * (H * W + 1024 * 1024),
        'ia_pyr_reduce_f64 (k_pyr_wave + k_pyr_clip_p) 2048^2 -> 1024^2')
    Ap_lg, Ap_sm = img[None].clone(), sm[None].clone()
    N = H * W
    ix = algorithms.LevelIndex(sm, img, Ap_sm, Ap_lg, rows=True)

    def build():
        _ia.check(lib.ia_db_build(ctypes.byref(ix.src), 0, ix.nrows, _ia.ptr(ix.center),
                                  _ia.ptr(ix.db), _ia.ptr(ix.amax), _ia.stream()), 'ia_db_build')
    put('db_build', timed(build), N * 224 + 8 * 2 * (N + 1024 * 1024),
        'ia_db_build (k_db_range + k_db_bound + LDS-tiled k_db_build_t), 4,194,304 rows')
    if ix.dbi is not None:
        def build_image():
            _ia.check(lib.ia_db_build_image(ctypes.byref(ix.src), 0, ix.nrows, _ia.ptr(ix.center),
                                            None, _ia.ptr(ix.amax), _ia.ptr(ix.dbi), _ia.stream()),
                      'ia_db_build_image')
        put('db_image', timed(build_image), N * 34,
            'ia_db_build_image without rows (k_db_range_at + one-pass k_img_build: pads, norm '
            'slots and the bound), 4,194,304 rows')
    return out


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(('127.0.0.1', 0))
        return sk.getsockname()[1]


def share_gpu():
    """IA_SHARE_GPU=1 (tests on a one-GPU box only): every rank runs on cuda:0.  The
    device-side exchange works between processes of one GPU; RCCL refuses it."""
    return os.environ.get('IA_SHARE_GPU', '0') == '1'


def launch_ranks(args):
    """`--gpus N` (N > 1) outside torch.distributed.run: start the N rank processes with it
    as a child (this process has made no GPU call: torch.cuda.device_count() does not
    initialise the device on this image) and exit with its status."""
    if not args.dry_run and not share_gpu():
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print('bench.py: --gpus %d but only %d GPU(s) visible' % (args.gpus, ndev),
                  file=sys.stderr, flush=True)
            sys.exit(2)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='c4', choices=sorted(CONFIGS))
    ap.add_argument('--jobs', type=int, default=32,
                    help='c5: jobs per GPU per step (32 = the per-GPU share of the 256-job '
                         'batch over 8 GPUs)')
    ap.add_argument('--batch', type=int, default=0,
                    help='c5: jobs per batched launch set (ia_synth_levels_batch; 0 = all of '
                         'the GPU\'s jobs in one batch; 1 = one job per synthesis call, run '
                         '--streams at a time)')
    ap.add_argument('--streams', type=int, default=4,
                    help='c5 with --batch 1: jobs run concurrently per GPU (one HIP stream + '
                         'host thread each; 4 = the HIP hardware queues per process)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0,
                    help='CPU work per leg of the CPU baseline (1 thread, all threads)')
    ap.add_argument('--matcher', default='brute', choices=['brute', 'lsh'],
                    help="lsh: the approximate E2LSH matcher (SURVEY §8(f)1, config c2)")
    ap.add_argument('--lsh', default='16,4,1.0', help='tables,hashes,width for --matcher lsh')
    ap.add_argument('--strict-exchange', action='store_true',
                    help='exit non-zero when the device-side exchange times out instead of '
                         'measuring again over RCCL')
    ap.add_argument('--dry-run', action='store_true',
                    help='launcher check without a GPU: ranks meet over gloo, rank 0 prints '
                         'the world it saw')
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        launch_ranks(args)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        print('bench.py: world size %d != --gpus %d' % (world, args.gpus), file=sys.stderr,
              flush=True)
        sys.exit(2)
    if world > 1:
        # gloo prints its connection report on stdout: keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group('gloo')
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if args.dry_run:
        t = torch.tensor([float(rank)])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({'dry_run': True, 'n_gpus': world, 'gpus': args.gpus,
                              'rank_sum': float(t.item()), 'config': args.config}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if share_gpu():
        local = 0
    if torch.cuda.device_count() <= local:
        print('bench.py: rank %d needs GPU %d, %d visible' % (rank, local,
                                                            torch.cuda.device_count()),
              file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    conf = CONFIGS[args.config]

    comm = None
    if world > 1 and args.config != 'c5':
        # one exchange per sharded level (the levels run pipelined, each exchange ordered
        # on its own level's stream): the device-side exchange (IA_EXCHANGE=peer, default)
        # or one RCCL all-gather per wave (IA_EXCHANGE=rccl)
        j0 = Job(conf, 0, dev)
        comm = ia.level_exchanges([ip.gaussian_pyramid_dev(j0.Ap, cfg.n_sm, j0.levels)],
                                  j0.max_levels, rank, world)
        del j0

    lsh = None
    if args.matcher == 'lsh':
        t_, h_, w_ = args.lsh.split(',')
        lsh = dict(tables=int(t_), hashes=int(h_), width=float(w_), seed=0)
    if args.config == 'c5':
        # the whole batch is args.jobs per GPU; this rank's share by the package's split
        # (image_analogies.rank_jobs: job j on rank j mod world, seed 1000 + 3 j)
        my_jobs = ia.rank_jobs(args.jobs * world, rank, world)
        jobs = [Job(conf, 1000 + 3 * j, dev, lsh) for j in my_jobs]
    else:
        jobs = [Job(conf, 0, dev, lsh)]

    # c5: --streams S runs the GPU's jobs S at a time, each on its own HIP stream driven by
    # its own host thread (ctypes drops the GIL inside ia_synth_level, so the threads enqueue
    # their latency-bound waves concurrently); results are per job and stream-independent
    batch = (args.batch or len(jobs)) if args.config == 'c5' and lsh is None else 1
    # --batch B < jobs: the batches run --streams at a time, each on its own stream and host
    # thread (one batch's latency-bound per-wave tails beside another's HBM-bound screens)
    nbatches = (len(jobs) + batch - 1) // batch
    if args.config != 'c5':
        nstreams = 1
    elif batch == 1:
        nstreams = max(1, min(args.streams, len(jobs)))
    else:
        nstreams = max(1, min(args.streams, nbatches))
    pool = streams = None
    if nstreams > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(nstreams)
        streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]

    def run_jobs(fn):
        if pool is None:
            return [fn(jb) for jb in jobs]
        main = torch.cuda.current_stream(dev)

        def lane(i):
            torch.cuda.set_device(dev)
            st = streams[i]
            st.wait_stream(main)
            with torch.cuda.stream(st):
                return [fn(jb) for jb in jobs[i::nstreams]]
        res = list(pool.map(lane, range(nstreams)))
        for st in streams:
            main.wait_stream(st)
        return [r for part in res for r in part]

    def run_batches(prof=False, check=True):
        groups = [jobs[b0:b0 + batch] for b0 in range(0, len(jobs), batch)]

        def one(part):
            ins = [jb.prepare() for jb in part]
            return ia.synthesize_batch_dev(ins, part[0].max_levels, [jb.k for jb in part],
                                           part[0].weights, prof=prof, check=check)
        if pool is None:
            # the package's multi-GPU batch entry: the whole job list with this rank's entries
            # (the others' are never read), split j = rank (mod world), `batch` per launch set
            whole = [None] * (len(jobs) * world)
            for j, jb in zip(my_jobs, jobs):
                whole[j] = jb.prepare
            res = ia.synthesize_jobs(whole, jobs[0].max_levels, [jobs[0].k] * len(whole),
                                     jobs[0].weights, rank, world, batch=batch, prof=prof,
                                     check=check)
            return [res[j] for j in my_jobs]
        main = torch.cuda.current_stream(dev)

        def lane(i):
            torch.cuda.set_device(dev)
            st = streams[i]
            st.wait_stream(main)
            with torch.cuda.stream(st):
                return [one(part) for part in groups[i::nstreams]]
        res = list(pool.map(lane, range(nstreams)))
        for st in streams:
            main.wait_stream(st)
        outs = [None] * len(groups)
        for i, r in enumerate(res):
            for j, o in enumerate(r):
                outs[i + j * nstreams] = o
        return [o for part in outs for o in part]

    def run_step(prof=False):
        # no per-step ia_synth_status (a host sync per step): every level folds its error
        # word into the device's sticky word, checked once after each timed pass
        if batch > 1:
            return run_batches(prof, check=False)
        run_jobs(lambda jb: jb.step(comm, rank, world, prof, check=False))

    def pass_status():
        pass_check(comm)

    def timed_pass(prof):
        """K steps between two barrier + synchronize brackets; prof: HIP events around
        every screen launch and the matcher statistics, read back after the region."""
        if prof:
            _ia.prof_begin()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_step(prof)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        return dt, (_ia.prof_end() if prof else None)

    def measure():
        # warm-up steps run profiled too; the event pool is created before any timed region
        nev = 3 * args.steps * sum(jb.waves for jb in jobs)
        _ia.prof_begin(nev)
        for _ in range(args.warmup):
            run_step(True)
        _ia.prof_end()
        pass_status()
        # `value`: the product path alone; then the same K steps with the HIP events of the
        # roofline (their cost is reported as events_overhead)
        plain, _ = timed_pass(False)
        pass_status()
        evented, prof = timed_pass(True)
        pass_status()
        return plain, evented, prof

    exchange_fallback = None
    try:
        elapsed, elapsed_ev, prof = measure()
    except _ia.ExchangeTimeout as e:
        # another rank's records never came over the device-side exchange: every rank
        # agrees, takes the RCCL exchange and measures again from scratch (every step
        # rebuilds pyramids, DBs, B').  A ScheduleFault (a neighbour-decision wait inside
        # the fused kernel) is a bug of the kernel, not of the exchange: it propagates.
        if not (comm and _ia.exchange_kind() == 'peer') or args.strict_exchange:
            raise
        exchange_fallback = 'device-side exchange wait timed out: %s' % e
    if comm and exchange_fallback is None and _ia.exchange_kind() == 'peer':
        ok = all(_ia.lib().ia_peer_status(cm) == 0 for cm in comm)
        if not _ia._all_ok(ok, world):
            exchange_fallback = 'device-side exchange wait timed out on some rank'
    if exchange_fallback is not None:
        if args.strict_exchange:
            print('bench.py: %s (--strict-exchange)' % exchange_fallback, file=sys.stderr, flush=True)
            sys.exit(3)
        for cm in comm:
            _ia.lib().ia_comm_destroy(cm)
        _ia._EXCHANGE_FALLBACK.append(exchange_fallback)
        print('bench.py: %s; measuring again over RCCL' % exchange_fallback, file=sys.stderr, flush=True)
        comm = [_ia.exchange(rank, world, 'rccl') for _ in comm]
        elapsed, elapsed_ev, prof = measure()
    for cm in comm or []:
        _ia.exchange_status(cm)     # raises if a device-side exchange wait timed out
    own_elapsed = elapsed
    t = torch.tensor([elapsed, elapsed_ev], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, elapsed_ev = float(t[0].item()), float(t[1].item())

    # consistency of the result (outside the timed region): B' == A'[im][s] per level and
    # identical replicas across ranks
    batch_ok = None

    def job_sum(jb, out):
        return sum(float(jb.Bp[l].sum().item()) + float(s_.double().sum().item())
                   for l, (s_, _) in out.items())
    job_sums = None
    if batch > 1:
        # every job of a batch equals its own one-job synthesis (same inputs, same B' init)
        outs = run_batches()
        torch.cuda.synchronize()
        bsums = [job_sum(jb, o) for jb, o in zip(jobs, outs)]
        batch_ok = all(b == job_sum(jb, jb.step()) for b, jb in zip(bsums, jobs))
        job_sums = {str(jb.seed): b for jb, b in zip(jobs, bsums)}
    elif args.config == 'c5':
        job_sums = {str(jb.seed): job_sum(jb, jb.step()) for jb in jobs}
    out = jobs[0].step(comm, rank, world)
    chk = 0.0
    consistent = True
    for l, (s, im) in out.items():
        chk += float(jobs[0].Bp[l].sum().item()) + float(s.double().sum().item())
        src = jobs[0].Ap_pyr_last[l]
        consistent &= bool(torch.equal(jobs[0].Bp[l].flatten(),
                                       src[s[:, 0].long(), s[:, 1].long()]))
    ct = torch.tensor([chk], dtype=torch.float64)
    concurrent_ok = None
    if pool is not None:   # every job's result: concurrent streams == one stream, in order
        outs = run_jobs(lambda jb: jb.step(comm, rank, world))
        torch.cuda.synchronize()
        order = [j for i in range(nstreams) for j in jobs[i::nstreams]]
        conc = [job_sum(jb, o) for jb, o in zip(order, outs)]
        seq = {id(jb): job_sum(jb, jb.step(comm, rank, world)) for jb in jobs}
        concurrent_ok = all(c == seq[id(jb)] for c, jb in zip(conc, order))
    replicas_ok = True
    if world > 1 and args.config != 'c5':
        lo, hi = ct.clone(), ct.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        replicas_ok = bool(lo.item() == hi.item())

    pixels_per_step = sum(jb.pixels for jb in jobs) * (world if args.config == 'c5' else 1)
    value = pixels_per_step * args.steps / elapsed
    # roofline of the dominant kernel: the screen instance k_screen16<G> (G = query tiles
    # per block) with the most time over the timed steps, from the HIP events on its
    # stream around each of its launches; also the whole finest level and all levels
    # 2*D = 110 algorithmic flop per (query, row) pair; the split-f16 screen
    # issues 3 f16 products per feature (a_h q_h + a_h q_l + a_l q_h), 330 flop per pair, so
    # its algorithmic fraction of the f16 dense peak is capped at 1/3; the
    # MFMA pipe's utilisation is reported beside it as pipe_frac
    per_pair = 2 * 55
    # the rotated screen (R16) on the fused kernel's levels of at least
    # rot_min_rows() rows: 4 MFMAs x 16 K-slots = 64 slots, 128 f16 flop issued per pair; else
    # the split-f16 screen's 3 products per feature, 330
    # (the finest level's DB, or this rank's shard of it, holds enough rows: level_index)
    fin_rows = max((p['rows'] for p in prof), default=0)
    rot_used = (_ia.db_rot_enabled() and lsh is None and fin_rows >= _ia.rot_min_rows() and
                (comm is None or _ia.exchange_kind() == 'peer'))
    pipe_per_pair = 2 * _ia.lib().ia_db_rot_slots() if rot_used else 3 * 2 * 55
    inst = {}
    lv = {}
    for p in prof:
        for ms, M in zip(p['launch_ms'], p['launch_M']):
            T = (int(M) + 31) // 32
            g = (T + 10) // 11
            G = (T + g - 1) // g
            d = inst.setdefault(G, [0.0, 0, 0.0, 0])
            nj = max(1, p.get('jobs', 1))      # a batch's launch screens every job's DB
            d[0] += ms; d[1] += 1; d[2] += float(M) * p['rows'] * nj; d[3] += int(M)
            e = lv.setdefault(p['level'], [0.0, 0, 0.0, p['rows']])
            e[0] += ms; e[1] += 1; e[2] += float(M) * p['rows'] * nj
    domG = max(inst, key=lambda G: inst[G][0]) if inst else None
    i_ms, i_n, i_pairs, i_q = inst[domG] if domG is not None else (0.0, 0, 0.0, 0)
    achieved = per_pair * i_pairs / (i_ms * 1e-3) / 1e12 if i_ms > 0 else 0.0
    fp32eq = 2.0 * 55 * i_pairs / (i_ms * 1e-3) / 1e12 if i_ms > 0 else 0.0
    fin = max(lv) if lv else None
    f_ms, f_n, f_pairs, f_rows = lv[fin] if fin is not None else (0.0, 0, 0.0, 0)
    screen_ms = sum(v[0] for v in lv.values())
    screens = sum(v[1] for v in lv.values())
    pairs = sum(v[2] for v in lv.values())
    traffic, pmc = None, screen_pmc()
    if pmc and args.config == 'c4' and world == 1 and domG == 11 and lsh is None and \
            ('k_screen16r' in pmc['kernel']) == bool(rot_used):
        traffic = pmc['bytes']
    # the finest level's screen streams the DB's image form when it applies (k_screen16i;
    # k_screen16p, the producer / consumer form, on strip-order levels: every c4 / c5 level)
    img_form = _ia.db_image_enabled() and jobs[0].A.shape[1] % 128 == 0 and lsh is None
    # (the producer / consumer form runs single-job, unsharded levels: a batch of jobs and a
    # sharded finest level take the 4-wave k_screen16i)
    pc_used = (_ia.lib().ia_diag_set_screen_pc(-1) and batch == 1 and
               comm is None)
    kname = 'k_screen16r<%s>' if rot_used else (('k_screen16p<%s>' if pc_used else 'k_screen16i<%s>')
                                                if img_form else 'k_screen16<%s>')
    roof = {'bound': 'mfma', 'kernel': kname % domG,
            'achieved': achieved,
            'peak': F16_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': achieved / F16_MFMA_PEAK_TFLOPS, 'traffic': traffic,
            'algorithmic': '%d flop per (query,row) pair (2 x D, D = 55; SURVEY 8(d)); %d launches, '
                           '%.4g pairs (mean M %.1f queries)' % (per_pair, i_n, i_pairs,
                                                                 i_q / max(i_n, 1)),
            'pipe_frac': achieved * pipe_per_pair / per_pair / F16_MFMA_PEAK_TFLOPS,
            'pipe_note': ('f16 MFMA pipe utilisation: the rotated split screen (R16) issues %d f16 '
                          'flop per pair (16 K-slots per MFMA x 2), so frac <= pipe_frac x 110 / that'
                          if rot_used else
                          'f16 MFMA pipe utilisation: the split issues %d f16 flop per pair '
                          '(3 products x 2 x 55), so frac <= pipe_frac / 3') % pipe_per_pair,
            'screen_avg_us': i_ms * 1e3 / max(i_n, 1),
            'source': 'HIP events around every launch of this kernel in the timed steps',
            'fp32_equivalent_tflops': fp32eq,
            'fp32_equivalent_frac_of_fp32_mfma_peak': fp32eq / FP32_MFMA_PEAK_TFLOPS,
            'finest_level': {'level': fin, 'rows': f_rows, 'launches': f_n,
                             'screen_avg_us': f_ms * 1e3 / max(f_n, 1),
                             'frac': (per_pair * f_pairs / (f_ms * 1e-3) / 1e12 /
                                      F16_MFMA_PEAK_TFLOPS) if f_ms else 0.0,
                             'pipe_frac': (pipe_per_pair * f_pairs / (f_ms * 1e-3) / 1e12 /
                                           F16_MFMA_PEAK_TFLOPS) if f_ms else 0.0},
            'all_levels': {'launches': screens, 'pairs': pairs,
                           'screen_avg_us': screen_ms * 1e3 / max(screens, 1),
                           'screen_ms_per_step': screen_ms / args.steps,
                           'fp32_equivalent_tflops':
                               2.0 * 55 * pairs / (screen_ms * 1e-3) / 1e12 if screen_ms else 0.0}}
    if traffic is not None:
        roof['traffic_note'] = ('HBM bytes per launch (mean of %d dispatches of %s), PMC FETCH_SIZE '
                                'x 2 + WRITE_SIZE of bench.py under rocprofv3 (%s); algorithmic: '
                                'the DB read once (R16 rotated rows: 128 B x 4,194,304 = 536.9 MB; '
                                'split-f16 row form: 939.5 MB) + 11 MB of segment minima'
                                % (pmc['dispatches'], pmc['kernel'], pmc['source']))
        sq = screen_sq()
        if sq is not None:
            # the same kernel's SQ/GRBM pass: why frac is what it is
            roof['pmc'] = sq
    if lsh is not None:
        # k_lsh_query is a gather: each examined row costs its 55 fp64 features (440 B)
        examined = sum(p['rows_rescored'] for p in prof if p['timed_screens'])
        screen_ms = sum(float(p['launch_ms'].sum()) for p in prof)
        gbs = examined * 440.0 / (screen_ms * 1e-3) / 1e9 if screen_ms > 0 else 0.0
        roof = {'bound': 'hbm', 'kernel': 'k_lsh_query', 'achieved': gbs,
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': gbs / HBM_PEAK_GBS,
                'traffic': None,
                'algorithmic': '440 B (55 fp64) per examined row; %d rows over %d launches'
                               % (examined, screens),
                'screen_avg_us': screen_ms * 1e3 / max(screens, 1),
                'source': 'HIP events around every LSH query launch of the timed steps'}

    result = {
        'metric': "B' pixels/sec (brute-force match, 5-level pyramid) + MFMA util @1/2/4/8 GPU"
                  + (' [LSH matcher]' if lsh is not None else ''),
        'value': value,
        'unit': "B' pixels/s",
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak' if args.config == 'c5' else 'strong',
        'vs_baseline': None,
        'dtype': ('f16 rotated split (R16 MFMA screen: %d principal components as f16 pairs, %d as '
                  'f16, f32 accumulate) + f64 (rotation, exact rescore, pyramids)'
                  % (_ia.lib().ia_db_rot_components(), 55 - _ia.lib().ia_db_rot_components()) if rot_used else
                  'f16x3 split (MFMA screen, f32 accumulate) + f32 (re-screen) + f64 (exact '
                  'rescore, pyramids)'),
        'data': 'synthetic (gaussian-filtered noise; A\' = blur(A)); seeded',
        'config': {'workload': args.config + ': ' + conf['name'] +
                               (', LSH matcher' if lsh is not None else ', brute force'),
                   'A': list(conf['A']), 'B': list(conf['B']), 'kappa': conf['k'],
                   'levels_cap': conf['levels'], 'jobs_per_gpu': len(jobs), 'streams_per_gpu': nstreams,
                   'jobs_per_launch': batch,
                   'pixels_per_step': pixels_per_step,
                   'parallelism': ('jobs%d' % world) if args.config == 'c5' else
                                  ('db-shard%d' % world if world > 1 else 'single'),
                   **({'exchange': _ia.exchange_kind() + (' (ranks share one GPU)' if share_gpu() else '')}
                      if comm is not None else {})},
        'roofline': roof,
        # N > 1 with DB sharding: whether a device-side exchange wait timed out and the
        # numbers are the RCCL exchange's (null: no fallback happened)
        **({'exchange_fallback': exchange_fallback or (_ia._EXCHANGE_FALLBACK[-1]
                                                       if _ia._EXCHANGE_FALLBACK else None)}
           if comm is not None else {}),
        'matcher': {'kind': 'lsh' if lsh is not None else 'exact',
                    'rows_rescored_fp64': sum(p['rows_rescored'] for p in prof),
                    'candidate_segments': sum(p['candidate_segments'] for p in prof),
                    'full_scans': sum(p['full_scans'] for p in prof),
                    'queries': pixels_per_step * args.steps // (world if args.config == 'c5' else 1),
                    # time the fused per-wave kernel's pixels spent waiting, summed over pixels
                    # and divided by them: for the other ranks' records (device-side exchange)
                    # and for the upper neighbour's decision (its next-query build)
                    'peer_wait_us_per_pixel': sum(p['peer_wait_us'] for p in prof) /
                        max(1, pixels_per_step * args.steps // (world if args.config == 'c5' else 1)),
                    'neighbour_wait_us_per_pixel': sum(p['neighbour_wait_us'] for p in prof) /
                        max(1, pixels_per_step * args.steps // (world if args.config == 'c5' else 1))},
        'events_pass': {'ms_per_step': elapsed_ev / args.steps * 1e3,
                        'overhead': (elapsed_ev - elapsed) / elapsed,
                        # the finest level's wave spacing on its stream (HIP events, no
                        # profiler): screen, end of screen -> end of the fused kernel, and
                        # end of the fused kernel -> start of the next screen
                        'finest_wave_us': wave_spacing(prof, fin),
                        'note': 'the same K steps again with HIP events around every screen '
                                'launch and the matcher statistics (the roofline\'s source); '
                                '`value` is the pass without them'},
        'checks': {'replicas_identical': replicas_ok, 'bp_equals_ap_at_s': consistent,
                   'checksum': chk,
                   **({'exchange_fallback': exchange_fallback or _ia._EXCHANGE_FALLBACK[-1]}
                      if (exchange_fallback or _ia._EXCHANGE_FALLBACK) else {}),
                   **({'concurrent_streams': nstreams, 'concurrent_identical': concurrent_ok}
                      if concurrent_ok is not None else {}),
                   **({'batch_jobs': batch, 'batch_identical': batch_ok}
                      if batch_ok is not None else {}),
                   # c5: every job's checksum by its seed (1000 + 3 (rank + world j)), so that
                   # any job can be compared with the same seed's run at another world size
                   **({'job_sums': job_sums} if job_sums is not None and world == 1 else {})},
    }
    if world > 1:
        # per-rank facts, so that the first run across GPUs explains itself
        rq = pixels_per_step * args.steps // (world if args.config == 'c5' else 1)
        mine = {'rank': rank, 'local_rank': local, 'device': torch.cuda.get_device_name(dev),
                'ms_per_step': own_elapsed / args.steps * 1e3,
                'jobs': len(jobs), 'pixels_per_step': sum(jb.pixels for jb in jobs),
                'exchanges': list(_ia.EXCHANGE_INFO),
                'exchange_fallback': list(_ia._EXCHANGE_FALLBACK),
                # this rank's dominant screen (the MFMA utilisation at N GPUs): launch mean,
                # algorithmic fraction of the f16 dense peak and the pipe's
                'kernel': roof.get('kernel'), 'screen_avg_us': roof.get('screen_avg_us'),
                'frac': roof.get('frac'), 'pipe_frac': roof.get('pipe_frac'),
                'peer_wait_us_per_pixel': sum(p['peer_wait_us'] for p in prof) / max(1, rq),
                'neighbour_wait_us_per_pixel': sum(p['neighbour_wait_us'] for p in prof) / max(1, rq),
                'checksum': chk, **({'job_sums': job_sums} if job_sums is not None else {})}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        result['ranks'] = allr
    if lsh is not None:
        result['lsh_quality'] = jobs[0].lsh_quality()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(jobs[0], args.cpu_seconds)
    if rank == 0 and world == 1 and args.config == 'c4':
        result['hbm_kernels'] = hbm_kernels(dev)
    if comm is not None:
        for cm in comm:
            _ia.lib().ia_comm_destroy(cm)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not (replicas_ok and consistent and batch_ok is not False and concurrent_ok is not False):
        print('bench.py: result check failed (replicas_identical=%s, bp_equals_ap_at_s=%s)'
              % (replicas_ok, consistent), file=sys.stderr, flush=True)
        sys.exit(4)


if __name__ == '__main__':
    main()
