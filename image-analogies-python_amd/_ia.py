"""ctypes binding of libia.so (include/ia.h) and device-memory plumbing.

PyTorch is used only as plumbing: device allocations (``torch.empty(..., device='cuda')``),
the current HIP stream and ``torch.distributed`` for rendezvous.  ``torch`` is imported
BEFORE libia.so is loaded so that the library's ``libamdhip64.so.7`` / ``librccl.so.1``
dependencies resolve (by SONAME) to the copies torch already loaded: one HIP runtime per
process, and torch's stream handles are valid inside libia.

There is no CPU fallback anywhere in the product: every entry point raises if the
library or a HIP device is missing.
"""
import ctypes
import os
import re
import sys

import numpy as np
import torch  # noqa: F401  (must precede libia.so, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
# IA_LIB_PATH: another build of the same library (A/B of build variants, `tools/gpu.sh ablib`)
LIB_PATH = os.environ.get('IA_LIB_PATH') or os.path.join(_HERE, 'libia.so')
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'ia.h')

IA_D = 55
IA_DP = 56

_dp = ctypes.c_void_p


class IaSrcLevel(ctypes.Structure):
    _fields_ = [('A_sm', _dp), ('A_lg', _dp), ('Ap_sm', _dp), ('Ap_lg', _dp),
                ('A_hs', ctypes.c_int), ('A_ws', ctypes.c_int), ('Ah', ctypes.c_int),
                ('Aw', ctypes.c_int), ('nAp', ctypes.c_int)]


class IaLsh(ctypes.Structure):
    _fields_ = [('mem', _dp), ('proj', _dp), ('L', ctypes.c_int), ('k', ctypes.c_int),
                ('w', ctypes.c_float)]


class IaMatchArgs(ctypes.Structure):
    _fields_ = [('src', IaSrcLevel), ('db', _dp), ('row0', ctypes.c_long),
                ('nrows', ctypes.c_long), ('center', _dp), ('amax', _dp), ('q64', _dp),
                ('M', ctypes.c_int), ('idx', _dp), ('dist', _dp), ('workspace', _dp),
                ('lsh', ctypes.POINTER(IaLsh)), ('dbi', _dp)]


class IaSynthArgs(ctypes.Structure):
    _fields_ = [('src', IaSrcLevel), ('db', _dp), ('row0', ctypes.c_long),
                ('nrows', ctypes.c_long), ('N_total', ctypes.c_long), ('center', _dp),
                ('amax', _dp), ('B_sm', _dp), ('B_lg', _dp), ('B_hs', ctypes.c_int),
                ('B_ws', ctypes.c_int), ('H', ctypes.c_int), ('W', ctypes.c_int),
                ('Bp_sm', _dp), ('Bp_lg', _dp), ('weights', _dp),
                ('kappa_factor', ctypes.c_double), ('s', _dp), ('im', _dp),
                ('workspace', _dp), ('comm', _dp), ('lsh', ctypes.POINTER(IaLsh)),
                ('flags', ctypes.c_int), ('tag', ctypes.c_int), ('dbg_px', _dp),
                ('dbg_dist', _dp), ('dbi', _dp), ('dbr', _dp), ('rot', _dp)]


class IaShardDb(ctypes.Structure):
    _fields_ = [('db', _dp), ('row0', ctypes.c_long), ('nrows', ctypes.c_long), ('amax', _dp),
                ('dbi', _dp)]


IA_SYNTH_EAGER = 1
IA_SYNTH_PROF = 2
IA_PROF_FIELDS = 11

_SIGS = {
    'ia_last_error': (ctypes.c_char_p, []),
    'ia_version': (ctypes.c_int, []),
    'ia_rgb_to_yiq': (ctypes.c_int, [_dp, ctypes.c_int, ctypes.c_long, ctypes.c_double, _dp, _dp, _dp]),
    'ia_yiq_to_rgb': (ctypes.c_int, [_dp, ctypes.c_long, _dp, _dp]),
    'ia_color_output': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]),
    'ia_scale_to_f64': (ctypes.c_int, [_dp, ctypes.c_int, ctypes.c_long, ctypes.c_double, _dp, _dp]),
    'ia_axpb_f64': (ctypes.c_int, [_dp, ctypes.c_long, ctypes.c_int, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, _dp, _dp]),
    'ia_pyr_workspace_bytes': (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    'ia_pyr_reduce_f64': (ctypes.c_int, [_dp, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), _dp, _dp]),
    'ia_mean_workspace_bytes': (ctypes.c_size_t, [ctypes.c_long]),
    'ia_mean_f64': (ctypes.c_int, [_dp, ctypes.c_long, _dp, _dp, _dp]),
    'ia_var_f64': (ctypes.c_int, [_dp, ctypes.c_long, _dp, _dp, _dp]),
    'ia_level_features_f64': (ctypes.c_int, [_dp, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, _dp, _dp]),
    'ia_db_rows_padded': (ctypes.c_long, [ctypes.c_long]),
    'ia_db_bytes': (ctypes.c_size_t, [ctypes.c_long]),
    'ia_db_chunk_rows': (ctypes.c_int, [ctypes.c_long]),
    'ia_set_chunk_target': (ctypes.c_long, [ctypes.c_long]),
    'ia_db_rot_applies': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long]),
    'ia_db_rot_bytes': (ctypes.c_size_t, [ctypes.c_long]),
    'ia_db_rot_components': (ctypes.c_int, []),
    'ia_screen_resources': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    'ia_fused_resources': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    'ia_level_resources': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), ctypes.POINTER(ctypes.c_int)]),
    'ia_db_rot_slots': (ctypes.c_int, []),
    'ia_db_rot_eps_a2': (ctypes.c_double, []),
    'ia_db_cov_bytes': (ctypes.c_size_t, []),
    'ia_db_cov': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long, _dp, _dp, _dp]),
    'ia_db_build_rot': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long, _dp, _dp,
                                       _dp, _dp, _dp]),
    'ia_db_build': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long,
                                   _dp, _dp, _dp, _dp]),
    'ia_db_image_bytes': (ctypes.c_size_t, [ctypes.POINTER(IaSrcLevel), ctypes.c_long,
                                            ctypes.c_long]),
    'ia_db_build_image': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long,
                                         _dp, _dp, _dp, _dp, _dp]),
    'ia_center_fill': (ctypes.c_int, [_dp, ctypes.c_double, ctypes.c_double, _dp]),
    'ia_match_workspace_bytes': (ctypes.c_size_t, [ctypes.c_int, ctypes.c_long]),
    'ia_match_batch': (ctypes.c_int, [ctypes.POINTER(IaMatchArgs), _dp]),
    'ia_coherence_pick': (ctypes.c_int, [_dp, ctypes.c_int, _dp, _dp, _dp]),
    'ia_wdist_batch': (ctypes.c_int, [_dp, _dp, _dp, ctypes.c_int, _dp, _dp]),
    'ia_synth_workspace_bytes': (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_long,
                                                   ctypes.c_int]),
    'ia_synth_level': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), _dp]),
    'ia_synth_level3': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), _dp]),
    'ia_synth3_status': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), ctypes.c_int, _dp]),
    'ia_synth_levels3': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), ctypes.c_int, _dp]),
    'ia_db3_rot_bytes': (ctypes.c_size_t, [ctypes.c_long]),
    'ia_db3_rot_components': (ctypes.c_int, []),
    'ia_db3_rot_floats': (ctypes.c_int, []),
    'ia_db3_cov_bytes': (ctypes.c_size_t, []),
    'ia_db3_cov': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]),
    'ia_db3_build_rot': (ctypes.c_int, [_dp, ctypes.c_long, _dp, _dp, _dp]),
    'ia_synth3_workspace_bytes': (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_long]),
    'ia_db3_bytes': (ctypes.c_size_t, [ctypes.c_long]),
    'ia_match3_workspace_bytes': (ctypes.c_size_t, [ctypes.c_int, ctypes.c_long]),
    'ia_match3_batch': (ctypes.c_int, [_dp, ctypes.c_long, _dp, ctypes.c_int, _dp, _dp, _dp, _dp]),
    'ia_coherence_pick3': (ctypes.c_int, [_dp, ctypes.c_int, _dp, _dp, _dp]),
    'ia_wdist3_batch': (ctypes.c_int, [_dp, _dp, _dp, ctypes.c_int, _dp, _dp]),
    'ia_db3_build': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long, _dp,
                                    _dp]),
    'ia_level_features3_f64': (ctypes.c_int, [_dp, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, _dp, _dp]),
    'ia_synth_levels': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), ctypes.c_int, _dp]),
    'ia_synth_status': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), ctypes.c_int, _dp]),
    'ia_sched_status': (ctypes.c_int, [ctypes.c_int]),
    'ia_synth_levels_batch': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs), ctypes.c_int, ctypes.c_int,
                                             _dp]),
    'ia_lsh_bytes': (ctypes.c_size_t, [ctypes.c_long, ctypes.c_int]),
    'ia_lsh_build': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long, _dp,
                                    ctypes.POINTER(IaLsh), _dp]),
    'ia_lsh_bits': (ctypes.c_int, [ctypes.c_long]),
    'ia_comm_unique_id': (ctypes.c_int, [ctypes.c_char_p]),
    'ia_comm_init': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_void_p)]),
    'ia_comm_destroy': (ctypes.c_int, [_dp]),
    'ia_comm_nranks': (ctypes.c_int, [_dp]),
    'ia_peer_create': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p]),
    'ia_peer_connect': (ctypes.c_int, [_dp, ctypes.c_char_p]),
    'ia_peer_check': (ctypes.c_int, [_dp, _dp]),
    'ia_peer_status': (ctypes.c_int, [_dp]),
    'ia_peer_mem_kind': (ctypes.c_int, [_dp]),
    'ia_prof_begin': (ctypes.c_int, []),
    'ia_prof_prepare': (ctypes.c_int, [ctypes.c_long]),
    'ia_prof_waves': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                     ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    'ia_prof_end': (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    'ia_prof_launches': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                        ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    'ia_release_thread_resources': (ctypes.c_int, []),
    # diagnostics (include/ia_diag.h)
    'ia_diag_set_rescore_mode': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_graph_mode': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_xwave': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_screen_sched': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_screen_pc': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_r16_form': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_img_fused': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_screen_trace': (ctypes.c_int, [_dp]),
    'ia_diag_set_color16': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_color16_stats': (ctypes.c_int, [_dp]),
    'ia_diag_screen3': (ctypes.c_int, [_dp, ctypes.c_long, _dp, ctypes.c_int, _dp, _dp, _dp]),
    'ia_diag_xwave_trace': (ctypes.c_int, [_dp]),
    'ia_diag_set_db_build_form': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_set_pyr_form': (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    'ia_diag_qp_rows': (ctypes.c_int, [ctypes.c_int]),
    'ia_diag_query_rows16': (ctypes.c_int, [_dp, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp]),
    'ia_diag_screen16': (ctypes.c_int, [_dp, ctypes.c_long, _dp, ctypes.c_int, _dp, _dp]),
    'ia_diag_stage_map': (ctypes.c_int, [ctypes.c_long, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_int)]),
    'ia_diag_screen16_rows': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long,
                                             _dp, _dp, ctypes.c_int, _dp, _dp]),
    'ia_diag_screen16_image': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long,
                                              ctypes.c_long, _dp, _dp, ctypes.c_int, _dp, _dp]),
    'ia_diag_peer_stress': (ctypes.c_int, [_dp, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int), _dp]),
    'ia_diag_peer_trace': (ctypes.c_int, [_dp, _dp]),
    'ia_diag_screen16r': (ctypes.c_int, [ctypes.POINTER(IaSrcLevel), ctypes.c_long, ctypes.c_long, _dp, _dp,
                                         _dp, _dp, _dp, ctypes.c_int, _dp, _dp, _dp, _dp, _dp]),
    'ia_diag_db3_askip': (ctypes.c_int, [_dp, ctypes.c_long, _dp]),
    'ia_diag_screen3r': (ctypes.c_int, [_dp, _dp, _dp, ctypes.c_long, _dp, ctypes.c_int, _dp, _dp, _dp]),
    'ia_diag_synth_level_shards': (ctypes.c_int, [ctypes.POINTER(IaSynthArgs),
                                                  ctypes.POINTER(IaShardDb), ctypes.c_int, _dp]),
}

_lib = None


def declared_symbols(header=None):
    """Function names declared in include/ia.h (the C-ABI contract), or in every header
    under include/ when header == 'all' (ia.h + the diagnostic ia_diag.h)."""
    inc = os.path.dirname(HEADER)
    if header == 'all':
        paths = [os.path.join(inc, f) for f in sorted(os.listdir(inc)) if f.endswith('.h')]
    else:
        paths = [header or HEADER]
    names = set()
    for p in paths:
        src = re.sub(r'/\*.*?\*/', '', open(p).read(), flags=re.S)
        names.update(re.findall(r'\b(ia_[a-z0-9_]+)\s*\(', src))
    return sorted(names)


def lib():
    """Load libia.so (no fallback: raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                'libia.so not found at %s — build it with `make -C %s/csrc` '
                '(the MI355X core has no CPU fallback)' % (LIB_PATH, _HERE))
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def rescore_mode(mode=-2):
    """Select the exact stage's form for this process (0 per-query workgroups, 1 work list,
    -1 default); returns the previous value."""
    return lib().ia_diag_set_rescore_mode(int(mode))


def graph_mode(mode=-1):
    """HIP-graph capture of the synthesis wave loop for this process (0 off [default],
    1 levels <= 2^18 rows, 2 all single-GPU levels); returns the previous value."""
    return lib().ia_diag_set_graph_mode(int(mode))


def xwave(on=-1):
    """The fused per-wave kernel for this process (2 [default, IA_XWAVE]: one launch per wave
    after the screen runs the exact stage, the device-side exchange, the per-pixel tail and
    the next wave's query rows, in its strip form k_xstrip on strip-order image-form levels;
    1: k_xwave everywhere; 0: the separate kernels); returns the previous value."""
    return lib().ia_diag_set_xwave(int(on))


def db_image_enabled():
    """The screen streams the DB's image form where it applies (IA_DB_IMAGE, default 1;
    0: always the 224-B rows).  Both give the same results bit for bit."""
    return os.environ.get('IA_DB_IMAGE', '1') != '0'


def rot_min_rows():
    """Levels (shards) with fewer DB rows keep the split-f16 screen (IA_ROT_MIN_ROWS, default
    131072): their waves are latency-bound, and the rotated form's per-level build (a
    covariance read back for the host eigh) and per-wave query rotation cost more than its
    faster screen saves there (c1: 19.5 -> 21.9 ms/step with R16 on every level)."""
    return int(os.environ.get('IA_ROT_MIN_ROWS', '131072'))


def db_rot_enabled():
    """The synthesis screen streams the rotated split DB (R16, DESIGN.md §4d: 5 MFMAs per tile
    instead of 11) where it applies (IA_DB_ROT, default 1; 0: the split-f16 image form).
    Both give the same results bit for bit."""
    return os.environ.get('IA_DB_ROT', '1') != '0'


R16_ROT_FLOATS = 13 * 256     # the rotation buffer (ia_rot16.h): 56 x 56 fp32, padded


def db_build_form(tiled=-1):
    """ia_db_build's kernels for this process (1 LDS-tiled where width and row0 are
    multiples of 32 [default], 0 per-row gathers); returns the previous value."""
    return lib().ia_diag_set_db_build_form(int(tiled))


PROF_KEYS = ('level', 'rows', 'pairs', 'screen_ms', 'timed_screens', 'rows_rescored',
             'candidate_segments', 'full_scans', 'peer_wait_us', 'neighbour_wait_us', 'jobs')


def prof_begin(nevents=0):
    """Open a profile: every ia_synth_level call flagged IA_SYNTH_PROF from now on records
    HIP events around its screen launches and its matcher statistics, without
    synchronising (include/ia.h).  nevents: create that many events up front."""
    if nevents:
        check(lib().ia_prof_prepare(int(nevents)), 'ia_prof_prepare')
    check(lib().ia_prof_begin(), 'ia_prof_begin')


def waves(H, W):
    """Skewed waves t = x + 3y of an H x W level: (W - 1) + 3 (H - 1) + 1."""
    return (W - 1) + 3 * (H - 1) + 1


def prof_end():
    """Synchronise the device and read the open profile: one dict per profiled level call
    (PROF_KEYS), in call order."""
    n = lib().ia_prof_end(None, 0)
    if n < 0:
        check(n, 'ia_prof_end')
    buf = (ctypes.c_double * (IA_PROF_FIELDS * max(n, 1)))()
    n = lib().ia_prof_end(buf, n)
    if n < 0:
        check(n, 'ia_prof_end')
    out = []
    for r in range(n):
        rec = dict(zip(PROF_KEYS, buf[r * IA_PROF_FIELDS:(r + 1) * IA_PROF_FIELDS]))
        for k in ('level', 'rows', 'timed_screens', 'rows_rescored', 'candidate_segments',
                  'full_scans', 'jobs'):
            rec[k] = int(rec[k])
        nl = rec['timed_screens']
        ms = (ctypes.c_float * max(nl, 1))()
        Ms = (ctypes.c_int * max(nl, 1))()
        got = lib().ia_prof_launches(r, ms, Ms, nl)
        if got < 0:
            check(got, 'ia_prof_launches')
        rec['launch_ms'] = np.array(ms[:got], dtype=np.float64)
        rec['launch_M'] = np.array(Ms[:got], dtype=np.int64)
        tl = (ctypes.c_float * max(nl, 1))()
        gp = (ctypes.c_float * max(nl, 1))()
        got = lib().ia_prof_waves(r, tl, gp, nl)
        if got < 0:
            check(got, 'ia_prof_waves')
        rec['tail_ms'] = np.array(tl[:got], dtype=np.float64)
        rec['gap_ms'] = np.array(gp[:got], dtype=np.float64)
        out.append(rec)
    return out


IA_E_ARG = -1          # include/ia.h: a bad argument, shape or precondition
IA_E_TIMEOUT = -5      # include/ia.h: a device-side exchange wait for another rank
IA_E_SCHED = -6        # include/ia.h: a neighbour-decision wait inside the fused kernel


class ExchangeTimeout(RuntimeError):
    """Another rank's records never reached this rank's receive box (IA_E_TIMEOUT)."""


class ScheduleFault(RuntimeError):
    """A wait for a neighbouring pixel's decision timed out inside the fused per-wave kernel
    (IA_E_SCHED): a fault of the device schedule itself, never an exchange problem."""


def check(rc, what):
    if rc != 0:
        msg = '%s failed (%d): %s' % (what, rc, lib().ia_last_error().decode())
        raise {IA_E_TIMEOUT: ExchangeTimeout, IA_E_SCHED: ScheduleFault}.get(rc, RuntimeError)(msg)


def sched_status(clear=True):
    """Raise ScheduleFault if any fused level run on this device since the last clear had a
    neighbour-decision wait time out (ia_sched_status; synchronises the device)."""
    check(lib().ia_sched_status(1 if clear else 0), 'ia_sched_status')


def require_device():
    if not torch.cuda.is_available():
        raise RuntimeError('a HIP (MI355X) device is required: this image-analogies core has '
                           'no CPU path')
    lib()
    return torch.device('cuda', torch.cuda.current_device())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def to_dev(a, dtype=torch.float64):
    """numpy -> contiguous device tensor."""
    dev = require_device()
    return torch.as_tensor(np.ascontiguousarray(a)).to(device=dev, dtype=dtype)


def workspace(nbytes):
    dev = require_device()
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)


def src_level(A_sm, A_lg, Ap_sm, Ap_lg):
    """IaSrcLevel over device tensors (Ap_*: stacked (nAp, h, w))."""
    s = IaSrcLevel()
    s.A_sm, s.A_lg, s.Ap_sm, s.Ap_lg = (ptr(A_sm).value, ptr(A_lg).value, ptr(Ap_sm).value,
                                        ptr(Ap_lg).value)
    s.A_hs, s.A_ws = A_sm.shape[-2:]
    s.Ah, s.Aw = A_lg.shape[-2:]
    s.nAp = Ap_lg.shape[0]
    return s


def mean_dev(t):
    """Deterministic device mean of a fp64 tensor (ia_mean_f64) -> python float."""
    t = t.contiguous()
    out = torch.empty(1, dtype=torch.float64, device=t.device)
    ws = workspace(lib().ia_mean_workspace_bytes(t.numel()))
    check(lib().ia_mean_f64(ptr(t), t.numel(), ptr(out), ptr(ws), stream()), 'ia_mean_f64')
    return float(out.item())


def var_f64(t):
    """Unbiased device variance of a fp64 tensor (ia_var_f64, two passes) -> python float."""
    t = t.contiguous()
    out = torch.empty(2, dtype=torch.float64, device=t.device)
    ws = workspace(lib().ia_mean_workspace_bytes(t.numel()))
    check(lib().ia_var_f64(ptr(t), t.numel(), ptr(out), ptr(ws), stream()), 'ia_var_f64')
    return float(out[0].item())


_EXCHANGE_FALLBACK = []   # reasons the device-side exchange was replaced by RCCL
PEER_MAX = 16             # ranks of one device-side exchange (IA_PEER_MAX, ia_internal.h)


def exchange_kind():
    """The per-wave exchange of sharded levels (IA_EXCHANGE): 'peer' [default] the
    device-side exchange (IPC-mapped receive boxes written by the exact stage's kernel),
    'rccl' one ncclAllGather per wave plus a finish kernel.  Same results.  'peer' reads
    'peer->rccl' once a peer exchange could not be set up on every rank (exchange())."""
    k = os.environ.get('IA_EXCHANGE', 'peer')
    if k not in ('peer', 'rccl'):
        raise ValueError('IA_EXCHANGE must be peer or rccl, not %r' % k)
    return 'peer->rccl' if k == 'peer' and _EXCHANGE_FALLBACK else k


def _all_ok(ok, world):
    """Every rank's flag (gloo/RCCL process group): True only if all ranks are ok."""
    if world == 1:
        return ok
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


# what each exchange() of this process ended up as (bench.py reports it per rank at N > 1)
EXCHANGE_INFO = []
PEER_MEM_KINDS = {0: 'uncached device memory', 1: 'fine-grained device memory',
                  2: 'plain device memory'}


def exchange(rank, world, kind=None, mcap=4096):
    """One exchange object (the IaSynthArgs.comm of one sharded level) over the initialised
    torch.distributed process group: every rank calls it at the same point.  'rccl': an
    RCCL communicator (the unique id broadcast from rank 0).  'peer': receive boxes for
    waves of up to mcap queries, handles all-gathered, mapped, then a handshake wave
    (include/ia.h).  If mapping or the handshake fails on any rank, every rank agrees on
    it and falls back to RCCL (the reason is kept in _EXCHANGE_FALLBACK; exchange_kind()
    then reports 'peer->rccl').  Release with ia_comm_destroy."""
    import torch.distributed as dist
    kind = kind or exchange_kind()
    h = ctypes.c_void_p()
    if kind == 'peer->rccl':
        kind = 'rccl'
    if kind == 'rccl':
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            check(lib().ia_comm_unique_id(buf), 'ia_comm_unique_id')
            uid = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        if world > 1:
            dist.broadcast(uid, 0)
        check(lib().ia_comm_init(uid.numpy().tobytes(), world, rank, ctypes.byref(h)),
              'ia_comm_init')
        EXCHANGE_INFO.append({'kind': 'rccl'})
        return h
    if world > PEER_MAX:
        _EXCHANGE_FALLBACK.append('%d ranks > the device-side exchange\'s %d' % (world, PEER_MAX))
        return exchange(rank, world, 'rccl', mcap)
    hd = ctypes.create_string_buffer(64)
    rc = lib().ia_peer_create(world, rank, mcap, ctypes.byref(h), hd)
    if not _all_ok(rc == 0, world):
        # no usable receive box on some rank: every rank takes the RCCL exchange
        if rc == 0:
            lib().ia_comm_destroy(h)
        _EXCHANGE_FALLBACK.append('rank %d: %s' % (rank, lib().ia_last_error().decode())
                                  if rc else 'ia_peer_create failed on another rank')
        print('ia: device-side exchange unusable (%s); falling back to RCCL' % _EXCHANGE_FALLBACK[-1],
              file=sys.stderr, flush=True)
        return exchange(rank, world, 'rccl', mcap)
    mine = torch.frombuffer(bytearray(hd.raw[:64]), dtype=torch.uint8).clone()
    parts = [torch.zeros(64, dtype=torch.uint8) for _ in range(world)]
    if world > 1:
        dist.all_gather(parts, mine)
    else:
        parts = [mine]
    why = None
    if lib().ia_peer_connect(h, b''.join(p.numpy().tobytes() for p in parts)) != 0:
        why = 'rank %d: %s' % (rank, lib().ia_last_error().decode())
    if _all_ok(why is None, world):
        if lib().ia_peer_check(h, stream()) != 0:
            why = 'rank %d: %s' % (rank, lib().ia_last_error().decode())
        elif world > 1:
            # many waves of known records through the boxes (a one-wave handshake can pass
            # on cold caches where later waves would go stale)
            bad = ctypes.c_int(0)
            if lib().ia_diag_peer_stress(h, 16, min(mcap, 256), ctypes.byref(bad), stream()) != 0:
                why = 'rank %d: %s' % (rank, lib().ia_last_error().decode())
            elif bad.value:
                why = 'rank %d: %d of 16 x %d stress records wrong' % (rank, bad.value, min(mcap, 256))
            stress = 'ok: 16 waves x %d records' % min(mcap, 256) if why is None else why
        if _all_ok(why is None, world):
            EXCHANGE_INFO.append({'kind': 'peer', 'peer_mem_kind': int(lib().ia_peer_mem_kind(h)),
                                  'peer_mem': PEER_MEM_KINDS.get(int(lib().ia_peer_mem_kind(h))),
                                  'handshake': 'ok',
                                  'stress': stress if world > 1 else 'skipped (1 rank)'})
            return h
    # some rank could not map or reach the others' boxes: every rank drops its peer
    # exchange and takes the RCCL one
    torch.cuda.synchronize()
    lib().ia_comm_destroy(h)
    _EXCHANGE_FALLBACK.append(why or 'another rank failed')
    print('ia: device-side exchange unusable (%s); falling back to RCCL' % _EXCHANGE_FALLBACK[-1],
          file=sys.stderr, flush=True)
    return exchange(rank, world, 'rccl', mcap)


def exchange_status(comm):
    """Raise if a device-side exchange timed out waiting for another rank (no-op for RCCL)."""
    if comm and lib().ia_peer_mem_kind(comm) >= 0:
        check(lib().ia_peer_status(comm), 'ia_peer_status')


def pyr_form(stream=-1, oh=0):
    """ia_pyr_reduce_f64's kernels for this process (1 the one-pass k_pyr_wave where the
    coefficients are a halving [default], 0 the tiled k_pyr_reduce only); returns the
    previous flag."""
    return lib().ia_diag_set_pyr_form(int(stream), int(oh))
