"""ia_pyr_reduce_f64 at 2048^2 -> 1024^2 (the c4 A level): HIP-event time of the C entry
per form / streaming block height, median of 50 (diagnostic; `python tools/pyr_sweep.py` on the GPU box)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (sets up the package path)
import torch  # noqa: E402

import _ia  # noqa: E402
import img_preprocess as ip  # noqa: E402


def main():
    lib = _ia.lib()
    H = W = 2048
    img = torch.rand((H, W), dtype=torch.float64, device='cuda')
    out = torch.empty((1024, 1024), dtype=torch.float64, device='cuda')
    ws = _ia.workspace(lib.ia_pyr_workspace_bytes(H, W))
    coef = (ctypes.c_double * 4)(*ip.resize_coeffs((H, W), (1024, 1024)))
    taps = (ctypes.c_double * 4)(*ip.PYR_TAPS)
    st = torch.cuda.current_stream()
    ref = None
    forms = [(0, 16), (1, 16)]
    if os.environ.get('PYR_FORMS'):      # e.g. "1:16,0:16"
        forms = [tuple(int(v) for v in f.split(':')) for f in os.environ['PYR_FORMS'].split(',')]
    for form, oh in forms:
        _ia.pyr_form(form, oh)
        def call():
            _ia.check(lib.ia_pyr_reduce_f64(_ia.ptr(img), H, W, _ia.ptr(out), 1024, 1024, coef, taps,
                                            _ia.ptr(ws), _ia.stream()), 'ia_pyr_reduce_f64')

        def med(batch):
            ts = []
            for _ in range(22):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(batch):
                    call()
                e1.record(st)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / batch)
            ts = sorted(ts[2:])
            return ts[len(ts) // 2], ts[0]
        lone, _ = med(1)
        us, tmin = med(10)
        ts = [tmin]
        same = ref is None or torch.equal(out, ref)
        if ref is None:
            ref = out.clone()
        print('form %d: %6.1f us per call in batches of 10 (min %6.1f) %7.1f GB/s; lone call %6.1f us; same=%s'
              % (form, us, ts[0], 8 * (H * W + 1024 * 1024) / us / 1e3, lone, same), flush=True)


if __name__ == '__main__':
    main()
