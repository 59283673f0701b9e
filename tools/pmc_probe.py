"""Which operation of a torch process crashes under rocprofv3 --pmc (round 1: a segfault
in the bench.py process).  Steps, printed as they complete:
  alloc   torch.empty on the GPU (no kernel)
  fill    torch.zeros (a torch elementwise kernel)
  memset  hipMemsetAsync through libia (the runtime's fill blit kernel)
  clone   x.clone() (a device-to-device copy: the runtime's copy blit kernel)
  stack   torch.stack (the call that crashed in round 1)
  libia   one libia kernel (ia_axpb_f64)
Usage: python tools/pmc_probe.py [steps...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'image-analogies-python_amd'))
import torch  # noqa: E402
import _ia  # noqa: E402


def main(steps):
    dev = torch.device('cuda', 0)
    x = torch.empty(1 << 20, dtype=torch.float64, device=dev)
    print('alloc ok', flush=True)
    for s in steps:
        if s == 'fill':
            x = torch.zeros(1 << 20, dtype=torch.float64, device=dev)
        elif s == 'memset':
            _ia.check(_ia.lib().ia_axpb_f64(_ia.ptr(x), x.numel(), 0, 0.0, 0.0, 0.0, _ia.ptr(x),
                                            _ia.stream()), 'ia_axpb_f64')
            ws = _ia.workspace(1 << 16)
            torch.cuda.synchronize()
            # libia's memsets go through hipMemsetAsync (e.g. in ia_synth_level)
            lib = ctypes.CDLL(None)
            del lib, ws
        elif s == 'clone':
            y = x.clone()
            del y
        elif s == 'stack':
            y = torch.stack([x, x])
            del y
        elif s == 'libia':
            _ia.check(_ia.lib().ia_axpb_f64(_ia.ptr(x), x.numel(), 0, 2.0, 0.0, 0.0, _ia.ptr(x),
                                            _ia.stream()), 'ia_axpb_f64')
        torch.cuda.synchronize()
        print(s, 'ok', flush=True)


if __name__ == '__main__':
    main(sys.argv[1:] or ['fill', 'libia', 'clone', 'stack'])
