"""Pyramid-reduce kernels (k_blur + k_resample) at 2048^2 and 4096^2, for rocprofv3
--kernel-trace --stats runs (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'image-analogies-python_amd'))
import torch  # noqa: E402
import img_preprocess as ip  # noqa: E402

for n in (2048, 4096):
    img = torch.rand((n, n), dtype=torch.float64, device='cuda')
    for _ in range(20):
        ip.pyramid_reduce_dev(img)
    torch.cuda.synchronize()
print('done')
