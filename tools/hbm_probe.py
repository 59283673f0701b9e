"""Run bench.hbm_kernels once (the bandwidth-bound kernels: YIQ, pyramid reduce, DB build)
as a short process for rocprofv3 kernel traces / PMC passes (`tools/gpu.sh trace TAG -- python tools/hbm_probe.py`)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

print(json.dumps(bench.hbm_kernels(torch.device('cuda:0'), reps=int(os.environ.get('REPS', 5))),
                 indent=1))
