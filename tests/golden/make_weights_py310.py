"""Golden weights of the reference's config.py:68-79 under THIS image's Python 3.10 /
numpy 2.2.6 (config.py imports cleanly on 3.10; compute_weights is called with the int
n_half that config_test.py:7,37 uses).  np.exp differs by 1 ulp between numpy 1.26 and
2.2, so the weights are pinned per numpy version: ref_golden.npz holds the 1.26.4 values.

    python tests/golden/make_weights_py310.py
"""
import importlib.util
import os

import numpy as np

spec = importlib.util.spec_from_file_location('ref_config', '/root/reference/config.py')
ref = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ref)
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ref_weights_py310.npz')
np.savez(out, ch1=ref.compute_weights(3, 5, 12, 1), ch3=ref.compute_weights(3, 5, 12, 3),
         numpy_version=np.array(np.__version__))
print('wrote', out)
