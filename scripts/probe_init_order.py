"""Does torch still see the GPU when libdfmi initialised HIP first (a host-memory EKF call
before any torch.cuda use)? Prints one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepfmkit_amd import _lib  # noqa: E402

lib = _lib.load()
x = np.cos(np.arange(8192) * 0.03)
st = np.zeros((2, 5))
rc = lib.dfmi_ekf_fit(_lib.ptr(x), 1, x.size, x.size, _lib.ptr(np.array([1.0, 6.0, 0.0, 0.0])), _lib.ptr(np.ones(5)),
                      _lib.ptr(np.full(5, 1e-8)), None, 2 * np.pi * 1000.0, 200000.0, 4000, 2, _lib.ptr(st),
                      _lib.DFMI_MEM_HOST, None)
import torch  # noqa: E402

print(json.dumps({"dfmi_rc": rc, "torch_cuda_available": torch.cuda.is_available(),
                  "device_count": torch.cuda.device_count()}))
