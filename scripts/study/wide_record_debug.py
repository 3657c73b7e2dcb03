"""Debug: noiseless m = 12 record at ndata 30 through nls_records, wide vs fold demodulation."""
import numpy as np
import torch
from deepfmkit_amd import _lib
from deepfmkit_amd.fitters import nls_records

lib = _lib.load()
nseg, R = 4000, 4000
t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
seg_phi = torch.linspace(-0.4, 0.4, nseg, dtype=torch.float64, device="cuda")
x = (1.0 + torch.cos(seg_phi[:, None] + 12.0 * torch.cos(2 * np.pi * 1000.0 * t[None, :] + 0.2))).reshape(1, -1)
for wide in (1, 0):
    _lib.check(lib.dfmi_set_tuning(b"demod_wide", wide), "tune")
    for nd in (30, 20):
        cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, nd, init_guess=(1.6, 12.0, 0.0, 0.2))
        k = lib.dfmi_last_demod_kernel().decode()
        cols, ok = cols.cpu().numpy(), ok.cpu().numpy()
        bad = np.where(ok != 0)[0]
        print(wide, nd, k, "bad", bad.size, bad[:10], "m", cols[1][bad[:5]], "ssq", cols[5][bad[:5]],
              "max|dm| ok", np.abs(cols[1][ok == 0] - 12).max() if (ok == 0).any() else None, flush=True)
