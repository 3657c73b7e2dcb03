"""Seed / demodulation timestamp probe (diagnostics): runs record-pipeline steps
with dfmi_set_tuning("probe", 1) and prints, per step, when the seed wave and the
bulk demodulation's first/last workgroups started, relative to the demod start (us)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from deepfmkit_amd import _lib  # noqa: E402
from deepfmkit_amd import fit as F  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402


def main():
    torch.cuda.set_device(0)
    lib = _lib.load()
    nseg, R, nd = 100000, 4000, 10
    x = bench.gen_shard(torch, torch.device("cuda", 0), 0, nseg, R, seed=1)
    st = torch.cuda.current_stream()
    out = torch.empty((6, nseg), dtype=torch.float64, device="cuda")
    ok = torch.empty(nseg, dtype=torch.int32, device="cuda")
    guess = np.array([1.6, 6.0, 0.0, 0.0])
    cfg = F.lm_config()
    for k, v in [kv.split("=") for kv in filter(None, os.environ.get("SETTINGS", "").split(","))]:
        _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), k)
    _lib.check(lib.dfmi_set_tuning(b"probe", 1), "probe")
    buf = (ctypes.c_int64 * 16)()
    rows = []
    for i in range(8):
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0_of(1000.0, 200000.0), 0,
                                       _lib.ptr(guess), 1, nseg - 1, cfg, out.data_ptr(), ok.data_ptr(),
                                       _lib.DFMI_MEM_DEVICE, st.cuda_stream), "nls_record")
        _lib.check(lib.dfmi_probe_read(buf, 6), "probe_read")
        t = [int(v) for v in buf[:6]]
        d0 = t[3]
        rows.append({"seed_in": (t[0] - d0) / 100, "seed_folded": (t[1] - d0) / 100, "seed_fitted": (t[2] - d0) / 100,
                     "demod_last_wg_in": (t[4] - d0) / 100, "demod_wg0_out": (t[5] - d0) / 100})
    print(json.dumps({"us_rel_to_demod_wg0_entry": rows}, indent=1))


if __name__ == "__main__":
    main()
