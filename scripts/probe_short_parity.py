"""Short-segment parity study (round 6): at R = 200 / 1000 (1 and 5 modulation cycles per
segment), how far the record pipeline's fits land from the numpy oracle for

  wide   the default record path (demod_wide_kernel QI),
  bins   demod_wide = 0 (the bin / fold kernels),
  exact  the LM alone (dfmi_lm) fed numpy's own QI (oracle.demod_buffer, computed here on
         the host): what an exact-order demodulation would give.

One JSON line per (R, ndata, variant): fits beyond 1e-9 / 5e-10, max |d|, and the QI's
distance from numpy's (max abs, fraction of components bit-identical)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def np_qi(X, nd, w0):
    """numpy's QI of every row of X (nseg, R): the reference's products and np.mean."""
    R = X.shape[1]
    t = np.arange(R)
    out = np.empty((2 * nd, X.shape[0]))
    for k in range(nd):
        ang = (k + 1) * w0 * t
        c, s = np.cos(ang), np.sin(ang)
        for i0 in range(0, X.shape[0], 4096):
            blk = X[i0:i0 + 4096]
            out[k, i0:i0 + 4096] = np.array([(row * c).mean() for row in blk])
            out[k + nd, i0:i0 + 4096] = np.array([(row * s).mean() for row in blk])
    return out


def dist(gp, ref):
    d = np.abs(gp[:, :4] - ref[:, :4])
    d[:, 2] = np.abs((gp[:, 2] - ref[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    return d


def main():
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    from oracle import nls_oracle as O
    import tempfile
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    w0 = w0_of(1000.0, 200000.0)
    cfg = F.lm_config()
    cases = [(200, 10, 100_000), (200, 15, 50_000), (1000, 10, 50_000)]
    if len(sys.argv) > 1:
        cases = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1].split(":")]
    for r, nd, nseg in cases:
        xd = bench.gen_shard(torch, dev, 0, nseg, r, seed=bench.SEED)
        x = xd.cpu().numpy()
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "x.f64")
            x.tofile(path)
            ref = O.fit_file_chunk1(path, nseg, r, nd, 1000.0, 200000.0, max(1, bench.cpu_share()[0]))
        ok = ref[:, 6] == 0
        qn = np_qi(x.reshape(nseg, r), nd, w0)
        for i in (0, 1, nseg // 2, nseg - 1):  # the vectorised QI are numpy's per-buffer ones
            assert np.array_equal(qn[:, i], O.demod_buffer(x[i * r:(i + 1) * r], nd, w0))

        def record(tune):
            for k, v in tune.items():
                _lib.check(lib.dfmi_set_tuning(k.encode(), v), "tune")
            out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
            sk = torch.empty(nseg, dtype=torch.int32, device=dev)
            g = np.array([1.6, 6.0, 0.0, 0.0])
            _lib.check(lib.dfmi_nls_record(xd.data_ptr(), 1, nseg * r, nseg, r, nd, w0, 0, _lib.ptr(g), 1, nseg - 1,
                                           cfg, out.data_ptr(), sk.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "rec")
            qd = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
            dd = torch.empty(nseg, dtype=torch.float64, device=dev)
            _lib.check(lib.dfmi_demod(xd.data_ptr(), nseg, r, r, nd, w0, 0, qd.data_ptr(), dd.data_ptr(),
                                      _lib.DFMI_MEM_DEVICE, st), "demod")
            torch.cuda.synchronize()
            kn = lib.dfmi_last_demod_kernel().decode()
            for k in tune:
                _lib.check(lib.dfmi_set_tuning(k.encode(), 1), "tune")
            return out.cpu().numpy().T, sk.cpu().numpy(), qd.cpu().numpy(), kn

        def exact():
            qd = torch.from_numpy(np.ascontiguousarray(qn[:, 1:])).to(dev)
            n1 = nseg - 1
            prm = torch.empty((4, n1), dtype=torch.float64, device=dev)
            ssq = torch.empty(n1, dtype=torch.float64, device=dev)
            sk = torch.empty(n1, dtype=torch.int32, device=dev)
            gd = torch.from_numpy(np.ascontiguousarray(ref[0, :4])).to(dev)
            _lib.check(lib.dfmi_lm(qd.data_ptr(), n1, nd, gd.data_ptr(), 0, n1, cfg, prm.data_ptr(), ssq.data_ptr(),
                                   sk.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "lm")
            torch.cuda.synchronize()
            gp = np.zeros((nseg, 6))
            gp[0, :4] = ref[0, :4]
            gp[1:, :4] = prm.cpu().numpy().T
            gp[1:, 5] = ssq.cpu().numpy()
            gs = np.zeros(nseg, dtype=np.int32)
            gs[1:] = sk.cpu().numpy()
            gs[0] = int(ref[0, 6])
            return gp, gs, qn, "host numpy QI + dfmi_lm"

        for name, fn in (("wide", lambda: record({})), ("bins", lambda: record({"demod_wide": 0})), ("exact", exact)):
            gp, gs, qi, kn = fn()
            d = dist(gp, ref)
            d[~ok] = 0
            dm = d.max(axis=1)
            qdiff = np.abs(qi - qn)
            print(json.dumps({"R": r, "ndata": nd, "segments": nseg, "variant": name, "kernel": kn,
                              "status_equal": bool(np.array_equal(gs, ref[:, 6].astype(int))),
                              "status_mismatch": int(np.sum(gs != ref[:, 6].astype(int))),
                              "beyond_1e-9": int(np.sum(dm > 1e-9)), "beyond_5e-10": int(np.sum(dm > 5e-10)),
                              "max_d": [float(v) for v in d.max(axis=0)],
                              "qi_max_abs_vs_numpy": float(qdiff.max()),
                              "qi_bit_identical_frac": float(np.mean(qi == qn))}), flush=True)
        del xd


if __name__ == "__main__":
    main()
