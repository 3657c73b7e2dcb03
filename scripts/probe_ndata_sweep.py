"""Config 2 (100,000 segments x R = 4000, 40 dB snr-mode record resident in HBM) at ndata 10 ..
62 ("for ndata >= 20 the demodulation crosses the ridge; report that
separately"). Per ndata: the record pipeline's step (dfmi_nls_record, parallel semantics),
the row demodulation alone (dfmi_demod_rows) and the LM alone over component-major QI
(dfmi_lm), HIP events on the launch stream, mean over many launches; the demodulation's
HBM fraction at 8R + 8(2 ndata + 1) bytes per segment, and the status-0 fraction.

The binned demodulation folds each segment into L phase bins (R adds) and contracts the bins
with the basis (2 ndata L FMAs, L = 200): at ndata 62 that is 24,800 FMAs per 4,000 samples
read, so the demodulation stays HBM-bound where a per-sample basis product (4 ndata R flops)
would not; what grows with ndata is the LM (Bessel orders, harmonic sums).
env: MTRUE (the record's m, 6.0; the step's buffer 0 is fitted from the default guess m = 6 either
way), NDS (the ndata list)."""
import json
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of

    lib = _lib.load()
    dev = torch.device("cuda", 0)
    R = 4000
    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    tune = dict(kv.split("=") for kv in sys.argv[2].split("+")) if len(sys.argv) > 2 and sys.argv[2] else {}
    for k, v in tune.items():  # e.g. lm_onepass=0
        _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), "tune")
    m_true = float(os.environ.get("MTRUE", 6.0))  # the record's m (31.4: the reference quickstart's)
    nds = [int(v) for v in os.environ.get("NDS", "10,12,16,20,30,40,62").split(",")]
    x = torch.empty(nseg * R, dtype=torch.float64, device=dev)
    bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED, m_true=m_true, out=x)
    w0 = w0_of(1000.0, 200000.0)
    cfg = F.lm_config()
    stream = torch.cuda.current_stream()
    guess = np.array([1.6, 6.0, 0.0, 0.0])
    out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
    ok = torch.empty(nseg, dtype=torch.int32, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, n):
        for _ in range(5):
            fn()
        ev0.record(stream)
        for _ in range(n):
            fn()
        ev1.record(stream)
        ev1.synchronize()
        return ev0.elapsed_time(ev1) / n

    for nd in nds:
        rows = torch.empty((nseg, lib.dfmi_qi_row_stride(nd)), dtype=torch.float64, device=dev)
        qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
        dcb = torch.empty(nseg, dtype=torch.float64, device=dev)
        lo = torch.empty((4, nseg), dtype=torch.float64, device=dev)
        ls = torch.empty(nseg, dtype=torch.float64, device=dev)
        lk = torch.empty(nseg, dtype=torch.int32, device=dev)
        g = torch.tensor([1.0, m_true, 0.0, 0.0], dtype=torch.float64, device=dev)

        def step():
            _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, _lib.ptr(guess), 1,
                                           nseg - 1, cfg, out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                           stream.cuda_stream), "dfmi_nls_record")

        def demod():
            _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0, 0, rows.data_ptr(),
                                           _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_demod_rows")

        def lm():
            _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, g.data_ptr(), 0, nseg, cfg, lo.data_ptr(), ls.data_ptr(),
                                   lk.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_lm")

        step_ms = timed(step, 60)
        step_kernel = lib.dfmi_last_demod_kernel().decode()
        st = ok.cpu().numpy()
        m = out[1].cpu().numpy()
        def demod_cm():  # component-major QI (the layout of the record pipeline beyond the row layout)
            _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dcb.data_ptr(),
                                      _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_demod")

        try:
            demod_ms = timed(demod, 60)
            layout = "rows"
        except _lib.DFMIError:
            demod_ms = timed(demod_cm, 60)
            layout = "component-major"
        demod_kernel = lib.dfmi_last_demod_kernel().decode()
        demod_cm()
        lm_ms = timed(lm, 60)
        import hashlib  # bit-identity across tuning variants: digests of the step's and the LM's outputs
        out_sha = hashlib.sha256(out.cpu().numpy().tobytes() + ok.cpu().numpy().tobytes()).hexdigest()[:16]
        lm_sha = hashlib.sha256(lo.cpu().numpy().tobytes() + ls.cpu().numpy().tobytes()
                                + lk.cpu().numpy().tobytes()).hexdigest()[:16]
        bytes_seg = 8 * R + 8 * (2 * nd + 1)
        print(json.dumps({
            "ndata": nd, "m": m_true, "segments": nseg, "R": R, "tune": tune,
            "step_ms": round(step_ms, 4), "segments_per_s": round(nseg / step_ms * 1e3, 1),
            "step_demod_kernel": step_kernel, "demod_layout": layout, "demod_ms": round(demod_ms, 4), "demod_kernel": demod_kernel,
            "demod_hbm_frac": round(nseg * bytes_seg / (demod_ms * 1e-3) / 8e12, 4),
            "lm_ms": round(lm_ms, 4), "end_to_end_frac": round(nseg * (8 * R + 56) / (step_ms * 1e-3) / 8e12, 4),
            "status0_frac": float(np.mean(st == 0)), "mean_m": float(np.mean(m[st == 0])), "out_sha16": out_sha, "lm_sha16": lm_sha}), flush=True)
        del rows, qi, dcb, lo, ls, lk


if __name__ == "__main__":
    main()
