"""Short segments (n = 1..5 modulation cycles per segment: R = 200..1000 at 200 kS/s / 1 kHz, the
notebooks' CRLB setting StandardNLSFitter({'n': 1, 'ndata': 15})): the record pipeline's step
over 16e7 samples (1.28 GB) at ndata 10 and 15, parallel semantics; HIP-event timing, status-0
fraction and the mean m. One JSON line per point."""
import json
import os
import sys

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
    ns = 160_000_000
    x = torch.empty(ns, dtype=torch.float64, device=dev)
    bench.gen_shard(torch, dev, 0, ns // 4000, 4000, seed=bench.SEED, out=x)
    w0 = w0_of(1000.0, 200000.0)
    cfg = F.lm_config()
    st = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # argv[1]: cycles per segment "1:2:5:20"; argv[2]: tuning variants "/"-separated, each
    # "key=value+key=value" ("" = the defaults)
    cycles = [int(v) for v in sys.argv[1].split(":")] if len(sys.argv) > 1 else [1, 2, 5, 20]
    tunes = [dict(kv.split("=") for kv in a.split("+")) if a else {} for a in
             (sys.argv[2].split("/") if len(sys.argv) > 2 else [""])]
    for ncyc in cycles:
        R = 200 * ncyc
        nseg = ns // R
        out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
        ok = torch.empty(nseg, dtype=torch.int32, device=dev)
        for nd, tune in [(nd, tu) for nd in (10, 15) for tu in tunes]:
            g = np.array([1.6, 6.0, 0.0, 0.0])
            for kk, vv in tune.items():
                _lib.check(lib.dfmi_set_tuning(kk.encode(), int(vv)), "tune")

            def step():
                _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, _lib.ptr(g), 1, nseg - 1,
                                               cfg, out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                               st.cuda_stream), "dfmi_nls_record")
            for _ in range(3):
                step()
            ev0.record(st)
            for _ in range(10):
                step()
            ev1.record(st)
            ev1.synchronize()
            ms = ev0.elapsed_time(ev1) / 10
            k = ok.cpu().numpy()
            m = out[1].cpu().numpy()
            # the demodulation alone (component-major QI) and the LM alone over it
            qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
            dcb = torch.empty(nseg, dtype=torch.float64, device=dev)
            lo = torch.empty((4, nseg), dtype=torch.float64, device=dev)
            ls = torch.empty(nseg, dtype=torch.float64, device=dev)
            lk = torch.empty(nseg, dtype=torch.int32, device=dev)
            gd = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)

            def dem():
                _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dcb.data_ptr(),
                                          _lib.DFMI_MEM_DEVICE, st.cuda_stream), "dfmi_demod")

            def lmf():
                _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, gd.data_ptr(), 0, nseg, cfg, lo.data_ptr(),
                                       ls.data_ptr(), lk.data_ptr(), _lib.DFMI_MEM_DEVICE, st.cuda_stream), "dfmi_lm")
            res = {}
            for name, fn in (("demod_ms", dem), ("lm_ms", lmf)):
                for _ in range(2):
                    fn()
                ev0.record(st)
                for _ in range(10):
                    fn()
                ev1.record(st)
                ev1.synchronize()
                res[name] = round(ev0.elapsed_time(ev1) / 10, 4)
            res["demod_alone_kernel"] = lib.dfmi_last_demod_kernel().decode()
            del qi, dcb, lo, ls, lk
            for kk in tune:
                _lib.check(lib.dfmi_set_tuning(kk.encode(), {"demod_wide": 1, "demod_wide_dbg": 0, "demod_wide_k": 0,
                                                             "demod_wide_half": 1}[kk]), "tune")
            print(json.dumps({"tune": tune, "cycles_per_segment": ncyc, "R": R, "ndata": nd, "segments": nseg, "ms_per_step": round(ms, 4),
                              "segments_per_s": round(nseg / ms * 1e3, 1),
                              "hbm_frac_end_to_end": round(nseg * (8 * R + 56) / (ms * 1e-3) / 8e12, 4),
                              "demod_kernel": lib.dfmi_last_demod_kernel().decode(),
                              "status0_frac": float(np.mean(k == 0)), "mean_m": float(np.mean(m[k == 0])), **res}),
                  flush=True)
        del out, ok


if __name__ == "__main__":
    main()
