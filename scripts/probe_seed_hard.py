"""Where a hard record's step goes (records whose phase the default guess does not reach):
the fused seed + demodulation launch vs the LM launch (dfmi_step_timing events), and inside
the fused launch the seed workgroup's own timestamps (dfmi_set_tuning('probe', 1):
s_memrealtime at entry / after the fold / after the fit, 100 MHz). One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    R = 4000
    nseg = int(os.environ.get("NSEG", 20000))
    res = {}
    x = torch.empty(nseg * R, dtype=torch.float64, device=dev)
    out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
    ok = torch.empty(nseg, dtype=torch.int32, device=dev)
    g = np.array([1.6, 6.0, 0.0, 0.0])
    st = torch.cuda.current_stream().cuda_stream
    for phi, psi in ((0.0, 0.0), (1.3, 0.4), (1.0, 1.0)):
        synth_snr(SnrSpec(seed=bench.SEED, f_samp=200000.0, f_mod=1000.0, m=6.0, phi=phi, psi=psi, snr_db=40.0), 0,
                  nseg * R, out=x)

        def step():
            _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, 10, w0_of(1000.0, 200000.0), 0,
                                           _lib.ptr(g), 1, nseg - 1, F.lm_config(), out.data_ptr(), ok.data_ptr(),
                                           _lib.DFMI_MEM_DEVICE, st), "nls")
        step()
        _lib.check(lib.dfmi_set_tuning(b"probe", 1), "probe")
        _lib.check(lib.dfmi_step_timing(1), "t")
        step()
        _lib.check(lib.dfmi_step_timing(0), "t")
        torch.cuda.synchronize()
        pr = np.zeros(6, dtype=np.int64)
        _lib.check(lib.dfmi_probe_read(_lib.ptr(pr), 6), "probe_read")
        _lib.check(lib.dfmi_set_tuning(b"probe", 0), "probe")
        td, tl, tn = np.zeros(1), np.zeros(1), np.zeros(1, dtype=np.int64)
        _lib.check(lib.dfmi_step_timing_read(_lib.ptr(td), _lib.ptr(tl), _lib.ptr(tn)), "read")
        res[f"phi={phi},psi={psi}"] = {"fused_ms": round(float(td[0]), 4), "lm_ms": round(float(tl[0]), 4),
                                       "seed_fold_us": round((pr[1] - pr[0]) / 100.0, 2),
                                       "seed_fit_us": round((pr[2] - pr[1]) / 100.0, 2),
                                       "seed_status": int(ok[0].item()), "status_counts":
                                       np.bincount(ok.cpu().numpy(), minlength=3).tolist()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
