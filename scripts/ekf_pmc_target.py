"""Profile target for the config-5 EKF (rocprofv3 --pmc passes, scripts/gpu_ekf_pmc.sh):
EKFFitter.fit on ONE 2 s = 400,000-sample channel (m = 6, 40 dB, counter-based input),
through dfmi_ekf_fit with the default kernel (ekf_rot_kernel<16> for one channel), REPS
fits after one warm fit. Prints one JSON line (kernel name, s per fit, samples)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    nch = int(os.environ.get("NCH", 1))
    reps = int(os.environ.get("REPS", 3))
    ns, R = 400_000, 4000
    xe = torch.empty(nch * ns, dtype=torch.float64, device=dev)
    for c in range(nch):
        synth_snr(SnrSpec(seed=1234, stream=100 + c, f_samp=200000.0, f_mod=1000.0, m=6.0, snr_db=40.0), 0, ns,
                  out=xe[c * ns:(c + 1) * ns])
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0 = torch.ones(5, dtype=torch.float64, device=dev)
    qd = torch.tensor([1e-8, 1e-8, 1e-6, 1e-6, 1e-8], dtype=torch.float64, device=dev)
    st = torch.empty((nch, ns // R, 5), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()

    def fit():
        _lib.check(lib.dfmi_ekf_fit(xe.data_ptr(), nch, ns, ns, init4.data_ptr(), p0.data_ptr(), qd.data_ptr(), None,
                                    2 * np.pi * 1000.0, 200000.0, R, ns // R, st.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                    s.cuda_stream), "dfmi_ekf_fit")

    fit()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fit()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"kernel": lib.dfmi_last_demod_kernel().decode(), "channels": nch, "samples": ns,
                      "s_per_fit": dt, "samples_per_s_per_channel": ns / dt, "fits": reps + 1}), flush=True)


if __name__ == "__main__":
    main()
