"""A/B of the many-harmonic demodulation (demod_wide_kernel) at config 2 (100,000 x 4000):
segments per wave (demod_wide_k) and the fold / contraction / store split (demod_wide_dbg), at ndata 10 / 16 (forced, against the
bin kernel) and 20 / 30 / 62. HIP events over 40 launches after 5 warm ones."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import w0_of
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    R, nseg = 4000, 100_000
    x = torch.empty(nseg * R, dtype=torch.float64, device=dev)
    bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED, out=x)
    w0 = w0_of(1000.0, 200000.0)
    st = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def tune(**kw):
        for k, v in kw.items():
            _lib.check(lib.dfmi_set_tuning(k.encode(), v), "tune")

    for nd in (10, 20, 30, 62):
        qi = torch.empty((2 * nd + 1, nseg), dtype=torch.float64, device=dev)  # +1 row: dbg 8 writes nseg x (2 nd + 1)
        dc = torch.empty(nseg, dtype=torch.float64, device=dev)

        def run():
            _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(),
                                      _lib.DFMI_MEM_DEVICE, st.cuda_stream), "dfmi_demod")
        variants = [dict(demod_wide=0)] + [dict(demod_wide=2, demod_wide_k=k, demod_wide_dbg=d)
                                          for k in (4, 8) for d in (0, 1, 2, 3)]
        for v in variants:
            tune(**v)
            for _ in range(5):
                run()
            ev0.record(st)
            for _ in range(40):
                run()
            ev1.record(st)
            ev1.synchronize()
            ms = ev0.elapsed_time(ev1) / 40
            print(json.dumps({"ndata": nd, **v, "kernel": lib.dfmi_last_demod_kernel().decode(), "ms": round(ms, 4),
                              "hbm_frac": round(nseg * (8 * R + 8 * (2 * nd + 1)) / (ms * 1e-3) / 8e12, 4)}), flush=True)
            tune(demod_wide=1, demod_wide_k=0, demod_wide_dbg=0)
        del qi, dc


if __name__ == "__main__":
    main()
