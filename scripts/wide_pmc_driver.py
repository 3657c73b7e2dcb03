"""PMC driver: the many-harmonic demodulation alone at config 2 (100,000 x 4000), N launches.
python scripts/wide_pmc_driver.py NDATA DBG [N] (DBG = demod_wide_dbg)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import w0_of
    nd, dbg = int(sys.argv[1]), int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    lib = _lib.load()
    R, nseg = 4000, 100_000
    x = torch.empty(nseg * R, dtype=torch.float64, device="cuda")
    bench.gen_shard(torch, torch.device("cuda", 0), 0, nseg, R, seed=bench.SEED, out=x)
    qi = torch.empty((2 * nd + 1, nseg), dtype=torch.float64, device="cuda")
    dc = torch.empty(nseg, dtype=torch.float64, device="cuda")
    _lib.check(lib.dfmi_set_tuning(b"demod_wide", 2), "tune")
    _lib.check(lib.dfmi_set_tuning(b"demod_wide_dbg", dbg), "tune")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(n):
        _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, qi.data_ptr(),
                                  dc.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "dfmi_demod")
    torch.cuda.synchronize()
    print(lib.dfmi_last_demod_kernel().decode())


if __name__ == "__main__":
    main()
