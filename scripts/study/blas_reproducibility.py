"""Is the reference's own fit reproducible to 1e-9 across x86 CPUs? The reference's LM
(fit.py:68-258) calls BLAS / LAPACK through numpy: np.dot(r, r) (ddot), J.T @ J (dgemm /
dsyrk), J.T @ r (dgemv), np.linalg.solve (dgesv). numpy's OpenBLAS picks its kernels by
CPU (DYNAMIC_ARCH; OPENBLAS_CORETYPE overrides). This fits the same record with the numpy
oracle (bit-exact with the reference on the golden vectors) under several core types and
reports how far the answers move between them.

usage: python scripts/study/blas_reproducibility.py fit CORETYPE R ND NSEG OUT.npy
       python scripts/study/blas_reproducibility.py compare R ND NSEG A.npy B.npy ..."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def record(r, nseg):
    from deepfmkit_amd.physics import SnrSpec
    from oracle import philox
    spec = SnrSpec(seed=1234, stream=0, f_samp=200000.0, f_mod=1000.0, m=6.0, snr_db=40.0)
    return philox.snr_samples(spec, 0, nseg * r)


def main():
    if sys.argv[1] == "fit":
        core, r, nd, nseg, out = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
        from oracle import nls_oracle as O
        import threadpoolctl
        arch = [i.get("architecture") for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"]
        x = record(r, nseg)
        path = f"/tmp/blas/x_{r}_{nseg}.f64"
        if not os.path.exists(path):
            x.tofile(path)
        res = O.fit_file_chunk1(path, nseg, r, nd, 1000.0, 200000.0, 8)
        np.save(out, res)
        print(core, "->", arch)
        return
    r, nd, nseg = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    base = np.load(sys.argv[5])
    for f in sys.argv[6:]:
        o = np.load(f)
        ok = (base[:, 6] == 0) & (o[:, 6] == 0)
        d = np.abs(o[:, :4] - base[:, :4])
        d[:, 2] = np.abs((o[:, 2] - base[:, 2] + np.pi) % (2 * np.pi) - np.pi)
        d[~ok] = 0
        dm = d.max(axis=1)
        print(f"{os.path.basename(f)} vs {os.path.basename(sys.argv[5])}: status differ {int(np.sum(o[:, 6] != base[:, 6]))}, "
              f"identical {int(np.sum(dm == 0))}, >5e-10 {int(np.sum(dm > 5e-10))}, >1e-9 {int(np.sum(dm > 1e-9))}, "
              f"max {d.max(axis=0).tolist()}")


if __name__ == "__main__":
    main()
