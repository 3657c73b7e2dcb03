"""CPU restatement of dfmi_synth_snr (deepfmkit_amd/csrc/snrgen.hip) — TEST
INFRASTRUCTURE ONLY: checks the device generator of the bench's sharded records.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC'11; the Random123 reference algorithm, no third-party code in this
image) in numpy uint64 arithmetic — bit-exact; the Box-Muller transform and the
signal use numpy's log / cos / sin, so the floats agree with the device's to a few
ulps (checked in tests/test_gpu_config4.py). The known-answer vectors of Random123's
kat_vectors file pin the integer part (tests/test_philox.py)."""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over the counter words (uint64 arrays holding 32-bit values)."""
    c = [np.asarray(v, dtype=np.uint64) & MASK for v in (c0, c1, c2, c3)]
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
    return c


def normals(seed, stream, idx0, n):
    """z_i for i in [idx0, idx0 + n) (Box-Muller pairs over counter i >> 1)."""
    i = np.arange(idx0, idx0 + n, dtype=np.int64)
    j = (i >> 1).astype(np.uint64)
    c = philox4x32_10(j & MASK, j >> np.uint64(32), np.full(j.shape, stream, np.uint64),
                      np.zeros(j.shape, np.uint64), seed & 0xFFFFFFFF, seed >> 32)
    b1 = ((c[0] >> np.uint64(5)) << np.uint64(26)) | (c[1] >> np.uint64(6))
    b2 = ((c[2] >> np.uint64(5)) << np.uint64(26)) | (c[3] >> np.uint64(6))
    u1 = (b1.astype(np.float64) + 1.0) * 2.0 ** -53
    u2 = b2.astype(np.float64) * 2.0 ** -53
    r = np.sqrt(-2.0 * np.log(u1))
    return np.where(i & 1, r * np.sin(2 * np.pi * u2), r * np.cos(2 * np.pi * u2))


def snr_samples(spec, idx0, n):
    """The record of a deepfmkit_amd.physics.SnrSpec, restated on the host."""
    i = np.arange(idx0, idx0 + n, dtype=np.int64)
    ti = i % spec.period if spec.period > 0 else i
    t = ti.astype(np.float64) / spec.f_samp
    w = 2.0 * np.pi * spec.f_mod
    clean = spec.amp * (1.0 + spec.visibility * np.cos(spec.phi + spec.m * np.cos(w * t + spec.psi)))
    return clean + spec.noise_std() * normals(spec.seed, spec.stream, idx0, n)
