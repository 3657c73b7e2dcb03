"""The LM inside the seed + demodulation launch (seed.h demod_seed_bins_lm_kernel,
dfmi_set_tuning("lm_fused", 1)) against the two-kernel record pipeline (the fused seed +
demodulation launch, then lm_chunks_kernel): the same register-path LM on the same rows,
so every column and status must be bit-identical (StandardNLSFitter._fit_parallel,
fitters.py:403-423). Layouts: one config-2 record (100,000 segments), several records whose
64-segment LM tiles straddle record boundaries (seed buffers inside tiles), a segment
count that is not a multiple of 64, and back-to-back calls (the per-tile counters reset
by the LM waves, the seed flags' epochs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _records(nrec, nbuf, seed):
    import torch
    R = 4000
    t = torch.arange(nbuf * R, dtype=torch.float64, device="cuda") / 200000.0
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    ms = torch.linspace(5.0, 7.0, nrec, dtype=torch.float64, device="cuda")[:, None]
    x = 1.0 + torch.cos(0.3 + ms * torch.cos(2 * np.pi * 1000.0 * t[None, :] + 0.1))
    x += 1e-2 * torch.randn(x.shape, dtype=torch.float64, device="cuda", generator=g)
    return x.contiguous()


def _fit(lib, x, fused, nbuf):
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import nls_records
    _lib.check(lib.dfmi_set_tuning(b"lm_fused", fused), "tune")
    try:
        cols, ok = nls_records(x, 200000.0, 1000.0, 4000, nbuf, 10)
        name = lib.dfmi_last_demod_kernel().decode()
    finally:
        _lib.check(lib.dfmi_set_tuning(b"lm_fused", 1), "tune")
    return cols.cpu().numpy(), ok.cpu().numpy(), name


@pytest.mark.parametrize("nrec,nbuf", [(1, 100000), (3, 20000), (2, 12345)])
def test_fused_lm_bit_identical_to_two_kernel_path(nrec, nbuf):
    import torch  # noqa: F401  (torch's HIP runtime first, then libdfmi)
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = _records(nrec, nbuf, 3 + nrec)
    a_cols, a_ok, a_name = _fit(lib, x, 1, nbuf)
    assert a_name.startswith("demod_seed_bins_lm_kernel"), a_name
    b_cols, b_ok, b_name = _fit(lib, x, 0, nbuf)
    assert b_name.startswith("demod_seed_bins_kernel"), b_name
    assert not (a_ok == -3).any(), "an LM wait timed out"
    np.testing.assert_array_equal(a_ok, b_ok)
    np.testing.assert_array_equal(a_cols, b_cols)
    assert (a_ok == 0).mean() > 0.99
    # back to back: the tile counters and seed epochs of the previous call must not leak
    c_cols, c_ok, _ = _fit(lib, x, 1, nbuf)
    np.testing.assert_array_equal(c_cols, a_cols)
    np.testing.assert_array_equal(c_ok, a_ok)


def test_fused_lm_steps_aside_below_ladder_threshold():
    """Small batches (at most lm_ladder x CUs fits) keep the latency-bound ladder LM after
    the fused seed + demodulation launch."""
    import torch  # noqa: F401
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = _records(1, 2000, 9)
    _, ok, name = _fit(lib, x, 1, 2000)
    assert name.startswith("demod_seed_bins_kernel"), name
    assert (ok == 0).all()
