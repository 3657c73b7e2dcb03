"""The aperture-checked debug build (ab/libdfmi_dbg.so, -DDFMI_DEBUG_ROWS: every
demodulation-row store traps unless its pointer lies in the address space the store is
compiled for, demod.h row_put) runs the record pipeline — the fused seed + demodulation
kernel whose seed writes its row to LDS and whose bulk waves write rows to global memory,
then the LM — and gives the product build's bits. Round 3 met an aperture-violation fault
when an A/B variant stored the seed's LDS row with a global-only instruction; this build
would trap on any such store."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(ROOT, "ab", "libdfmi_dbg.so")


def test_debug_rows_build_runs_the_pipeline_bit_identically():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(DBG):
        pytest.fail("ab/libdfmi_dbg.so missing: run __graft_entry__.build()")
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    lib = _lib.load()
    dbg = ctypes.CDLL(DBG, mode=ctypes.RTLD_LOCAL)
    dbg.dfmi_nls_record.argtypes = lib.dfmi_nls_record.argtypes
    dbg.dfmi_nls_record.restype = ctypes.c_int
    dbg.dfmi_last_demod_kernel.restype = ctypes.c_char_p
    R, nseg = 4000, 3001
    dev = torch.device("cuda", 0)
    x = torch.empty(2 * nseg * R, dtype=torch.float64, device=dev)
    for c, m in enumerate((6.0, 4.3)):  # two records: two seed workgroups
        bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED, m_true=m, stream=c, out=x[c * nseg * R:(c + 1) * nseg * R])
    g = np.ascontiguousarray(np.tile([1.6, 6.0, 0.0, 0.0], (2, 1)))
    outs = []
    for L in (lib, dbg):
        out = torch.empty((6, 2 * nseg), dtype=torch.float64, device=dev)
        st = torch.empty(2 * nseg, dtype=torch.int32, device=dev)
        rc = L.dfmi_nls_record(x.data_ptr(), 2, nseg * R, nseg, R, 10, w0_of(1000.0, 200000.0), 0, _lib.ptr(g), 1,
                               nseg - 1, F.lm_config(), out.data_ptr(), st.data_ptr(), _lib.DFMI_MEM_DEVICE,
                               torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        assert L.dfmi_last_demod_kernel().decode().startswith("demod_seed_bins_kernel")
        outs.append((out.cpu().numpy(), st.cpu().numpy()))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert (outs[0][1] == 0).all()
