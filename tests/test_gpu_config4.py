"""GPU checks of BASELINE config 4 (one 10M-segment record split over 8 GPUs,
1.25M segments = 40 GB per GPU) and of the counter-based input generator the
sharded bench uses (dfmi_synth_snr, csrc/snrgen.hip).

- the device generator vs its CPU restatement (oracle/philox.py): integer stream
  bit-exact by construction (Random123 known answers pinned in
  tests/test_api_contract.py), floats within a few ulps (device log/sin/cos);
  any window regenerated alone is bit-identical to the same samples of a longer one;
- a full 1.25M-segment shard on one GPU: noiseless known answer in every segment,
  seed independence (a slice refitted alone == the same segments of the shard,
  bit for bit) and, on the noisy record, parity of a far-end subset with the CPU
  oracle on the same bytes (tolerances of SURVEY.md §8d);
- two ranks (gloo, both on this one GPU) fitting contiguous shards of one record,
  each regenerating and fitting buffer 0 itself: the union equals the unsharded
  fit bit for bit (fitters.py:403-416: every chunk is seeded from buffer 0).
"""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import compare_fit, wrapped

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R = 4000


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_snr_generator_matches_restatement():
    import torch
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    from oracle.philox import snr_samples
    spec = SnrSpec(seed=1234, m=6.0, snr_db=40.0)
    # windows: record start, an odd start/length, the last segment of a 10M-segment record
    for idx0, n in ((0, 8000), (4000 * 1234567 + 3, 4001), (4000 * 9_999_999, 4000)):
        dev = synth_snr(spec, idx0, n, out=torch.empty(n, dtype=torch.float64, device="cuda")).cpu().numpy()
        host = snr_samples(spec, idx0, n)
        assert np.abs(dev - host).max() <= 1e-13, (idx0, np.abs(dev - host).max())
        assert np.mean(dev == host) > 0.5
    # split invariance on the device: any window == the same samples of a longer draw
    big = synth_snr(spec, 1000, 20001, out=torch.empty(20001, dtype=torch.float64, device="cuda")).cpu().numpy()
    for a, b in ((1000, 1001), (1001, 9000), (4000, 21001), (7777, 7778)):
        part = synth_snr(spec, a, b - a, out=torch.empty(b - a, dtype=torch.float64, device="cuda")).cpu().numpy()
        np.testing.assert_array_equal(part, big[a - 1000:b - 1000])
    # the host-memory path returns the same bytes
    np.testing.assert_array_equal(synth_snr(spec, 1001, 8000), big[1:8001])


def _shard_record(spec, nseg):
    import torch
    from deepfmkit_amd.physics import synth_snr
    x = torch.empty(nseg * R, dtype=torch.float64, device="cuda")
    synth_snr(spec, 0, nseg * R, out=x)
    return x.reshape(1, -1)


def test_config4_shard_known_answer_and_seed_independence():
    """1,250,000 segments (config 4's per-GPU shard, 40 GB resident) in one call."""
    import torch
    from deepfmkit_amd.fitters import nls_records
    from deepfmkit_amd.physics import SnrSpec
    nseg = 1_250_000
    x = _shard_record(SnrSpec(seed=5, m=6.0, phi=0.3, psi=0.1, snr_db=None), nseg)
    cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, 10)
    c = cols.cpu().numpy()
    assert (ok.cpu().numpy() == 0).all()
    assert np.abs(c[0] - 1.0).max() < 1e-9
    assert np.abs(c[1] - 6.0).max() < 1e-9
    assert wrapped(c[2] - 0.3).max() < 1e-9
    assert np.abs(c[3] - 0.1).max() < 1e-9
    # seed independence: buffer 0 + segments [1_000_000, 1_000_100) fitted alone
    sub = torch.cat([x[:, :R], x[:, 1_000_000 * R:1_000_100 * R]], dim=1).contiguous()
    c2, _ = nls_records(sub, 200000.0, 1000.0, R, 101, 10)
    np.testing.assert_array_equal(c2.cpu().numpy()[:, 1:], c[:, 1_000_000:1_000_100])
    del x, sub, cols
    torch.cuda.empty_cache()


def test_config4_shard_noisy_parity_far_end():
    """The noisy 40 dB shard: every segment converges (status 0); its last 48 segments
    agree with the CPU oracle fitting the same bytes, seeded by buffer 0 as
    _fit_parallel seeds every chunk (chunk size 1)."""
    import torch
    from deepfmkit_amd.fitters import nls_records, w0_of
    from deepfmkit_amd.physics import SnrSpec
    from oracle import nls_oracle as O
    nseg = 1_250_000
    x = _shard_record(SnrSpec(seed=1234, m=6.0, snr_db=40.0), nseg)
    cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, 10)
    ok = ok.cpu().numpy()
    c = cols.cpu().numpy()
    assert (ok == 0).all()
    assert abs(c[1].mean() - 6.0) < 1e-5
    buf0 = x[0, :R].cpu().numpy()
    tail = x[0, (nseg - 48) * R:].cpu().numpy().reshape(48, R)
    del x, cols
    torch.cuda.empty_cache()
    w0 = w0_of(1000.0, 200000.0)
    st0, p0, _ = O.fit_segment(10, O.demod_buffer(buf0, 10, w0), np.array([1.6, 6.0, 0.0, 0.0]))
    ref = np.array([O.fit_chunk((tail[i:i + 1], p0[:4], 10, 1000.0, 200000.0, dict(O.C0)))[0] for i in range(48)])
    ours = {k: c[i, nseg - 48:] for i, k in enumerate(("amp", "m", "phi", "psi", "dc", "ssq"))}
    ours["fitok"] = ok[nseg - 48:]
    compare_fit(ours, {"amp": ref[:, 0], "m": ref[:, 1], "phi": ref[:, 2], "psi": ref[:, 3], "dc": ref[:, 4],
                       "ssq": ref[:, 5], "fitok": ref[:, 6]}, tol=1e-9)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, nseg, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from deepfmkit_amd.fitters import nls_records
        torch.cuda.set_device(0)
        seg0, nbuf, prepend = bench.shard_plan(rank, world, nseg)
        x = torch.empty(nbuf * R, dtype=torch.float64, device="cuda")
        if prepend:
            bench.gen_shard(torch, "cuda", 0, 1, R, seed=77, out=x[:R])
        bench.gen_shard(torch, "cuda", seg0, nseg, R, seed=77, out=x[(nbuf - nseg) * R:])
        cols, ok = nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, nbuf, 10)
        cols, ok = cols.cpu().numpy(), ok.cpu().numpy()
        mine = (seg0, cols[:, 1:] if prepend else cols, ok[1:] if prepend else ok)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        if rank == 0:
            q.put(gathered)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_equal_unsharded_bit_for_bit():
    import torch
    import torch.multiprocessing as mp
    import bench
    from deepfmkit_amd.fitters import nls_records
    world, nseg = 2, 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, nseg, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        gathered = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    gathered.sort(key=lambda g: g[0])
    assert [g[0] for g in gathered] == [0, nseg]
    sharded = np.concatenate([g[1] for g in gathered], axis=1)
    sharded_ok = np.concatenate([g[2] for g in gathered])
    x = bench.gen_shard(torch, "cuda", 0, world * nseg, R, seed=77)
    cols, ok = nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, world * nseg, 10)
    np.testing.assert_array_equal(sharded, cols.cpu().numpy())
    np.testing.assert_array_equal(sharded_ok, ok.cpu().numpy())
