"""Multi-process (gloo, world_size 2, CPU) rehearsal of bench.py's sharded path:
every rank fits its contiguous shard seeded from the record's buffer 0 with no
data-path collective, and the union equals the unsharded _fit_parallel with chunk
size 1 (here with the oracle as the engine — the GPU engine is covered by
tests/test_gpu_parity.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nseg, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    import bench
    from oracle import nls_oracle as O
    from tests.conftest import make_record  # noqa: F401
    import deepfmkit_amd as dfm
    R = 4000
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    sim = dfm.DFMIObject("mp", laser, ifo, f_samp=200000.0)
    x = dfm.SignalGenerator().generate(sim, world * nseg * R / 200000.0, mode="snr", snr_db=40.0,
                                       trial_num=3)["main"].samples()
    seg0, nbuf, prepend = bench.shard_plan(rank, world, nseg)
    local = x[seg0 * R:(seg0 + nseg) * R]
    if prepend:
        local = np.concatenate([x[:R], local])
    assert local.size == nbuf * R
    # _fit_parallel semantics on the local batch, chunk size 1 (every buffer its own chunk)
    out = O.fit_record_parallel(local, 200000.0, 1000.0, 20, n_cores=max(nbuf - 1, 1),
                                pool=type("P", (), {"imap": lambda self, f, j: map(f, j)})())
    mine = out[1:] if prepend else out
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's timing reduction
    gathered = [None] * world
    dist.all_gather_object(gathered, (seg0, mine))
    if rank == 0:
        q.put((float(t.item()), gathered, x))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_unsharded():
    world, nseg = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nseg, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, gathered, x = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert tmax == 2.0
    gathered.sort(key=lambda g: g[0])
    assert [g[0] for g in gathered] == [0, nseg]
    sharded = np.concatenate([g[1] for g in gathered])
    from oracle import nls_oracle as O
    whole = O.fit_record_parallel(x, 200000.0, 1000.0, 20, n_cores=world * nseg - 1,
                                  pool=type("P", (), {"imap": lambda self, f, j: map(f, j)})())
    np.testing.assert_array_equal(sharded, whole)


def test_shard_plan_covers_record_once():
    import bench
    for world in (1, 2, 4, 8):
        seen = []
        for r in range(world):
            s0, nbuf, pre = bench.shard_plan(r, world, 100)
            assert nbuf == 100 + (1 if pre else 0)
            assert pre == (r > 0)
            seen.extend(range(s0, s0 + 100))
        assert seen == list(range(world * 100))
