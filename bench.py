"""bench.py — segments fitted per second, MI355X DFMI NLS readout (BASELINE.json metric).

One step = one pass of the hot path (StandardNLSFitter._fit_parallel semantics,
fitters.py:395-428) over one batch of synthetic input resident in HBM:
demodulation of every segment, the seed LM fit of buffer 0, and the LM fits of
all remaining segments seeded from it — i.e. (amp, m, phi, psi, dc, ssq, fitok)
for every segment. Workload at N=1: BASELINE config 2 — 100,000 segments of
R = 4000 samples (200 kS/s, f_mod = 1 kHz, n = 20), ndata = 10, fp64.

Multi-GPU (torchrun, one process per GPU): BASELINE config 4 by default — ONE
record of 10,000,000 segments split into contiguous shards of 10M/world segments
(strong scaling; 1.25M = 40 GB per GPU at 8); with --segments, that many per GPU
(weak scaling). No data-path collective: each rank also demodulates/fits the
record's buffer 0 to get the seed, exactly what every reference Pool worker
receives, and regenerates it bit for bit (the input is the counter-based
dfmi_synth_snr record: sample i is a function of (seed, i) only). Timing: barrier
+ synchronize on both sides of exactly K steps, MAX over ranks (all_reduce MAX of
the elapsed time).

Extra JSON fields: roofline (demod kernel, HIP events on the launch stream),
cpu_baseline (oracle restatement of _fit_parallel with a Pool on the host's
cores, rank 0 at N=1 only, bounded sample), parity (max |dphi| of the GPU vs that
oracle on the same sample).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "segments fitted/sec (m,phi,psi,amp) @200 kS/s, 1/2/4/8 GPU; max|Δphi| vs ref"
F_SAMP, F_MOD, N_CYC, NDATA = 200000.0, 1000.0, 20, 10
M_TRUE, SNR_DB = 6.0, 40.0
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CONFIG4_SEGMENTS = 10_000_000  # BASELINE.json config 4: 10M segments over the node's GPUs
SEED = 1234  # key of the counter-based generator (one record for every rank)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps (~63 ms): a 20-step window carries ~0.5 ms of one-time cost
    # (0.658 vs 0.630 ms/step measured on the same box)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--segments", type=int, default=None,
                    help="segments per GPU (default: 100,000 = config 2 on one GPU; with WORLD_SIZE > 1, "
                         "10,000,000 / world = config 4, one 10M-segment record split over the ranks)")
    ap.add_argument("--channels", type=int, default=1,
                    help="records in the batch (config 3: 2 channels, main m=6 and witness m=4.3, each "
                         "seeded by its own buffer 0), segments split evenly; 1 GPU only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="segments in the CPU-baseline sample (default max(8000, 500 per process))")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="Pool size of the CPU baseline (0: every CPU this process may use, bench.cpu_share)")
    ap.add_argument("--demod-only", action="store_true", help="profile helper: time only the demod kernel")
    ap.add_argument("--tune", default="", help="A/B helper: dfmi_set_tuning knobs as key=value[,key=value]")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the extra config keys (config 3, config 5, config 1 sequential) after the timed window")
    ap.add_argument("--rdzv-timeout", type=float, default=120.0,
                    help="seconds a rank waits for the others in init_process_group before it fails")
    ap.add_argument("--launch-timeout", type=float, default=None,
                    help="seconds the self-launcher (--gpus N without torchrun) waits for its ranks "
                         "(default: launch_timeout(), from --steps, --warmup and the segments per rank)")
    return ap.parse_args()


def gen_shard(torch, dev, seg0, nseg, R, seed, chunk=None, m_true=None, stream=0, out=None):
    """Global segments [seg0, seg0+nseg) of the snr-mode record (physics.py:493-530
    formula: A(1 + C cos(phi + m cos(w t + psi))) + white noise at SNR_DB) generated on
    the device by the counter-based dfmi_synth_snr: sample i of the record depends only
    on (seed, stream, i), so every rank regenerates any segment (buffer 0 included) bit
    for bit at any world size."""
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    spec = SnrSpec(seed=seed, stream=stream, f_samp=F_SAMP, f_mod=F_MOD, m=M_TRUE if m_true is None else m_true,
                   snr_db=SNR_DB)
    x = torch.empty(nseg * R, dtype=torch.float64, device=dev) if out is None else out
    synth_snr(spec, seg0 * R, nseg * R, out=x)
    return x


def shard_plan(rank, world, nseg):
    """Static shard of one long record: rank r owns global segments
    [r*nseg, (r+1)*nseg). Rank 0's shard starts with the record's buffer 0, which
    seeds every chunk (fitters.py:403-410); the other ranks prepend that buffer
    (regenerated bit for bit by the counter-based generator) and fit it themselves
    (no collective). Returns (first global segment, buffers in the local batch,
    whether the seed buffer is prepended)."""
    if rank == 0:
        return 0, nseg, False
    return rank * nseg, nseg + 1, True


def plan_workload(world, segments=None, channels=1):
    """What one rank of `bench.py --gpus world` fits, and how its line names it. Config 4
    (BASELINE.json): ONE 10,000,000-segment record split over the ranks (total work fixed:
    strong scaling; 1.25 M segments = 40 GB per GPU at 8); config 2: 100,000 segments on one
    GPU; an explicit --segments is per GPU (weak scaling). The workload string names the
    per-GPU shard only, so the N = 1 scaling anchor (config 4's 8-way shard on one GPU) and
    rank 0 at N = 8 carry the same string (tests/test_bench_launch.py)."""
    R = int(F_SAMP / F_MOD * N_CYC)
    config4 = world > 1 and segments is None
    if config4:
        if CONFIG4_SEGMENTS % world:
            raise SystemExit(f"config 4: {CONFIG4_SEGMENTS} segments do not split over {world} ranks")
        nseg = CONFIG4_SEGMENTS // world
    else:
        nseg = segments if segments is not None else 100_000
    nrec = max(1, channels) if world == 1 else 1
    if config4:
        name = "config4"
    elif nrec == 2:
        name = "config3"
    else:
        name = {100_000: "config2", 1_250_000: "config4 shard"}.get(nseg, "config2-shape")
    workload = (f"{name}: {nseg} segments/GPU x R={R} @200 kS/s, ndata={NDATA}, {nrec} channel"
                f"{'s' if nrec > 1 else ''}, _fit_parallel chunk size 1")
    return {"name": name, "config4": config4, "nseg": nseg, "nrec": nrec, "R": R, "workload": workload,
            "record_segments": CONFIG4_SEGMENTS if config4 else nseg * nrec, "scaling": "strong" if config4 else "weak"}


ANCHOR_WORLD = 8  # the driver's largest scaling point: config 4's shard at N = 8 is the N = 1 anchor


def cpu_share():
    """The host CPUs this process may use: affinity, capped by a cgroup CPU quota
    (a GPU box's share is far below os.cpu_count(), which counts the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    share = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return share, {"os_cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "model": model}


def cpu_baseline(args):
    """Oracle restatement of StandardNLSFitter._fit_parallel (Pool over np.array_split
    chunks, fitters.py:395-428) timed on this host. Runs BEFORE the GPU is touched
    (the Pool forks). Returns the sample, the oracle result and the baseline record."""
    from multiprocessing import get_context

    import deepfmkit_amd as dfm
    from oracle import nls_oracle as O

    R = int(F_SAMP / F_MOD * N_CYC)
    share, host = cpu_share()
    procs = args.cpu_procs if args.cpu_procs > 0 else share
    nseg = args.cpu_sample if args.cpu_sample else max(8000, 500 * procs)
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, M_TRUE)
    sim = dfm.DFMIObject("cpu", laser, ifo, f_samp=F_SAMP)
    raw = dfm.SignalGenerator().generate(sim, nseg * R / F_SAMP, mode="snr", snr_db=SNR_DB, trial_num=0)["main"]
    x = raw.samples()
    # close + join (not the context manager's terminate): the workers exit on their own,
    # so a profiled run (rocprofv3) records no SIGTERM abort stacks for them
    pool = get_context("fork").Pool(procs)
    try:
        O.fit_record_parallel(x[: 4 * R * procs], F_SAMP, F_MOD, N_CYC, n_cores=procs, pool=pool)  # warm
        t0 = time.perf_counter()
        ref = O.fit_record_parallel(x, F_SAMP, F_MOD, N_CYC, n_cores=procs, pool=pool)
        dt = time.perf_counter() - t0
    finally:
        pool.close()
        pool.join()
    base = {"value": round(nseg / dt, 1), "unit": "segments/s", "cores": procs, "kind": "port",
            "sample": f"{nseg} segments of config 2 (R=4000, ndata=10, m=6, 40 dB; the reference's own snr "
                      f"generator, RandomState(0)), numpy restatement of StandardNLSFitter._fit_parallel with "
                      f"multiprocessing.Pool({procs}); {dt:.2f} s wall",
            "host": host}
    base_c = cpu_baseline_c(x, nseg, R, procs, ref)
    return raw, ref, procs, base, base_c


def cpu_baseline_c(x, nseg, R, threads, ref):
    """Second CPU baseline (optional): the scalar C restatement of the same
    readout (oracle/csrc/nls_scalar.c: chunk size 1, J_n by one Miller pass per
    evaluation, the quadratures through the basis period's phase bins) with OpenMP over
    the same host CPU share, on the same sample fitted 50 times over (one fit of the sample
    takes milliseconds); status-0 parameters against the numpy port's."""
    path = os.path.join(ROOT, "oracle", "libnls_scalar.so")
    if not os.path.exists(path):
        return {"error": "oracle/libnls_scalar.so not built"}
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    lib.nls_scalar_record.argtypes = [P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double, P,
                                      ctypes.c_int, P]
    xs = np.ascontiguousarray(x[: nseg * R], dtype=np.float64)
    g = np.array([1.6, 6.0, 0.0, 0.0])
    out = np.zeros((nseg, 7))
    reps = 50
    lib.nls_scalar_record(xs.ctypes.data, nseg, R, NDATA, 2.0 * np.pi * F_MOD / F_SAMP, g.ctypes.data, threads,
                          out.ctypes.data)  # warm (threads, pages)
    t0 = time.perf_counter()
    for _ in range(reps):
        rc = lib.nls_scalar_record(xs.ctypes.data, nseg, R, NDATA, 2.0 * np.pi * F_MOD / F_SAMP, g.ctypes.data,
                                   threads, out.ctypes.data)
        if rc != 0:
            return {"error": f"nls_scalar_record rc {rc}"}
    dt = (time.perf_counter() - t0) / reps
    ok = (out[:, 6] == 0) & (ref[:, 6] == 0)
    return {"value": round(nseg / dt, 1), "unit": "segments/s", "cores": threads, "kind": "port",
            "sample": f"the same {nseg} segments; scalar C restatement (oracle/csrc/nls_scalar.c, gcc -O2, "
                      f"OpenMP {threads} threads, chunk size 1), fitted {reps} times: {dt * 1e3:.2f} ms each",
            "max_dm_vs_numpy_port": float(np.abs(out[ok, 1] - ref[ok, 1]).max()) if ok.any() else None,
            "status_match": float(np.mean(out[:, 6] == ref[:, 6]))}


def parity_vs_oracle(df, ref):
    st_ok = (df["fitok"].to_numpy() == ref[:, 6]) & (ref[:, 6] == 0)
    dphi = np.abs((df["phi"].to_numpy() - ref[:, 2] + np.pi) % (2 * np.pi) - np.pi)[st_ok]
    dm = np.abs(df["m"].to_numpy() - ref[:, 1])[st_ok]
    da = np.abs(df["amp"].to_numpy() - ref[:, 0])[st_ok]
    dpsi = np.abs(df["psi"].to_numpy() - ref[:, 3])[st_ok]
    return {"segments": int(ref.shape[0]), "max_dphi": float(dphi.max()), "max_dm": float(dm.max()),
            "max_damp": float(da.max()), "max_dpsi": float(dpsi.max()),
            "status_match": float(np.mean(df["fitok"].to_numpy() == ref[:, 6])),
            "vs": "oracle restatement of fit.py/fitters.py, pinned to the reference by tests/golden"}


_ROCTX = None


def _roctx():
    """ROCm's marker API (rocprofiler-sdk's roctx, which rocprofv3 --marker-trace records) or
    False when absent: markers are diagnostics only."""
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except (OSError, AttributeError):
                continue
    return _ROCTX


def roctx_push(name):
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(name.encode())


def roctx_pop():
    lib = _roctx()
    if lib:
        lib.roctxRangePop()


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_timeout(args, world):
    """Wall-clock bound of a self-launched N-rank job: process start-up and imports (180 s),
    the rendezvous (--rdzv-timeout), the CPU baseline leg (rank 0 only at N = 1: not here),
    input generation and the timed / side windows at a generous 100 ns per segment per step
    (the measured step is ~5 ns per segment: BENCH_r04) plus the extra configs (300 s)."""
    nseg = args.segments if args.segments is not None else CONFIG4_SEGMENTS // max(world, 1)
    steps = args.steps + args.warmup + max(200, args.steps) + 40
    return 180.0 + args.rdzv_timeout + steps * nseg * 1e-7 + (0.0 if args.no_extra else 300.0)


def join_group(dist, backend, dev, timeout_s):
    """init_process_group with a bounded rendezvous: a rank that does not arrive within
    timeout_s makes the others raise instead of waiting forever (then self_launch reports
    which rank never arrived: every rank leaves a marker in DFMI_RDZV_DIR when it reaches the
    rendezvous and another when it has joined).
    DFMI_RDZV_DELAY="rank:seconds" delays that rank before it joins (test hook:
    tests/test_bench_launch.py)."""
    from datetime import timedelta
    rank = int(os.environ.get("RANK", "0"))
    delay = os.environ.get("DFMI_RDZV_DELAY", "")
    if delay:
        r, sec = delay.split(":")
        if int(r) == rank:
            time.sleep(float(sec))
    mark = os.environ.get("DFMI_RDZV_DIR")

    def stamp(what):
        if mark:
            with open(os.path.join(mark, f"rank{rank}.{what}"), "w") as f:
                f.write(str(os.getpid()))
    stamp("arrived")
    kw = {"timeout": timedelta(seconds=timeout_s)}
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev, **kw)
    else:
        dist.init_process_group(backend, **kw)
    stamp("joined")


def self_launch(n, argv, script=None, env_extra=None, timeout=None):
    """`python bench.py --gpus N` without torchrun: start N rank processes, one per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), BEFORE this process
    touches any GPU, wait for all of them and return the worst exit code. The reference's
    parallel width is likewise an explicit argument (n_cores -> Pool(n_cores),
    fitters.py:397-399,416-423), and its Pool context manager propagates a worker's failure
    (fitters.py:421-423): here rank 0 prints the JSON line; a rank that fails takes the
    others down with it; past `timeout` seconds every rank is killed (exit 124). On any
    failure the ranks that never reached the rendezvous (no marker, join_group) are named
    on stderr."""
    import shutil
    import subprocess
    import tempfile
    port = str(free_port())
    mark = tempfile.mkdtemp(prefix="dfmi_rdzv_")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, DFMI_SELF_LAUNCHED="1", DFMI_RDZV_DIR=mark,
                   **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    why = ""
    t_end = None if timeout is None else time.monotonic() + timeout
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0:
                    if not rc:
                        why = f"rank {procs.index(p)} exited with {code}"
                    rc = rc or code
                    for q in pending:  # one rank failed: the barrier would hang the others
                        q.terminate()
            if t_end is not None and time.monotonic() > t_end and pending:
                if not rc:
                    why = f"launch timeout {timeout:.0f} s"
                rc = rc or 124
                for q in pending:
                    q.kill()
            if pending:
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
        if rc:
            def without(what):
                return [r for r in range(n) if not os.path.exists(os.path.join(mark, f"rank{r}.{what}"))]
            print(f"bench: {n}-rank job failed ({why}); ranks that never reached the rendezvous: {without('arrived')}; "
                  f"ranks that did not complete it: {without('joined')}", file=sys.stderr, flush=True)
        shutil.rmtree(mark, ignore_errors=True)
    return rc


def rank_topology(dist, dev, world):
    """Every rank's (rank, local rank, host, device) all-gathered onto rank 0, and the
    process-group backend: evidence that N ranks ran on N distinct GPUs."""
    import socket
    me = {"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "host": socket.gethostname(), "device": str(dev)}
    if dev is not None and getattr(dev, "type", "") == "cuda":
        import torch
        props = torch.cuda.get_device_properties(dev)
        me["device_index"] = dev.index
        me["pci_bus_id"] = getattr(props, "pci_bus_id", None)
        me["uuid"] = str(getattr(props, "uuid", ""))
    if world == 1:
        return [me], None
    allr = [None] * world
    dist.all_gather_object(allr, me)
    return allr, dist.get_backend()


def window_breakdown(torch, lib, _lib, fn, stream, k):
    """Where a K-step window's wall time goes (diagnostic, run AFTER the timed window, same
    K): the same synchronize -> K steps -> synchronize wall clock, split into the GPU span
    (an event recorded before the first launch to one after the last: the launch lag of the
    first step after an idle GPU included) and the kernels themselves (dfmi_step_timing events
    around each step's two launches). wall - span = the host-side sync costs; span - kernels
    = the first launch's lag plus the gaps between launches."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    _lib.check(lib.dfmi_step_timing(1), "dfmi_step_timing")
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(k):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    _lib.check(lib.dfmi_step_timing(0), "dfmi_step_timing")
    td, tl, tn = np.zeros(1), np.zeros(1), np.zeros(1, dtype=np.int64)
    _lib.check(lib.dfmi_step_timing_read(_lib.ptr(td), _lib.ptr(tl), _lib.ptr(tn)), "dfmi_step_timing_read")
    span = e0.elapsed_time(e1)
    kern = float(td[0] + tl[0])
    return {"steps": k, "wall_ms_per_step": round(wall * 1e3 / k, 4), "gpu_span_ms_per_step": round(span / k, 4),
            "kernels_ms_per_step": round(kern / k, 4), "marked_steps": int(tn[0]),
            "host_sync_ms": round(wall * 1e3 - span, 4), "launch_lag_and_gaps_ms": round(span - kern, 4),
            "note": "a second K-step window after the timed one, with events: wall = host sync + GPU span; "
                    "span = kernels + the first launch's lag + inter-launch gaps"}


def _timed_steps(torch, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def facade_end_to_end(torch, x, nseg, R, calls=11, host_calls=5):
    """DeepFitFramework.fit(label, n=20) on a record already on the GPU and on the same
    record in host memory: wall time per call (each call returns the DeepFitObject, i.e.
    after the results' D2H), median of `calls` (host: `host_calls`) calls after three warm
    calls; both give the same bits."""
    import deepfmkit_amd as dfm
    res = {}
    cols = {}
    xh = x.cpu().numpy()
    for name, data in (("device_resident", x), ("host_resident", xh)):
        raw = dfm.DeepRawObject(data)
        raw.f_samp, raw.f_mod, raw.label = F_SAMP, F_MOD, name
        dff = dfm.DeepFitFramework()
        dff.raws[name] = raw
        for _ in range(3):
            dff.fit(name, n=N_CYC, fit_label="e2e")
        ts = []
        for _ in range(calls if name == "device_resident" else host_calls):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fo = dff.fit(name, n=N_CYC, fit_label="e2e")
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        cols[name] = np.stack([fo.amp, fo.m, fo.phi, fo.psi, fo.dc, fo.ssq])
        res[name] = {"ms_per_call": round(t * 1e3, 3), "segments_per_s": round(nseg / t, 1),
                     "calls": len(ts), "nbuf": int(fo.nbuf)}
    res["device_resident"]["includes"] = ("StandardNLSFitter dispatch, dfmi_nls_record (seed + demodulation + LM), "
                                          "D2H of the 7 result columns, DataFrame, tau, DeepFitObject")
    res["host_resident"]["includes"] = "the same plus H2D of the 3.2 GB record (pinned staging)"
    res["bit_identical"] = bool(np.array_equal(cols["device_resident"], cols["host_resident"]))
    res["workload"] = f"config 2: {nseg} segments x R={R}, DeepFitFramework.fit(label, n={N_CYC}) (parallel=True)"
    del xh
    return res


def extra_configs(torch, dev, lib, _lib, stream, cfg, cpu_leg):
    """The other BASELINE.json configs on this GPU, timed after the main window (same
    process, steady clocks): config 3 (two channels, main m = 6 and witness m = 4.3, as
    two records of one dfmi_nls_record call, each seeded by its own buffer 0: 2 x 50,000
    segments), config 5 (EKFFitter.fit over a 2 s = 400,000-sample record, one channel,
    and 1,024 channels in one launch; with the scalar C restatement of the same loop
    timed on one host core beside it when the CPU leg runs) and config 1 through the
    sequential path (_fit_sequential: one warm-start chain over 500 buffers), and config 2's
    100,000-segment record through the same sequential path."""
    from deepfmkit_amd.fitters import w0_of
    R = int(F_SAMP / F_MOD * N_CYC)
    w0 = w0_of(F_MOD, F_SAMP)
    out = {}
    # ---- config 3
    nbuf = 50_000
    x = torch.empty(2 * nbuf * R, dtype=torch.float64, device=dev)
    for c, m in enumerate((M_TRUE, 4.3)):
        gen_shard(torch, dev, 0, nbuf, R, seed=SEED, m_true=m, stream=c, out=x[c * nbuf * R:(c + 1) * nbuf * R])
    g2 = np.ascontiguousarray(np.tile([1.6, 6.0, 0.0, 0.0], (2, 1)))
    o2 = torch.empty((6, 2 * nbuf), dtype=torch.float64, device=dev)
    k2 = torch.empty(2 * nbuf, dtype=torch.int32, device=dev)

    def step3():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 2, nbuf * R, nbuf, R, NDATA, w0, 0, _lib.ptr(g2), 1, nbuf - 1, cfg,
                                       o2.data_ptr(), k2.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream),
                   "dfmi_nls_record")

    s3 = _timed_steps(torch, step3, 20, 5)
    st = k2.cpu().numpy()
    mm = o2[1].cpu().numpy()
    out["config3"] = {"workload": "2 channels (main m=6, witness m=4.3) x 50,000 segments, one dfmi_nls_record call",
                      "value": round(2 * nbuf / s3, 1), "unit": "segments/s", "ms_per_step": round(s3 * 1e3, 4),
                      "steps": 20, "status0_frac": float(np.mean(st == 0)),
                      "m_mean_per_channel": [float(mm[:nbuf].mean()), float(mm[nbuf:].mean())]}
    del o2, k2  # x is reused by the 100k sequential chain below
    # ---- config 5: EKF, 2 s @ 200 kS/s
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    ns = int(2.0 * F_SAMP)
    nb5 = ns // R
    p0 = np.ones(5)
    qd = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0d = torch.from_numpy(p0).to(dev)
    qdd = torch.from_numpy(qd).to(dev)
    res5 = {}
    for nch in (1, 1024):
        xe = torch.empty(nch * ns, dtype=torch.float64, device=dev)
        for c in range(nch):
            synth_snr(SnrSpec(seed=SEED, stream=100 + c, f_samp=F_SAMP, f_mod=F_MOD, m=M_TRUE, snr_db=SNR_DB), 0, ns,
                      out=xe[c * ns:(c + 1) * ns])
        stt = torch.empty((nch, nb5, 5), dtype=torch.float64, device=dev)

        def ekf():
            _lib.check(lib.dfmi_ekf_fit(xe.data_ptr(), nch, ns, ns, init4.data_ptr(), p0d.data_ptr(), qdd.data_ptr(),
                                        None, 2 * np.pi * F_MOD, F_SAMP, R, nb5, stt.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                        stream.cuda_stream), "dfmi_ekf_fit")

        t = _timed_steps(torch, ekf, 3, 1)
        res5[nch] = {"channels": nch, "s_per_fit": round(t, 5), "samples_per_s_per_channel": round(ns / t, 1),
                     "samples_per_s_aggregate": round(nch * ns / t, 1),
                     "kernel": lib.dfmi_last_demod_kernel().decode()}
        if nch == 1:
            passes = (ctypes.c_int32 * 1)()
            _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), 1), "dfmi_ekf_pit_passes")
            res5[1]["pit_passes"] = int(passes[0])
            x1 = xe.cpu().numpy()
            s1 = stt[0].cpu().numpy()
            # the same channel through the sequential row kernel (ekf_pit off)
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit", 0), "tune")
            ts = _timed_steps(torch, ekf, 3, 1)
            res5["seq"] = {"s_per_fit": round(ts, 5), "samples_per_s_per_channel": round(ns / ts, 1),
                           "kernel": lib.dfmi_last_demod_kernel().decode(),
                           "max_abs_dstate_vs_parallel_in_time": float(np.max(np.abs(stt[0].cpu().numpy() - s1)))}
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit", 1024), "tune")
        del xe, stt
    c5 = {"workload": "EKFFitter.fit, 2 s = 400,000 samples @200 kS/s (m=6, 40 dB), snapshots every R=4000",
          "one_channel": res5[1], "one_channel_sequential": res5["seq"], "channels_1024": res5[1024],
          "unit": "samples/s"}
    if cpu_leg:  # the host baseline: the oracle's scalar C restatement of the same loop, one core
        lib_c = os.path.join(ROOT, "oracle", "libekf_scalar.so")
        if os.path.exists(lib_c):
            cl = ctypes.CDLL(lib_c)
            P_ = ctypes.c_void_p
            cl.ekf_scalar.argtypes = [P_, ctypes.c_int64, P_, P_, P_, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_int64, ctypes.c_int64, P_]
            cx0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x1)])
            cst = np.zeros((nb5, 5))
            t0 = time.perf_counter()
            cl.ekf_scalar(x1.ctypes.data, ns, cx0.ctypes.data, p0.ctypes.data, qd.ctypes.data, float(np.var(x1)),
                          2 * np.pi * F_MOD, F_SAMP, R, nb5, cst.ctypes.data)
            tc = time.perf_counter() - t0
            c5["cpu_baseline"] = {"value": round(ns / tc, 1), "unit": "samples/s per channel", "cores": 1,
                                  "kind": "port", "sample": "the same 400,000-sample record, oracle/csrc/ekf_scalar.c "
                                                            "(gcc -O2, libm), the numpy loop's operation order"}
            c5["max_abs_dstate_gpu_vs_cpu"] = float(np.max(np.abs(s1 - cst)))
    out["config5"] = c5
    out["config5_handover"] = ekf_handover_point(torch, dev, lib, _lib, stream)
    # ---- config 1 through the sequential path (one warm-start chain, fitters.py:370-393)
    nb1 = 500
    x1r = torch.empty(nb1 * R, dtype=torch.float64, device=dev)
    gen_shard(torch, dev, 0, nb1, R, seed=SEED, out=x1r)
    g1 = np.array([1.6, 6.0, 0.0, 0.0])
    o1 = torch.empty((6, nb1), dtype=torch.float64, device=dev)
    k1 = torch.empty(nb1, dtype=torch.int32, device=dev)

    def seq():
        _lib.check(lib.dfmi_nls_record(x1r.data_ptr(), 1, nb1 * R, nb1, R, NDATA, w0, 0, _lib.ptr(g1), 0, 1, cfg,
                                       o1.data_ptr(), k1.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream),
                   "dfmi_nls_record")

    t1 = _timed_steps(torch, seq, 5, 1)
    out["config1_sequential"] = {"workload": "500 segments (10 s @200 kS/s), parallel=False: one warm-start chain",
                                 "value": round(nb1 / t1, 1), "unit": "segments/s", "ms_per_fit": round(t1 * 1e3, 3),
                                 "status0_frac": float(np.mean(k1.cpu().numpy() == 0)),
                                 "reference_same_path": "724 segments/s on one core of the survey container "
                                                        "(SURVEY.md §6)"}
    # ---- config 2 end to end through the drop-in facade (SURVEY.md §8(d) "Timing":
    # end-to-end incl. D2H of the results, reported separately): DeepFitFramework.fit on
    # the 100,000-segment record (core.py:424-517 -> StandardNLSFitter -> dfmi_nls_record ->
    # D2H of the 7 columns -> DataFrame -> tau -> DeepFitObject), device-resident and
    # host-resident (+ H2D of the 3.2 GB record through pinned staging)
    nb2 = 2 * nbuf
    gen_shard(torch, dev, 0, nb2, R, seed=SEED, out=x)
    out["config2_end_to_end"] = facade_end_to_end(torch, x, nb2, R)
    # ---- config 2's record through the sequential path: ONE warm-start chain of 100,000 fits
    o4 = torch.empty((6, nb2), dtype=torch.float64, device=dev)
    k4 = torch.empty(nb2, dtype=torch.int32, device=dev)

    def seq2():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nb2 * R, nb2, R, NDATA, w0, 0, _lib.ptr(g1), 0, 1, cfg,
                                       o4.data_ptr(), k4.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream),
                   "dfmi_nls_record")

    t2 = _timed_steps(torch, seq2, 1, 1)
    out["config2_sequential"] = {"workload": "100,000 segments (config 2's record), parallel=False: one warm-start "
                                             "chain", "value": round(nb2 / t2, 1), "unit": "segments/s",
                                 "s_per_record": round(t2, 4), "status0_frac": float(np.mean(k4.cpu().numpy() == 0))}
    # ---- config 2 at more harmonics ("for ndata >= 20 the demodulation
    # crosses the ridge; report that separately"): the record pipeline's step and the
    # demodulation alone (component-major QI: demod_wide_kernel beyond 16 harmonics)
    sweep = []
    # (ndata, m): config 2's record at more harmonics, and the reference quickstart's own
    # setting (notebooks/0.0_quickstart.ipynb: m_target = 10*3.14, ndata = int(2*m_target) = 62,
    # and ndata 30) on a 100,000-segment record of m = 31.4, buffer 0 through the m-grid seed
    m_rec = M_TRUE
    for nd, m in ((16, M_TRUE), (20, M_TRUE), (30, M_TRUE), (62, M_TRUE), (30, 31.4), (62, 31.4)):
        if m != m_rec:
            gen_shard(torch, dev, 0, nb2, R, seed=SEED, m_true=m, out=x)
            m_rec = m

        def stepn():
            _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nb2 * R, nb2, R, nd, w0, 0, _lib.ptr(g1), 1, nb2 - 1, cfg,
                                           o4.data_ptr(), k4.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream),
                       "dfmi_nls_record")
        tn = _timed_steps(torch, stepn, 20, 5)
        kstep = lib.dfmi_last_demod_kernel().decode()
        okn = float(np.mean(k4.cpu().numpy() == 0))
        m_fit = float(o4[1].mean().item())
        qn = torch.empty((2 * nd, nb2), dtype=torch.float64, device=dev)
        dn = torch.empty(nb2, dtype=torch.float64, device=dev)

        def demn():
            _lib.check(lib.dfmi_demod(x.data_ptr(), nb2, R, R, nd, w0, 0, qn.data_ptr(), dn.data_ptr(),
                                      _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_demod")
        td = _timed_steps(torch, demn, 20, 5)
        lo = torch.empty((4, nb2), dtype=torch.float64, device=dev)
        ls = torch.empty(nb2, dtype=torch.float64, device=dev)
        lk = torch.empty(nb2, dtype=torch.int32, device=dev)
        gm = torch.tensor([1.0, m, 0.0, 0.0], dtype=torch.float64, device=dev)

        def lmn():  # the LM alone over these QI, every segment seeded near its m (chunk size 1)
            _lib.check(lib.dfmi_lm(qn.data_ptr(), nb2, nd, gm.data_ptr(), 0, nb2, cfg, lo.data_ptr(), ls.data_ptr(),
                                   lk.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_lm")
        tl = _timed_steps(torch, lmn, 20, 5)
        sweep.append({"ndata": nd, "m": m, "value": round(nb2 / tn, 1), "unit": "segments/s",
                      "ms_per_step": round(tn * 1e3, 4), "step_demod_kernel": kstep, "status0_frac": okn,
                      "mean_m": m_fit, "demod_component_major_ms": round(td * 1e3, 4),
                      "demod_kernel": lib.dfmi_last_demod_kernel().decode(), "lm_alone_ms": round(tl * 1e3, 4),
                      "demod_hbm_frac": round(nb2 * (8 * R + 8 * (2 * nd + 1)) / td / 1e9 / HBM_PEAK_GBS, 4),
                      "hbm_frac_end_to_end": round(nb2 * (8 * R + 56) / tn / 1e9 / HBM_PEAK_GBS, 4)})
        del qn, dn, lo, ls, lk
    out["config2_ndata_sweep"] = {"workload": "config 2 (100,000 x R=4000, 40 dB) at ndata 16 / 20 / 30 / 62 (m = 6), "
                                              "and the reference quickstart's m = 31.4 at ndata 30 / 62; "
                                              "dfmi_nls_record parallel", "points": sweep}
    del x, o4, k4
    torch.cuda.empty_cache()
    return out


def ekf_handover_point(torch, dev, lib, _lib, stream, ns=400_000, nch=1024, n_bad=64):
    """The EKF parallel in time's hand-over (dfmi_capi.hip ekf_pit_run, round 6): channels whose
    iteration does not lock (here m = 20 records fitted from init_m = 6: the filter never
    locks, moves O(1) every pass) are re-run in place by the sequential kernel, in one launch
    after the last pass (ekf_pit_overlap 0; launching at each check beside the passes measured
    slower). One such channel alone: its time against the sequential kernel's alone (the passes before
    the hand-over are the overhead). A batch of nch config-5 channels with n_bad of those among
    them: its time against the passes alone (the same batch with the re-run switched off,
    ekf_pit_seq 0: diagnostics) and the n_bad channels' sequential run alone."""
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    R = int(F_SAMP / F_MOD * N_CYC)
    nb5 = ns // R
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0d = torch.ones(5, dtype=torch.float64, device=dev)
    qdd = torch.tensor([1e-8, 1e-8, 1e-6, 1e-6, 1e-8], dtype=torch.float64, device=dev)

    def records(ms):
        xe = torch.empty(len(ms) * ns, dtype=torch.float64, device=dev)
        for c, m in enumerate(ms):
            synth_snr(SnrSpec(seed=SEED, stream=300 + c, f_samp=F_SAMP, f_mod=F_MOD, m=m, snr_db=SNR_DB), 0, ns,
                      out=xe[c * ns:(c + 1) * ns])
        return xe

    def run(xe, n, tune=None, reps=3):
        stt = torch.empty((n, nb5, 5), dtype=torch.float64, device=dev)
        for k, v in (tune or {}).items():
            _lib.check(lib.dfmi_set_tuning(k.encode(), v), "tune")

        def ekf():
            _lib.check(lib.dfmi_ekf_fit(xe.data_ptr(), n, ns, ns, init4.data_ptr(), p0d.data_ptr(), qdd.data_ptr(),
                                        None, 2 * np.pi * F_MOD, F_SAMP, R, nb5, stt.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                        stream.cuda_stream), "dfmi_ekf_fit")
        try:
            t = _timed_steps(torch, ekf, reps, 1)
            kname = lib.dfmi_last_demod_kernel().decode()
            passes = (ctypes.c_int32 * n)()
            _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), n), "passes")
        finally:
            for k in (tune or {}):
                _lib.check(lib.dfmi_set_tuning(k.encode(), {"ekf_pit": 1024, "ekf_pit_seq": 1}[k]), "tune")
        return t, kname, np.array(list(passes)), stt
    bad = records([20.0])
    t1, k1, p1, s1 = run(bad, 1)
    ts1, ks1, _, q1 = run(bad, 1, {"ekf_pit": 0})
    one = {"channels": 1, "record": "m = 20 fitted from init_m = 6 (never locks)", "ms": round(t1 * 1e3, 3),
           "passes": int(p1[0]), "kernel": k1, "sequential_alone_ms": round(ts1 * 1e3, 3),
           "overhead_ms": round((t1 - ts1) * 1e3, 3),
           "bit_identical_to_sequential": bool(torch.equal(s1, q1))}
    del bad, s1, q1
    ms = [M_TRUE] * nch
    for i in range(n_bad):  # spread over the batch
        ms[(i * nch) // n_bad + 3] = 20.0
    xe = records(ms)
    tb, kb, pb, sb = run(xe, nch, reps=2)
    tp, _, _, _ = run(xe, nch, {"ekf_pit_seq": 0}, reps=2)
    idx = [i for i, m in enumerate(ms) if m != M_TRUE]
    xs = torch.stack([xe[i * ns:(i + 1) * ns] for i in idx]).reshape(-1).contiguous()
    del xe
    tsq, ksq, _, ss = run(xs, n_bad, {"ekf_pit": 0}, reps=2)
    handed = int(np.sum(pb < 0))
    batch = {"channels": nch, "samples_per_channel": ns, "non_locking": n_bad, "handed_over": handed,
             "ms": round(tb * 1e3, 3), "kernel": kb, "passes_alone_ms": round(tp * 1e3, 3),
             "sequential_alone_ms": round(tsq * 1e3, 3), "sequential_kernel": ksq,
             "ratio_to_max_of_parts": round(tb / max(tp, tsq), 4),
             "ratio_to_sum_of_parts": round(tb / (tp + tsq), 4),
             "handed_states_bit_identical_to_sequential": bool(torch.equal(sb[idx], ss))}
    del sb, ss, xs
    torch.cuda.empty_cache()
    return {"workload": f"EKFFitter.fit hand-over: {ns} samples per channel, m = 20 channels from init_m = 6",
            "one_channel": one, "batch": batch}


def scaling_anchor(torch, dev, lib, _lib, stream, cfg, steps, warmup):
    """The N = 1 anchor of the driver's strong-scaling curve: bench.py's step
    and timed window (W warmup steps, synchronize, exactly K steps, synchronize) over the shard
    rank 0 fits at N = ANCHOR_WORLD = 8 (global segments [0, 1.25 M) of the 10M-segment record,
    40 GB resident, buffer 0 first), on this one GPU. At N ranks each GPU fits 10M / N segments,
    and a rank's per-segment cost is flat in its shard size from ~10^5 segments up, so
    value_N / (N x this value) is the scaling efficiency of the curve's N-th point; the headline
    stays config 2."""
    from deepfmkit_amd.fitters import w0_of
    plan = plan_workload(ANCHOR_WORLD)
    R, nseg = plan["R"], plan["nseg"]
    seg0, nbuf, prepend = shard_plan(0, ANCHOR_WORLD, nseg)
    x = torch.empty(nbuf * R, dtype=torch.float64, device=dev)
    gen_shard(torch, dev, seg0, nseg, R, seed=SEED, out=x)
    g = np.array([1.6, 6.0, 0.0, 0.0])
    o = torch.empty((6, nbuf), dtype=torch.float64, device=dev)
    k = torch.empty(nbuf, dtype=torch.int32, device=dev)
    w0 = w0_of(F_MOD, F_SAMP)

    def step():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nbuf * R, nbuf, R, NDATA, w0, 0, _lib.ptr(g), 1, nbuf - 1, cfg,
                                       o.data_ptr(), k.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream),
                   "dfmi_nls_record")

    t = _timed_steps(torch, step, steps, warmup)
    st = k.cpu().numpy()
    res = {"workload": plan["workload"], "n_gpus": 1, "of_world": ANCHOR_WORLD, "record_segments": CONFIG4_SEGMENTS,
           "value": round(nseg / t, 1), "unit": "segments/s", "ms_per_step": round(t * 1e3, 4), "steps": steps,
           "warmup": warmup, "status0_frac": float(np.mean(st == 0)),
           "hbm_frac_end_to_end": round(nseg * (8 * R + 56) / t / 1e9 / HBM_PEAK_GBS, 4),
           "note": "rank 0's shard of config 4 at N = 8, timed on one GPU: the curve's N-th point has "
                   "efficiency value_N / (N x value)"}
    del x, o, k
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no torchrun: one rank process per GPU, launched here before any GPU call
            t = args.launch_timeout if args.launch_timeout is not None else launch_timeout(args, args.gpus)
            return self_launch(args.gpus, sys.argv[1:], timeout=t)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: the launcher and the "
                         "flag disagree")
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    want_base = rank == 0 and world == 1 and not args.no_cpu_baseline and not args.demod_only
    pre = cpu_baseline(args) if want_base else None
    # one process per GPU: bind the device first, so RCCL's barrier / all_reduce run
    # on this rank's GPU
    # (local rank modulo the visible GPUs: only a gloo rehearsal puts two ranks on one card;
    # under RCCL that is refused below)
    ndev = torch.cuda.device_count()  # counting devices does not initialise HIP
    dev_index = local % ndev if ndev > 0 else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        # RCCL; DFMI_DIST_BACKEND=gloo rehearses N ranks that share one card (RCCL
        # refuses two ranks on one device)
        join_group(dist, os.environ.get("DFMI_DIST_BACKEND", "nccl"), dev, args.rdzv_timeout)

    ranks, backend = rank_topology(dist, dev, world)
    if world > 1 and len({(r["host"], r.get("pci_bus_id"), r["device"]) for r in ranks}) < world \
            and os.environ.get("DFMI_DIST_BACKEND", "nccl") == "nccl":
        raise SystemExit(f"{world} ranks on fewer distinct GPUs: {ranks}")

    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import StandardNLSFitter, w0_of

    lib = _lib.load()
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), "dfmi_set_tuning")
    plan = plan_workload(world, args.segments, args.channels)
    R, nseg, nrec, config4 = plan["R"], plan["nseg"], plan["nrec"], plan["config4"]
    if nrec > 1:  # config 3: channels as records of one batch (fit_many), each with its own seed
        if nseg % nrec:
            raise SystemExit("--segments must be a multiple of --channels")
        nbuf, prepend_seed = nseg // nrec, False
        ms_true = [M_TRUE, 4.3] + [M_TRUE] * (nrec - 2)
        x = torch.empty(nrec * nbuf * R, dtype=torch.float64, device=dev)
        for c in range(nrec):  # channel c: its own Philox stream under the seed
            gen_shard(torch, dev, 0, nbuf, R, seed=SEED, m_true=ms_true[c], stream=c,
                      out=x[c * nbuf * R:(c + 1) * nbuf * R])
    else:
        seg0, nbuf, prepend_seed = shard_plan(rank, world, nseg)
        x = torch.empty(nbuf * R, dtype=torch.float64, device=dev)
        if prepend_seed:  # the record's buffer 0, bit for bit what rank 0 holds
            gen_shard(torch, dev, 0, 1, R, seed=SEED, out=x[:R])
        gen_shard(torch, dev, seg0, nseg, R, seed=SEED, out=x[(nbuf - nseg) * R:])
    torch.cuda.synchronize()
    w0 = w0_of(F_MOD, F_SAMP)
    cfg = F.lm_config()
    guess = np.ascontiguousarray(np.tile([1.6, 6.0, 0.0, 0.0], (nrec, 1)))  # per-record default seed
    out = torch.empty((6, nrec * nbuf), dtype=torch.float64, device=dev)
    ok = torch.empty(nrec * nbuf, dtype=torch.int32, device=dev)
    nall = nrec * nbuf  # segments in the batch (demodulation / LM-only timings run over all of them)
    qi = torch.empty((2 * NDATA, nall), dtype=torch.float64, device=dev)
    dcb = torch.empty(nall, dtype=torch.float64, device=dev)
    rows = torch.empty((nall, lib.dfmi_qi_row_stride(NDATA)), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        rc = lib.dfmi_nls_record(x.data_ptr(), nrec, nbuf * R, nbuf, R, NDATA, w0, 0, _lib.ptr(guess), 1, nbuf - 1,
                                 cfg, out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream)
        _lib.check(rc, "dfmi_nls_record")

    def demod():  # the record pipeline's demodulation (row layout): the roofline kernel
        rc = lib.dfmi_demod_rows(x.data_ptr(), nall, R, R, NDATA, w0, 0, rows.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                 stream.cuda_stream)
        _lib.check(rc, "dfmi_demod_rows")

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nrep = max(200, args.steps)
    # ---- side measurements first (untimed): the standalone row demodulation (dfmi_demod_rows,
    # no seed: the same bulk code) and the LM kernel alone over component-major QI
    for _ in range(5):
        demod()
    ev0.record(stream)
    for _ in range(nrep):
        demod()
    ev1.record(stream)
    ev1.synchronize()
    rows_ms = ev0.elapsed_time(ev1) / nrep
    if args.demod_only:  # profile helper: nothing but the timed demodulation kernel
        if rank == 0:
            print(json.dumps({"metric": "demod only (profile helper)", "kernel": lib.dfmi_last_demod_kernel().decode(),
                              "avg_launch_ms": rows_ms, "roofline": {"kernel": lib.dfmi_last_demod_kernel().decode()}}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    lm_out = torch.empty((4, nall), dtype=torch.float64, device=dev)
    lm_ssq = torch.empty(nall, dtype=torch.float64, device=dev)
    lm_st = torch.empty(nall, dtype=torch.int32, device=dev)
    gdev = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)

    def lm_only():
        rc = lib.dfmi_lm(qi.data_ptr(), nall, NDATA, gdev.data_ptr(), 0, nall, cfg, lm_out.data_ptr(),
                         lm_ssq.data_ptr(), lm_st.data_ptr(), _lib.DFMI_MEM_DEVICE, stream.cuda_stream)
        _lib.check(rc, "dfmi_lm")

    _lib.check(lib.dfmi_demod(x.data_ptr(), nall, R, R, NDATA, w0, 0, qi.data_ptr(), dcb.data_ptr(),
                              _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_demod")
    lm_only()
    ev0.record(stream)
    for _ in range(nrep):
        lm_only()
    ev1.record(stream)
    ev1.synchronize()
    lm_ms = ev0.elapsed_time(ev1) / nrep
    # ---- roofline of the step's dominant kernel, HIP events on the launch stream, over
    # whole steps: these untimed steps are also the ramp immediately before the window (the
    # clocks come up over the first ~35 demodulation-sized launches, 0.58 -> 0.50 ms,
    # profiles/r02m kernel trace), so a short driver window carries no ramp-up
    for _ in range(40):
        step()
    # nrep >= 200 steps (~0.11 s): the kernel's mean over these dominates any rocprofv3 average
    # of the same run, ramp launches included (profiles/r03*_frac_check.json); dfmi_step_timing
    # records events around the fused seed + demodulation launch (the dominant kernel) and
    # the LM launch of every step, on the step's stream
    _lib.check(lib.dfmi_step_timing(1), "dfmi_step_timing")
    for _ in range(nrep):
        step()
    _lib.check(lib.dfmi_step_timing(0), "dfmi_step_timing")
    td, tl, tn = np.zeros(1), np.zeros(1), np.zeros(1, dtype=np.int64)
    _lib.check(lib.dfmi_step_timing_read(_lib.ptr(td), _lib.ptr(tl), _lib.ptr(tn)), "dfmi_step_timing_read")
    step_kname = lib.dfmi_last_demod_kernel().decode()
    if int(tn[0]) != nrep:
        raise SystemExit(f"step timing: {int(tn[0])} marked steps of {nrep} (pipeline not fused: {step_kname})")
    demod_ms, lm_step_ms = float(td[0]) / nrep, float(tl[0]) / nrep
    demod_ms_max = demod_ms
    per_rank = [{"rank": rank, "step_demod_seed_ms": round(demod_ms, 4), "step_lm_ms": round(lm_step_ms, 4)}]
    if world > 1:  # the slowest rank's dominant kernel (every rank runs the same shape)
        tt = torch.tensor([demod_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        demod_ms_max = float(tt.item())
        # every rank's fused launch carries its own fit of the record's buffer 0 (the seed):
        # reported per rank, so a rank whose seed fit runs long shows here
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "step_demod_seed_ms": round(demod_ms, 4),
                                          "step_lm_ms": round(lm_step_ms, 4)})
    kname = step_kname
    fn = step
    # ---- the timed window: W untimed warmup steps, barrier + synchronize, exactly K steps,
    # synchronize + barrier, MAX over ranks. A roctx range "timed_window" brackets it (seen by
    # rocprofv3 --marker-trace; scripts/window_check.py accounts the window from a trace).
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    roctx_push("timed_window")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    roctx_pop()
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    window_diag = window_breakdown(torch, lib, _lib, fn, stream, args.steps)
    ms = el / args.steps * 1e3
    total_segments = nseg * world  # units of work; the seed replicas on ranks > 0 are not counted
    value = total_segments * args.steps / el
    bytes_per_seg = 8 * R + 8 * (2 * NDATA + 1)  # read the segment, write QI + dc
    achieved = nall * bytes_per_seg / (demod_ms * 1e-3) / 1e9
    family = kname.split("<")[0]
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_demod.json")
    if os.path.exists(pmc):  # PMC pass of the same kernel and workload (scripts/profile_round.sh)
        with open(pmc) as f:
            rec = json.load(f)
        if family and family in rec.get("kernel", "") and rec.get("algorithmic_bytes_per_launch") == \
                nall * bytes_per_seg:
            traffic, traffic_src = rec.get("hbm_bytes_per_launch"), "profiles/pmc_demod.json"
    # the whole step (seed + demodulation + LM) at SURVEY.md §8(d)'s algorithmic bytes per
    # segment: 8 R read + 56 B of results (6 fp64 + the status padded to 8 B); the 168-B
    # demodulation rows are an intermediate of the step, not its output
    e2e_bytes_per_seg = 8 * R + 56
    e2e = nall * e2e_bytes_per_seg / (ms * 1e-3) / 1e9
    roof = {"kernel": kname, "bound": "hbm", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": traffic_src, "avg_launch_ms": round(demod_ms, 4),
            "timing": f"HIP events around the step's own {kname} launch inside dfmi_nls_record "
                      f"(dfmi_step_timing), mean over {nrep} steps",
            "algorithmic_bytes_per_launch": nall * bytes_per_seg,
            "end_to_end_frac": round(e2e / HBM_PEAK_GBS, 4),
            "end_to_end_note": "SURVEY.md §8(d) algorithmic bytes of the step (8 R + 56 B per segment) / "
                               "ms_per_step / peak: the seed and the LM after the demodulation included"}
    if world > 1:
        roof["avg_launch_ms_max_over_ranks"] = round(demod_ms_max, 4)
        roof["frac_min_over_ranks"] = round(nall * bytes_per_seg / (demod_ms_max * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    # parity on the timed batch itself: status-0 fraction and a sanity check of the estimates
    st = ok.cpu().numpy()
    res = out.cpu().numpy()

    line = {"metric": METRIC, "value": round(value, 1), "unit": "segments/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": plan["scaling"], "vs_baseline": None, "dtype": "f64",
            "data": "synthetic snr-mode DFMI (m=6, 40 dB white noise) generated on device by the counter-based "
                    "dfmi_synth_snr (Philox4x32-10 keyed by (seed, sample index): every rank regenerates buffer 0 "
                    "bit for bit)",
            "config": {"workload": plan["workload"], "record_segments": plan["record_segments"],
                       "segments_per_gpu": nseg, "channels": nrec, "R": R, "ndata": NDATA,
                       "parallelism": f"shard{world}"},
            "world": {"size": world, "backend": backend, "ranks": ranks,
                      "launcher": "bench.py self-launch" if os.environ.get("DFMI_SELF_LAUNCHED") else
                      ("torchrun" if world > 1 else "single process")},
            "roofline": roof,
            "kernels_ms": {"step_demod_seed": round(demod_ms, 4), "step_lm": round(lm_step_ms, 4),
                           "demod_rows_alone": round(rows_ms, 4), "lm_alone_all_segments": round(lm_ms, 4)},
            "window_breakdown": window_diag,
            "per_rank_kernels_ms": per_rank,
            "batch_status0_frac": float(np.mean(st == 0)),
            "batch_m_mean": float(res[1].mean())}
    if args.tune:
        line["tuning"] = args.tune
    if world == 1 and nrec == 1 and args.segments is None:
        # the N = 1 point of the driver's 1 -> 8 curve, on the workload rank 0 fits at N = 8
        del x, out, ok, qi, dcb, rows, lm_out, lm_ssq, lm_st
        torch.cuda.empty_cache()
        line["scaling_anchor"] = scaling_anchor(torch, dev, lib, _lib, stream, cfg, args.steps, args.warmup)
    if world == 1 and not args.no_extra and nrec == 1 and args.segments is None:
        line["extra_configs"] = extra_configs(torch, dev, lib, _lib, stream, cfg, want_base)
    if pre is not None:
        raw, ref, procs, base, base_c = pre
        df = StandardNLSFitter({"n": N_CYC}).fit(raw, parallel=True, n_cores=procs)  # same chunking, on GPU
        line["cpu_baseline"] = base
        line["cpu_baseline_c"] = base_c
        line["parity"] = parity_vs_oracle(df, ref)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
