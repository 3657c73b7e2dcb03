"""Replay the EKF parallel-in-time stop rule (ekf_pit.h pit_decide) on recorded per-pass moves
(scripts/probe_pit_moves.py output) for rule variants, on the host: per variant, how many
channels converge, after how many passes, how many are handed to the sequential kernel, and how
many of those are well-conditioned (S <= 1e-14). The default variant is checked against the host
build of pit_decide itself (tests/hostcheck hc_pit_decide).
usage: python scripts/study/pit_rule_replay.py pit_moves.jsonl"""
import ctypes
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIG = 1.7976931348623157e308


def fmax(a, b):
    """C fmax: a NaN operand is ignored."""
    if a != a:
        return b
    if b != b:
        return a
    return max(a, b)


def decide(moves, tol=1e-13, stall_max=3, cap=48, trend=4, min_pass=0, slow_floor=0.5, slow_from=16, env=True):
    """pit_decide over a channel's move sequence: (passes when the status left 0, status).
    slow_from / env: round 6's transient grace and envelope test (slow_from=0, env=False: the
    round-5 rule)."""
    dprev, rho_c, stall = math.nan, -1.0, 0
    dold = [math.nan] * trend
    for pass_ in range(min(cap, len(moves))):
        d = math.nan if pass_ == 0 else moves[pass_]
        if d is None:
            d = math.nan
        status = 0
        if d == 0.0:
            status = 1
        elif not (d <= BIG):
            if pass_ >= 1:
                status = 2
        else:
            rho = -1.0
            if dprev > 0.0 and dprev <= BIG:
                q = d / dprev
                if dprev > tol and d > tol:
                    rho = max(q, rho_c) if rho_c >= 0.0 else q
                    rho_c = q
                elif d > tol:
                    rho = q
                else:
                    rho = rho_c
            if rho < 0.0:
                if d <= tol:
                    status = 1
            elif rho < 1.0 and rho / (1.0 - rho) * d <= tol:
                status = 1
            if env and status == 0 and pass_ >= 3:
                dk, dk2 = fmax(d, dold[0]), fmax(dold[1], dold[2])
                if 0.0 < dk <= BIG and 0.0 < dk2 <= BIG:
                    r = math.sqrt(dk / dk2)
                    if r < 1.0 and 2.0 * dk * r / (1.0 - r) <= tol:
                        status = 1
            if status == 0 and d > tol:
                w, dw = 0, 0.0
                for i in range(trend):
                    if dold[i] > 0.0 and dold[i] <= BIG:
                        w, dw = i + 1, dold[i]
                if w > 0:
                    rt = (d / dw) ** (1.0 / w)
                    slow = rt >= 1.0
                    if not slow and rt >= slow_floor and pass_ + 1 >= slow_from:
                        need = math.log(tol * (1.0 - rt) / (rt * d)) / math.log(rt)
                        slow = pass_ + 1 + need > cap
                    stall = stall + 1 if slow else 0
                    if stall >= stall_max and pass_ + 1 >= min_pass:
                        status = 2
        dold = [d] + dold[:-1]
        dprev = d
        if status:
            return pass_ + 1, status
    return min(cap, len(moves)), 0


def main():
    rows = [json.loads(v) for v in open(sys.argv[1])]
    hc = ctypes.CDLL(os.path.join(ROOT, "tests", "hostcheck", "libhostcheck.so"))
    hc.hc_pit_decide.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
    variants = [dict(), dict(slow_from=0, env=False), dict(env=False), dict(slow_from=0), dict(slow_from=20),
                dict(slow_from=24)]
    for v in variants:
        tot = dict(ch=0, conv=0, seq=0, seq_well=0, well=0, passes_conv=0, seq_pass=[])
        for r in rows:
            cap = r["cap"]
            for c, mv in enumerate(r["moves"]):
                p, st = decide(mv, cap=cap, **v)
                if not v:  # the host build of pit_decide agrees with this replica
                    arr = np.array([np.nan if a is None else a for a in mv], dtype=np.float64)
                    po, so = ctypes.c_int(), ctypes.c_int()
                    hc.hc_pit_decide(arr.ctypes.data, len(mv), 1e-13, 3, cap, ctypes.byref(po), ctypes.byref(so))
                    assert (po.value, so.value) == ((p, st) if st else (0, 0)), (r["batch"], c, p, st, po.value, so.value)
                well = r["sens"][c] <= 1e-14
                tot["ch"] += 1
                tot["well"] += well
                if st == 1:
                    tot["conv"] += 1
                    tot["passes_conv"] += p
                else:
                    tot["seq"] += 1
                    tot["seq_well"] += well
                    tot["seq_pass"].append(p)
        sp = np.array(tot.pop("seq_pass"))
        print(v or "default", {k: int(x) for k, x in tot.items()},
              "mean passes when converged", round(tot["passes_conv"] / max(1, tot["conv"]), 1),
              "hand-over pass median", float(np.median(sp)) if sp.size else None)


if __name__ == "__main__":
    main()
