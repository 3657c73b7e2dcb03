"""EKF parallel-in-time stop rule study (round 6): the per-pass moves d_k (the stop rule's own
input, dfmi_ekf_pit_trace) of every channel of the stress set (tests/helpers/ekf_stress.py) with
the stall hand-over switched off (ekf_pit_stall 1000: a channel passes until it converges or
reaches the cap), and whether the channel is well-conditioned (the C oracle's one-ulp
sensitivity S <= 1e-14, tests/test_gpu_ekf_pit_stress.py). The moves do not depend on the rule
(each channel's iteration is its own), so the rule can be replayed on the host
(tests/hostcheck hc_pit_decide) for any parameters: scripts/study/pit_rule_replay.py.
Writes one JSON line per batch to stdout."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
import ekf_stress as S  # noqa: E402


def main():
    from deepfmkit_amd import _lib
    lib = _lib.load()
    cl = S.c_oracle()
    for k, v in (("ekf_pit_trace", 1), ("ekf_pit_stall", 1000)):
        _lib.check(lib.dfmi_set_tuning(k.encode(), v), k)
    for bi, (n, nch, R) in enumerate(S.BATCHES):
        x, x0, rv, qd, meta = S.batch_inputs(bi, n, nch)
        nbuf = n // R
        got, kname, passes = S.gpu_states(lib, x, x0, rv, qd, R, nbuf)
        cap = int(min(256, max(48, n // 1600)))
        moves = np.zeros((nch, cap))
        _lib.check(lib.dfmi_ekf_pit_trace(moves.ctypes.data, nch, cap), "trace")
        ref, sens = S.oracle_batch(cl, x, x0, rv, qd, R, nbuf)
        err = S.rel_err(got, ref)
        print(json.dumps({"batch": bi, "n": n, "channels": nch, "R": R, "cap": cap, "kernel": kname,
                          "passes": passes.tolist(), "sens": sens.tolist(), "err": err.tolist(),
                          "moves": [[None if not np.isfinite(v) else float(v) for v in row] for row in moves]}),
              flush=True)


if __name__ == "__main__":
    main()
