"""Host-side checks of the algebra the parallel-in-time EKF (deepfmkit_amd/csrc/ekf_pit.h)
rests on, in numpy (no GPU):

* the filtering elements of a linear-Gaussian model with F = I and their associative
  combine (Sarkka & Garcia-Fernandez 2021, Lemma 8) scanned in any grouping give the
  sequential Kalman filter's means and covariances;
* the rank-1 fold ekf_pit_aggregate_kernel applies per sample equals the general combine
  with that sample's element;
* the whole scheme — linearize at xbar, fold blocks, scan the block aggregates, re-run the
  true EKF per block from the scanned entry states, repeat — converges to the sequential EKF
  of fitters.py:274-302 (oracle/nls_oracle.py ekf_record's loop) on a short record.
"""
import numpy as np

I5 = np.eye(5)


def combine(ei, ej):
    """ei (earlier) (x) ej: M = (I + C_i J_j)^-1 ... (the kernel's pit_combine)."""
    Ai, bi, Ci, hi, Ji = ei
    Aj, bj, Cj, hj, Jj = ej
    M = np.linalg.inv(I5 + Ci @ Jj)
    A = Aj @ M @ Ai
    b = Aj @ M @ (bi + Ci @ hj) + bj
    C = Aj @ M @ Ci @ Aj.T + Cj
    eta = Ai.T @ M.T @ (hj - Jj @ bi) + hi
    J = Ai.T @ M.T @ Jj @ Ai + Ji
    return A, b, C, eta, J


def element(h, e, q, Rv):
    Q = np.diag(q)
    S = h @ Q @ h + Rv
    K = Q @ h / S
    return I5 - np.outer(K, h), K * e, Q - np.outer(Q @ h, Q @ h) / S, h * e / S, np.outer(h, h) / S


def fold(agg, h, e, q, Rv):
    """ekf_pit_aggregate_kernel's rank-1 fold of one sample into the aggregate."""
    A, b, C, eta, J = agg
    g = q * h + C @ h
    gam = Rv + h @ g
    r = A.T @ h
    v = g / gam
    eps = e - h @ b
    return (A - np.outer(v, r), b + v * eps, C + np.diag(q) - np.outer(g, v), eta + r * (eps / gam),
            J + np.outer(r / gam, r))


def identity():
    return I5.copy(), np.zeros(5), np.zeros((5, 5)), np.zeros(5), np.zeros((5, 5))


def test_rank1_fold_equals_general_combine():
    rng = np.random.default_rng(3)
    for _ in range(50):
        X = rng.standard_normal((5, 5))
        Y = rng.standard_normal((5, 5))
        agg = (rng.standard_normal((5, 5)), rng.standard_normal(5), X @ X.T, rng.standard_normal(5), Y @ Y.T)
        h, e = rng.standard_normal(5), rng.standard_normal()
        q, Rv = np.abs(rng.standard_normal(5)) + 1e-3, 0.1 + abs(rng.standard_normal())
        want = combine(agg, element(h, e, q, Rv))
        got = fold(agg, h, e, q, Rv)
        for w, g in zip(want, got):
            np.testing.assert_allclose(g, w, rtol=1e-9, atol=1e-9)


def test_scan_equals_sequential_kalman_filter():
    """Linear model, random H_k: the prior element (A = 0, b = m0, C = P0) folded with the
    samples, in blocks and then scanned, gives the sequential KF's filtered means/covs."""
    rng = np.random.default_rng(5)
    n, q, Rv = 96, np.array([1e-3, 2e-3, 1e-2, 1e-2, 1e-3]), 0.05
    H = rng.standard_normal((n, 5))
    y = rng.standard_normal(n)
    m, P = np.zeros(5), I5.copy()
    seq_m, seq_P = [], []
    for k in range(n):
        P = P + np.diag(q)
        S = H[k] @ P @ H[k] + Rv
        K = P @ H[k] / S
        m = m + K * (y[k] - H[k] @ m)
        P = P - np.outer(K, H[k] @ P)
        seq_m.append(m)
        seq_P.append(P)
    B = 12
    aggs = []
    for b in range(n // B):
        a = (np.zeros((5, 5)), np.zeros(5), I5.copy(), np.zeros(5), np.zeros((5, 5))) if b == 0 else identity()
        for k in range(b * B, (b + 1) * B):
            a = fold(a, H[k], y[k], q, Rv)
        aggs.append(a)
    pre = [aggs[0]]
    for a in aggs[1:]:
        pre.append(combine(pre[-1], a))
    for b in range(n // B):
        k = (b + 1) * B - 1
        np.testing.assert_allclose(pre[b][1], seq_m[k], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(pre[b][2], seq_P[k], rtol=1e-10, atol=1e-12)
    # regrouped (Hillis-Steele order): the same prefixes
    el = list(aggs)
    off = 1
    while off < len(el):
        el = [el[i] if i < off else combine(el[i - off], el[i]) for i in range(len(el))]
        off *= 2
    for b in range(len(el)):
        np.testing.assert_allclose(el[b][1], pre[b][1], rtol=1e-10, atol=1e-12)


def _ekf_step(st, P, xk, wt, q, Rv):
    """fitters.py:276-302 (one sample)."""
    P = P + np.diag(q)
    a, m, phi, psi, dc = st
    th = wt + psi
    arg = phi + m * np.cos(th)
    sa = np.sin(arg)
    H = np.array([np.cos(arg), -a * sa * np.cos(th), -a * sa, a * m * sa * np.sin(th), 1.0])
    S = H @ P @ H + Rv
    K = P @ H / S
    return st + K * (xk - (a * np.cos(arg) + dc)), P - np.outer(K, H @ P)


def _step_h(st, P, xk, wt, q, Rv):
    """_ekf_step that also returns H and h at the predicted state (ekf_step_h)."""
    P = P + np.diag(q)
    a, m, phi, psi, dc = st
    th = wt + psi
    arg = phi + m * np.cos(th)
    sa = np.sin(arg)
    H = np.array([np.cos(arg), -a * sa * np.cos(th), -a * sa, a * m * sa * np.sin(th), 1.0])
    h = a * np.cos(arg) + dc
    S = H @ P @ H + Rv
    K = P @ H / S
    return st + K * (xk - h), P - np.outer(K, H @ P), H, h


def test_fused_pass_converges_to_sequential_ekf():
    """ekf_pit_pass_kernel's iteration: each block runs the EKF from its scanned entry and
    folds every sample's element linearized at the EKF's own predicted state (its H, h), the
    new aggregates are scanned for the next pass; converged when the entry states stop moving
    (1e-11): the states equal the sequential EKF's to ~1e-13."""
    fs, fm, n, B = 200000.0, 1000.0, 2400, 48
    wt = 2 * np.pi * fm * (np.arange(n) / fs)
    rng = np.random.default_rng(9)
    x = 1.1 * np.cos(0.4 + 6.0 * np.cos(wt + 0.1)) + 0.5 + 0.01 * rng.standard_normal(n)
    q, Rv = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8]), float(np.var(x))
    x0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x)])
    st, P, seq = x0.copy(), I5.copy(), []
    for k in range(n):
        st, P = _ekf_step(st, P, x[k], wt[k], q, Rv)
        seq.append(st)
    seq = np.array(seq)
    nb = n // B
    # first aggregates at the trajectory held at x0 (no head here)
    aggs = []
    for b in range(nb):
        a = (np.zeros((5, 5)), x0.copy(), I5.copy(), np.zeros(5), np.zeros((5, 5))) if b == 0 else identity()
        for k in range(b * B, (b + 1) * B):
            xa, m, phi, psi, dc = x0
            th = wt[k] + psi
            arg = phi + m * np.cos(th)
            sa = np.sin(arg)
            h = np.array([np.cos(arg), -xa * sa * np.cos(th), -xa * sa, xa * m * sa * np.sin(th), 1.0])
            a = fold(a, h, x[k] - (xa * np.cos(arg) + dc) + h @ x0, q, Rv)
        aggs.append(a)
    prev = None
    for it in range(14):
        pre = [aggs[0]]
        for a in aggs[1:]:
            pre.append(combine(pre[-1], a))
        ent = [(x0.copy(), I5.copy())] + [(pre[b - 1][1].copy(), pre[b - 1][2].copy()) for b in range(1, nb)]
        new, aggs = np.empty_like(seq), []
        for b in range(nb):
            st, P = ent[b]
            a = (np.zeros((5, 5)), x0.copy(), I5.copy(), np.zeros(5), np.zeros((5, 5))) if b == 0 else identity()
            for k in range(b * B, (b + 1) * B):
                xp = st.copy()
                st, P, H, h = _step_h(st, P, x[k], wt[k], q, Rv)
                a = fold(a, H, x[k] - h + H @ xp, q, Rv)
                new[k] = st
            aggs.append(a)
        e = np.array([v[0] for v in ent])
        moved = np.inf if prev is None else np.max(np.abs(e - prev) / np.maximum(1.0, np.abs(e)))
        prev = e
        if moved <= 1e-11:
            break
    assert moved <= 1e-11, (it, moved)
    assert np.max(np.abs(new - seq)) <= 1e-12, np.max(np.abs(new - seq))


def test_relinearized_scan_converges_to_sequential_ekf():
    """The kernel sequence on a 2,400-sample record (a = 1.1, m = 6, phi = 0.4, psi = 0.1,
    dc = 0.5, 40 dB white noise; fitters.py defaults: Q, P0 = I, x0 = (1.6, 6, 0, 0, mean),
    R = var): xbar within 1e-11 after a few passes, block entry
    states then equal the sequential EKF's to ~1e-13."""
    fs, fm, n, B = 200000.0, 1000.0, 2400, 48
    wt = 2 * np.pi * fm * (np.arange(n) / fs)
    rng = np.random.default_rng(9)
    x = 1.1 * np.cos(0.4 + 6.0 * np.cos(wt + 0.1)) + 0.5 + 0.01 * rng.standard_normal(n)
    q, Rv = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8]), float(np.var(x))
    x0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x)])
    st, P, seq = x0.copy(), I5.copy(), []
    for k in range(n):
        st, P = _ekf_step(st, P, x[k], wt[k], q, Rv)
        seq.append(st)
    seq = np.array(seq)
    xbar = np.tile(x0, (n, 1))
    nb = n // B
    for it in range(12):
        aggs = []
        for b in range(nb):
            a = (np.zeros((5, 5)), x0.copy(), I5.copy(), np.zeros(5), np.zeros((5, 5))) if b == 0 else identity()
            for k in range(b * B, (b + 1) * B):
                xa, m, phi, psi, dc = xbar[k]
                th = wt[k] + psi
                arg = phi + m * np.cos(th)
                sa = np.sin(arg)
                h = np.array([np.cos(arg), -xa * sa * np.cos(th), -xa * sa, xa * m * sa * np.sin(th), 1.0])
                e = x[k] - (xa * np.cos(arg) + dc) + h @ xbar[k]
                a = fold(a, h, e, q, Rv)
            aggs.append(a)
        pre = [aggs[0]]
        for a in aggs[1:]:
            pre.append(combine(pre[-1], a))
        new = np.empty_like(seq)
        for b in range(nb):
            st, P = (x0.copy(), I5.copy()) if b == 0 else (pre[b - 1][1].copy(), pre[b - 1][2].copy())
            for k in range(b * B, (b + 1) * B):
                st, P = _ekf_step(st, P, x[k], wt[k], q, Rv)
                new[k] = st
        moved = np.max(np.abs(new[:-1] - xbar[1:]) / np.maximum(1.0, np.abs(new[:-1])))
        xbar[1:] = new[:-1]
        if moved <= 1e-11:
            break
    assert moved <= 1e-11, (it, moved)
    assert it <= 8, it
    assert np.max(np.abs(new - seq)) <= 1e-12, np.max(np.abs(new - seq))


def _hier_scan(el, W):
    """ekf_pit_run's scan hierarchy in numpy: Hillis-Steele within groups of W, group totals
    one level up (recursively until one group holds a level), then the fix-ups top-down with
    the (0, b, C, 0, 0) form of a prefix from element 0. Returns levels 0 and 1 as the pass
    kernels read them."""
    levels = [list(el)]
    while len(levels[-1]) > W:
        cur = levels[-1]
        tot = []
        for g0 in range(0, len(cur), W):
            grp = cur[g0:g0 + W]
            off = 1
            while off < len(grp):
                grp = [grp[i] if i < off else combine(grp[i - off], grp[i]) for i in range(len(grp))]
                off *= 2
            cur[g0:g0 + W] = grp
            tot.append(grp[-1])
        levels.append(tot)
    top = levels[-1]
    off = 1
    while off < len(top):
        top = [top[i] if i < off else combine(top[i - off], top[i]) for i in range(len(top))]
        off *= 2
    levels[-1] = top
    for lv in range(len(levels) - 2, 0, -1):
        up, cur = levels[lv + 1], levels[lv]
        for g in range(W, len(cur)):
            _, b, C, _, _ = combine(up[g // W - 1], cur[g])
            cur[g] = (np.zeros((5, 5)), b, C, np.zeros(5), np.zeros((5, 5)))
    return levels


def test_scan_hierarchy_with_fixups_gives_every_entry_state():
    """37 block aggregates, groups of 4 (levels 37 -> 10 -> 3, two fix-up levels): the entry
    state of every block read as the pass kernels do (level 0 within its group, preceded by
    the fixed level-1 prefix of the earlier groups) equals the sequential prefix."""
    rng = np.random.default_rng(11)
    q, Rv = np.array([1e-3, 2e-3, 1e-2, 1e-2, 1e-3]), 0.05
    aggs = []
    for b in range(37):
        a = (np.zeros((5, 5)), rng.standard_normal(5), I5.copy(), np.zeros(5), np.zeros((5, 5))) if b == 0 \
            else identity()
        for _ in range(3):
            a = fold(a, rng.standard_normal(5), rng.standard_normal(), q, Rv)
        aggs.append(a)
    seq = [aggs[0]]
    for a in aggs[1:]:
        seq.append(combine(seq[-1], a))
    W = 4
    levels = _hier_scan(aggs, W)
    for b in range(1, 37):
        p = b - 1
        loc = levels[0][p]
        if p // W == 0:
            st, C = loc[1], loc[2]
        else:
            _, st, C, _, _ = combine(levels[1][p // W - 1], loc)
        np.testing.assert_allclose(st, seq[p][1], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(C, seq[p][2], rtol=1e-9, atol=1e-11)
