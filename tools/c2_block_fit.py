"""VERDICT r3 item 1 / VERDICT r4 item 1 / ADVICE r4 (CPU only): which failure
explains round 3's wrong C2 covariance (step 6 of
test_c2_full_size_lockstep_vs_oracle, gpurun_out/var3e/pytest.log:92-103)?

Step 6 is a resample step.  Both likelihood modes on two handles returned the
same matrix (ACTUAL below, 4.5e-4 relative off), with x_est, the argmax and the
separately checked resample indices right.  The lockstep had loaded the
oracle's step-6 prior state with set_state, so only device state that
set_state does not rewrite can be stale: the other ping-pong particle buffer,
the run marks and block carries of step 3's resample, the block partials of
step 5, the weights.

Recomputes the oracle trajectory of the C2 fixture (tests/conftest.py
c2_trajectory) to step 6 and fits each hypothesis to ACTUAL, per 512-particle
fused block (or per resample run) where it is local:

  lost      one block's partial missing from the sums (round 4's test);
  stale5    one block's partial is its step-5 value (a relaxed
            ticket that let the finalize read the previous step's record);
  pingpong  one block gathers its sources from the non-current particle
            buffer (the step-5 prior state: set_state rewrote the current one);
  nogather  one block skips the gather (its own un-resampled particles);
  carry3    one block starts its running max from step 3's carry;
  marks3    one block also accepts step 3's run marks (a tag test that fails);
  misrun    one run's start mark missed: its positions take the previous
            run's source;
  noreset   (global) the post-resample weights are not reset to 1/NP;
  lost / stale5 again per 128-, 256-, 1024-, 2048-, 4096- and 8192-element unit;
  (round 6)
  torn65    one block's record torn: its max from step 6 with its scaled sums
            from step 5 (the finalize rescales step 5's sums by M6_b / M);
  torn56    the reverse: step 5's max with step 6's scaled sums;
  tornf     one block, one field (S0, one of S1's 3, one of S2's 6) from step 5,
            the rest of the record from step 6;
  refp4     one block (or a group of 16 / 128 / 512 blocks, or an XCD) formed
            its moments about the wrong reference point, the estimate two steps
            back (the other refp slot) instead of the previous one.

Prints the best fit of each (max relative error over the six distinct entries
of ACTUAL, which the log printed to 7 digits: a true cause fits to ~1e-6).
Reference: /root/reference/particle_filter.py:200-224 (resampling),
:226-237 (normalisation)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import pf_oracle as po  # noqa: E402

ACTUAL = np.array([[6.645246e-06, -3.528556e-05, -2.212189e-06],
                   [-3.528556e-05, 3.669996e-04, 2.066460e-05],
                   [-2.212189e-06, 2.066460e-05, 5.692706e-06]])
DESIRED = np.array([[6.645041e-06, -3.530142e-05, -2.212044e-06],
                    [-3.530142e-05, 3.671349e-04, 2.067047e-05],
                    [-2.212044e-06, 2.067047e-05, 5.692871e-06]])
IU = np.triu_indices(3)
B = 512                                   # fused block (kPartPer)


def lik(p, x, y, th, z, chunk=1 << 17):
    out = np.empty(x.size)
    for a in range(0, x.size, chunk):
        f = po.landmark_factors(x[a:a + chunk], y[a:a + chunk], th[a:a + chunk], p.lm, z, p.r)
        out[a:a + chunk] = f.prod(axis=1)
    return out


def moments(w, P, nb):
    """per-block S0 (nb), S1 (nb,3), S2 (nb,3,3) of weights w and centred P (3, n)."""
    wb = w.reshape(nb, -1)
    Pb = P.reshape(3, nb, -1)
    return wb.sum(1), np.einsum("nb,inb->ni", wb, Pb), np.einsum("nb,inb,jnb->nij", wb, Pb, Pb)


def cov_of(S0, S1, S2):
    mu = S1 / S0
    return S2 / S0 - np.outer(mu, mu)


def err(C):
    return float(np.max(np.abs(C[IU] - ACTUAL[IU]) / np.abs(ACTUAL[IU])))


def best_local(name, tot, alt_b, base_b):
    """Replace one unit's moments (alt for base), fit each; report the best.
    Also every unit of one XCD at once (blockIdx % 8: the eight L2s are not
    coherent with each other for plain stores), and every unit."""
    S0, S1, S2 = tot
    a0, a1, a2 = alt_b
    b0, b1, b2 = base_b
    n = a0.shape[0]
    e = np.empty(n)
    for k in range(n):
        e[k] = err(cov_of(S0 - b0[k] + a0[k], S1 - b1[k] + a1[k], S2 - b2[k] + a2[k]))
    k = int(np.argmin(e))
    changed = int(np.count_nonzero((a0 != b0) | np.any(a1 != b1, axis=1)))
    xcd = [err(cov_of(S0 + (a0 - b0)[x::8].sum(0), S1 + (a1 - b1)[x::8].sum(0),
                      S2 + (a2 - b2)[x::8].sum(0))) for x in range(8)]
    every = err(cov_of(S0 + (a0 - b0).sum(0), S1 + (a1 - b1).sum(0), S2 + (a2 - b2).sum(0)))
    print(f"{name:9s} best single-unit fit {e[k]:.3g} (unit {k} of {n}; {changed} units differ); "
          f"best XCD {min(xcd):.3g} (xcd {int(np.argmin(xcd))}); every unit {every:.3g}")
    return e


def main():
    n, nl = 1 << 20, 100
    nb = n // B
    rs = np.random.RandomState(1)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm, motion="velocity")
    orc, world = po.PFOracle(p), po.PFWorld(p)
    np.random.seed(2)
    steps = []
    for _ in range(7):
        world.advance()
        state = (orc.x.copy(), orc.y.copy(), orc.th.copy(), orc.w.copy())
        u = np.random.rand() if orc.needs_resample() else None
        g = np.random.standard_normal(3 * n).reshape(n, 3)
        z = world.observe()
        out = orc.step(z, g, None if u is None else u * p.np_recip)
        steps.append(dict(state=state, g=g, z=z, out=out, u=u,
                          post=(orc.x.copy(), orc.y.copy(), orc.th.copy(), orc.w.copy())))
    s6 = steps[6]
    assert s6["out"]["resampled"] and steps[3]["out"]["resampled"]
    print("oracle step 6 vs the failing run's DESIRED:",
          float(np.max(np.abs(s6["out"]["cov"] - DESIRED) / np.abs(DESIRED))))
    print("DESIRED vs ACTUAL:", err(DESIRED))
    g6, z6 = s6["g"], s6["z"]
    idx6, idx3 = s6["out"]["idx"], steps[3]["out"]["idx"]
    x6, y6, t6, w6 = s6["state"]
    ref = np.ravel(steps[5]["out"]["x_est"])        # the device centres on the previous estimate

    def predict(x, y, th):
        return po.motion_velocity(x, y, th, p.vel, p.omega, p.dt, p.alphas, g6)

    def unit_moments(xs, ys, ts, w_un):
        return moments(w_un, np.vstack([xs - ref[0], ys - ref[1], ts - ref[2]]), nb)

    # the true step 6 (device-equivalent w_un = 1/NP * lik)
    X, Y, T = predict(x6[idx6], y6[idx6], t6[idx6])
    L = lik(p, X, Y, T, z6)
    w_un = p.np_recip * L
    base = unit_moments(X, Y, T, w_un)
    tot = tuple(m.sum(0) for m in base)
    print("true step 6 from block moments vs DESIRED:",
          float(np.max(np.abs(cov_of(*tot) - DESIRED) / np.abs(DESIRED))))
    zero = (np.zeros(nb), np.zeros((nb, 3)), np.zeros((nb, 3, 3)))
    results = {}
    results["lost"] = best_local("lost", tot, zero, base)

    # stale5: the block's step-5 partial (its own particles, w_un = w_prev * lik,
    # centred on the estimate before step 5), read as if it were step 6's
    X5, Y5, T5, _ = steps[5]["post"]
    w_prev5 = steps[5]["out"]["w_prev"]
    L5 = steps[5]["out"]["bn"]
    ref5 = np.ravel(steps[4]["out"]["x_est"])
    st5 = moments(w_prev5 * L5, np.vstack([X5 - ref5[0], Y5 - ref5[1], T5 - ref5[2]]), nb)
    results["stale5"] = best_local("stale5", tot, st5, base)

    # pingpong: sources read from the step-5 prior state
    x5, y5, t5, _ = steps[5]["state"]
    Xp, Yp, Tp = predict(x5[idx6], y5[idx6], t5[idx6])
    results["pingpong"] = best_local("pingpong", tot,
                                     unit_moments(Xp, Yp, Tp, p.np_recip * lik(p, Xp, Yp, Tp, z6)),
                                     base)

    # nogather: the block's own particles; weights still 1/NP (rflag read once)
    Xn, Yn, Tn = predict(x6, y6, t6)
    Ln = lik(p, Xn, Yn, Tn, z6)
    results["nogather"] = best_local("nogather", tot, unit_moments(Xn, Yn, Tn, p.np_recip * Ln), base)

    # carry3 / marks3: per block, the running max over step 6's marks started
    # from step 3's carry, or over the union of both steps' marks
    pos = np.arange(n)

    def run_starts(idx):
        st = np.ones(n, bool)
        st[1:] = idx[1:] != idx[:-1]
        return st

    m6 = np.where(run_starts(idx6), idx6, -1)
    m3 = np.where(run_starts(idx3), idx3, -1)

    def gather_by_marks(marks, carry):
        r = np.maximum.accumulate(marks.reshape(nb, B), axis=1)
        return np.maximum(r, carry[:, None]).ravel()

    carry6 = idx6[pos[::B]]
    carry3 = idx3[pos[::B]]
    assert np.array_equal(gather_by_marks(m6, carry6), idx6)

    def alt_from_src(src):
        Xa, Ya, Ta = predict(x6[src], y6[src], t6[src])
        return unit_moments(Xa, Ya, Ta, p.np_recip * lik(p, Xa, Ya, Ta, z6))

    results["carry3"] = best_local("carry3", tot, alt_from_src(gather_by_marks(m6, carry3)), base)
    results["marks3"] = best_local("marks3", tot,
                                   alt_from_src(gather_by_marks(np.maximum(m6, m3), carry6)), base)

    # misrun: run j's positions take run j-1's source (one run at a time)
    st = run_starts(idx6)
    rid = np.cumsum(st) - 1
    nr = int(rid[-1]) + 1
    src_of_run = idx6[st]
    prev_src = np.where(rid > 0, src_of_run[np.maximum(rid - 1, 0)], idx6)
    a = alt_from_src(prev_src)
    # per-run sums of (alt - base) at particle level
    Xb = np.vstack([X - ref[0], Y - ref[1], T - ref[2]])
    Xa, Ya, Ta = predict(x6[prev_src], y6[prev_src], t6[prev_src])
    wa = p.np_recip * lik(p, Xa, Ya, Ta, z6)
    Pa = np.vstack([Xa - ref[0], Ya - ref[1], Ta - ref[2]])
    d0 = np.bincount(rid, wa - w_un, nr)
    d1 = np.stack([np.bincount(rid, wa * Pa[i] - w_un * Xb[i], nr) for i in range(3)], 1)
    d2 = np.stack([np.stack([np.bincount(rid, wa * Pa[i] * Pa[j] - w_un * Xb[i] * Xb[j], nr)
                             for j in range(3)], 1) for i in range(3)], 1)
    del a
    e = np.array([err(cov_of(tot[0] + d0[k], tot[1] + d1[k], tot[2] + d2[k])) for k in range(nr)])
    k = int(np.argmin(e))
    print(f"{'misrun':9s} best single-run fit {e[k]:.3g} (run {k} of {nr}, source {src_of_run[k]}, "
          f"{int(np.sum(rid == k))} positions)")
    results["misrun"] = e

    # noise5: the block predicts with step 5's normals (a stale noise upload)
    Xg, Yg, Tg = po.motion_velocity(x6[idx6], y6[idx6], t6[idx6], p.vel, p.omega, p.dt,
                                    p.alphas, steps[5]["g"])
    results["noise5"] = best_local("noise5", tot,
                                   unit_moments(Xg, Yg, Tg, p.np_recip * lik(p, Xg, Yg, Tg, z6)),
                                   base)

    # one particle: removed, or its weight doubled (any single heavy particle)
    w1 = w_un[None, :]
    c0 = tot[0] - w_un
    c1 = tot[1][:, None] - w_un * Xb
    c2 = tot[2][:, :, None] - w_un * Xb[:, None, :] * Xb[None, :, :]
    mu = c1 / c0
    C = c2 / c0 - mu[:, None, :] * mu[None, :, :]
    e = np.max(np.abs(C[IU[0], IU[1], :] - ACTUAL[IU][:, None]) / np.abs(ACTUAL[IU][:, None]), 0)
    k = int(np.argmin(e))
    print(f"{'particle':9s} best single-particle removal {e[k]:.3g} (position {k}, weight share "
          f"{w_un[k] / tot[0]:.3g})")
    del C, c2, w1

    # noreset: w_un = w_prior[src] * lik, or w_prior (ungathered) * lik
    for nm, wp in (("noreset_g", w6[idx6]), ("noreset_u", w6)):
        S = tuple(m.sum(0) for m in unit_moments(X, Y, T, wp * L))
        print(f"{nm:9s} global fit {err(cov_of(*S)):.3g}")

    # the one-unit hypotheses at every granularity a hand-off could
    # have (a 128-element leaf ... an 8192-element np.sum buffer), lost and stale5
    Pb6 = np.vstack([X - ref[0], Y - ref[1], T - ref[2]])
    Pb5 = np.vstack([X5 - ref5[0], Y5 - ref5[1], T5 - ref5[2]])
    for size in (128, 256, 1024, 2048, 4096, 8192):
        m = n // size
        base_s = moments(w_un, Pb6, m)
        tot_s = tuple(q.sum(0) for q in base_s)
        zero_s = (np.zeros(m), np.zeros((m, 3)), np.zeros((m, 3, 3)))
        best_local(f"lost@{size}", tot_s, zero_s, base_s)
        best_local(f"stale5@{size}", tot_s, moments(w_prev5 * L5, Pb5, m), base_s)
    # round 6: torn records and the wrong reference point
    M6 = w_un.reshape(nb, B).max(1)
    M5 = (w_prev5 * L5).reshape(nb, B).max(1)
    r65 = (M6 / M5)
    b5 = st5                                             # step-5 raw moments (centred on ref5)
    results["torn65"] = best_local("torn65", tot, (b5[0] * r65, b5[1] * r65[:, None],
                                                   b5[2] * r65[:, None, None]), base)
    results["torn56"] = best_local("torn56", tot, (base[0] / r65, base[1] / r65[:, None],
                                                   base[2] / r65[:, None, None]), base)
    # one field of one block from step 5 (rescaled by M6_b / M5_b)
    best = (np.inf, None)
    fields = [("S0", None)] + [(f"S1[{i}]", i) for i in range(3)] + \
             [(f"S2[{i}{j}]", (i, j)) for i in range(3) for j in range(i, 3)]
    for name, f in fields:
        for k in range(nb):
            S0, S1, S2 = tot[0], tot[1].copy(), tot[2].copy()
            if f is None:
                S0 = S0 - base[0][k] + b5[0][k] * r65[k]
            elif isinstance(f, int):
                S1[f] += b5[1][k][f] * r65[k] - base[1][k][f]
            else:
                i, j = f
                d = b5[2][k][i, j] * r65[k] - base[2][k][i, j]
                S2[i, j] += d
                if i != j:
                    S2[j, i] += d
            e = err(cov_of(S0, S1, S2))
            if e < best[0]:
                best = (e, f"{name} of block {k}")
    print(f"{'tornf':9s} best single-field fit {best[0]:.3g} ({best[1]})")
    # refp4: moments about the estimate two steps back
    ref4 = np.ravel(steps[4]["out"]["x_est"])
    Pw = np.vstack([X - ref4[0], Y - ref4[1], T - ref4[2]])
    alt4 = moments(w_un, Pw, nb)
    results["refp4"] = best_local("refp4", tot, alt4, base)
    for g in (16, 128, 512):
        m = nb // g
        grp = lambda q: q.reshape((m, g) + q.shape[1:]).sum(1)
        best_local(f"refp4@{g}blk", tot, tuple(grp(q) for q in alt4), tuple(grp(q) for q in base))
    print("(a true cause fits to ~1e-6, the printing precision of ACTUAL)")
    return results


if __name__ == "__main__":
    main()
