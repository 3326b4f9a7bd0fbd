"""Comparison of decision traces (nifty_amd/minimization/trace.py) between a
build run and reference runs: shared by tests/test_geovi_trace_gpu.py (build
vs the reference's recorded traces) and tests/test_geovi_batch_gpu.py
(batched vs per-sample path).  Helpers only, no tests."""
import numpy as np

RTOL_FLOOR = 1e-9
CHAOS = 1e-3    # relative spread of the reference's own runs beyond which it does not reproduce itself


def our_events(events, s):
    from nifty_amd.minimization import trace
    bt = trace.by_tag(events)
    pair = s // 2
    lin = trace.solves(bt.get(("lin", pair), []))
    assert len(lin) == 1, f"linear solve of pair {pair}: {len(lin)} solves traced"
    newton = [v for _, v in bt.get(("newton", s), [])]
    dirs = trace.solves(bt.get(("dir", s), []))
    trials = trace.trials(bt.get(("trial", s), []))
    trialE = trace.trials(bt.get(("trialE", s), []))
    ev = [("lin", lin[0]), ("newton", newton[:1])]
    for j, d in enumerate(dirs):
        ev += [("dir", d), ("trial", trials[j] if j < len(trials) else []),
               ("trialE", trialE[j] if j < len(trialE) else [])]
        if j + 1 < len(newton):
            ev.append(("newton", newton[j + 1:j + 2]))
    return ev


def envelope(vb, perts, n, window=3):
    """per index j < n: 10x the largest |base - perturbed| over the perturbed
    runs and the indices j-window..j+window (the reference's own local
    rounding sensitivity), floor RTOL_FLOOR |base|"""
    s = np.zeros(n)
    for vp in perts:
        m = min(n, len(vp))
        s[:m] = np.maximum(s[:m], np.abs(np.asarray(vb[:m]) - np.asarray(vp[:m])))
    env = np.array([s[max(0, j - window):j + window + 1].max() for j in range(n)]) if n else s
    return 10 * env + RTOL_FLOOR * np.abs(np.asarray(vb[:n]))


def compare(ours, base, perts, stop_at=None):
    """Walk the events of one sample while the reference reproduces itself.

    Per event, with n checks common to all runs:
    * values: the build's within the reference's envelope (envelope) up to
      the first check where the reference's own runs spread by more than
      CHAOS (relative) -- past it the reference does not reproduce itself;
    * decision (number of checks / Newton steps / trial steps):
      - values never chaotic and all reference runs agree: the build's equals
        it exactly;
      - values never chaotic but the reference runs disagree (a threshold
        decision on values that agree to CHAOS, e.g. AbsDelta(0.05) on
        energies of 2e3): the build's lies in the range they span;
      - values chaotic inside the event (e.g. a near-zero-curvature CG step
        of the geoVI Newton metric): the decision follows the chaotic values
        and is only required to be a valid one.
    The walk stops after an event whose decision or values the reference
    does not reproduce: everything after it depends on that outcome.
    ``stop_at`` = (event, check): a diagnosed defect of the reference at that
    point (its values there are not a valid target); compared up to it.
    Returns (n events compared, stable throughout, worst value ratio, log)."""
    worst, log = 0.0, []
    for i, (kb, vb) in enumerate(base):
        pv = [p[i][1] for p in perts if i < len(p)]
        assert all(p[i][0] == kb for p in perts if i < len(p))
        assert i < len(ours), f"event {i} ({kb}) missing in the build's trace"
        ko, vo = ours[i]
        assert ko == kb, (i, ko, kb)
        n = min([len(vo), len(vb)] + [len(v) for v in pv])
        if stop_at is not None and i == stop_at[0]:
            n = min(n, stop_at[1])
        # non-finite values (inf energies of a line-search trial step past an
        # overflow, EnergyAdapter(nanisinf=True)) must coincide
        fin = [j for j in range(n) if np.isfinite(vb[j]) and all(np.isfinite(v[j]) for v in pv)]
        for j in range(n):
            if j not in fin:
                assert np.isfinite(vo[j]) == np.isfinite(vb[j]), \
                    f"event {i} ({kb}) index {j}: build {vo[j]!r}, reference {vb[j]!r}"
        vb = [x if np.isfinite(x) else 0.0 for x in vb]
        pv = [[x if np.isfinite(x) else 0.0 for x in v] for v in pv]
        vo = [x if np.isfinite(x) else 0.0 for x in vo]
        chaos = n
        for j in range(n):
            spread = max(abs(v[j] - vb[j]) for v in pv) if pv else 0.0
            if spread > CHAOS * max(abs(vb[j]), 1e-300):
                chaos = j
                break
        if chaos:
            tol = envelope(vb, pv, chaos)
            err = np.abs(np.asarray(vo[:chaos]) - np.asarray(vb[:chaos]))
            ratio = np.where(err == 0, 0.0, err / np.maximum(tol, 1e-300))
            r = float(ratio.max())
            worst = max(worst, r)
            j = int(ratio.argmax())
            assert r <= 1.0, (f"event {i} ({kb}) index {j}: build {vo[j]!r} vs reference {vb[j]!r} "
                              f"(perturbed {[v[j] for v in pv if j < len(v)]}), ratio {r:.3g}")
        lens = [len(vb)] + [len(v) for v in pv]
        if stop_at is not None and i == stop_at[0]:
            log.append(f"event {i} ({kb}): compared up to check {n}, the reference's diagnosed defect: stop")
            return i + 1, False, worst, log
        if chaos < n:
            assert len(vo) >= 1
            log.append(f"event {i} ({kb}): reference values spread > {CHAOS:g} from check {chaos}, "
                       f"decisions {lens}, build {len(vo)}: stop")
            return i + 1, False, worst, log
        if len(set(lens)) > 1 or len(pv) < len(perts):
            assert min(lens) <= len(vo) <= max(lens), \
                f"event {i} ({kb}): build takes {len(vo)} steps, reference runs {lens}"
            log.append(f"event {i} ({kb}): reference decisions differ {lens}, build {len(vo)}: stop")
            return i + 1, False, worst, log
        assert len(vo) == len(vb), f"event {i} ({kb}): build takes {len(vo)} steps, reference {len(vb)}"
    stable = all(len(p) == len(base) for p in perts)
    if stable:
        assert len(ours) == len(base), f"build trace has {len(ours)} events, reference {len(base)}"
    return len(base), stable, worst, log
