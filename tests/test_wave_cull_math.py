"""CPU check of the geometry behind the wave-level shadow cull (trace_kernels.h step_cands).

The device skips an objList entry for a whole wave when every lane's shadow segment
[p_l, L] provably misses the entry's bounding sphere (or stays strictly on one side of a
quad's / plane's world plane). The argument: every lane segment lies within sp of the first
lane's segment [p_f, L], sp = max-norm spread of the hit points x sqrt 3. These tests restate
the device's formulas in numpy (same expressions, float64) and check on random waves that no
entry a lane's segment actually reaches is ever skipped -- the conservative direction is the
only one that matters for parity (a kept entry is still tested per lane).
"""
import numpy as np

SQRT3 = 1.7320508075688776


def wave_spread(p):
    pf = p[0]
    return np.max(np.abs(p - pf)) * SQRT3, pf


def sphere_candidate(pf, sp, L, c, R):
    """step_cands' sphere test for one (light, entry) pair, as the device evaluates it."""
    pn = np.max(np.abs(pf))
    v = L - pf
    vv = v @ v
    vl = np.sqrt(vv)
    w = c - pf
    wv = w @ v
    ww = w @ w
    Q = (R + sp + 1e-9 * (1 + vl + sp + pn + R)) * (1 + 1e-9)
    Q2 = Q * Q
    perp = ww * vv - wv * wv
    slackP = 1e-9 * (ww * vv + Q2 * vv)
    slackT = 1e-9 * (np.sqrt(ww) * vl + vv)
    qv = Q * vl
    return not (perp > Q2 * vv + slackP or wv < -qv - slackT or wv > vv + qv + slackT)


def plane_off(pf, sp, L, n, d):
    """step_cands' plane-side test (one plane): True when the wave's segments stay strictly on
    one side of n . y + d = 0."""
    pn = np.max(np.abs(pf))
    m = 1e-6 * (1 + pn + np.max(np.abs(L)))
    mm = m * (1 + abs(d))
    sP = n @ pf + d
    sL = n @ L + d
    return (sP - sp > mm and sL > mm) or (sP + sp < -mm and sL < -mm)


def seg_sphere_dist(a, b, c):
    ab = b - a
    t = np.clip((c - a) @ ab / (ab @ ab), 0.0, 1.0)
    q = a + t * ab
    return np.sqrt((c - q) @ (c - q))


def test_sphere_cull_never_skips_a_reachable_entry():
    rng = np.random.default_rng(1234)
    skipped = kept_hit = 0
    for _ in range(4000):
        centre = rng.uniform(-5, 5, 3)
        spread = 10 ** rng.uniform(-4, 0)
        p = centre + rng.uniform(-spread, spread, (64, 3))
        L = rng.uniform(-10, 10, 3)
        sp, pf = wave_spread(p)
        R = 10 ** rng.uniform(-2, 0.5)
        if rng.uniform() < 0.5:  # near some lane's segment: reachable or just missed
            pl = p[rng.integers(64)]
            c = pl + rng.uniform(0, 1) * (L - pl) + rng.normal(size=3) * R * rng.uniform(0.5, 1.5)
        else:
            c = rng.uniform(-8, 8, 3)
        cand = sphere_candidate(pf, sp, L, c, R)
        reach = min(seg_sphere_dist(pl, L, c) for pl in p) <= R
        if reach:
            kept_hit += 1
            assert cand, (centre, spread, L, c, R)
        elif not cand:
            skipped += 1
    # the test is useful (skips most unreachable entries) and was exercised on reachable ones
    assert skipped > 1000 and kept_hit > 100


def test_plane_side_never_skips_a_crossing_segment():
    rng = np.random.default_rng(99)
    off_count = crossing = 0
    for _ in range(4000):
        n = rng.normal(size=3)
        n /= np.sqrt(n @ n)
        d = rng.uniform(-3, 3)
        centre = rng.uniform(-5, 5, 3)
        spread = 10 ** rng.uniform(-4, 0.3)
        p = centre + rng.uniform(-spread, spread, (64, 3))
        if rng.uniform() < 0.2:  # hit points on the plane itself (shading a ground quad)
            p = p - np.outer(p @ n + d, n)
        L = rng.uniform(-10, 10, 3)
        sp, pf = wave_spread(p)
        off = plane_off(pf, sp, L, n, d)
        s = p @ n + d
        sL = L @ n + d
        crosses = np.any((s <= 0) != (sL <= 0)) or np.any(np.abs(s) < 1e-12)
        if crosses:
            crossing += 1
            assert not off
        elif off:
            off_count += 1
    assert off_count > 1000 and crossing > 500


def test_spread_bounds_every_lane_segment():
    """The hull argument itself: the point at fraction s of lane l's segment is within sp of the
    point at fraction s of the first lane's segment."""
    rng = np.random.default_rng(7)
    for _ in range(500):
        p = rng.uniform(-1, 1, 3) + rng.uniform(-0.3, 0.3, (64, 3))
        L = rng.uniform(-10, 10, 3)
        sp, pf = wave_spread(p)
        s = rng.uniform(0, 1, (64, 1))
        a = p + s * (L - p)
        b = pf + s * (L - pf)
        assert np.all(np.sqrt(np.sum((a - b) ** 2, axis=1)) <= sp * (1 + 1e-12))
