"""The fp32 triangle edge pre-test (csrc/trace_kernels.h tri_f32_out, RT_F32_TRI) never rejects a lane
that the fp64 triangle test accepts (CPU, numpy).

The pre-test may only say "this lane's triangle test returns false"; the GPU parity tests cover the
product kernels on every scene, and this test attacks the error bound itself where scenes rarely go:
hit points on the edges and within a few ulps of them, grazing rays (n.d near 0), far-off triangles
(|v| >> edge length), tiny and huge scales and unnormalised directions (instance transforms).

The fp64 side restates trace_device.h planar_test<3> (the reference's myPlanarObject.java:165-211
triangle test, with the orientation of Q5) in the same operation order; the fp32 side restates
tri_f32_out and the host's TriF record (trace.hip upload_scene), with each fmaf emulated as an fp64
product-sum rounded to fp32 (a double rounding: within one fp32 ulp of the fused result, well inside
the bound's 4x margin)."""
import numpy as np
import pytest

EPS = 1e-7
f32 = np.float32


def _dot(a, b):
    return ((a[..., 0] * b[..., 0]) + (a[..., 1] * b[..., 1])) + (a[..., 2] * b[..., 2])


def _cross(a, b):
    return np.stack([(a[..., 1] * b[..., 2]) - (a[..., 2] * b[..., 1]),
                     (a[..., 2] * b[..., 0]) - (a[..., 0] * b[..., 2]),
                     (a[..., 0] * b[..., 1]) - (a[..., 1] * b[..., 0])], -1)


def planar_eq(v):
    """scene_build.cpp planar_eq for a triangle: N = normalized(cross(P2P[1], P2P[0])), D = -N.v0."""
    p2p = [v[1] - v[0], v[2] - v[1], v[0] - v[2]]  # P2P[i-1] = v[i] - v[i-1]
    n = _cross(p2p[1], p2p[0])
    ln = np.sqrt(_dot(n, n))
    n = n / ln
    return n, -_dot(n, v[0])


def tri_records(v):
    n, dA = planar_eq(v)
    nB, dB = planar_eq(v[::-1].copy())
    assert np.array_equal(nB, -n)
    return n, dA, dB


def ref_test(v, n, dA, dB, o, d):
    """trace_device.h planar_test<3, false> with LimNone, vectorised over rays (o, d: [R, 3])."""
    pr = _dot(np.broadcast_to(n, d.shape), d)
    st = pr > 0
    N = np.where(st[:, None], -n, n)
    Dp = np.where(st, dB, dA)
    pr = _dot(N, d)
    ok = (np.abs(pr) > 0) & ~(pr > 0)
    with np.errstate(all="ignore"):
        t = -(_dot(N, o) + Dp) / pr
        ok &= t > EPS
        p = d * t[:, None] + o
        for i in range(3):
            vi0, pi0 = i, (2 if i == 0 else i - 1)
            vi1, pi1 = 2 - i, 2 - (2 if i == 0 else i - 1)
            w = np.where(st[:, None], v[vi1], v[vi0])
            wp = np.where(st[:, None], v[pi1], v[pi0])
            e = w - wp
            ir = p - w
            ok &= ~(_dot(_cross(ir, e), N) < -EPS)
    return ok


def _f32_up(x):
    u = x * (1 + 2.0 ** -20)
    return f32(u) if 0 <= u <= 3.0e38 else f32(np.inf)


def trif(v, n, dA):
    """trace.hip upload_scene's TriF record."""
    m, c = [], []
    mmax, tm = 0.0, abs(dA)
    for j in range(3):
        a, b = v[j], v[(j + 2) % 3]
        e = a - b
        mj = np.array([e[1] * n[2] - e[2] * n[1], e[2] * n[0] - e[0] * n[2], e[0] * n[1] - e[1] * n[0]])
        m.append(mj.astype(f32))
        c.append(f32(a[0] * mj[0] + a[1] * mj[1] + a[2] * mj[2]))
        mmax = max(mmax, float(np.sqrt(mj @ mj)))
        tm = max(tm, float(np.sqrt(a @ a)))
    nmag = float(np.sqrt(n @ n))
    return {"m": m, "c": c, "n": n.astype(f32), "d": f32(dA),
            "k": _f32_up(2.0 ** -17 * mmax * max(1.0, nmag)), "tm": _f32_up(tm)}


def fmaf(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f32)


def f32_out(T, o, d):
    """tri_f32_out + tri_ray_f32, vectorised over rays."""
    o32, d32 = o.astype(f32), d.astype(f32)
    O = (np.abs(o32[:, 0]) + np.abs(o32[:, 1])) + np.abs(o32[:, 2])
    D = (np.abs(d32[:, 0]) + np.abs(d32[:, 1])) + np.abs(d32[:, 2])
    n = T["n"]
    s = fmaf(n[2], d32[:, 2], fmaf(n[1], d32[:, 1], (n[0] * d32[:, 0]).astype(f32)))
    P = fmaf(n[2], o32[:, 2], fmaf(n[1], o32[:, 1], fmaf(n[0], o32[:, 0], T["d"])))
    a_s = np.abs(s)
    sP = np.where(s < 0, -P, P).astype(f32)
    with np.errstate(all="ignore"):
        B = fmaf(D, fmaf(T["k"], (O + T["tm"]).astype(f32), f32(2.0 ** -40)), f32(2.0 ** -100))
        thr = -fmaf(f32(1.00000001168609742e-07), a_s, B)
        out = np.zeros(len(o), bool)
        for j in range(3):
            m = T["m"][j]
            Q = fmaf(m[2], o32[:, 2], fmaf(m[1], o32[:, 1], fmaf(m[0], o32[:, 0], -T["c"][j])))
            R = fmaf(m[2], d32[:, 2], fmaf(m[1], d32[:, 1], (m[0] * d32[:, 0]).astype(f32)))
            out |= fmaf(a_s, Q, -(sP * R).astype(f32)) < thr
        return out & (a_s > f32(2.0 ** -20) * D) & (B < f32(2.0 ** 100))


def _rays(rng, v, n, R):
    """Rays at points on / near the triangle's edges and vertices, inside and outside it, from random
    origins, a share of them grazing, with unnormalised directions."""
    c = v.mean(0)
    size = max(np.linalg.norm(v[i] - v[j]) for i in range(3) for j in range(i))
    # target points: barycentric combinations pushed across the edges by a few ulps to a few sizes
    bary = rng.dirichlet([1, 1, 1], R)
    k = rng.integers(0, 3, R)
    bary[np.arange(R), k] = 0.0  # on an edge
    bary /= bary.sum(1, keepdims=True)
    p = bary @ v
    push = rng.choice([0.0, 1e-16, 1e-14, 1e-12, 1e-9, 1e-7, 1e-5, 1e-2, 1.0], R) * size
    push *= rng.choice([-1.0, 1.0], R)
    p += push[:, None] * (p - c) / np.maximum(np.linalg.norm(p - c, axis=1, keepdims=True), 1e-300)
    rnd = rng.random(R) < 0.3
    p[rnd] = c + rng.normal(size=(rnd.sum(), 3)) * size * 2  # anywhere near
    # origins: off the plane at distances from tiny to far, a share nearly in the plane (grazing)
    dist = size * 10.0 ** rng.uniform(-3, 4, R)
    dirn = rng.normal(size=(R, 3))
    dirn /= np.linalg.norm(dirn, axis=1, keepdims=True)
    graze = rng.random(R) < 0.3
    tang = dirn - (dirn @ n)[:, None] * n
    tang /= np.maximum(np.linalg.norm(tang, axis=1, keepdims=True), 1e-300)
    tilt = 10.0 ** rng.uniform(-12, -2, R)
    dirn[graze] = tang[graze] + tilt[graze, None] * n * rng.choice([-1.0, 1.0], graze.sum())[:, None]
    o = p - dirn * dist[:, None]
    d = (p - o) / np.linalg.norm(p - o, axis=1, keepdims=True)
    d *= 10.0 ** rng.uniform(-0.5, 0.5, R)[:, None]  # unnormalised (an instance's inverse CTM)
    return o, d


@pytest.mark.parametrize("scale,offset", [(1.0, 0.0), (1e-3, 0.0), (1e3, 0.0), (1.0, 1e2), (1e-2, 1e3), (1.0, 1e5),
                                          (1e-4, 1.0), (1e4, 1e7)])
def test_f32_pretest_never_rejects_a_hit(scale, offset):
    rng = np.random.default_rng(int(scale * 1e4 + offset) % (2**31))
    rejected = total = hits = 0
    for _ in range(150):
        base = rng.normal(size=3) * offset
        v = base + rng.normal(size=(3, 3)) * scale
        if rng.random() < 0.2:  # a sliver
            v[2] = v[0] + (v[1] - v[0]) * rng.uniform(0.2, 0.8) + rng.normal(size=3) * scale * 1e-4
        n, dA, dB = tri_records(v)
        if not np.all(np.isfinite(n)):
            continue
        o, d = _rays(rng, v, n, 400)
        ref = ref_test(v, n, dA, dB, o, d)
        out = f32_out(trif(v, n, dA), o, d)
        bad = out & ref
        assert not bad.any(), (scale, offset, v, o[bad][:3], d[bad][:3])
        rejected += int(out.sum())
        total += len(o)
        hits += int(ref.sum())
    # A sanity floor where the triangle is not tiny against its distance from the origin: the band
    # the pre-test leaves open is ~2^-17 (|o| + |v|) |d| / |n.d| wide (absolute coordinates), so a
    # 0.01-sized triangle 1e3 away settles little (C3: bunny in [-1, 1], 0.018 edges, eye 3 away --
    # a band of ~0.3 % of an edge). These rays are aimed within a few ulps of the edges, where
    # nothing can be settled.
    if offset <= 10 * scale:
        assert rejected >= 0.3 * (total - hits), (rejected, total, hits)


def test_f32_pretest_degenerate_records_reject_nothing():
    """Non-finite records (k = +inf) and rays parallel to the plane settle nothing."""
    v = np.array([[0.0, 0, 0], [1, 0, 0], [0, 1, 0]])
    n, dA, dB = tri_records(v)
    T = trif(v, n, dA)
    T["k"] = f32(np.inf)
    o = np.array([[5.0, 5.0, 1.0], [0.2, 0.2, 1.0]])
    d = np.array([[0.0, 0.0, -1.0], [0.0, 0.0, -1.0]])
    assert not f32_out(T, o, d).any()
    T = trif(v, n, dA)
    assert f32_out(T, o, d)[0] and not f32_out(T, o, d)[1]  # far outside: rejected; inside: not
    par = np.array([[1.0, 0.0, 0.0], [1.0, 0.0, 0.0]])  # n.d = 0
    assert not f32_out(T, o, par).any()
    huge = np.array([[1e30, 1e30, 1.0]])
    assert not f32_out(trif(v * 1e20, n, dA * 1e20), huge, d[:1]).any()
