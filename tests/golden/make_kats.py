#!/usr/bin/env python3
"""Reference-independent known answers: single pixels derived in plain float64 Python from the
Java reference's formulas (file:line at every step below, paths relative to
src/rayTracerDistAccelShdPhtnMap/), WITHOUT calling the oracle or the product. They pin the
shading branches the sky pin (tests/test_refpin.py) cannot reach:

  c2clear     `shiny` glass sphere: mySimpleReflObjShdr.calcSimpleTransClr (myObjShader.java:503-631)
              -- its index (the `shiny` Index token, currPerm) is 1, so n1 = n2, tr = 0 and the
              refraction child alone carries the weight (1 - tr) * KTrans = 1.5; the phong term
  trTrans     `surface` glass sphere (full shader): calcTransClr (myObjShader.java:157-276), entering
              and leaving the glass, weights (1 - tr) * permClr and tr * permClr (the skydome
              background line replaced by a plain colour, so no texture is involved)
  c3spotLight a ground pixel inside the spot fall-off band: mySpotLight.calcT_Mult
              (myLight.java:77-82,158-163), DEG_TO_RAD as Processing's float
  p2_t05      ground pixels lit by the disk light: getRandomDiskPos (myLight.java:251-266) drawn
              with the product's keyed RNG (Java's ThreadLocalRandom is not seedable,
              Q23), two draws per shadow ray (light direction, then the distance to the light, Q12)

Every scene here has identity transforms; the classes below keep the reference's mutable state
(the in-place re-normalisation of a ray's direction in getTransformedRay, myRay.java:93; the
in-place vertex reversal of a planar object hit from behind, myPlanarObject.java:110; the normal
normalised in place per hit, :130-136). Trig / pow come from the host libm, not fdlibm (within an
ulp of StrictMath); the tests therefore compare with a 2e-6 tolerance on the float32 RGB and
require the ARGB int exactly, which the script checks is not within 1e-9 of a truncation step.

  python tests/golden/make_kats.py          # writes tests/golden/kats.json
"""
from __future__ import annotations

import json
import math
from pathlib import Path

HERE = Path(__file__).resolve().parent
SCENES = HERE.parent.parent / "scenes"
EPS = 0.0000001                      # DistRayTracer.epsVal
NUM_RAYS = 8                         # myScene.numRays (myScene.java:27)
FLOAT_TWO_PI = 6.2831854820251465    # (double) PConstants.TWO_PI (a float)
FLOAT_DEG_TO_RAD = 0.01745329238474369  # (double) PConstants.DEG_TO_RAD (a float)
SEED = 0x5EED0001                    # the render seed the tests use
M64 = (1 << 64) - 1


# ---- myVector (myVector.java): Java evaluates left to right, no fused operations
def dot(a, b):
    return ((a[0] * b[0]) + (a[1] * b[1])) + (a[2] * b[2])           # :43


def mag(a):
    return math.sqrt(((a[0] * a[0]) + (a[1] * a[1])) + (a[2] * a[2]))  # :27-28


def normalize(a):  # in place (:30, :39)
    m = mag(a)
    if m == 0:
        return a
    a[0] /= m
    a[1] /= m
    a[2] /= m
    return a


def cross(a, b):  # :41
    return [(a[1] * b[2]) - (a[2] * b[1]), (a[2] * b[0]) - (a[0] * b[2]), (a[0] * b[1]) - (a[1] * b[0])]


def sub(a, b):
    return [a[0] - b[0], a[1] - b[1], a[2] - b[2]]


def mult(a, s):  # in place (:20)
    a[0] *= s
    a[1] *= s
    a[2] *= s
    return a


def dist(a, b):  # _dist (:37)
    return math.sqrt((((a[0] - b[0]) * (a[0] - b[0])) + ((a[1] - b[1]) * (a[1] - b[1]))) +
                     ((a[2] - b[2]) * (a[2] - b[2])))


def mult_vert_identity(v, w):
    """myMatrix.multVert (myVector.java:85-90) with the identity CTM of these scenes:
    each row accumulates from 0 over the four columns."""
    out = []
    for row in range(3):
        acc = 0.0
        for col in range(4):
            m = 1.0 if row == col else 0.0
            acc += m * (v[col] if col < 3 else w)
        out.append(acc)
    return out


def angle_between(v1, v2):  # DistRayTracer._angleBetween (:445-452)
    return math.acos(dot(v1, v2) / (mag(v1) * mag(v2)))


def rot_axis(v1, u, th):  # DistRayTracer.rotVecAroundAxis (:336-349)
    c, s = math.cos(th), math.sin(th)
    omc = 1 - c
    ux2, uy2, uz2 = u[0] * u[0], u[1] * u[1], u[2] * u[2]
    uxy, uxz, uyz = u[0] * u[1], u[0] * u[2], u[1] * u[2]
    uzS, uyS, uxS = u[2] * s, u[1] * s, u[0] * s
    uxzC1, uxyC1, uyzC1 = uxz * omc, uxy * omc, uyz * omc
    return [(ux2 * omc + c) * v1[0] + (uxyC1 - uzS) * v1[1] + (uxzC1 + uyS) * v1[2],
            (uxyC1 + uzS) * v1[0] + (uy2 * omc + c) * v1[1] + (uyzC1 - uxS) * v1[2],
            (uxzC1 - uyS) * v1[0] + (uyzC1 + uxS) * v1[1] + (uz2 * omc + c) * v1[2]]


def ortho_vec(v):  # DistRayTracer.getOrthoVec (:455-462)
    t = normalize([1.0, 1.0, 0.0])
    if abs(dot(t, v) - 1) < EPS:
        t = [0.0, 0.0, 1.0]
    return normalize(cross(v, t))


def clamp_color(r, g, b):  # myColor ctor (myObjShader.java:661)
    return [min(1.0, r), min(1.0, g), min(1.0, b)]


def argb(c):  # myColor.getInt (myObjShader.java:671): truncating casts, int arithmetic
    v = (255 << 24) + (int(c[0] * 255) << 16) + (int(c[1] * 255) << 8) + int(c[2] * 255)
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


# ---- the product's keyed counter RNG, JDK8 nextDouble(lo, hi) semantics
def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def rng(seed, a, b, c, site, k, lo, hi):
    h = mix64(seed ^ mix64(a))
    h = mix64(h ^ ((b << 32) | c))
    h = mix64(h ^ ((site << 32) | k))
    r = (h >> 11) * 2.0 ** -53
    r = r * (hi - lo) + lo
    return math.nextafter(hi, -math.inf) if r >= hi else r


SITE_DISK = 0x100
TRACE = []  # what the derivation went through (stored with each KAT, checked below)


# ---- rays (myRay.java)
class Ray:
    def __init__(self, o, d, gen):  # ctor :26-47: origin copied, direction normalised
        self.o = list(o)
        self.d = normalize(list(d))
        self.gen = gen
        self.kt = [1.0] * 5       # currKTrans (:31-36)
        self.node = 1             # the product's RNG key of the ray; not reference state

    def transformed(self):
        """getTransformedRay with the identity inverse CTM (:91-102): normalises THIS ray's
        direction in place, then the transformed ray's origin / direction are multVert results."""
        normalize(self.d)
        t = Ray(self.o, self.d, self.gen)
        t.o = mult_vert_identity(self.o, 1.0)
        t.d = mult_vert_identity(self.d, 0.0)
        t.kt = list(self.kt)
        t.node = self.node
        return t

    def point(self, t):  # pointOnRay (:82-87)
        return [(self.d[0] * t) + self.o[0], (self.d[1] * t) + self.o[1], (self.d[2] * t) + self.o[2]]


class Hit:
    """rayHit (myRay.java:147-161) via objHit (:119-125), identity CTMs."""

    def __init__(self, trans_ray, raw_dir, obj, normal, pt, t):
        self.trans_ray = trans_ray
        self.obj = obj
        self.t = t
        self.hit_loc = pt
        self.fwd_hit = mult_vert_identity(mult_vert_identity(pt, 1.0), 1.0)  # objHit, then the ctor again
        n = mult_vert_identity(normal, 0.0)                                  # adjoint (identity)
        self.nrm = normalize(n)
        self.fwd_dir = list(raw_dir)                                          # copy of _ray.direction


# ---- shaders (myObjShader.java)
class Shader:
    def __init__(self, diff, amb, spec, phong, krefl, ktrans=0.0, perm=0.0, perm_clr=(0.0, 0.0, 0.0), simple=False):
        self.diff = clamp_color(*diff)
        self.amb = clamp_color(*amb)
        self.spec = clamp_color(*spec)
        self.phong, self.krefl, self.ktrans, self.perm = phong, krefl, ktrans, perm
        self.perm_clr = clamp_color(*perm_clr)
        self.simple = simple
        self.has_caustic = (krefl > 0.0) or (perm > 0.0) or (ktrans > 0.0)  # setCurrColors :69
        self.diff_const = 1 - perm                                            # :73


def shader_from_tokens(tok, simple_flag):
    """setSurfaceShiny (myRTFileReader.java:358-378) / `diffuse` (:185-192) -> myScene.setSurface
    (myScene.java:817-840): KReflClr = (krefl, krefl, krefl); perm colour from tokens 14-16."""
    f = [float(x) for x in tok[1:]]
    if tok[0] == "diffuse":
        return Shader(f[0:3], f[3:6], (0, 0, 0), 0.0, 0.0, simple=simple_flag)
    kt = f[11] if len(f) > 11 else 0.0
    perm = f[12] if len(f) > 12 else 0.0
    pc = tuple(f[13:16]) if len(f) > 15 else (perm, perm, perm)
    return Shader(f[0:3], f[3:6], f[6:9], f[9], f[10], kt, perm, pc, simple=simple_flag)


# ---- geometry
class Sphere:  # mySphere (myImpObject.java:35-94)
    def __init__(self, r, c, shader):
        self.r, self.c, self.shader = r, list(c), shader

    def intersect(self, ray, tr):
        rx = ry = rz = self.r
        d, o, c = tr.d, tr.o, self.c
        a = ((d[0] / rx) * (d[0] / rx)) + ((d[1] / ry) * (d[1] / ry)) + ((d[2] / rz) * (d[2] / rz))
        pC = [(o[0] - c[0]) / rx, (o[1] - c[1]) / ry, (o[2] - c[2]) / rz]          # originRadCalc :19-23
        ta = 2 * a
        b = 2 * (((d[0] / rx) * pC[0]) + ((d[1] / ry) * pC[1]) + ((d[2] / rz) * pC[2]))
        cc = (pC[0] * pC[0]) + (pC[1] * pC[1]) + (pC[2] * pC[2]) - 1
        discr = ((b * b) - (2 * ta * cc))
        if discr < 0:
            return None
        d1 = discr ** .5
        t1, t2 = (-1 * b + d1) / ta, (-1 * b - d1) / ta
        tv = min(t1, t2)
        if tv < EPS:
            tv = max(t1, t2)
            if tv < EPS:
                return None
        pt = tr.point(tv)
        n = normalize(sub(pt, self.c))                                              # getNormalAtPoint :68-74
        return Hit(tr, ray.d, self, n, pt, tv)


class Planar:  # myPlanarObject / myTriangle (myPlanarObject.java)
    def __init__(self, verts, shader):
        self.v = [list(p) for p in verts]
        self.shader = shader
        self._setup()

    def _setup(self):  # setPointsAndNormal (:44-69) + setEQ (:90)
        n = len(self.v)
        self.p2p = [None] * n
        for i in range(n):
            idx = i - 1 if i != 0 else n - 1
            self.p2p[idx] = sub(self.v[i], self.v[idx])
        self.N = normalize(cross(self.p2p[1], self.p2p[0]))
        self.D = -((self.N[0] * self.v[0][0]) + (self.N[1] * self.v[0][1]) + (self.N[2] * self.v[0][2]))

    def _invert(self):  # invertNormal (:71-88): reverse the vertex order in place
        self.v = self.v[::-1]
        self._setup()

    def _inside(self, p):  # myTriangle.checkInside (:165-175)
        n = len(self.v)
        for i in range(n):
            pi = n - 1 if i == 0 else i - 1
            ir = [p[0] - self.v[i][0], p[1] - self.v[i][1], p[2] - self.v[i][2]]
            if dot(cross(ir, self.p2p[pi]), self.N) < -EPS:
                return False
        return True

    def intersect(self, ray, tr):  # intersectCheck (:104-115)
        pr = dot(self.N, tr.d)
        if abs(pr) > 0:
            if pr > 0:
                self._invert()
                return self.intersect(ray, tr)
            t = -(dot(self.N, tr.o) + self.D) / pr
            if t > EPS and self._inside(tr.point(t)):
                normalize(self.N)                                                   # getNormalAtPoint :130-136
                return Hit(tr, ray.d, self, list(self.N), tr.point(t), t)
        return None


# ---- lights (myLight.java)
class Light:
    def __init__(self, kind, index, origin, color, orient=(0.0, 0.0, 0.0), inner=0.0, outer=0.0, radius=0.0):
        self.kind, self.index = kind, index
        self.origin = list(origin)
        self.color = clamp_color(*color)                                            # setLightColor :51
        self.orient = normalize(list(orient))                                       # ctor :28-29
        if kind == "spot":                                                          # setSpotlightVals :150-157
            self.inner = inner * FLOAT_DEG_TO_RAD
            self.outer = outer * FLOAT_DEG_TO_RAD
            self.rad_diff = self.outer - self.inner
        if kind == "disk":                                                          # setDisklightVals :244-247
            self.radius = radius
            self.tangent = ortho_vec(self.orient)

    def position(self, key, k):
        """getOrigin (:87; disk :262-266 = getRandomDiskPos :251-258, keyed draws k, k+1)."""
        if self.kind != "disk":
            return list(self.origin)
        seed, pixel, sample, node = key
        th = rng(seed, pixel, sample, node, SITE_DISK + self.index, k, 0.0, FLOAT_TWO_PI)
        tmp = normalize(rot_axis(self.tangent, self.orient, th))
        m = rng(seed, pixel, sample, node, SITE_DISK + self.index, k + 1, 0.0, self.radius)
        mult(tmp, m)
        return [tmp[0] + self.origin[0], tmp[1] + self.origin[1], tmp[2] + self.origin[2]]


class Scene:
    def __init__(self, W, H, fov, objs, lights, bg):
        self.W, self.H = W, H
        self.objs, self.lights, self.bg = objs, lights, clamp_color(*bg)
        fov_rad = math.pi * fov / 180.0                                             # setSceneParams :1367-1381
        self.viewZ = -1 * (max(H, W) / 2.0) / math.tan(fov_rad / 2)

    # findClosestRayHit (myScene.java:888-903): the TreeMap keeps the first hit of an equal t
    def closest(self, ray):
        best = None
        for obj in self.objs:
            h = obj.intersect(ray, ray.transformed())
            if h is not None and (best is None or h.t < best.t):
                best = h
        return best

    # calcShadow (myScene.java:879-885) with mySceneObject.calcShadowHit (mySceneObject.java:33-38)
    def shadowed(self, ray, dist_to_light):
        for obj in self.objs:
            h = obj.intersect(ray, ray.transformed())
            if h is not None and (dist_to_light - h.t) > EPS:
                return True
        return False

    def reflect_ray(self, ray, key):  # reflectRay (myScene.java:907-914)
        h = self.closest(ray)
        if h is None:
            return list(self.bg)
        return self.color_at(h, key)

    def shadow_color(self, h, tex, key):  # calcShadowColor (myObjShader.java:98-153)
        sh = h.obj.shader
        r = g = b = 0.0
        for L in self.lights:
            lk = (key[0], key[1], key[2], h.trans_ray.node)
            ln = mult_vert_identity(L.position(lk, 0), 1.0)                         # :114
            ln = sub(ln, h.fwd_hit)                                                 # :115
            normalize(ln)
            sray = Ray(h.fwd_hit, ln, h.trans_ray.gen + 1)                          # :119
            t = dist(sray.o, L.position(lk, 2))                                     # intersectCheck :33-41
            lt_mult = 1.0
            if L.kind == "spot":                                                    # :159-163, calcT_Mult :79-82
                angle = math.acos(-1 * dot(sray.d, L.orient))
                lt_mult = 1 if angle < L.inner else 0 if angle > L.outer else (L.outer - angle) / L.rad_diff
            TRACE.append(("light", L.kind, L.index, h.trans_ray.node, lt_mult))
            if lt_mult == 0:
                continue
            if self.shadowed(sray, t):                                              # :125
                TRACE.append(("blocked", L.index, h.trans_ray.node))
                continue
            normalize(sray.d)                                                       # :128
            ldp = dot(sray.d, h.nrm) * lt_mult
            if ldp > EPS:
                r += tex[0] * L.color[0] * ldp
                g += tex[1] * L.color[1] * ldp
                b += tex[2] * L.color[2] * ldp
            if sh.phong == 0:
                continue
            hn = sub(sray.d, h.fwd_dir)                                             # :138-141
            normalize(hn)
            hdp = dot(hn, h.nrm) * lt_mult
            if hdp > EPS:
                ph = (hdp * hdp) ** sh.phong
                r += sh.spec[0] * L.color[0] * ph
                g += sh.spec[1] * L.color[1] * ph
                b += sh.spec[2] * L.color[2] * ph
        return [r, g, b]

    def refl_dir(self, eye, n):  # compReflDir (myObjShader.java:89-96)
        dp = 2 * dot(eye, n)
        tv = [n[0] * dp, n[1] * dp, n[2] * dp]
        return normalize(sub(tv, eye))

    def child(self, origin, d, parent, node, kt=None):
        ray = Ray(origin, d, parent.gen + 1)
        ray.node = node
        if kt is not None:
            ray.kt = list(kt)
        return ray

    def trans_color(self, h, key):
        """calcTransClr (myObjShader.java:157-276) or, for the simple shader, calcSimpleTransClr
        (:503-631): the Fresnel split, then the refraction child (node 2n) and the reflection
        child (node 2n + 1)."""
        sh = h.obj.shader
        back = mult(list(h.fwd_dir), -1)
        N = list(h.nrm)
        cos1 = dot(back, N)
        rnm = 1.0
        if cos1 < EPS:
            rnm = -1.0
            mult(N, -1)
        cos1 = dot(back, N)
        thetaI = angle_between(back, N)
        idx = sh.perm if sh.simple else sh.ktrans          # simple: currPerm as the index (:546,563)
        n, n1, n2, cos2, tr, omtr, TIR = 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, False
        if rnm < 0:                                        # leaving (:196-212 / :544-560)
            if thetaI < math.asin(1.0 / idx):
                n1, n2 = idx, 1.0
                n = n1 / n2
                cos2 = (1.0 - (n * n) * (1.0 - (cos1 * cos1))) ** .5
            else:
                tr, omtr, TIR, cos2 = 1.0, 0.0, True, 0.0
        else:                                              # entering (:213-222 / :561-570)
            n1 = h.trans_ray.kt[1] if sh.simple else h.trans_ray.kt[0]
            n2 = idx
            n = n1 / n2
            cos2 = (1.0 - (n * n) * (1.0 - (cos1 * cos1))) ** .5
        if not TIR:                                        # Fresnel, Q15 (:224-231 / :573-580)
            sa = math.sin(math.acos(cos1))
            rct = (1.0 - ((n1 / n2) * sa * sa)) ** .5
            a1, b1 = n1 * cos1, n2 * rct
            nd1 = (a1 - b1) / (a1 + b1)                    # calcFresPerp :78-81
            a2, b2 = n1 * rct, n2 * cos1
            nd2 = (a2 - b2) / (a2 + b2)                    # calcFresPlel :83-86
            tr = ((nd1 * nd1) + (nd2 * nd2)) / 2.0
            omtr = 1 - tr
        TRACE.append(("fresnel", "simple" if sh.simple else "full", "leave" if rnm < 0 else "enter", TIR, tr,
                      h.trans_ray.node))
        r = g = b = 0.0
        node = h.trans_ray.node
        medium = [sh.ktrans, sh.perm] + list(sh.perm_clr)  # setCurrKTrans (myRay.java:71-77)
        if (omtr > 0) if sh.simple else (omtr > EPS):
            u = mult(list(back), n * -1)
            nv = mult(list(N), (n * cos1) - cos2)
            refr = normalize([u[0] + nv[0], u[1] + nv[1], u[2] + nv[2]])
            c = self.reflect_ray(self.child(h.fwd_hit, refr, h.trans_ray, 2 * node, medium), key)
            if sh.simple:
                w = omtr * sh.ktrans                       # :605-608
                r += w * c[0]; g += w * c[1]; b += w * c[2]
            else:
                r += omtr * sh.perm_clr[0] * c[0]          # :251-253
                g += omtr * sh.perm_clr[1] * c[1]
                b += omtr * sh.perm_clr[2] * c[2]
        if (tr > 0) if sh.simple else (tr > EPS):
            rd = mult(self.refl_dir(back, N), rnm)         # :261-262 / :542,616
            kt = None if sh.simple else medium             # the simple shader's reflection ray: all 1s
            c = self.reflect_ray(self.child(h.fwd_hit, rd, h.trans_ray, 2 * node + 1, kt), key)
            if sh.simple:
                w = tr * sh.krefl                          # :624-627
                r += w * c[0]; g += w * c[1]; b += w * c[2]
            else:
                r += tr * sh.perm_clr[0] * c[0]            # :269-271
                g += tr * sh.perm_clr[1] * c[1]
                b += tr * sh.perm_clr[2] * c[2]
        return [r, g, b]

    def color_at(self, h, key):  # getColorAtPos (myObjShader.java:409-438; simple :635-651)
        sh = h.obj.shader
        r, g, b = sh.amb
        dc = 1.0 if sh.simple else sh.diff_const
        tex = [sh.diff[0] * dc, sh.diff[1] * dc, sh.diff[2] * dc]                   # myImageTexture :105-111
        s = self.shadow_color(h, tex, key)
        r += s[0]; g += s[1]; b += s[2]
        if h.trans_ray.gen < NUM_RAYS - 2 and sh.has_caustic:
            res = [0.0, 0.0, 0.0]
            if (sh.ktrans > 0) if sh.simple else ((sh.ktrans > 0) or (sh.perm > 0.0)):
                res = self.trans_color(h, key)
            elif sh.krefl > 0.0:                                                    # calcReflClr :278-294
                back = mult(list(h.fwd_dir), -1)
                rd = self.refl_dir(back, h.nrm)
                if dot(rd, h.nrm) >= 0:
                    c = self.reflect_ray(self.child(h.fwd_hit, rd, h.trans_ray, 2 * h.trans_ray.node), key)
                    res = [sh.krefl * c[0], sh.krefl * c[1], sh.krefl * c[2]]
            r += res[0]; g += res[1]; b += res[2]
        return clamp_color(r, g, b)

    def pixel(self, row, col, seed=SEED):
        """myFOVScene.draw's 1-spp path (myScene.java:1498-1508): one unjittered camera ray."""
        rayY = (-1 * (row - self.H / 2.0))
        rayX = col - self.W / 2.0
        ray = Ray([0.0, 0.0, 0.0], [rayX, rayY, self.viewZ], 0)
        return self.reflect_ray(ray, (seed, row * self.W + col, 0))


def load(cli_text, W, H):
    """The handful of .cli commands these scenes use (myRTFileReader.java:113-313)."""
    objs, lights, bg, fov = [], [], (0.0, 0.0, 0.0), 90.0
    shader, simple_flag, poly = None, False, None
    for line in cli_text.splitlines():
        tok = line.split()
        if not tok or tok[0].startswith("#"):
            continue
        c = tok[0]
        if c == "fov":
            fov = float(tok[1])
        elif c == "background":
            bg = tuple(float(x) for x in tok[1:4])
        elif c == "point_light":
            lights.append(Light("point", len(lights), map(float, tok[1:4]), map(float, tok[4:7])))
        elif c == "spotlight":
            lights.append(Light("spot", len(lights), map(float, tok[1:4]), map(float, tok[9:12]),
                                map(float, tok[4:7]), float(tok[7]), float(tok[8])))
        elif c == "disk_light":
            lights.append(Light("disk", len(lights), map(float, tok[1:4]), map(float, tok[8:11]),
                                map(float, tok[5:8]), radius=float(tok[4])))
        elif c in ("diffuse", "shiny", "surface"):
            if c == "shiny" and len(tok) > 12 and (float(tok[12]) > 0 or (len(tok) > 13 and float(tok[13]) > 0)):
                simple_flag = True  # scFlags[simpleRefrIDX] stays set for the rest of the scene (:377)
            shader = shader_from_tokens(tok, simple_flag)
        elif c == "sphere":
            objs.append(Sphere(float(tok[1]), [float(x) for x in tok[2:5]], shader))
        elif c == "begin":
            poly = []
        elif c == "vertex":
            poly.append([float(x) for x in tok[1:4]])
        elif c == "end":
            objs.append(Planar(poly, shader))
        elif c in ("refine", "write", "rays_per_pixel"):
            pass
        else:
            raise ValueError(f"make_kats: command {c!r} not restated here")
    return Scene(W, H, fov, objs, lights, bg)


TR_TRANS_PLAIN = "trTrans.cli with its skydome line replaced by `background 0.2 0.2 1`"
KATS = [
    # (name, scene, row, col, what it pins)
    ("c2clear_glass_simple", "c2clear.cli", 180, 115, "calcSimpleTransClr: index 1, refraction child x KTrans"),
    ("trTrans_glass_full", "trTrans_plain.cli", 138, 157, "calcTransClr: entering / leaving glass, permClr weights"),
    ("c3spotLight_falloff", "c3spotLight.cli", 208, 237, "mySpotLight.calcT_Mult inside the fall-off band"),
    ("p2_t05_disk_lit", "p2_t05.cli", 262, 118, "getRandomDiskPos light direction + distance draws"),
    ("p2_t05_disk_shadow", "p2_t05.cli", 222, 128, "the disk light's shadow ray to its drawn point blocked by the sphere"),
]


def scene_text(name):
    if name == "trTrans_plain.cli":
        txt = (SCENES / "trTrans.cli").read_text()
        return txt.replace("background texture nightSky.png 100 0 -1 -50", "background 0.2 0.2 1")
    return (SCENES / name).read_text()


def main():
    out = {"about": __doc__.split("\n\n")[0], "seed": SEED, "W": 300, "H": 300, "kats": []}
    for name, cli, row, col, what in KATS:
        sc = load(scene_text(cli), 300, 300)
        TRACE.clear()
        c = sc.pixel(row, col)
        path = [list(e) for e in TRACE]
        # each KAT goes through the branch it is meant to pin
        fr = [e for e in path if e[0] == "fresnel"]
        if "glass_full" in name:  # into and out of the glass, a real Fresnel split (both children)
            assert any(e[2] == "enter" for e in fr) and any(e[2] == "leave" for e in fr), path
            assert any(0 < e[4] < 1 for e in fr), path
        if "glass_simple" in name:  # c2clear's index is 1: tr = 0, the refraction child weighted by KTrans
            assert fr and all(e[1] == "simple" for e in fr), path
        if "spot" in name:
            assert any(e[1] == "spot" and 0 < e[4] < 1 for e in path if e[0] == "light"), path
        if "disk" in name:
            assert any(e[1] == "disk" for e in path if e[0] == "light"), path
            blocked = any(e[0] == "blocked" and e[1] == 0 for e in path)
            assert blocked == ("shadow" in name), path
        for ch in c:  # the ARGB int is exact only away from a truncation step
            frac = ch * 255 - math.floor(ch * 255)
            assert ch >= 1.0 or min(frac, 1 - frac) > 1e-9, (name, c)
        out["kats"].append({"name": name, "cli": cli, "row": row, "col": col, "what": what, "rgb": c,
                            "argb": argb(c), "path": path})
        print(f"{name:26s} {cli:18s} ({row},{col}) rgb {c} argb {argb(c) & 0xFFFFFFFF:08X}")
    out["trTrans_plain"] = TR_TRANS_PLAIN
    (HERE / "kats.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
