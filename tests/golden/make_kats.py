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
  kat_bvh     (round 5) C3's path in miniature: a 12-triangle `begin_list ... end_accel` under
              `translate 0 0 -3` (tests/golden/kat_scenes/kat_bvh.cli) -- the myBVH build with the
              root's dropped element (Q1, myGeomBase.java:361-381), the traversal with its local
              pruning (:407-421), the leaf hit re-derived with leafCTM x objCTM (Q4, :298,
              myRay.java:168-175: the "ghost" hit point every secondary ray starts from), a mirror
              child whose origin lies inside the BVH's root box (Q2, :157,218: the BVH is missed)
              and the two shadow rays (myBVH.calcShadowHit :397-404, no root-box test)
  earth       a bilinear texel of an image-textured sphere (myImageTexture.getTextureColor,
              myTextureHandler.java:84-117; mySphere.findTextureU/V, myImpObject.java:97-122)
  kat_photon  a photon irradiance at k = 5 over hand-placed photons (getIrradianceFromPhtnTree,
              myObjShader.java:441-458; find_near, myLight.java:389-445)

The first five scenes have identity transforms; the classes below keep the reference's mutable state
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
import struct
from pathlib import Path

HERE = Path(__file__).resolve().parent
SCENES = HERE.parent.parent / "scenes"
EPS = 0.0000001                      # DistRayTracer.epsVal
NUM_RAYS = 8                         # myScene.numRays (myScene.java:27)
FLOAT_TWO_PI = 6.2831854820251465    # (double) PConstants.TWO_PI (a float)
FLOAT_DEG_TO_RAD = 0.01745329238474369  # (double) PConstants.DEG_TO_RAD (a float)
FLOAT_PI = 3.1415927410125732        # (double) PConstants.PI (a float)
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


class Matrix:
    """myMatrix (myVector.java:65-223): row-major 4 x 4, Java evaluation order."""

    def __init__(self, m=None):
        self.m = [list(r) for r in m] if m else [[1.0 if r == c else 0.0 for c in range(4)] for r in range(4)]

    def mult_mat(self, b):  # [this] x [b], each entry accumulated from 0 (:76-81)
        out = Matrix()
        for row in range(4):
            for col in range(4):
                acc = 0.0
                for k in range(4):
                    acc += self.m[row][k] * b.m[k][col]
                out.m[row][col] = acc
        return out

    def mult_vert(self, v, w):  # multVert of (v, w) (:85-90); the 4th result is not read
        out = []
        for row in range(3):
            acc = 0.0
            for col in range(4):
                acc += self.m[row][col] * (v[col] if col < 3 else w)
            out.append(acc)
        return out

    def transpose(self):  # :93-97
        return Matrix([[self.m[c][r] for c in range(4)] for r in range(4)])

    def inverse(self):  # InvertMe (:111-196): cofactors of the transposed source, / det
        src = [0.0] * 16
        for row in range(4):
            for col in range(4):
                src[4 * col + row] = self.m[row][col]
        t = [src[10] * src[15], src[11] * src[14], src[9] * src[15], src[11] * src[13], src[9] * src[14],
             src[10] * src[13], src[8] * src[15], src[11] * src[12], src[8] * src[14], src[10] * src[12],
             src[8] * src[13], src[9] * src[12]]
        d = [0.0] * 16
        d[0] = t[0] * src[5] + t[3] * src[6] + t[4] * src[7]; d[0] -= t[1] * src[5] + t[2] * src[6] + t[5] * src[7]
        d[1] = t[1] * src[4] + t[6] * src[6] + t[9] * src[7]; d[1] -= t[0] * src[4] + t[7] * src[6] + t[8] * src[7]
        d[2] = t[2] * src[4] + t[7] * src[5] + t[10] * src[7]; d[2] -= t[3] * src[4] + t[6] * src[5] + t[11] * src[7]
        d[3] = t[5] * src[4] + t[8] * src[5] + t[11] * src[6]; d[3] -= t[4] * src[4] + t[9] * src[5] + t[10] * src[6]
        d[4] = t[1] * src[1] + t[2] * src[2] + t[5] * src[3]; d[4] -= t[0] * src[1] + t[3] * src[2] + t[4] * src[3]
        d[5] = t[0] * src[0] + t[7] * src[2] + t[8] * src[3]; d[5] -= t[1] * src[0] + t[6] * src[2] + t[9] * src[3]
        d[6] = t[3] * src[0] + t[6] * src[1] + t[11] * src[3]; d[6] -= t[2] * src[0] + t[7] * src[1] + t[10] * src[3]
        d[7] = t[4] * src[0] + t[9] * src[1] + t[10] * src[2]; d[7] -= t[5] * src[0] + t[8] * src[1] + t[11] * src[2]
        t = [src[2] * src[7], src[3] * src[6], src[1] * src[7], src[3] * src[5], src[1] * src[6], src[2] * src[5],
             src[0] * src[7], src[3] * src[4], src[0] * src[6], src[2] * src[4], src[0] * src[5], src[1] * src[4]]
        d[8] = t[0] * src[13] + t[3] * src[14] + t[4] * src[15]; d[8] -= t[1] * src[13] + t[2] * src[14] + t[5] * src[15]
        d[9] = t[1] * src[12] + t[6] * src[14] + t[9] * src[15]; d[9] -= t[0] * src[12] + t[7] * src[14] + t[8] * src[15]
        d[10] = t[2] * src[12] + t[7] * src[13] + t[10] * src[15]; d[10] -= t[3] * src[12] + t[6] * src[13] + t[11] * src[15]
        d[11] = t[5] * src[12] + t[8] * src[13] + t[11] * src[14]; d[11] -= t[4] * src[12] + t[9] * src[13] + t[10] * src[14]
        d[12] = t[2] * src[10] + t[5] * src[11] + t[1] * src[9]; d[12] -= t[4] * src[11] + t[0] * src[9] + t[3] * src[10]
        d[13] = t[8] * src[11] + t[0] * src[8] + t[7] * src[10]; d[13] -= t[6] * src[10] + t[9] * src[11] + t[1] * src[8]
        d[14] = t[6] * src[9] + t[11] * src[11] + t[3] * src[8]; d[14] -= t[10] * src[11] + t[2] * src[8] + t[7] * src[9]
        d[15] = t[10] * src[10] + t[4] * src[8] + t[9] * src[9]; d[15] -= t[8] * src[9] + t[11] * src[10] + t[5] * src[8]
        det = src[0] * d[0] + src[1] * d[1] + src[2] * d[2] + src[3] * d[3]
        out = Matrix()  # dstMat = new myMatrix(): the identity, kept when det ~ 0
        if abs(det) > .0000001:
            out = Matrix([[d[4 * r + c] / det for c in range(4)] for r in range(4)])
        return out


IDENT = Matrix()


def ctm_ara(glbl):
    """DistRayTracer.buildMatExt (:395): [CTM, inverse, transpose, adjoint = inverse^T]."""
    inv = glbl.inverse()
    return [glbl, inv, glbl.transpose(), inv.transpose()]


IDENT_ARA = ctm_ara(IDENT)


def xpt(M, p):  # getTransformedPt (myRay.java:105-109, DistRayTracer.java:380-384)
    return M.mult_vert(p, 1.0)


def xvec(M, v):  # getTransformedVec
    return M.mult_vert(v, 0.0)


def jdiv(a, b):
    """Java double division (IEEE: x / 0 is +-Inf, 0 / 0 NaN) -- Python raises instead."""
    if b != 0:
        return a / b
    if a == 0 or math.isnan(a):
        return math.nan
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


def jmax(vals):  # DistRayTracer.max (:420): NaN never replaces
    m = -1.7976931348623157e308
    for v in vals:
        if v > m:
            m = v
    return m


def jmin(vals):  # DistRayTracer.min (:421)
    m = 1.7976931348623157e308
    for v in vals:
        if v < m:
            m = v
    return m


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

    def transformed(self, inv=IDENT):
        """getTransformedRay (:91-102): normalises THIS ray's direction in place, then the new ray's
        origin / direction are inv x (o, 1) and inv x (d, 0), not re-normalised."""
        normalize(self.d)
        t = Ray(self.o, self.d, self.gen)
        t.o = xpt(inv, self.o)
        t.d = xvec(inv, self.d)
        t.kt = list(self.kt)
        t.node = self.node
        return t

    def point(self, t):  # pointOnRay (:82-87)
        return [(self.d[0] * t) + self.o[0], (self.d[1] * t) + self.o[1], (self.d[2] * t) + self.o[2]]


class Hit:
    """objHit (myRay.java:119-125) -> rayHit (:147-161): the object-space hit point, the world hit
    point fwdTransHitLoc = CTM x hitLoc, the normal through the adjoint, a copy of the world ray's
    direction."""

    def __init__(self, trans_ray, raw_dir, obj, ctm, pt, t, args=None):
        self.trans_ray = trans_ray
        self.obj = obj
        self.t = t
        self.hit_loc = pt
        self.args = args
        self.ctm = ctm
        xpt(ctm[0], pt)                                                       # objHit's fwdTransPt (unused)
        self.nrm = normalize(xvec(ctm[3], obj.normal_at(pt, args)))          # objHit :121-122
        self.fwd_hit = xpt(ctm[0], pt)                                        # rayHit ctor :157
        self.fwd_dir = list(raw_dir)                                          # copy of _ray.direction

    def recalc(self, ctm):  # reCalcCTMHitNorm (:168-175)
        self.ctm = ctm
        self.fwd_hit = xpt(ctm[0], self.hit_loc)
        self.nrm = normalize(xvec(ctm[3], self.obj.normal_at(self.hit_loc, self.args)))


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
        self.tex = None            # the image texture (`texture` before the shader's object), RGB rows
        self.use_photons = False   # shdrFlags[usePhotonMap]: a photon command before the shader


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
    def __init__(self, r, c, shader, ctm=IDENT_ARA):
        self.r, self.c, self.shader, self.ctm = r, list(c), shader, ctm

    def normal_at(self, pt, args):  # getNormalAtPoint :68-74 (pt - origin)
        return normalize(sub(pt, self.c))

    def intersect(self, ray, tr, ctm=None):
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
        return Hit(tr, ray.d, self, ctm or self.ctm, tr.point(tv), tv)

    def shadow_hit(self, ray, tr, ctm, dist):  # mySceneObject.calcShadowHit (mySceneObject.java:33-38)
        h = self.intersect(ray, tr, ctm)
        return h is not None and (dist - h.t) > EPS

    def tex_coords(self, p, tw, th):
        """findTxtrCoords (myImpObject.java:25-28): v = findTextureV (:111-121), then u = findTextureU
        (:97-109) with Processing's float TWO_PI and shWm1 / 2.0f."""
        a1 = (p[1] - self.c[1]) / self.r
        a1 = 1 if a1 > 1 else (-1 if a1 < -1 else a1)
        v = (th - 1) * math.acos(a1) / math.pi
        shWm1 = tw - 1.0
        z1 = p[2] - self.c[2]
        q = v / (th - 1)
        a0 = (p[0] - self.c[0]) / self.r
        a0 = 1 if a0 > 1 else (-1 if a0 < -1 else a0)
        s1 = math.sin(q * math.pi)
        a2 = 1 if abs(s1) < EPS else a0 / s1
        if z1 <= EPS:
            u = (shWm1 * math.acos(a2)) / FLOAT_TWO_PI + shWm1 / 2.0
        else:
            u = shWm1 - ((shWm1 * math.acos(a2)) / FLOAT_TWO_PI + shWm1 / 2.0)
        u = 0 if u < 0 else (shWm1 if u > shWm1 else u)
        TRACE.append(("texel", u, v))
        return u, v


class Planar:  # myPlanarObject / myTriangle (myPlanarObject.java)
    def __init__(self, verts, shader, ctm=IDENT_ARA):
        self.v = [list(p) for p in verts]
        self.shader = shader
        self.ctm = ctm
        self._setup()
        # centroid (setPointsAndNormal :45-51,67: coordinates summed from 0 in vertex order) through
        # the CTM: trans_origin, the BVH build's sort key (:68)
        n = len(self.v)
        tot = [0.0, 0.0, 0.0]
        for q in self.v:
            tot = [tot[0] + q[0], tot[1] + q[1], tot[2] + q[2]]
        self.trans_origin = xpt(ctm[0], [tot[0] / n, tot[1] / n, tot[2] / n])
        # the object-space box (finalizePoly :96-99)
        self.bmin = [jmin([q[c] for q in self.v]) for c in range(3)]
        self.bmax = [jmax([q[c] for q in self.v]) for c in range(3)]

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

    def normal_at(self, pt, args):  # getNormalAtPoint (:130-136): N normalised in place
        return normalize(self.N)

    def intersect(self, ray, tr, ctm=None):  # intersectCheck (:104-115)
        pr = dot(self.N, tr.d)
        if abs(pr) > 0:
            if pr > 0:
                self._invert()
                return self.intersect(ray, tr, ctm)
            t = -(dot(self.N, tr.o) + self.D) / pr
            if t > EPS and self._inside(tr.point(t)):
                return Hit(tr, ray.d, self, ctm or self.ctm, tr.point(t), t)
        return None

    def shadow_hit(self, ray, tr, ctm, dist):  # mySceneObject.calcShadowHit
        h = self.intersect(ray, tr, ctm)
        return h is not None and (dist - h.t) > EPS


# ---- acceleration structures (myGeomBase.java)
def expand_pt(box, p):  # DistRayTracer.expandBoxPt (:350-361)
    for c in range(3):
        box[0][c] = box[0][c] if box[0][c] < p[c] else p[c]
        box[1][c] = box[1][c] if box[1][c] > p[c] else p[c]


def new_box():  # a myBBox built around a fresh object's min / max (+-100000, myGeomBase.java:35-36)
    return [[100000.0] * 3, [-100000.0] * 3]


def box_hit(box, tr):
    """myBBox.intersectCheck (:132-162): slabs in the box's object space (tr), the miss test
    min(tMax) > max(tMin) AND biggestMin > 0 (a ray starting inside the box misses, Q2; IEEE
    divisions, NaN axes skipped by p.min / p.max, Q3). Returns the entry t or None."""
    t1 = [jdiv(box[0][i] - tr.o[i], tr.d[i]) for i in range(3)]
    t2 = [jdiv(box[1][i] - tr.o[i], tr.d[i]) for i in range(3)]
    tmin, tmax = [1.7976931348623157e308] * 3, [-1.7976931348623157e308] * 3
    big = -1.7976931348623157e308
    for i in range(3):
        if t1[i] < t2[i]:
            tmin[i], tmax[i] = t1[i], t2[i]
            if big < t1[i]:
                big = t1[i]
        else:
            tmin[i], tmax[i] = t2[i], t1[i]
            if big < t2[i]:
                big = t2[i]
    return big if (jmin(tmax) > jmax(tmin) and big > 0) else None


class GeomList:
    """myGeomList (:251-306): a BVH leaf's members."""

    def __init__(self, ctm):
        self.objs = []
        self.ctm = ctm
        self.box = new_box()

    def add(self, obj):  # addObj (:261-266): the member's box corners through inv(listCTM) x objCTM
        self.objs.append(obj)
        tmp = self.ctm[1].mult_mat(obj.ctm[0])
        expand_pt(self.box, xpt(tmp, obj.bmin))
        expand_pt(self.box, xpt(tmp, obj.bmax))

    def traverse(self, ray, tr, ctm):  # traverseStruct (:281-302)
        best, best_t = None, 1.7976931348623157e308
        for obj in self.objs:
            otr = ray.transformed(obj.ctm[1])
            h = obj.intersect(ray, otr, obj.ctm)
            if h is not None and h.t < best_t:
                best, best_t = h, h.t
        if best is None:
            return None
        best.recalc(ctm_ara(self.ctm[0].mult_mat(best.obj.ctm[0])))         # reBuildCTMara: Q4
        TRACE.append(("leaf_hit", best.obj.kat_id, best.t, best.fwd_hit))
        return best

    def shadow_hit(self, ray, tr, ctm, dist):  # calcShadowHit (:268-277): the leaf box first
        t = box_hit(self.box, tr)
        if t is None or not (dist - t) > EPS:
            return False
        for obj in self.objs:
            if obj.shadow_hit(ray, ray.transformed(obj.ctm[1]), ctm, dist):
                return True
        return False


class BVH:
    """myBVH (:309-423) built by myScene.endTmpObjList (myScene.java:305-324)."""
    MAX_PRIMS_PER_LEAF = 5  # DistRayTracer.maxPrimsPerLeaf

    def __init__(self, ctm, depth=0):
        self.ctm = ctm
        self.box = new_box()
        self.leaf = None
        self.left = self.right = None
        self.depth = depth

    @staticmethod
    def sorted_aras(objs, skip):
        """buildSortedObjAras (:338-357): per axis, a TreeMap<Double> of trans_origin (Double.compare
        order) with insertion-ordered buckets; the axis `skip` keeps the given order."""
        out = [None] * 3
        if skip != -1:
            out[skip] = list(objs)
        for i in range(3):
            if i == skip:
                continue
            out[i] = sorted(objs, key=lambda o: (o.trans_origin[i], math.copysign(1.0, o.trans_origin[i])))
        return out

    def add_list(self, lists, st, end):  # addObjList (:360-386), end exclusive
        size = end - st
        if size <= self.MAX_PRIMS_PER_LEAF:
            self.leaf = GeomList(self.ctm)
            for obj in lists[0]:  # every object of the list, however many (the root's N-1 aside)
                self.leaf.add(obj)
            expand_pt(self.box, self.leaf.box[0])
            expand_pt(self.box, self.leaf.box[1])
            return
        split = int(.5 * size)
        n = len(lists[0])
        axis, span = -1, -1.0  # DistRayTracer.getIDXofMaxBVHSpan (:409-418): strict >, over the whole list
        for i in range(3):
            diff = lists[i][n - 1].trans_origin[i] - lists[i][0].trans_origin[i]
            if span < diff:
                span, axis = diff, i
        self.axis = axis
        self.left, self.right = BVH(self.ctm, self.depth + 1), BVH(self.ctm, self.depth + 1)
        self.left.add_list(self.sorted_aras(lists[axis][0:split], axis), st, st + split)
        self.right.add_list(self.sorted_aras(lists[axis][split:size], axis), st + split, end)
        for ch in (self.left, self.right):
            expand_pt(self.box, ch.box[0])
            expand_pt(self.box, ch.box[1])

    @classmethod
    def build(cls, objs, ctm):
        root = cls(ctm)
        lists = cls.sorted_aras(objs, -1)
        root.add_list(lists, 0, len(lists[0]) - 1)  # N - 1: the root's last element is dropped (Q1)
        kept = set()
        root._collect(kept)
        root.dropped = [o for o in objs if id(o) not in kept]
        return root

    def _collect(self, kept):
        if self.leaf is not None:
            kept.update(id(o) for o in self.leaf.objs)
        else:
            self.left._collect(kept)
            self.right._collect(kept)

    def intersect(self, ray, tr, ctm=None):  # myAccelStruct.intersectCheck (:216-222): the root box first
        if box_hit(self.box, tr) is None:
            inside = all(self.box[0][i] < tr.o[i] < self.box[1][i] for i in range(3))
            TRACE.append(("bvh_root_miss", ray.gen, tr.o, inside))
            return None
        return self.traverse(ray, tr, ctm or self.ctm)

    def traverse(self, ray, tr, ctm):  # traverseStruct (:407-421)
        if self.leaf is not None:
            return self.leaf.traverse(ray, tr, ctm)
        h = None
        lt = box_hit(self.left.box, tr)
        if lt is not None:
            h = self.left.traverse(ray, tr, ctm)
        rt = box_hit(self.right.box, tr)
        ht = h.t if h is not None else 1.7976931348623157e308
        if rt is not None and (h is None or rt < ht):
            h2 = self.right.traverse(ray, tr, ctm)
            h2t = h2.t if h2 is not None else 1.7976931348623157e308
            return h if ht <= h2t else h2
        if rt is not None:
            TRACE.append(("bvh_right_pruned", self.depth))
        return h

    def shadow_hit(self, ray, tr, ctm, dist):  # calcShadowHit (:397-404): no root-box test
        if self.leaf is not None:
            return self.leaf.shadow_hit(ray, tr, ctm, dist)
        for ch in (self.left, self.right):
            t = box_hit(ch.box, tr)
            if t is not None and (dist - t) > EPS and ch.shadow_hit(ray, tr, ctm, dist):
                return True
        return False


# ---- lights (myLight.java)
class Light:
    def __init__(self, kind, index, origin, color, orient=(0.0, 0.0, 0.0), inner=0.0, outer=0.0, radius=0.0,
                 ctm=IDENT_ARA):
        self.kind, self.index = kind, index
        self.ctm = ctm
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
            h = obj.intersect(ray, ray.transformed(obj.ctm[1]), obj.ctm)
            if h is not None and (best is None or h.t < best.t):
                best = h
        return best

    # calcShadow (myScene.java:879-885): each entry's calcShadowHit (mySceneObject.java:33-38,
    # myBVH.calcShadowHit myGeomBase.java:397-404)
    def shadowed(self, ray, dist_to_light):
        for obj in self.objs:
            if obj.shadow_hit(ray, ray.transformed(obj.ctm[1]), obj.ctm, dist_to_light):
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
            ln = xpt(L.ctm[0], L.position(lk, 0))                                  # :114
            ln = sub(ln, h.fwd_hit)                                                 # :115
            normalize(ln)
            sray = Ray(h.fwd_hit, ln, h.trans_ray.gen + 1)                          # :119
            t = dist(sray.o, xpt(L.ctm[0], L.position(lk, 2)))                      # intersectCheck :33-41
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
            TRACE.append(("lit", L.index, h.trans_ray.node))
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

    def irradiance(self, p):
        """getIrradianceFromPhtnTree (myObjShader.java:441-458) over find_near (myLight.java:389-445):
        the k nearest photons with d2 < max_dist^2 (distinct distances here: no tie for the heap to
        decide), their powers summed in poll order (farthest first) over PI_f x the farthest d2."""
        near = []
        for q, w in zip(self.photons, self.photon_pwr):
            dx, dy, dz = p[0] - q[0], p[1] - q[1], p[2] - q[2]
            near.append((dx * dx + dy * dy + dz * dz, w))                       # len2 (:427-430)
        near = sorted(x for x in near if x[0] < self.photon_maxd2)[: self.photon_k]
        if not near:
            return [0.0, 0.0, 0.0]                                              # [null] -> 0 (Q20)
        res = [0.0, 0.0, 0.0]
        for d2, w in reversed(near):                                            # poll order
            res = [res[0] + w[0], res[1] + w[1], res[2] + w[2]]
        area = FLOAT_PI * near[-1][0]
        TRACE.append(("photons", len(near), near[-1][0]))
        return [res[0] / area, res[1] / area, res[2] / area]

    def tex_color(self, h):
        """myImageTexture.getTextureColor (myTextureHandler.java:84-103): bilinear between the four
        texels around (u, v) of findTxtrCoords, each myColor(int) / 255, interpColor in u then v."""
        img = h.obj.shader.tex
        th, tw = len(img), len(img[0])
        u, v = h.obj.tex_coords(h.hit_loc, tw, th)
        ui, vi = int(u), int(v)

        def texel(r, c):
            px = img[r][c]
            return [px[0] / 255.0, px[1] / 255.0, px[2] / 255.0]

        def interp(a, t, b):  # myColor.interpColor (myObjShader.java:667): clamped <= 1
            return clamp_color(a[0] + t * (b[0] - a[0]), a[1] + t * (b[1] - a[1]), a[2] + t * (b[2] - a[2]))
        c00, c10 = texel(vi, ui), texel(vi + 1, ui)
        c01, c11 = texel(vi, ui + 1), texel(vi + 1, ui + 1)
        fu, fv = u - ui, v - vi
        return interp(interp(c00, fu, c01), fv, interp(c10, fu, c11))

    def color_at(self, h, key):  # getColorAtPos (myObjShader.java:409-438; simple :635-651)
        sh = h.obj.shader
        r, g, b = sh.amb
        if sh.krefl == 0.0 and sh.use_photons:                                      # :415-424
            irr = self.irradiance(h.fwd_hit)
            r += sh.diff[0] * irr[0]; g += sh.diff[1] * irr[1]; b += sh.diff[2] * irr[2]
        dc = 1.0 if sh.simple else sh.diff_const
        base = self.tex_color(h) if sh.tex is not None else sh.diff                 # getDiffTxtrColor :105-111
        tex = [base[0] * dc, base[1] * dc, base[2] * dc]
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
                    TRACE.append(("mirror", h.trans_ray.node, h.fwd_hit))
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


def load(cli_text, W, H, scene_dir=None):
    """The handful of .cli commands these scenes use (myRTFileReader.java:113-313). Objects take the
    matrix-stack top (myGeomBase ctor, myGeomBase.java:37) and a shader of the current settings
    (getCurShader, myScene.java:524-528: the image texture and the photon flag included)."""
    import copy

    objs, lights, bg, fov = [], [], (0.0, 0.0, 0.0), 90.0
    shader, simple_flag, poly = None, False, None
    top = IDENT                                   # matrixStack.peek()
    tex, photons = None, None                     # currTextureTop (txtrType 1) / the photon command
    tmp_list = None                               # begin_list ... end_accel (addToTmpListIDX)

    def cur_shader():
        sh = copy.copy(shader)
        sh.tex = tex
        sh.use_photons = photons is not None
        return sh

    def add(obj):  # addObjectToScene (myScene.java:558-565)
        (tmp_list if tmp_list is not None else objs).append(obj)

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
            lights.append(Light("point", len(lights), map(float, tok[1:4]), map(float, tok[4:7]), ctm=ctm_ara(top)))
        elif c == "spotlight":
            lights.append(Light("spot", len(lights), map(float, tok[1:4]), map(float, tok[9:12]),
                                map(float, tok[4:7]), float(tok[7]), float(tok[8]), ctm=ctm_ara(top)))
        elif c == "disk_light":
            lights.append(Light("disk", len(lights), map(float, tok[1:4]), map(float, tok[8:11]),
                                map(float, tok[5:8]), radius=float(tok[4]), ctm=ctm_ara(top)))
        elif c in ("diffuse", "shiny", "surface"):
            if c == "shiny" and len(tok) > 12 and (float(tok[12]) > 0 or (len(tok) > 13 and float(tok[13]) > 0)):
                simple_flag = True  # scFlags[simpleRefrIDX] stays set for the rest of the scene (:377)
            shader = shader_from_tokens(tok, simple_flag)
        elif c in ("texture", "image_texture"):   # :257-272 (top texture), Pillow-decoded texels
            from PIL import Image
            name = tok[2] if tok[1].lower() == "top" else tok[1]
            im = Image.open(Path(scene_dir or SCENES) / "txtrs" / name).convert("RGB")
            w, h = im.size
            raw = im.tobytes()
            tex = [[tuple(raw[3 * (r * w + q):3 * (r * w + q) + 3]) for q in range(w)] for r in range(h)]
        elif c in ("diffuse_photons", "caustic_photons"):  # setPhotonHandling (myScene.java:919-931)
            photons = (int(tok[1]), int(tok[2]), float(tok[3]))
        elif c == "translate":                   # gtTranslate / updateCTM (myScene.java:1256-1264,1320-1323)
            T = Matrix()
            T.m[0][3], T.m[1][3], T.m[2][3] = float(tok[1]), float(tok[2]), float(tok[3])
            top = top.mult_mat(T)
        elif c == "sphere":
            objs_ctm = ctm_ara(top)
            add(Sphere(float(tok[1]), [float(x) for x in tok[2:5]], cur_shader(), objs_ctm))
        elif c == "begin":
            poly, poly_ctm = [], ctm_ara(top)    # the object exists (and takes its CTM) from `begin`
        elif c == "vertex":
            poly.append([float(x) for x in tok[1:4]])
        elif c == "end":
            add(Planar(poly, cur_shader(), poly_ctm))
        elif c == "begin_list":
            tmp_list = []
        elif c == "end_accel":
            for i, o in enumerate(tmp_list):
                o.kat_id = i
            members, tmp_list = tmp_list, None
            bvh = BVH.build(members, ctm_ara(top))
            bvh.members = members
            add(bvh)
        elif c in ("refine", "write", "rays_per_pixel", "reset_timer", "print_timer"):
            pass
        else:
            raise ValueError(f"make_kats: command {c!r} not restated here")
    sc = Scene(W, H, fov, objs, lights, bg)
    sc.photons, sc.photon_pwr = [], []
    if photons is not None:
        sc.photon_k = photons[1]
        md = float(struct.unpack("f", struct.pack("f", photons[2]))[0])  # Float.parseFloat, widened
        sc.photon_maxd2 = md * md                                               # _baseMaxDist2 (:311-315)
    return sc


TR_TRANS_PLAIN = "trTrans.cli with its skydome line replaced by `background 0.2 0.2 1`"
KAT_SCENES = HERE / "kat_scenes"  # KAT-only scenes (kat_*.cli), written for these derivations
KATS = [
    # (name, scene, row, col, what it pins)
    ("c2clear_glass_simple", "c2clear.cli", 180, 115, "calcSimpleTransClr: index 1, refraction child x KTrans"),
    ("trTrans_glass_full", "trTrans_plain.cli", 138, 157, "calcTransClr: entering / leaving glass, permClr weights"),
    ("c3spotLight_falloff", "c3spotLight.cli", 208, 237, "mySpotLight.calcT_Mult inside the fall-off band"),
    ("p2_t05_disk_lit", "p2_t05.cli", 262, 118, "getRandomDiskPos light direction + distance draws"),
    ("p2_t05_disk_shadow", "p2_t05.cli", 222, 128, "the disk light's shadow ray to its drawn point blocked by the sphere"),
    ("bvh_q1_q2_q4_tile", "kat_bvh.cli", 140, 156,
     "BVH under translate: the ray passes the dropped root element (Q1) to a tile; the hit point is the "
     "double-transformed ghost (Q4); its mirror ray starts inside the root box and misses the BVH (Q2); "
     "both shadow rays lit"),
    ("bvh_q4_ghost_blocked", "kat_bvh.cli", 150, 150,
     "BVH under translate: through the dropped element (Q1) to the backdrop; the ghost point (Q4) lies behind "
     "the backdrop, so both shadow rays are blocked and the mirror ray hits the backdrop from behind"),
    ("earth_bilinear_texel", "earth.cli", 120, 210,
     "myImageTexture.getTextureColor: bilinear texel of a sphere's (u, v) (findTextureU/V)"),
    ("photon_irradiance_k5", "kat_photon.cli", 200, 170,
     "getIrradianceFromPhtnTree at k = 5 over hand-placed photons (distinct distances, two beyond max_dist)"),
]
# hand-placed photons of photon_irradiance_k5: offsets (dx, dy, dz) from the KAT pixel's hit point,
# distinct distances (5 within the neighbourhood, 2 more within max_dist 0.5, 2 beyond it)
PHOTON_OFFSETS = [(0.05, 0.0, 0.02), (-0.11, 0.0, 0.07), (0.13, 0.0, -0.09), (-0.04, 0.0, -0.17), (0.21, 0.0, 0.12),
                  (-0.26, 0.0, -0.05), (0.02, 0.0, 0.31), (0.38, 0.0, -0.41), (-0.45, 0.0, 0.3), (0.0, 0.03, 0.045)]


def scene_text(name):
    if name == "trTrans_plain.cli":
        txt = (SCENES / "trTrans.cli").read_text()
        return txt.replace("background texture nightSky.png 100 0 -1 -50", "background 0.2 0.2 1")
    if (KAT_SCENES / name).exists():
        return (KAT_SCENES / name).read_text()
    return (SCENES / name).read_text()


def scene_dir(name):
    return KAT_SCENES if (KAT_SCENES / name).exists() else SCENES


def kat_scene(kat, W, H):
    """The derivation's scene of a KAT entry (with its photons, when it has any)."""
    sc = load(scene_text(kat["cli"]), W, H, scene_dir(kat["cli"]))
    if "photons" in kat:
        sc.photons, sc.photon_pwr = kat["photons"]["pos"], kat["photons"]["pwr"]
    return sc


def make_photons(name, row, col):
    """Photons around the KAT pixel's camera hit (the derivation's own hit point)."""
    sc = load(scene_text(name), 300, 300, scene_dir(name))
    ray = Ray([0.0, 0.0, 0.0], [col - 150.0, -1 * (row - 150.0), sc.viewZ], 0)
    p = sc.closest(ray).fwd_hit
    pos = [[p[0] + dx, p[1] + dy, p[2] + dz] for dx, dy, dz in PHOTON_OFFSETS]
    pwr = [[0.001 * (i + 1), 0.002 + 0.0003 * i, 0.0005 * (i + 2)] for i in range(len(pos))]
    return {"pos": pos, "pwr": pwr}


def check_path(name, path, sc):
    """Each KAT goes through the branch it is meant to pin."""
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
    if name.startswith("bvh"):
        bvh = [o for o in sc.objs if isinstance(o, BVH)][0]
        hits = [e for e in path if e[0] == "leaf_hit"]
        cam = hits[-1] if name.endswith("tile") else None
        assert bvh.dropped and bvh.dropped[0].kat_id == 11, "the root drops the front triangle (Q1)"
        # the camera ray's first BVH result is the tile / backdrop behind the dropped element
        mirrors = [e for e in path if e[0] == "mirror"]
        assert mirrors, path  # a mirror child
        assert sum(1 for e in path if e[0] in ("lit", "blocked") and e[2] == 1) == 2, path  # two shadow rays
        if name.endswith("tile"):
            assert any(e[0] == "bvh_root_miss" and e[3] for e in path), path  # Q2: origin inside the root box
            assert all(e[0] != "blocked" for e in path if len(e) > 2 and e[2] == 1), path
        else:
            assert all(e[0] == "blocked" for e in path if e[0] in ("lit", "blocked") and e[2] == 1), path
    if name.startswith("earth"):
        tx = [e for e in path if e[0] == "texel"]
        assert tx and all(0 < e[1] % 1 < 1 and 0 < e[2] % 1 < 1 for e in tx), path  # a true bilinear blend
    if name.startswith("photon"):
        ph = [e for e in path if e[0] == "photons"]
        assert ph and ph[0][1] == 5, path


def q1_q4_facts(sc, row, col):
    """The camera ray would hit the dropped element before the hit the reference keeps (Q1), and the
    kept hit's world point is the double-transformed ghost, not CTM x the object-space point (Q4)."""
    ray = Ray([0.0, 0.0, 0.0], [col - 150.0, -1 * (row - 150.0), sc.viewZ], 0)
    bvh = [o for o in sc.objs if isinstance(o, BVH)][0]
    h = sc.closest(ray)
    d = bvh.dropped[0]
    dh = d.intersect(ray, ray.transformed(d.ctm[1]), d.ctm)
    assert dh is not None and dh.t < h.t, (dh, h.t)
    true_pt = xpt(h.obj.ctm[0], h.hit_loc)
    assert abs(h.fwd_hit[2] - (true_pt[2] - 3.0)) < 1e-12, (h.fwd_hit, true_pt)
    return {"dropped_t": dh.t, "hit_t": h.t, "hit_member": h.obj.kat_id, "ghost": h.fwd_hit, "true_point": true_pt}


def main():
    out = {"about": __doc__.split("\n\n")[0], "seed": SEED, "W": 300, "H": 300, "kats": []}
    for name, cli, row, col, what in KATS:
        kat = {"name": name, "cli": cli, "row": row, "col": col, "what": what}
        if name.startswith("photon"):
            kat["photons"] = make_photons(cli, row, col)
        sc = kat_scene(kat, 300, 300)
        TRACE.clear()
        c = sc.pixel(row, col)
        path = [list(e) for e in TRACE]
        check_path(name, path, sc)
        if name.startswith("bvh"):
            kat["facts"] = q1_q4_facts(kat_scene(kat, 300, 300), row, col)
        for ch in c:  # the ARGB int is exact only away from a truncation step
            frac = ch * 255 - math.floor(ch * 255)
            assert ch >= 1.0 or min(frac, 1 - frac) > 1e-9, (name, c)
        kat.update({"rgb": c, "argb": argb(c), "path": path})
        out["kats"].append(kat)
        print(f"{name:26s} {cli:18s} ({row},{col}) rgb {c} argb {argb(c) & 0xFFFFFFFF:08X}")
    out["trTrans_plain"] = TR_TRANS_PLAIN
    (HERE / "kats.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
