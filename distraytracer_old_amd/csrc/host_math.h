// Host-side double math with the reference's evaluation order (built with
// -ffp-contract=off). Used by the scene builder to precompute CTM inverses,
// planar equations, boxes and BVH keys exactly as the Java builder does.
//   myVector / myMatrix: src/rayTracerDistAccelShdPhtnMap/myVector.java
//   expandBoxPt / getTransformedPt: DistRayTracer.java:353-397
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

#include "jfdlibm.h"  // sin / cos: the fdlibm sequences the oracle and the device share

namespace rt {
namespace hm {

static const double EPS = 0.0000001;
static const double TWO_PI_F = (double)6.28318530717958647692f;  // PConstants.TWO_PI (float)
static const double DEG_TO_RAD_F = (double)(3.14159265358979323846f / 180.0f);
static const double DMAX = std::numeric_limits<double>::max();

static inline double jmin(double a, double b) {  // java.lang.Math.min
  if (a != a) return a;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? a : b;
  return (a <= b) ? a : b;
}
static inline double jmax(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
  return (a >= b) ? a : b;
}
static inline int jcompare(double a, double b) {  // Double.compare
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x, y;
  std::memcpy(&x, &a, 8);
  std::memcpy(&y, &b, 8);
  if (a != a) x = 0x7ff8000000000000LL;
  if (b != b) y = 0x7ff8000000000000LL;
  return x == y ? 0 : (x < y ? -1 : 1);
}

struct D3 {
  double x, y, z;
};
static inline D3 d3(double x, double y, double z) { return D3{x, y, z}; }
static inline double dot(D3 a, D3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
static inline D3 cross(D3 a, D3 b) { return d3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)); }
static inline D3 normalized(D3 a) {
  double m = std::sqrt(((a.x * a.x) + (a.y * a.y)) + (a.z * a.z));
  if (m == 0) return a;
  return d3(a.x / m, a.y / m, a.z / m);
}

struct Mat {
  double m[16];  // row-major
  static Mat ident() {
    Mat r;
    for (int i = 0; i < 16; ++i) r.m[i] = (i % 5 == 0) ? 1.0 : 0.0;
    return r;
  }
  bool operator==(const Mat& o) const { return std::memcmp(m, o.m, sizeof(m)) == 0; }
};
static inline Mat mul(const Mat& a, const Mat& b) {
  Mat r;
  for (int row = 0; row < 4; ++row)
    for (int col = 0; col < 4; ++col) {
      double acc = 0;
      for (int k = 0; k < 4; ++k) acc += a.m[row * 4 + k] * b.m[k * 4 + col];
      r.m[row * 4 + col] = acc;
    }
  return r;
}
static inline D3 xform(const Mat& a, D3 p, double w) {
  double b[4] = {p.x, p.y, p.z, w}, o[3];
  for (int row = 0; row < 3; ++row) {
    double acc = 0;
    for (int col = 0; col < 4; ++col) acc += a.m[row * 4 + col] * b[col];
    o[row] = acc;
  }
  return d3(o[0], o[1], o[2]);
}
static inline Mat transpose(const Mat& a) {
  Mat r;
  for (int row = 0; row < 4; ++row)
    for (int col = 0; col < 4; ++col) r.m[col * 4 + row] = a.m[row * 4 + col];
  return r;
}
// Cramer-by-pairs inverse of myMatrix.InvertMe; singular (|det| <= 1e-7) -> identity
static inline Mat inverse(const Mat& a) {
  double s[16], p[12], d[16];
  for (int row = 0; row < 4; ++row)
    for (int col = 0; col < 4; ++col) s[4 * col + row] = a.m[row * 4 + col];
  p[0] = s[10] * s[15]; p[1] = s[11] * s[14]; p[2] = s[9] * s[15]; p[3] = s[11] * s[13];
  p[4] = s[9] * s[14]; p[5] = s[10] * s[13]; p[6] = s[8] * s[15]; p[7] = s[11] * s[12];
  p[8] = s[8] * s[14]; p[9] = s[10] * s[12]; p[10] = s[8] * s[13]; p[11] = s[9] * s[12];
  d[0] = p[0] * s[5] + p[3] * s[6] + p[4] * s[7];    d[0] -= p[1] * s[5] + p[2] * s[6] + p[5] * s[7];
  d[1] = p[1] * s[4] + p[6] * s[6] + p[9] * s[7];    d[1] -= p[0] * s[4] + p[7] * s[6] + p[8] * s[7];
  d[2] = p[2] * s[4] + p[7] * s[5] + p[10] * s[7];   d[2] -= p[3] * s[4] + p[6] * s[5] + p[11] * s[7];
  d[3] = p[5] * s[4] + p[8] * s[5] + p[11] * s[6];   d[3] -= p[4] * s[4] + p[9] * s[5] + p[10] * s[6];
  d[4] = p[1] * s[1] + p[2] * s[2] + p[5] * s[3];    d[4] -= p[0] * s[1] + p[3] * s[2] + p[4] * s[3];
  d[5] = p[0] * s[0] + p[7] * s[2] + p[8] * s[3];    d[5] -= p[1] * s[0] + p[6] * s[2] + p[9] * s[3];
  d[6] = p[3] * s[0] + p[6] * s[1] + p[11] * s[3];   d[6] -= p[2] * s[0] + p[7] * s[1] + p[10] * s[3];
  d[7] = p[4] * s[0] + p[9] * s[1] + p[10] * s[2];   d[7] -= p[5] * s[0] + p[8] * s[1] + p[11] * s[2];
  p[0] = s[2] * s[7]; p[1] = s[3] * s[6]; p[2] = s[1] * s[7]; p[3] = s[3] * s[5];
  p[4] = s[1] * s[6]; p[5] = s[2] * s[5]; p[6] = s[0] * s[7]; p[7] = s[3] * s[4];
  p[8] = s[0] * s[6]; p[9] = s[2] * s[4]; p[10] = s[0] * s[5]; p[11] = s[1] * s[4];
  d[8] = p[0] * s[13] + p[3] * s[14] + p[4] * s[15];    d[8] -= p[1] * s[13] + p[2] * s[14] + p[5] * s[15];
  d[9] = p[1] * s[12] + p[6] * s[14] + p[9] * s[15];    d[9] -= p[0] * s[12] + p[7] * s[14] + p[8] * s[15];
  d[10] = p[2] * s[12] + p[7] * s[13] + p[10] * s[15];  d[10] -= p[3] * s[12] + p[6] * s[13] + p[11] * s[15];
  d[11] = p[5] * s[12] + p[8] * s[13] + p[11] * s[14];  d[11] -= p[4] * s[12] + p[9] * s[13] + p[10] * s[14];
  d[12] = p[2] * s[10] + p[5] * s[11] + p[1] * s[9];    d[12] -= p[4] * s[11] + p[0] * s[9] + p[3] * s[10];
  d[13] = p[8] * s[11] + p[0] * s[8] + p[7] * s[10];    d[13] -= p[6] * s[10] + p[9] * s[11] + p[1] * s[8];
  d[14] = p[6] * s[9] + p[11] * s[11] + p[3] * s[8];    d[14] -= p[10] * s[11] + p[2] * s[8] + p[7] * s[9];
  d[15] = p[10] * s[10] + p[4] * s[8] + p[9] * s[9];    d[15] -= p[8] * s[9] + p[11] * s[10] + p[5] * s[8];
  double det = s[0] * d[0] + s[1] * d[1] + s[2] * d[2] + s[3] * d[3];
  Mat r = Mat::ident();
  if (std::fabs(det) > .0000001) {
    for (int j = 0; j < 16; j++) d[j] /= det;
    for (int j = 0; j < 16; j++) r.m[j] = d[j];
  }
  return r;
}
static inline D3 rot_axis(D3 v1, D3 u, double thet) {  // rotVecAroundAxis
  double cT = jf::cos(thet), sT = jf::sin(thet), oneMC = 1 - cT, ux2 = u.x * u.x, uy2 = u.y * u.y,
         uz2 = u.z * u.z, uxy = u.x * u.y, uxz = u.x * u.z, uyz = u.y * u.z, uzS = u.z * sT, uyS = u.y * sT,
         uxS = u.x * sT, uxzC1 = uxz * oneMC, uxyC1 = uxy * oneMC, uyzC1 = uyz * oneMC;
  return d3((ux2 * oneMC + cT) * v1.x + (uxyC1 - uzS) * v1.y + (uxzC1 + uyS) * v1.z,
            (uxyC1 + uzS) * v1.x + (uy2 * oneMC + cT) * v1.y + (uyzC1 - uxS) * v1.z,
            (uxzC1 - uyS) * v1.x + (uyzC1 + uxS) * v1.y + (uz2 * oneMC + cT) * v1.z);
}
static inline D3 ortho(D3 v) {  // getOrthoVec
  D3 t = normalized(d3(1, 1, 0));
  if (std::fabs(dot(t, v) - 1) < EPS) t = d3(0, 0, 1);
  return normalized(cross(v, t));
}

}  // namespace hm
}  // namespace rt
