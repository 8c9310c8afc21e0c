// tests/test_jfdlibm.py: csrc/jfdlibm.h (host build) vs glibc over arguments spanning every
// branch; prints "<fn> <n> <max_ulp> <n_diff>" per function, and with an argument file
// writes the jf:: results (bit patterns) for the device comparison.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../distraytracer_old_amd/csrc/jfdlibm.h"

static int64_t ulps(double a, double b) {
  if (a == b) return 0;
  if (std::isnan(a) && std::isnan(b)) return 0;
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8); std::memcpy(&ib, &b, 8);
  if (ia < 0) ia = INT64_MIN - ia;
  if (ib < 0) ib = INT64_MIN - ib;
  return ia > ib ? ia - ib : ib - ia;
}

int main(int argc, char** argv) {
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> u01(0, 1);
  std::vector<double> trig, inv;
  for (int i = 0; i < 400000; ++i) trig.push_back((u01(g) * 2 - 1) * 7.0);          // [-7, 7]: n = 0..4
  for (int i = 0; i < 200000; ++i) trig.push_back(u01(g) * 6.2831854820251465);     // draws in [0, TWO_PI_F)
  for (int i = 0; i < 200000; ++i) trig.push_back((u01(g) * 2 - 1) * 1e5);          // medium range
  for (int i = 0; i < 100000; ++i) trig.push_back(std::ldexp(u01(g), -(int)(u01(g) * 40)));  // tiny
  for (int k = 1; k < 2000; ++k)  // near multiples of pi/2 (cancellation paths)
    for (int d = -3; d <= 3; ++d) trig.push_back(std::nextafter(k * 1.5707963267948966, d < 0 ? 0.0 : 1e9) + d * 1e-16 * k);
  for (int i = 0; i < 600000; ++i) inv.push_back(u01(g) * 2 - 1);                   // [-1, 1]
  for (int i = 0; i < 100000; ++i) inv.push_back(1 - std::ldexp(u01(g), -(int)(u01(g) * 50)));  // near 1
  for (int i = 0; i < 100000; ++i) inv.push_back(-1 + std::ldexp(u01(g), -(int)(u01(g) * 50)));
  for (double v : {0.0, -0.0, 0.5, -0.5, 0.975, -0.975, 1.0, -1.0, 1e-30, -1e-30, 0.4999999999999999, 0.5000000000000001})
    inv.push_back(v);
  struct F { const char* name; double (*jf)(double); double (*ref)(double); std::vector<double>* xs; };
  F fs[] = {{"sin", jf::sin, ::sin, &trig}, {"cos", jf::cos, ::cos, &trig}, {"asin", jf::asin, ::asin, &inv},
            {"acos", jf::acos, ::acos, &inv}};
  for (auto& f : fs) {
    int64_t mx = 0, nd = 0;
    for (double x : *f.xs) {
      int64_t d = ulps(f.jf(x), f.ref(x));
      if (d > mx) mx = d;
      nd += d != 0;
    }
    std::printf("%s %zu %lld %lld\n", f.name, f.xs->size(), (long long)mx, (long long)nd);
  }
  if (argc > 2) {  // argv[1]: doubles in, argv[2]: jf results out (4 per argument: sin cos asin acos)
    FILE* fi = std::fopen(argv[1], "rb");
    std::vector<double> xs;
    double v;
    while (std::fread(&v, 8, 1, fi) == 1) xs.push_back(v);
    std::fclose(fi);
    FILE* fo = std::fopen(argv[2], "wb");
    for (double x : xs) {
      double r[4] = {jf::sin(x), jf::cos(x), jf::asin(x), jf::acos(x)};
      std::fwrite(r, 8, 4, fo);
    }
    std::fclose(fo);
  }
  return 0;
}
