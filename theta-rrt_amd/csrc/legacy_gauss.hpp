// numpy RandomState's gaussian (np.random.normal -> legacy_gauss) restated for the device: the
// stream rand_conf draws three values of per iteration (rrt.py:58,66).  Host-and-device code so the
// CPU tests can check the same arithmetic against np.random without a GPU.
//
//   MT19937 output word: tempering of the state word (numpy mt19937_next)
//   legacy_double:       (a >> 5) * 2^26 + (b >> 6), / 2^53, from two successive words a, b
//   legacy_gauss:        x1 = 2 d1 - 1, x2 = 2 d2 - 1, r2 = x1 x1 + x2 x2, retry while r2 >= 1 or
//                        r2 == 0; f = sqrt(-2 log(r2) / r2); return f x2, keep f x1 for the next
//                        call (has_gauss)
//
// `log` is glibc's (numpy calls libm): not correctly rounded (~0.3 % of the r2 values differ from
// the correctly rounded log), so legacy_log() below restates it operation for operation, with the
// fused multiply-adds of glibc's x86-64 FMA variant (__log_fma, the one the ifunc picks on
// FMA/AVX2 hosts).  Compile without contraction: every product and sum below is a separate IEEE op
// unless written as fma().
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "legacy_log.hpp"

#if defined(__HIPCC__)
#define TR_LG __host__ __device__ inline
#else
#define TR_LG inline
#endif

namespace tr {

TR_LG uint64_t lg_bits(double v) {
  uint64_t u;
  memcpy(&u, &v, 8);
  return u;
}
TR_LG double lg_double(uint64_t u) {
  double v;
  memcpy(&v, &u, 8);
  return v;
}

// glibc log for a positive normal finite x (the polar method's r2 is in [2^-104, 1)).
TR_LG double legacy_log(double x) {
  using namespace glibc_log;
  const uint64_t ix = lg_bits(x);
  if (ix - 0x3fee000000000000ull <= 0x308ffffffffffull) {   // x in [1 - 2^-4, 1 + 0x1.09p-4)
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double r = x - 1.0;
    const double r2 = r * r, r3 = r * r2;
    double p2 = fma(r, kB[2], kB[1]);
    double p3 = fma(r, kB[5], kB[4]);
    const double p5 = fma(r, kB[8], kB[7]);
    p2 = fma(r2, kB[3], p2);
    p3 = fma(r2, kB[6], p3);
    double p = fma(r2, kB[9], p5);
    p = fma(r3, kB[10], p);
    p = fma(p, r3, p3);
    p = fma(p, r3, p2);                                      // B1 + r B2 + ... + r^9 B10
    const double t = fma(r, 0x1p27, r);
    const double rhi = fma(-0x1p27, r, t);                   // r rounded to 26 bits
    const double rhi2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = fma(rhi2, kB[0], r);
    double lo = fma(rhi2, kB[0], r - hi);
    lo = fma(kB[0] * rlo, r + rhi, lo);
    return hi + fma(p, r3, lo);
  }
  // x = 2^k z, z in [0x1.6p-1, 0x1.6p0); log x = k ln2 + log c + log1p(z / c - 1)
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const double z = lg_double(ix - (tmp & 0xfff0000000000000ull));
  const double invc = kTab[2 * i], logc = kTab[2 * i + 1];
  const double kd = (double)k;
  const double r = fma(z, invc, -1.0);
  const double w = fma(kd, kLn2hi, logc);
  const double q1 = fma(r, kA[2], kA[1]);
  const double hi = r + w;
  const double r2 = r * r;
  const double lo = fma(kd, kLn2lo, (w - hi) + r);
  const double r3 = r * r2;
  double q = fma(r, kA[4], kA[3]);
  const double y0 = fma(r2, kA[0], lo);
  q = fma(q, r2, q1);
  return fma(r3, q, y0) + hi;
}

TR_LG uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// One polar-method attempt from four successive tempered words; true when accepted, with the two
// gaussians in stream order (first = f x2, returned; second = f x1, kept in has_gauss).
TR_LG bool legacy_attempt(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, double* first,
                          double* second) {
  const double d1 = ((double)(int32_t)(w0 >> 5) * 67108864.0 + (double)(int32_t)(w1 >> 6)) / 9007199254740992.0;
  const double d2 = ((double)(int32_t)(w2 >> 5) * 67108864.0 + (double)(int32_t)(w3 >> 6)) / 9007199254740992.0;
  const double x1 = 2.0 * d1 - 1.0, x2 = 2.0 * d2 - 1.0;
  const double r2 = x1 * x1 + x2 * x2;
  if (r2 >= 1.0 || r2 == 0.0) return false;
  const double f = sqrt(-2.0 * legacy_log(r2) / r2);
  *first = f * x2;
  *second = f * x1;
  return true;
}

// MT19937 twist element: new key[i] from key[i], key[i + 1] and key[i + 397] (mod 624; the last two
// already twisted where the reference loop has overwritten them).
TR_LG uint32_t mt_mix(uint32_t cur, uint32_t next, uint32_t far) {
  const uint32_t y = (cur & 0x80000000u) | (next & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

}  // namespace tr
