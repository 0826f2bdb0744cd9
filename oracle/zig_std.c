/*
 * ORACLE — test infrastructure only (see zig_std.h).  Build flags:
 * -ffp-contract=off, no fast-math: every f32 operation rounds once, as Zig's
 * (which never contracts a*b+c into an fma) does.
 */
#include "zig_std.h"

#include <math.h>
#include <string.h>

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint64_t rotl64(uint64_t x, unsigned k) { return (x << k) | (x >> (64 - k)); }

/* ---- std.rand ----------------------------------------------------------- */

/* std/rand/SplitMix64.zig: next() */
uint64_t zs_splitmix64_next(uint64_t* state) {
  *state += 0x9e3779b97f4a7c15ULL;
  uint64_t z = *state;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

/* Xoroshiro128.seed / Xoshiro256.seed: the state words are successive
 * SplitMix64 outputs of init_s. */
void zs_rng_init(zs_rng* r, int kind, uint64_t init_s) {
  uint64_t g = init_s;
  r->kind = kind;
  int n = kind == 0 ? 2 : 4;
  for (int i = 0; i < 4; ++i) r->s[i] = 0;
  for (int i = 0; i < n; ++i) r->s[i] = zs_splitmix64_next(&g);
}

uint64_t zs_rng_next(zs_rng* r) {
  if (r->kind == 0) {
    /* std/rand/Xoroshiro128.zig: next() */
    const uint64_t s0 = r->s[0];
    uint64_t s1 = r->s[1];
    const uint64_t res = s0 + s1;
    s1 ^= s0;
    r->s[0] = rotl64(s0, 55) ^ s1 ^ (s1 << 14);
    r->s[1] = rotl64(s1, 36);
    return res;
  }
  /* std/rand/Xoshiro256.zig: next() */
  uint64_t* s = r->s;
  const uint64_t res = rotl64(s[0] + s[3], 23) + s[0];
  const uint64_t t = s[1] << 17;
  s[2] ^= s[0];
  s[3] ^= s[1];
  s[1] ^= s[2];
  s[0] ^= s[3];
  s[2] ^= t;
  s[3] = rotl64(s[3], 45);
  return res;
}

/* Random.float(f32): int(u32) takes 4 little-endian bytes of one next()
 * (fill() consumes one whole next() per call), then
 * bitcast(0x7f<<23 | s>>9) - 1.0. */
float zs_random_float(zs_rng* r) {
  const uint32_t s = (uint32_t)zs_rng_next(r);
  return u2f((0x7fu << 23) | (s >> 9)) - 1.0f;
}

/* Random.boolean(): int(u1) reads one byte of one next() and truncates. */
int zs_random_boolean(zs_rng* r) { return (int)(zs_rng_next(r) & 1u); }

/* ---- std.math ----------------------------------------------------------- */

float zs_sqrt(float x) { return sqrtf(x); }
float zs_min(float x, float y) { return x < y ? x : y; }
float zs_max(float x, float y) { return x > y ? x : y; }

/* std/math/sin.zig + cos.zig (Zig <= 0.9): Go's port of Cephes sin/cos,
 * evaluated in the argument's type (f32).  The comptime_float coefficients
 * are coerced to f32 at each use. */
static const float S0 = 1.58962301576546568060E-10f;
static const float S1 = -2.50507477628578072866E-8f;
static const float S2 = 2.75573136213857245213E-6f;
static const float S3 = -1.98412698295895385996E-4f;
static const float S4 = 8.33333333332211858878E-3f;
static const float S5 = -1.66666666666666307295E-1f;
static const float C0 = -1.13585365213876817300E-11f;
static const float C1 = 2.08757008419747316778E-9f;
static const float C2 = -2.75573141792967388112E-7f;
static const float C3 = 2.48015872888517045348E-5f;
static const float C4 = -1.38888888888730564116E-3f;
static const float C5 = 4.16666666666665929218E-2f;
static const float pi4a = 7.85398125648498535156e-1f;
static const float pi4b = 3.77489470793079817668e-8f;
static const float pi4c = 2.69515142907905952645e-15f;
static const float m4pi = 1.273239544735162542821171882678754627704620361328125f;

float zs_sin(float x) {
  if (x == 0.0f || isnan(x)) return x;
  if (isinf(x)) return NAN;
  int sign = x < 0.0f;
  x = fabsf(x);
  float y = floorf(x * m4pi);
  int32_t j = (int32_t)y;
  if (j & 1) { j += 1; y += 1.0f; }
  j &= 7;
  if (j > 3) { j -= 4; sign = !sign; }
  const float z = ((x - y * pi4a) - y * pi4b) - y * pi4c;
  const float w = z * z;
  float r;
  if (j == 1 || j == 2)
    r = 1.0f - 0.5f * w + w * w * (C5 + w * (C4 + w * (C3 + w * (C2 + w * (C1 + w * C0)))));
  else
    r = z + z * w * (S5 + w * (S4 + w * (S3 + w * (S2 + w * (S1 + w * S0)))));
  return sign ? -r : r;
}

float zs_cos(float x) {
  if (isnan(x) || isinf(x)) return NAN;
  int sign = 0;
  x = fabsf(x);
  float y = floorf(x * m4pi);
  int32_t j = (int32_t)y;
  if (j & 1) { j += 1; y += 1.0f; }
  j &= 7;
  if (j > 3) { j -= 4; sign = !sign; }
  if (j > 1) sign = !sign;
  const float z = ((x - y * pi4a) - y * pi4b) - y * pi4c;
  const float w = z * z;
  float r;
  if (j == 1 || j == 2)
    r = z + z * w * (S5 + w * (S4 + w * (S3 + w * (S2 + w * (S1 + w * S0)))));
  else
    r = 1.0f - 0.5f * w + w * w * (C5 + w * (C4 + w * (C3 + w * (C2 + w * (C1 + w * C0)))));
  return sign ? -r : r;
}

/* std/math/acos.zig acos32 = musl acosf. */
static float acos_r32(float z) {
  const float pS0 = 1.6666586697e-01f;
  const float pS1 = -4.2743422091e-02f;
  const float pS2 = -8.6563630030e-03f;
  const float qS1 = -7.0662963390e-01f;
  const float p = z * (pS0 + z * (pS1 + z * pS2));
  const float q = 1.0f + z * qS1;
  return p / q;
}

float zs_acos(float x) {
  const float pio2_hi = 1.5707962513e+00f;
  const float pio2_lo = 7.5497894159e-08f;
  const uint32_t hx = f2u(x);
  const uint32_t ix = hx & 0x7fffffffu;
  if (ix >= 0x3f800000u) {
    if (ix == 0x3f800000u) {
      if (hx >> 31) return 2.0f * pio2_hi + 0x1.0p-120f;
      return 0.0f;
    }
    return NAN;
  }
  if (ix < 0x3f000000u) {
    if (ix <= 0x32800000u) return pio2_hi + 0x1.0p-120f;
    return pio2_hi - (x - (pio2_lo - x * acos_r32(x * x)));
  }
  if (hx >> 31) {
    const float z = (1.0f + x) * 0.5f;
    const float s = sqrtf(z);
    const float w = acos_r32(z) * s - pio2_lo;
    return 2.0f * (pio2_hi - (s + w));
  }
  const float z = (1.0f - x) * 0.5f;
  const float s = sqrtf(z);
  const float df = u2f(f2u(s) & 0xfffff000u);
  const float c = (z - df * df) / (s + df);
  const float w = acos_r32(z) * s + c;
  return 2.0f * (df + w);
}

/* std/math/atan.zig atan32 = musl atanf. */
float zs_atan(float x_) {
  static const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f,
                                  9.8279368877e-01f, 1.5707962513e+00f};
  static const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f,
                                  3.4473217170e-08f, 7.5497894159e-08f};
  static const float aT[5] = {3.3333328366e-01f, -1.9999158382e-01f, 1.4253635705e-01f,
                              -1.0648017377e-01f, 6.1687607318e-02f};
  float x = x_;
  uint32_t ix = f2u(x);
  const uint32_t sign = ix >> 31;
  ix &= 0x7fffffffu;
  int id;
  if (ix >= 0x4c800000u) {
    if (isnan(x)) return x;
    const float z = atanhi[3] + 0x1.0p-120f;
    return sign ? -z : z;
  }
  if (ix < 0x3ee00000u) {
    if (ix < 0x39800000u) return x;
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000u) {
      if (ix < 0x3f300000u) {
        id = 0;
        x = (2.0f * x - 1.0f) / (2.0f + x);
      } else {
        id = 1;
        x = (x - 1.0f) / (x + 1.0f);
      }
    } else {
      if (ix < 0x401c0000u) {
        id = 2;
        x = (x - 1.5f) / (1.0f + 1.5f * x);
      } else {
        id = 3;
        x = -1.0f / x;
      }
    }
  }
  float z = x * x;
  const float w = z * z;
  const float s1 = z * (aT[0] + w * (aT[2] + w * aT[4]));
  const float s2 = w * (aT[1] + w * aT[3]);
  if (id < 0) return x - x * (s1 + s2);
  z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return sign ? -z : z;
}

/* std/math/atan2.zig atan2_32 = musl atan2f. */
float zs_atan2(float y, float x) {
  const float pi = 3.1415927410e+00f;
  const float pi_lo = -8.7422776573e-08f;
  if (isnan(x) || isnan(y)) return x + y;
  uint32_t ix = f2u(x);
  uint32_t iy = f2u(y);
  if (ix == 0x3f800000u) return zs_atan(y);
  const uint32_t m = ((iy >> 31) & 1u) | ((ix >> 30) & 2u);
  ix &= 0x7fffffffu;
  iy &= 0x7fffffffu;
  if (iy == 0) {
    switch (m) {
      case 0: case 1: return y;
      case 2: return pi;
      default: return -pi;
    }
  }
  if (ix == 0) return (m & 1) ? -pi / 2.0f : pi / 2.0f;
  if (ix == 0x7f800000u) {
    if (iy == 0x7f800000u) {
      switch (m) {
        case 0: return pi / 4.0f;
        case 1: return -pi / 4.0f;
        case 2: return 3.0f * pi / 4.0f;
        default: return -3.0f * pi / 4.0f;
      }
    }
    switch (m) {
      case 0: return 0.0f;
      case 1: return -0.0f;
      case 2: return pi;
      default: return -pi;
    }
  }
  if (ix + (26u << 23) < iy || iy == 0x7f800000u) return (m & 1) ? -pi / 2.0f : pi / 2.0f;
  float z;
  if ((m & 2) && iy + (26u << 23) < ix)
    z = 0.0f;
  else
    z = zs_atan(fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

/* std/math/pow.zig (Go port), restated for integral y > 0 (the path only
 * calls pow(f32, 1 - cosine, 5.0), material.zig:127).  ans = a1 * 2^ae by
 * repeated squaring of frexp's significand. */
float zs_pow(float x, float y) {
  if (y == 0.0f || x == 1.0f) return 1.0f;
  if (isnan(x) || isnan(y)) return NAN;
  if (y == 1.0f) return x;
  const float yi_f = truncf(fabsf(y));
  const int y_odd = fmodf(yi_f, 2.0f) == 1.0f;
  if (x == 0.0f) {
    if (y < 0.0f) return y_odd ? copysignf(INFINITY, x) : INFINITY;
    return y_odd ? x : 0.0f;
  }
  if (isinf(x) || isinf(y) || yi_f != fabsf(y) || y < 0.0f) {
    return powf(x, y); /* not on the path: only y = 5, x in [0, 2] occurs */
  }
  float a1 = 1.0f;
  int ae = 0;
  int xe;
  float x1 = frexpf(x, &xe);
  int32_t i = (int32_t)yi_f;
  while (i != 0) {
    const int overflow_shift = 8 + 1; /* floatExponentBits(f32) + 1 */
    if (xe < -(1 << overflow_shift) || (1 << overflow_shift) < xe) {
      ae += xe;
      break;
    }
    if (i & 1) {
      a1 *= x1;
      ae += xe;
    }
    x1 *= x1;
    xe *= 2; /* xe << 1 without the UB of shifting a negative value */
    if (x1 < 0.5f) {
      x1 += x1;
      xe -= 1;
    }
    i >>= 1;
  }
  return ldexpf(a1, ae);
}
