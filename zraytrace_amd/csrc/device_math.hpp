// device_math.hpp — f32 math of the reference's hot path, on the device.
//
// Every function is built from IEEE-correctly-rounded +,-,*,/,sqrt (HIP's
// default for f32 division and sqrtf), exact bit operations and exact
// conversions, and the file is compiled with -ffp-contract=off, so results are
// bit-identical to the same algorithms on any IEEE host.  The algorithms are
// those of the Zig 0.9 standard library the reference calls:
//   sin/cos    std/math/sin.zig, cos.zig (Go port of Cephes)   sample.zig:51
//   acos       std/math/acos.zig (musl acosf)                   sphere.zig:47
//   atan2      std/math/atan2.zig, atan.zig (musl atan2f/atanf) sphere.zig:48
//   pow(x, 5)  std/math/pow.zig (Go port; frexp + squaring)     material.zig:127
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace zrt {
namespace dev {

__device__ __forceinline__ float fmin_z(float x, float y) { return x < y ? x : y; }  // math.min
__device__ __forceinline__ float fmax_z(float x, float y) { return x > y ? x : y; }  // math.max


__device__ __forceinline__ bool is_nan(float x) { return x != x; }
__device__ __forceinline__ bool is_inf(float x) { return __builtin_fabsf(x) == __builtin_inff(); }

// ---- correctly rounded reciprocal and division in fewer instructions ----
// HIP's f32 `/` (and 1.0f / b) is v_div_scale x2, v_rcp, five FMA/MUL, v_div_fmas,
// v_div_fixup: 10 VALU, its scaling steps there for operands near the ends of the
// exponent range.  Inside the range two shorter sequences give the same bits:
//
// rcp_core(b) = v_rcp_f32 (1 ulp) + one Newton step: 3 VALU.  Equal to IEEE 1.0f / b
//   for EVERY b with 2^-126 <= |b| < 2^126: checked on an MI355X over all 2^32
//   inputs (tools/div_exact.hip, zrt_debug_division; profiles/r02/div_exact.json);
//   the only other inputs where it differs are zeros, subnormals, |b| >= 2^126, inf.
// div_core(a, b, y) with y = RN(1/b): Markstein's correction, q = a*y, r = a - b*q
//   (exact by FMA), q + r*y: 3 VALU, RN(a / b) whenever nothing under- or overflows
//   (Markstein's theorem: y within 1/2 ulp of 1/b and q within 1 ulp of a/b);
//   3.4e10 random and near-midpoint pairs with exponents in [-50, 50] checked on the
//   device, no difference.  Callers keep every operand in [2^-50, 2^50] (or prove it).
__device__ __forceinline__ float rcp_core(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float div_core(float a, float b, float y) {
  const float q = a * y;
  return __builtin_fmaf(__builtin_fmaf(-q, b, a), y, q);
}
#ifndef ZRT_FAST_DIV
#define ZRT_FAST_DIV 1  // 0: every reciprocal / division through HIP's IEEE `/` (A/B builds)
#endif
#ifndef ZRT_FAST_SQRT
#define ZRT_FAST_SQRT ZRT_FAST_DIV  // 0: HIP's IEEE sqrtf
#endif
__device__ __forceinline__ bool rcp_core_ok(float b) {
  const float m = __builtin_fabsf(b);
  return ZRT_FAST_DIV && m >= 0x1p-126f && m < 0x1p126f;  // false for NaN
}
// a / b for a caller-proven range, y = RN(1/b) known (a constant or per frame)
__device__ __forceinline__ float div_known(float a, float b, float y) {
  return ZRT_FAST_DIV ? div_core(a, b, y) : a / b;
}
// 1.0f / b, bit for bit
__device__ __forceinline__ float rcp_rn(float b) {
  if (__builtin_expect(rcp_core_ok(b), 1)) return rcp_core(b);
  return 1.0f / b;
}
// sqrt_core: v_sqrt_f32 (1 ulp) and LLVM's +-1 ulp fix-up by FMA residuals, without
//   the scaling of small inputs and the zero / inf class select HIP's IEEE sqrtf adds
//   (9 VALU instead of 16).  Equal to IEEE sqrtf for every x >= 2^-104 (and +inf):
//   all 2^32 inputs checked on an MI355X (tools/div_exact.hip, zrt_debug_division).
__device__ __forceinline__ float sqrt_core(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __uint_as_float(__float_as_uint(s) - 1u);
  const float su = __uint_as_float(__float_as_uint(s) + 1u);
  const float f = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
  return __builtin_fmaf(-su, s, x) > 0.0f ? su : f;
}
// sqrt, bit for bit (IEEE for zero, subnormal, negative and NaN inputs)
__device__ __forceinline__ float sqrt_rn(float x) {
  if (__builtin_expect(ZRT_FAST_SQRT && x >= 0x1p-100f, 1)) return sqrt_core(x);
  return __builtin_sqrtf(x);
}

// a / b, bit for bit
__device__ __forceinline__ float div_rn(float a, float b) {
  const float mb = __builtin_fabsf(b);
  if (__builtin_expect(ZRT_FAST_DIV && mb >= 0x1p-50f && mb <= 0x1p50f, 1)) {
    const float y = rcp_core(b);
    const float mq = __builtin_fabsf(a * y);
    if (__builtin_expect(mq >= 0x1p-50f && mq <= 0x1p50f, 1)) return div_core(a, b, y);
  }
  return a / b;
}

// Go/Cephes sin & cos as Zig <= 0.9 evaluates them in f32.
namespace cephes {
constexpr float S0 = 1.58962301576546568060E-10f;
constexpr float S1 = -2.50507477628578072866E-8f;
constexpr float S2 = 2.75573136213857245213E-6f;
constexpr float S3 = -1.98412698295895385996E-4f;
constexpr float S4 = 8.33333333332211858878E-3f;
constexpr float S5 = -1.66666666666666307295E-1f;
constexpr float C0 = -1.13585365213876817300E-11f;
constexpr float C1 = 2.08757008419747316778E-9f;
constexpr float C2 = -2.75573141792967388112E-7f;
constexpr float C3 = 2.48015872888517045348E-5f;
constexpr float C4 = -1.38888888888730564116E-3f;
constexpr float C5 = 4.16666666666665929218E-2f;
constexpr float pi4a = 7.85398125648498535156e-1f;
constexpr float pi4b = 3.77489470793079817668e-8f;
constexpr float pi4c = 2.69515142907905952645e-15f;
constexpr float m4pi = 1.273239544735162542821171882678754627704620361328125f;
}  // namespace cephes

// One argument reduction shared by sin and cos (both evaluate the same z, w, j).
__device__ __forceinline__ void sincos_z(float xin, float* s_out, float* c_out) {
  using namespace cephes;
  const bool sneg = xin < 0.0f;
  const float x = __builtin_fabsf(xin);
  float y = __builtin_floorf(x * m4pi);
  int32_t j = (int32_t)y;
  if (j & 1) {
    j += 1;
    y += 1.0f;
  }
  j &= 7;
  bool s_sign = sneg, c_sign = false;
  if (j > 3) {
    j -= 4;
    s_sign = !s_sign;
    c_sign = !c_sign;
  }
  if (j > 1) c_sign = !c_sign;
  const float z = ((x - y * pi4a) - y * pi4b) - y * pi4c;
  const float w = z * z;
  const float pc = 1.0f - 0.5f * w + w * w * (C5 + w * (C4 + w * (C3 + w * (C2 + w * (C1 + w * C0)))));
  const float ps = z + z * w * (S5 + w * (S4 + w * (S3 + w * (S2 + w * (S1 + w * S0)))));
  const bool swap = (j == 1 || j == 2);
  const float rs = swap ? pc : ps;
  const float rc = swap ? ps : pc;
  float s = s_sign ? -rs : rs;
  float c = c_sign ? -rc : rc;
  // special cases of sin.zig / cos.zig
  if (xin == 0.0f || is_nan(xin)) s = xin;
  else if (is_inf(xin)) s = __builtin_nanf("");
  if (is_nan(xin) || is_inf(xin)) c = __builtin_nanf("");
  *s_out = s;
  *c_out = c;
}

// musl acosf
__device__ __forceinline__ float acos_r32(float z) {
  const float p = z * (1.6666586697e-01f + z * (-4.2743422091e-02f + z * -8.6563630030e-03f));
  const float q = 1.0f + z * -7.0662963390e-01f;
  return p / q;
}
__device__ __forceinline__ float acos_z(float x) {
  const float pio2_hi = 1.5707962513e+00f;
  const float pio2_lo = 7.5497894159e-08f;
  const uint32_t hx = __float_as_uint(x);
  const uint32_t ix = hx & 0x7fffffffu;
  if (ix >= 0x3f800000u) {
    if (ix == 0x3f800000u) return (hx >> 31) ? 2.0f * pio2_hi + 0x1.0p-120f : 0.0f;
    return __builtin_nanf("");
  }
  if (ix < 0x3f000000u) {
    if (ix <= 0x32800000u) return pio2_hi + 0x1.0p-120f;
    return pio2_hi - (x - (pio2_lo - x * acos_r32(x * x)));
  }
  if (hx >> 31) {
    const float z = (1.0f + x) * 0.5f;
    const float s = sqrt_rn(z);
    const float w = acos_r32(z) * s - pio2_lo;
    return 2.0f * (pio2_hi - (s + w));
  }
  const float z = (1.0f - x) * 0.5f;
  const float s = sqrt_rn(z);
  const float df = __uint_as_float(__float_as_uint(s) & 0xfffff000u);
  const float c = (z - df * df) / (s + df);
  const float w = acos_r32(z) * s + c;
  return 2.0f * (df + w);
}

// musl atanf
__device__ __forceinline__ float atan_z(float xin) {
  float x = xin;
  uint32_t ix = __float_as_uint(x);
  const uint32_t sign = ix >> 31;
  ix &= 0x7fffffffu;
  int id;
  if (ix >= 0x4c800000u) {
    if (is_nan(x)) return x;
    const float z = 1.5707962513e+00f + 0x1.0p-120f;
    return sign ? -z : z;
  }
  if (ix < 0x3ee00000u) {
    if (ix < 0x39800000u) return x;
    id = -1;
  } else {
    x = __builtin_fabsf(x);
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
  const float s1 = z * (3.3333328366e-01f + w * (1.4253635705e-01f + w * 6.1687607318e-02f));
  const float s2 = w * (-1.9999158382e-01f + w * -1.0648017377e-01f);
  if (id < 0) return x - x * (s1 + s2);
  const float hi = id == 0 ? 4.6364760399e-01f : id == 1 ? 7.8539812565e-01f
                 : id == 2 ? 9.8279368877e-01f : 1.5707962513e+00f;
  const float lo = id == 0 ? 5.0121582440e-09f : id == 1 ? 3.7748947079e-08f
                 : id == 2 ? 3.4473217170e-08f : 7.5497894159e-08f;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return sign ? -z : z;
}

// musl atan2f
__device__ __forceinline__ float atan2_z(float y, float x) {
  const float pi = 3.1415927410e+00f;
  const float pi_lo = -8.7422776573e-08f;
  if (is_nan(x) || is_nan(y)) return x + y;
  uint32_t ix = __float_as_uint(x);
  uint32_t iy = __float_as_uint(y);
  if (ix == 0x3f800000u) return atan_z(y);
  const uint32_t m = ((iy >> 31) & 1u) | ((ix >> 30) & 2u);
  ix &= 0x7fffffffu;
  iy &= 0x7fffffffu;
  if (iy == 0) {
    if (m < 2) return y;
    return m == 2 ? pi : -pi;
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
  if ((m & 2) && iy + (26u << 23) < ix) z = 0.0f;
  else z = atan_z(__builtin_fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// std.math.pow(f32, x, 5.0): Go algorithm, a1 * 2^ae by squaring frexp(x)'s
// significand (pow.zig), for the path's only exponent.
__device__ __forceinline__ float pow5_z(float x) {
  if (x == 1.0f) return 1.0f;
  if (is_nan(x)) return x;
  if (x == 0.0f) return x;  // y = 5 is an odd integer: pow(+-0, 5) = +-0
  int xe;
  float x1 = __builtin_frexpf(x, &xe);
  float a1 = 1.0f;
  int ae = 0;
  // i = 5 (binary 101)
  a1 *= x1;
  ae += xe;
  x1 *= x1;
  xe *= 2;
  if (x1 < 0.5f) { x1 += x1; xe -= 1; }
  // i = 2
  x1 *= x1;
  xe *= 2;
  if (x1 < 0.5f) { x1 += x1; xe -= 1; }
  // i = 1
  a1 *= x1;
  ae += xe;
  return __builtin_ldexpf(a1, ae);
}

}  // namespace dev
}  // namespace zrt
