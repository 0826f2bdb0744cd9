// Exhaustive / randomized check of cheap correctly-rounded f32 reciprocal and
// division sequences against HIP's IEEE `/` (v_div_scale .. v_div_fixup, 10 VALU)
// on the device itself.  Candidates:
//   rcp3(b)    y0 = v_rcp_f32(b); e = fma(-b, y0, 1); y = fma(e, y0, y0)
//   div(a, b)  y = RN(1/b); q = a*y; r = fma(-q, b, a); q' = fma(r, y, q)   (Markstein)
// Output: JSON with mismatch counts per binade class and the first mismatches.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__device__ __forceinline__ float rcp3(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, y0, 1.0f);
  return __builtin_fmaf(e, y0, y0);
}

__device__ __forceinline__ bool same(float x, float y) {
  return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}

// all 2^32 patterns: counts[e] = mismatches of rcp3 for biased exponent e
__global__ void rcp_all(unsigned long long* counts, uint32_t* first, unsigned int* n_first) {
  const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = tid; i < (1ull << 32); i += stride) {
    const float b = __uint_as_float(uint32_t(i));
    const float ref = 1.0f / b;
    const float got = rcp3(b);
    if (!same(ref, got)) {
      atomicAdd(&counts[(uint32_t(i) >> 23) & 0xff], 1ull);
      const unsigned k = atomicAdd(n_first, 1u);
      if (k < 64) first[k] = uint32_t(i);
    }
  }
}

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return uint32_t(x);
}

// Markstein division with y = IEEE RN(1/b), a and b with exponents in
// [127-E, 127+E] (both signs), plus a = b * k +- few ulps (hard cases near
// midpoints come from quotients with short significands).
__global__ void div_rand(uint64_t n, int E, unsigned long long* bad, uint32_t* first, unsigned int* n_first) {
  const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = tid; i < n; i += stride) {
    const uint32_t h1 = hash32(2 * i), h2 = hash32(2 * i + 1);
    const uint32_t ea = 127 - E + (h1 >> 24) % uint32_t(2 * E + 1);
    const uint32_t eb = 127 - E + (h2 >> 24) % uint32_t(2 * E + 1);
    float a = __uint_as_float((h1 & 0x807fffffu) | (ea << 23));
    const float b = __uint_as_float((h2 & 0x807fffffu) | (eb << 23));
    if (i & 1) {  // a near a short-significand multiple of b
      const float k = float(int(h1 & 0xfff) + 1) * 0.0009765625f;
      a = __uint_as_float(__float_as_uint(b * k) + int((h2 >> 8) & 7) - 3);
    }
    const float y = 1.0f / b;
    const float q = a * y;
    const float r = __builtin_fmaf(-q, b, a);
    const float got = __builtin_fmaf(r, y, q);
    const float ref = a / b;
    if (!same(ref, got)) {
      atomicAdd(bad, 1ull);
      const unsigned k = atomicAdd(n_first, 1u);
      if (k < 32) {
        first[2 * k] = __float_as_uint(a);
        first[2 * k + 1] = __float_as_uint(b);
      }
    }
  }
}

// v_sqrt_f32 alone, and v_sqrt + LLVM's +-1 ulp fix-up without the range scaling,
// against IEEE sqrtf over all 2^32 patterns: counts[e] per biased exponent
__global__ void sqrt_all(unsigned long long* raw, unsigned long long* fix) {
  const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = tid; i < (1ull << 32); i += stride) {
    const float x = __uint_as_float(uint32_t(i));
    const float ref = __builtin_sqrtf(x);
    const float s = __builtin_amdgcn_sqrtf(x);
    if (!same(ref, s)) atomicAdd(&raw[(uint32_t(i) >> 23) & 0xff], 1ull);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    float f = s;
    if (__builtin_fmaf(-sd, s, x) <= 0.0f) f = sd;
    if (__builtin_fmaf(-su, s, x) > 0.0f) f = su;
    if (!same(ref, f)) atomicAdd(&fix[(uint32_t(i) >> 23) & 0xff], 1ull);
  }
}

static void print_counts(const char* name, const unsigned long long* h) {
  unsigned long long tot = 0;
  for (int e = 0; e < 256; ++e) tot += h[e];
  std::printf(", \"%s\": {\"mismatches\": %llu, \"by_exponent\": {", name, tot);
  bool c = false;
  for (int e = 0; e < 256; ++e)
    if (h[e]) {
      std::printf("%s\"%d\": %llu", c ? ", " : "", e, h[e]);
      c = true;
    }
  std::printf("}}");
}

int main(int argc, char** argv) {
  const uint64_t n_div = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1ull << 34);
  unsigned long long* counts;
  uint32_t* first;
  unsigned int* nf;
  CHK(hipMalloc(&counts, 256 * sizeof(unsigned long long)));
  CHK(hipMalloc(&first, 128 * sizeof(uint32_t)));
  CHK(hipMalloc(&nf, sizeof(unsigned int)));
  CHK(hipMemset(counts, 0, 256 * sizeof(unsigned long long)));
  CHK(hipMemset(nf, 0, sizeof(unsigned int)));
  rcp_all<<<8192, 256>>>(counts, first, nf);
  CHK(hipDeviceSynchronize());
  unsigned long long h[256];
  uint32_t hf[128];
  unsigned int hn;
  CHK(hipMemcpy(h, counts, sizeof h, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(&hn, nf, sizeof hn, hipMemcpyDeviceToHost));
  std::printf("{\"rcp3\": {\"mismatches\": %u, \"by_exponent\": {", hn);
  bool c = false;
  for (int e = 0; e < 256; ++e)
    if (h[e]) {
      std::printf("%s\"%d\": %llu", c ? ", " : "", e, h[e]);
      c = true;
    }
  std::printf("}, \"first\": [");
  for (unsigned k = 0; k < hn && k < 64; ++k) std::printf("%s\"0x%08x\"", k ? ", " : "", hf[k]);
  std::printf("]}");
  for (int E : {20, 50}) {
    CHK(hipMemset(counts, 0, sizeof(unsigned long long)));
    CHK(hipMemset(nf, 0, sizeof(unsigned int)));
    div_rand<<<8192, 256>>>(n_div, E, counts, first, nf);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h, counts, sizeof(unsigned long long), hipMemcpyDeviceToHost));
    CHK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&hn, nf, sizeof hn, hipMemcpyDeviceToHost));
    std::printf(", \"markstein_E%d\": {\"pairs\": %llu, \"mismatches\": %llu, \"first\": [", E,
                (unsigned long long)n_div, h[0]);
    for (unsigned k = 0; k < hn && k < 32; ++k) std::printf("%s[\"0x%08x\", \"0x%08x\"]", k ? ", " : "", hf[2 * k], hf[2 * k + 1]);
    std::printf("]}");
  }
  {
    unsigned long long *raw, *fix;
    CHK(hipMalloc(&raw, 256 * sizeof(unsigned long long)));
    CHK(hipMalloc(&fix, 256 * sizeof(unsigned long long)));
    CHK(hipMemset(raw, 0, 256 * sizeof(unsigned long long)));
    CHK(hipMemset(fix, 0, 256 * sizeof(unsigned long long)));
    sqrt_all<<<8192, 256>>>(raw, fix);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h, raw, sizeof h, hipMemcpyDeviceToHost));
    print_counts("v_sqrt", h);
    CHK(hipMemcpy(h, fix, sizeof h, hipMemcpyDeviceToHost));
    print_counts("v_sqrt_fixup", h);
  }
  std::printf("}\n");
  return 0;
}
