// ubench.hip — measured ceilings of the resources render_kernel can be bound by
// (bench.py's roofline.ceilings): VALU issue, L1 (TCP) access rate, L2 read
// rate.  Each kernel saturates one resource with the whole chip; the rates are
// reported per second from HIP events and, under rocprofv3 --pmc, the same
// counters bench.py reads for render_kernel (SQ_INSTS_VALU,
// TCP_TOTAL_CACHE_ACCESSES_sum, TCP_TCC_READ_REQ_sum) calibrate them.
//
// build: hipcc --offload-arch=gfx950 -O3 -o abvar/ubench tools/ubench.hip
// run:   abvar/ubench > profiles/r02/ubench.json
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int kIters = 4096;

// 8 independent f32 multiply-add chains (the compiler fuses each into one
// v_fma_f32): 8 VALU per iteration, no memory traffic.
__global__ void __launch_bounds__(256) valu_kernel(float* out, float a, float b) {
  float x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 0.001f + k;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = __fadd_rn(__fmul_rn(x[k], a), b);
  }
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  if (s == 12345.678f) out[blockIdx.x] = s;  // keep the chains alive
}

// One VALU instruction class at a time (inline asm, so the compiler neither
// fuses nor packs): 16 independent chains per wave, 16 instructions per
// iteration.  Which classes issue at one wave64 instruction per 2 cycles per
// SIMD and which take longer decides the VALU ceiling of a kernel's mix.
#define ZRT_UB_VALU(NAME, ASM)                                                               \
  __global__ void __launch_bounds__(256) NAME(float* out, float a) {                         \
    float x[16];                                                                            \
    _Pragma("unroll") for (int k = 0; k < 16; ++k) x[k] = threadIdx.x * 0.001f + k;          \
    for (int i = 0; i < kIters / 2; ++i) {                                                  \
      _Pragma("unroll") for (int k = 0; k < 16; ++k) asm volatile(ASM : "+v"(x[k]) : "v"(a)); \
    }                                                                                       \
    float s = 0.0f;                                                                         \
    _Pragma("unroll") for (int k = 0; k < 16; ++k) s += x[k];                               \
    if (s == 12345.678f) out[blockIdx.x] = s;                                               \
  }
ZRT_UB_VALU(valu_add_f32, "v_add_f32 %0, %0, %1")
ZRT_UB_VALU(valu_mul_f32, "v_mul_f32 %0, %0, %1")
ZRT_UB_VALU(valu_fma_f32, "v_fma_f32 %0, %0, %1, %1")
ZRT_UB_VALU(valu_max3_f32, "v_max3_f32 %0, %0, %1, %1")
ZRT_UB_VALU(valu_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
ZRT_UB_VALU(valu_add_u32, "v_add_u32 %0, %0, %1")
ZRT_UB_VALU(valu_xor_b32, "v_xor_b32 %0, %0, %1")
ZRT_UB_VALU(valu_rcp_f32, "v_rcp_f32 %0, %0")

// Does scalar work take VALU issue?  The same 16 v_fma_f32 chains with NS scalar ALU
// instructions per iteration beside them (4 independent SGPR chains): render_kernel
// issues 0.39 SALU per VALU on C4 (PMC SQ_INSTS_SALU / SQ_INSTS_VALU), mostly exec-mask
// and uniform-branch work.  If the VALU rate holds as NS grows, SALU is free.
constexpr int kMixIters = kIters * 4;
template <int NS>
__global__ void __launch_bounds__(256) valu_salu_mix(float* out, float a) {
  float x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = threadIdx.x * 0.001f + k;
  uint32_t s0 = blockIdx.x, s1 = blockIdx.x + 1u, s2 = blockIdx.x + 2u, s3 = blockIdx.x + 3u;
  for (int i = 0; i < kMixIters; ++i) {  // (milliseconds per launch: ramp-up and launch cost negligible)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x[k]) : "v"(a));
      if (NS > 0 && (k * NS) % 16 + NS > 15) {  // NS of the 16 slots, spread evenly
        switch ((k * NS / 16) & 3) {
          case 0: asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(s0) : : "scc"); break;
          case 1: asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(s1) : : "scc"); break;
          case 2: asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(s2) : : "scc"); break;
          default: asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(s3) : : "scc"); break;
        }
      }
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += x[k];
  if (s == 12345.678f || (s0 ^ s1 ^ s2 ^ s3) == 0x12345u) out[blockIdx.x] = s;
}

// float4 loads from a table of `mask + 1` float4 (a power of two), index
// advancing by `step` float4 per lane and per iteration: with a 16 KiB table
// every access hits the CU's L1; with a 2 MiB table and a 2 KiB lane stride
// they miss L1 and hit the XCD's L2.  `spread` = float4 between neighbouring
// lanes: 1 -> a wave reads 1 KiB contiguous (16 x 64-B lines), 8 -> 64 lanes
// in 64 different 128-B lines.
__global__ void __launch_bounds__(256) load_kernel(const float4* __restrict__ t, uint32_t mask, uint32_t spread,
                                                   uint32_t step, int iters, float* out) {
  uint32_t idx = (threadIdx.x * spread + blockIdx.x * 977u) & mask;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 v = t[(idx + u * 64u * spread) & mask];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    idx = (idx + step) & mask;
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.678f) out[blockIdx.x] = acc.x;
}

static float time_ms(void (*launch)(void*), void* arg, int reps) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  launch(arg);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch(arg);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

struct LoadArgs {
  const float4* t;
  uint32_t mask, spread, step;
  int iters, grid;
  float* out;
};
static void launch_load(void* p) {
  const LoadArgs* a = static_cast<const LoadArgs*>(p);
  hipLaunchKernelGGL(load_kernel, dim3(a->grid), dim3(256), 0, 0, a->t, a->mask, a->spread, a->step, a->iters, a->out);
}
struct ValuArgs {
  int grid;
  float* out;
};
static void launch_valu(void* p) {
  const ValuArgs* a = static_cast<const ValuArgs*>(p);
  hipLaunchKernelGGL(valu_kernel, dim3(a->grid), dim3(256), 0, 0, a->out, 0.999f, 0.001f);
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int grid = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  float* out = nullptr;
  CHK(hipMalloc(&out, grid * sizeof(float)));
  float4* t = nullptr;
  const size_t big = (32u << 20) / sizeof(float4);
  CHK(hipMalloc(&t, big * sizeof(float4)));
  CHK(hipMemset(t, 0, big * sizeof(float4)));

  std::printf("{\n \"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d,\n", prop.gcnArchName, cus, prop.clockRate);
  {
    ValuArgs a{grid, out};
    const float ms = time_ms(launch_valu, &a, 5);
    const double waves = double(grid) * 4;
    const double insts = waves * kIters * 8.0;  // VALU wave-instructions in the loop (8 v_fma_f32)
    std::printf(" \"valu\": {\"ms\": %.4f, \"wave_insts\": %.0f, \"wave_insts_per_s\": %.4e},\n", ms, insts,
                insts / (ms * 1e-3));
  }
  {
    struct {
      const char* name;
      void (*fn)(float*, float);
    } ops[] = {{"add_f32", valu_add_f32}, {"mul_f32", valu_mul_f32}, {"fma_f32", valu_fma_f32},
               {"max3_f32", valu_max3_f32}, {"cndmask", valu_cndmask}, {"add_u32", valu_add_u32},
               {"xor_b32", valu_xor_b32}, {"rcp_f32", valu_rcp_f32}};
    std::printf(" \"valu_ops\": {\n");
    const int nops = int(sizeof(ops) / sizeof(ops[0]));
    for (int o = 0; o < nops; ++o) {
      hipEvent_t e0, e1;
      CHK(hipEventCreate(&e0));
      CHK(hipEventCreate(&e1));
      hipLaunchKernelGGL(ops[o].fn, dim3(grid), dim3(256), 0, 0, out, 0.999f);
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ops[o].fn, dim3(grid), dim3(256), 0, 0, out, 0.999f);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double insts = double(grid) * 4 * (kIters / 2) * 16.0;
      // per SIMD per cycle at the nominal 2.4 GHz (the PMC pass gives the real clock)
      std::printf("  \"%s\": {\"ms\": %.4f, \"wave_insts_per_s\": %.4e, \"per_simd_per_clk_2400\": %.4f}%s\n",
                  ops[o].name, ms, insts / (ms * 1e-3), insts / (ms * 1e-3) / (cus * 4.0) / 2.4e9,
                  o + 1 < nops ? "," : "");
    }
    std::printf(" },\n");
  }
  {
    struct {
      int ns;
      void (*fn)(float*, float);
    } mix[] = {{0, valu_salu_mix<0>}, {4, valu_salu_mix<4>}, {8, valu_salu_mix<8>}, {16, valu_salu_mix<16>}};
    std::printf(" \"valu_salu_mix\": {\n");
    for (int o = 0; o < 12; ++o) {  // three interleaved rounds of the four mixes
      hipEvent_t e0, e1;
      CHK(hipEventCreate(&e0));
      CHK(hipEventCreate(&e1));
      hipLaunchKernelGGL(mix[o % 4].fn, dim3(grid), dim3(256), 0, 0, out, 0.999f);
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(mix[o % 4].fn, dim3(grid), dim3(256), 0, 0, out, 0.999f);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double valu = double(grid) * 4 * kMixIters * 16.0, salu = valu * mix[o % 4].ns / 16.0;
      std::printf("  \"salu_per_16_valu_%d_r%d\": {\"ms\": %.4f, \"valu_per_simd_per_clk_2400\": %.4f, "
                  "\"salu_per_simd_per_clk_2400\": %.4f}%s\n",
                  mix[o % 4].ns, o / 4, ms, valu / (ms * 1e-3) / (cus * 4.0) / 2.4e9,
                  salu / (ms * 1e-3) / (cus * 4.0) / 2.4e9, o + 1 < 12 ? "," : "");
    }
    std::printf(" },\n");
  }
  struct Case {
    const char* name;
    uint32_t table_f4, spread, step;
    int iters;
  } cases[] = {
      {"l1_coalesced", 1024, 1, 64, 512},      // 16 KiB, 1 KiB contiguous per wave-instruction
      {"l1_divergent", 1024, 8, 8, 512},       // 16 KiB, 64 distinct 128-B lines per wave-instruction
      {"l2_divergent", 131072, 128, 4096, 64},  // 2 MiB, lanes 2 KiB apart: 64 lines per wave-instruction, all L1 misses
  };
  std::printf(" \"loads\": {\n");
  for (size_t i = 0; i < sizeof(cases) / sizeof(cases[0]); ++i) {
    const Case& c = cases[i];
    LoadArgs a{t, c.table_f4 - 1, c.spread, c.step, c.iters, grid, out};
    const float ms = time_ms(launch_load, &a, 5);
    const double wave_insts = double(grid) * 4 * c.iters * 8;
    const double bytes = wave_insts * 64 * 16;  // bytes delivered to lanes
    std::printf("  \"%s\": {\"ms\": %.4f, \"vmem_wave_insts\": %.0f, \"lane_bytes_per_s\": %.4e, "
                "\"vmem_insts_per_s\": %.4e}%s\n",
                c.name, ms, wave_insts, bytes / (ms * 1e-3), wave_insts / (ms * 1e-3),
                i + 1 < sizeof(cases) / sizeof(cases[0]) ? "," : "");
  }
  std::printf(" }\n}\n");
  CHK(hipFree(t));
  CHK(hipFree(out));
  return 0;
}
