// ubench_shapes.hip — the render kernel's own vector-memory shapes, measured
// alone with the whole chip: what one wave-instruction of
// each shape costs the CU's data-return path (TA / TD) when the shape saturates
// it, and what a dependent hop costs in latency.  tools/ubench.hip measured
// generic patterns (1 KiB contiguous, 64 lines per instruction); the lockstep
// FAST loop (render.hip render_loop, wide_iter) issues other shapes:
//
//   node<K, TABLE, CHAIN, WPS>  a 128-B wide node (8 x global_load_dwordx4) read
//       by every lane of a wave, K distinct nodes per wave (lanes l*K/64 share
//       one; K = 1 is the wave-coherent fetch, 64 every lane its own node), from a
//       table of TABLE nodes (128 = 16 KiB, L1-resident; 12 800 = 1.6 MB, the
//       bunny's eight octant copies, L2-resident), the next node's index either
//       independent of the loaded record (CHAIN = 0: throughput) or computed from
//       it (CHAIN = 1: a dependent hop, as the traversal's next node), at WPS
//       waves per SIMD (6: the lockstep kernel's occupancy; 1: one wave alone).
//   prim<K>  a 48-B triangle record (3 x dwordx4), K distinct per wave.
//   lane_dwords<MODE>  spill-shaped traffic: one dword per lane at consecutive
//       lanes (256 B per wave-instruction, the layout scratch uses), in a per-wave
//       region of 25 rows x 256 B (the kernel's 100 B/lane private segment):
//       MODE 0 8 stores then their 8 reloads, 1 stores only, 2 loads only.
//
// Each case is its own kernel instantiation, so rocprofv3 --pmc attributes TD /
// TA busy, TCP accesses and SQ_INSTS_VMEM_* per case (tools/gpu_ubench.sh,
// tools/ubench_summary.py).  Output: JSON of HIP-event times per case.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_shapes.bin tools/ubench_shapes.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t fold(float4 v) {
  return __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
}

// The table is all zeros, so `s` is 0 and the index sequence is the same for
// CHAIN = 0 and 1; the compiler cannot know it, so with CHAIN the next address
// waits for the loaded record.  `zero` (a kernel argument, 0) keeps the index in
// a VGPR: the loads stay vector loads even where every lane's index is equal.
template <int K, uint32_t TABLE, bool CHAIN, int WPS>
__global__ void __launch_bounds__(kBlock) node(const float4* __restrict__ t, uint32_t zero, int iters,
                                               uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const uint32_t grp = (lane * (uint32_t)K) >> 6;
  uint32_t h = wave * 0x9E3779B9u + grp * 0x85EBCA6Bu + 0x165667B1u;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const uint32_t n = ((h >> 9) & (TABLE - 1u)) | (lane & zero);
    const float4* q = t + 8u * n;
    const float4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3], v4 = q[4], v5 = q[5], v6 = q[6], v7 = q[7];
    const uint32_t s = fold(v0) ^ fold(v1) ^ fold(v2) ^ fold(v3) ^ fold(v4) ^ fold(v5) ^ fold(v6) ^ fold(v7);
    acc += s;
    h = h * 1664525u + 1013904223u + (CHAIN ? s : 0u);
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// K = 1 with only the first ACT lanes active (exec-masked loads): does the data
// return scale with the active lanes?
template <int ACT>
__global__ void __launch_bounds__(kBlock) node_act(const float4* __restrict__ t, uint32_t zero, int iters,
                                                   uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  uint32_t h = wave * 0x9E3779B9u + 0x165667B1u;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const uint32_t n = ((h >> 9) & 12799u) | (lane & zero);
    if (lane < (uint32_t)ACT) {
      const float4* q = t + 8u * n;
      const float4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3], v4 = q[4], v5 = q[5], v6 = q[6], v7 = q[7];
      acc += fold(v0) ^ fold(v1) ^ fold(v2) ^ fold(v3) ^ fold(v4) ^ fold(v5) ^ fold(v6) ^ fold(v7);
    }
    h = h * 1664525u + 1013904223u;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// A node read from LDS (a 16 KiB table filled at kernel start), K distinct per
// wave: FLAT = 1 through a generic pointer that may point to LDS or global memory
// (flat_load_dwordx4: the render kernel's loads of LDS-resident top nodes and
// materials), FLAT = 0 as ds_read_b128.
template <int K, bool FLAT>
__global__ void __launch_bounds__(kBlock) node_lds(const float4* __restrict__ t, uint32_t zero, int iters,
                                                   uint32_t* out) {
  __shared__ float4 tab[128 * 8];
  for (uint32_t i = threadIdx.x; i < 128u * 8u; i += kBlock) tab[i] = t[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const uint32_t grp = (lane * (uint32_t)K) >> 6;
  uint32_t h = wave * 0x9E3779B9u + grp * 0x85EBCA6Bu + 0x165667B1u;
  const float4* base = (zero == 12345u) ? t : tab;  // generic: LDS at run time
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const uint32_t n = ((h >> 9) & 127u) | (lane & zero);
    const float4* q = FLAT ? base + 8u * n : tab + 8u * n;
    const float4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3], v4 = q[4], v5 = q[5], v6 = q[6], v7 = q[7];
    acc += fold(v0) ^ fold(v1) ^ fold(v2) ^ fold(v3) ^ fold(v4) ^ fold(v5) ^ fold(v6) ^ fold(v7);
    h = h * 1664525u + 1013904223u;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// a triangle record: 3 float4 (prims[3 * slot .. 3 * slot + 2]), 4 969 of them (the bunny)
template <int K>
__global__ void __launch_bounds__(kBlock) prim(const float4* __restrict__ t, uint32_t zero, int iters, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const uint32_t grp = (lane * (uint32_t)K) >> 6;
  uint32_t h = wave * 0x9E3779B9u + grp * 0x85EBCA6Bu + 0x165667B1u;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const uint32_t n = ((h >> 9) % 4969u) | (lane & zero);
    const float4* q = t + 3u * n;
    const float4 v0 = q[0], v1 = q[1], v2 = q[2];
    acc += fold(v0) ^ fold(v1) ^ fold(v2);
    h = h * 1664525u + 1013904223u;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// Spill-shaped: per wave 25 rows of 64 consecutive dwords.  The empty asm with a
// memory clobber keeps the compiler from forwarding the stored values to the
// reloads (they are issued as loads after the stores, as a spill's reload is).
constexpr int kRows = 25;
template <int MODE>
__global__ void __launch_bounds__(kBlock) lane_dwords(uint32_t* buf, int iters, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  uint32_t* w = buf + (size_t)wave * kRows * 64u + lane;
  uint32_t acc = lane;
  for (int i = 0; i < iters; ++i) {
    const uint32_t r0 = (uint32_t)(i * 8) % (kRows - 7);
    if (MODE != 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) w[(r0 + k) * 64u] = acc + k;
    }
    asm volatile("" ::: "memory");
    if (MODE != 1) {
      uint32_t s = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) s ^= w[(r0 + k) * 64u];
      acc += s;
    } else {
      acc = acc * 1664525u + 1013904223u;
    }
    asm volatile("" ::: "memory");
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

struct Case {
  const char* name;
  void (*launch)(int grid, int iters);
  int wps;       // waves per SIMD (blocks per CU = wps: 4 waves per block, one per SIMD)
  int iters;
  double loads;  // vector-memory wave-instructions per wave per iteration
  int chain;     // 1: a dependent hop per iteration (latency = time per iteration)
};

static float4* g_tab;
static uint32_t* g_buf;
static uint32_t* g_out;

#define NODE_CASE(K, TABLE, CHAIN, WPS)                                                                  \
  [](int grid, int iters) {                                                                              \
    hipLaunchKernelGGL((node<K, TABLE, CHAIN, WPS>), dim3(grid), dim3(kBlock), 0, 0, g_tab, 0u, iters, g_out); \
  }
#define ACT_CASE(A) \
  [](int grid, int iters) { hipLaunchKernelGGL((node_act<A>), dim3(grid), dim3(kBlock), 0, 0, g_tab, 0u, iters, g_out); }
#define LDS_CASE(K, F)                                                                                   \
  [](int grid, int iters) {                                                                              \
    hipLaunchKernelGGL((node_lds<K, F>), dim3(grid), dim3(kBlock), 0, 0, g_tab, 0u, iters, g_out);       \
  }
#define PRIM_CASE(K) \
  [](int grid, int iters) { hipLaunchKernelGGL((prim<K>), dim3(grid), dim3(kBlock), 0, 0, g_tab, 0u, iters, g_out); }
#define LANE_CASE(M) \
  [](int grid, int iters) { hipLaunchKernelGGL((lane_dwords<M>), dim3(grid), dim3(kBlock), 0, 0, g_buf, iters, g_out); }

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t tab_f4 = 12800u * 8u;
  CHK(hipMalloc(&g_tab, tab_f4 * sizeof(float4)));
  CHK(hipMemset(g_tab, 0, tab_f4 * sizeof(float4)));
  const size_t waves_max = (size_t)cus * 8 * 4;
  CHK(hipMalloc(&g_buf, waves_max * kRows * 64 * sizeof(uint32_t)));
  CHK(hipMemset(g_buf, 0, waves_max * kRows * 64 * sizeof(uint32_t)));
  CHK(hipMalloc(&g_out, (size_t)cus * 8 * sizeof(uint32_t)));

  const Case cases[] = {
      {"node_k1_l1", NODE_CASE(1, 128, false, 6), 6, 1000, 8, 0},
      {"node_k2_l1", NODE_CASE(2, 128, false, 6), 6, 1000, 8, 0},
      {"node_k4_l1", NODE_CASE(4, 128, false, 6), 6, 1000, 8, 0},
      {"node_k64_l1", NODE_CASE(64, 128, false, 6), 6, 250, 8, 0},
      {"node_k1_l2", NODE_CASE(1, 12800, false, 6), 6, 1000, 8, 0},
      {"node_k2_l2", NODE_CASE(2, 12800, false, 6), 6, 1000, 8, 0},
      {"node_k4_l2", NODE_CASE(4, 12800, false, 6), 6, 1000, 8, 0},
      {"node_k64_l2", NODE_CASE(64, 12800, false, 6), 6, 100, 8, 0},
      {"node_k8_l2", NODE_CASE(8, 12800, false, 6), 6, 1000, 8, 0},
      {"node_k16_l2", NODE_CASE(16, 12800, false, 6), 6, 500, 8, 0},
      {"node_k32_l2", NODE_CASE(32, 12800, false, 6), 6, 250, 8, 0},
      {"node_k1_l2_chain", NODE_CASE(1, 12800, true, 6), 6, 1000, 8, 1},
      {"node_k4_l2_chain", NODE_CASE(4, 12800, true, 6), 6, 1000, 8, 1},
      {"node_k1_l1_chain_w1", NODE_CASE(1, 128, true, 1), 1, 2000, 8, 1},
      {"node_k1_l2_chain_w1", NODE_CASE(1, 12800, true, 1), 1, 2000, 8, 1},
      {"node_act1", ACT_CASE(1), 6, 1000, 8, 0},
      {"node_act8", ACT_CASE(8), 6, 1000, 8, 0},
      {"node_act32", ACT_CASE(32), 6, 1000, 8, 0},
      {"node_lds_flat_k1", LDS_CASE(1, true), 6, 1000, 8, 0},
      {"node_lds_flat_k64", LDS_CASE(64, true), 6, 250, 8, 0},
      {"node_lds_ds_k1", LDS_CASE(1, false), 6, 1000, 8, 0},
      {"node_lds_ds_k64", LDS_CASE(64, false), 6, 250, 8, 0},
      {"prim_k1", PRIM_CASE(1), 6, 2000, 3, 0},
      {"prim_k4", PRIM_CASE(4), 6, 2000, 3, 0},
      {"prim_k64", PRIM_CASE(64), 6, 500, 3, 0},
      {"lane_dwords_store_reload", LANE_CASE(0), 6, 2000, 16, 0},
      {"lane_dwords_store", LANE_CASE(1), 6, 2000, 8, 0},
      {"lane_dwords_load", LANE_CASE(2), 6, 2000, 8, 0},
  };
  const int n = (int)(sizeof(cases) / sizeof(cases[0]));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  std::printf("{\n \"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d,\n \"shapes\": {\n", prop.gcnArchName, cus,
              prop.clockRate);
  for (int c = 0; c < n; ++c) {
    const Case& k = cases[c];
    const int grid = cus * k.wps;  // one block = 4 waves, one per SIMD
    k.launch(grid, k.iters);       // warm (the first of 6 dispatches; ubench_summary skips it)
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) k.launch(grid, k.iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipGetLastError());
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    const double waves = (double)grid * 4;
    const double insts = waves * k.iters * k.loads;
    const double cyc = ms * 1e-3 * 2.4e9;  // nominal clock; the PMC pass gives the real one
    std::printf("  \"%s\": {\"ms\": %.4f, \"waves_per_simd\": %d, \"vmem_wave_insts\": %.0f, "
                "\"cu_cycles_per_inst_2400\": %.3f, \"wave_cycles_per_iter_2400\": %.1f}%s\n",
                k.name, ms, k.wps, insts, cyc * cus / insts, cyc / k.iters, c + 1 < n ? "," : "");
  }
  std::printf(" }\n}\n");
  CHK(hipFree(g_tab));
  CHK(hipFree(g_buf));
  CHK(hipFree(g_out));
  return 0;
}
