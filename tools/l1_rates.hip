// l1_rates.hip -- what a vector-memory load costs the L1 path (TA/TD) on gfx950, by width, active lanes and
// address pattern. Measurement tool for DESIGN.md §4 (the C4 kernel is bound by the L1 address/data path):
// does a wave's load cost per active lane or per instruction, and per byte or per instruction?
//
// Every wave runs kIters iterations of 8 independent loads from a 16 KiB table (L1-resident) at addresses
// from a per-lane LCG; the results are folded into a register that is written once. Reported: shader-clock
// cycles per wave-load instruction per CU (event time x clock / loads per CU), for
//   width: 4, 8, 16 bytes per lane (global_load_dword / dwordx2 / dwordx4);
//   lanes: 64, 32, 16, 4 active (the others skip the loop body: exec-masked);
//   pattern: random (every lane its own 16-byte slot) or uniform (all lanes the same address).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

constexpr int kIters = 1024;
constexpr int kSlots = 1024;  // 16 KiB of 16-byte slots

template <int W, bool UNIFORM>
__device__ __forceinline__ uint32_t load(const uint4* tb, uint32_t i) {
  if constexpr (W == 4) return ((const uint32_t*)tb)[4 * i];
  if constexpr (W == 8) {
    const uint2 v = ((const uint2*)tb)[2 * i];
    return v.x ^ v.y;
  }
  const uint4 v = tb[i];
  return v.x ^ v.y ^ v.z ^ v.w;
}

template <int W, int LANES, bool UNIFORM>
__global__ __launch_bounds__(256) void k_l1(const uint4* tb, uint32_t* out, uint32_t seed) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t acc = 0;
  if (lane < (uint32_t)LANES) {
    uint32_t x = UNIFORM ? seed : seed * 2654435761u + threadIdx.x * 40503u + blockIdx.x * 977u;
#pragma unroll 1
    for (int it = 0; it < kIters; it++) {
      x = x * 1664525u + 1013904223u;
      const uint32_t i = (UNIFORM ? __builtin_amdgcn_readfirstlane(x) : x) >> 22;  // 10 bits: a slot
      // 8 loads from slots i, i + 129, ... (independent, distinct lines)
      acc ^= load<W, UNIFORM>(tb, i) ^ load<W, UNIFORM>(tb, (i + 129u) & (kSlots - 1)) ^
             load<W, UNIFORM>(tb, (i + 258u) & (kSlots - 1)) ^ load<W, UNIFORM>(tb, (i + 387u) & (kSlots - 1)) ^
             load<W, UNIFORM>(tb, (i + 516u) & (kSlots - 1)) ^ load<W, UNIFORM>(tb, (i + 645u) & (kSlots - 1)) ^
             load<W, UNIFORM>(tb, (i + 774u) & (kSlots - 1)) ^ load<W, UNIFORM>(tb, (i + 903u) & (kSlots - 1));
      x ^= acc & 1u;  // a dependence so the loop is not folded
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

struct Entry {
  const char* name;
  void (*k)(const uint4*, uint32_t*, uint32_t);
  int width, lanes;
  bool uniform;
};

int main() {
  const Entry es[] = {
      {"dwordx4 64 random", k_l1<16, 64, false>, 16, 64, false}, {"dwordx4 32 random", k_l1<16, 32, false>, 16, 32, false},
      {"dwordx4 16 random", k_l1<16, 16, false>, 16, 16, false}, {"dwordx4 4 random", k_l1<16, 4, false>, 16, 4, false},
      {"dwordx2 64 random", k_l1<8, 64, false>, 8, 64, false},   {"dwordx2 32 random", k_l1<8, 32, false>, 8, 32, false},
      {"dword 64 random", k_l1<4, 64, false>, 4, 64, false},     {"dword 32 random", k_l1<4, 32, false>, 4, 32, false},
      {"dwordx4 64 uniform", k_l1<16, 64, true>, 16, 64, true},  {"dword 64 uniform", k_l1<4, 64, true>, 4, 64, true},
  };
  int ncu = 0, clk_khz = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const int waves_per_simd = 8, blocks = ncu * waves_per_simd;
  uint4* tb;
  uint32_t* out;
  CHECK(hipMalloc(&tb, sizeof(uint4) * kSlots));
  CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
  std::vector<uint4> h(kSlots);
  for (int i = 0; i < kSlots; i++) h[i] = make_uint4(i, 3 * i, 5 * i, 7 * i);
  CHECK(hipMemcpy(tb, h.data(), sizeof(uint4) * kSlots, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"rows\": [", ncu, clk_khz / 1e3);
  for (size_t i = 0; i < sizeof(es) / sizeof(es[0]); i++) {
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(es[i].k, dim3(blocks), dim3(256), 0, 0, tb, out, 12345u);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    // wave-load instructions per CU: 4 SIMDs x 8 waves x kIters x 8
    const double loads_per_cu = 4.0 * waves_per_simd * kIters * 8;
    const double cycles = ms * 1e-3 * clk_khz * 1e3;  // at the nominal peak clock
    const double cpl = cycles / loads_per_cu;
    std::printf("%s{\"load\": \"%s\", \"bytes_per_lane\": %d, \"active_lanes\": %d, \"ms\": %.3f, "
                "\"cycles_per_wave_load_per_cu\": %.2f, \"active_bytes_per_cycle_per_cu\": %.1f}",
                i ? ", " : "", es[i].name, es[i].width, es[i].lanes, ms, cpl, es[i].width * es[i].lanes / cpl);
  }
  std::printf("], \"note\": \"cycles at the nominal clock (hipDeviceAttributeClockRate); 8 waves/SIMD; 16 KiB table\"}\n");
  CHECK(hipFree(tb));
  CHECK(hipFree(out));
  return 0;
}
