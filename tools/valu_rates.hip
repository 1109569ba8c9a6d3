// valu_rates -- issue cost of single VALU opcodes on gfx950 (MI355X), measured.
//
// Why: bench.py prices the fp64 headline kernel's VALU issue in SIMD cycles, weighting the fp64
// add/mul/fma/transcendental instructions (SQ_INSTS_VALU_*_F64) at 4 cycles per wave64 instruction and
// everything else at 2. The kernel also issues fp64 compares, min/max, conversions, 64-bit moves and
// 64-bit integer ops, whose costs no document gives. This program measures them: for every opcode a
// kernel runs 8 independent dependency chains of that one instruction (inline asm) in a loop, with
// 8 waves on every SIMD, and each wave reads the shader clock around its loop; cycles per wave64
// instruction per SIMD = wave cycles / (waves per SIMD x instructions per wave).
// Run under rocprofv3 --pmc as well to see how SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU /
// SQ_THREAD_CYCLES_VALU count each opcode (scripts/valu_rates.sh).
//   build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

constexpr int kIters = 2048;  // loop trips (~131k instructions per wave: launch costs vanish)
constexpr int kPerIter = 64;  // instructions per trip (8 chains x 8)

// one op on chain register r (double / uint64 pairs, float / uint32 singles)
#define OP8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

template <int K>
__device__ __forceinline__ void body(double& a0, double& a1, double& a2, double& a3, double& a4, double& a5,
                                     double& a6, double& a7, double b, double c, float fc, float& f0, float& f1, float& f2, float& f3,
                                     float& f4, float& f5, float& f6, float& f7, float fb, uint64_t& s0, uint64_t& s1,
                                     uint64_t& s2, uint64_t& s3, uint64_t& s4, uint64_t& s5, uint64_t& s6,
                                     uint64_t& s7, uint64_t m) {
#pragma unroll
  for (int rep = 0; rep < 8; rep++) {
    if constexpr (K == 0) {
#define X(r) asm volatile("v_add_f64 %0, %0, %1" : "+v"(r) : "v"(b));
      OP8(X)
#undef X
    } else if constexpr (K == 1) {
#define X(r) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r) : "v"(b));
      OP8(X)
#undef X
    } else if constexpr (K == 2) {
#define X(r) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
      OP8(X)
#undef X
    } else if constexpr (K == 3) {
#define X(r) asm volatile("v_max_f64 %0, %0, %1" : "+v"(r) : "v"(b));
      OP8(X)
#undef X
    } else if constexpr (K == 4) {
#define X(r) { uint64_t t; asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "=s"(t) : "v"(a##r), "v"(b)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 5) {
#define X(r) asm volatile("v_mov_b64 %0, %0" : "+v"(r));
      OP8(X)
#undef X
    } else if constexpr (K == 6) {
#define X(r) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f##r) : "v"(a##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 7) {
#define X(r) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 8) {
#define X(r) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 9) {
#define X(r) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "s"(m));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 10) {
#define X(r) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(r) : "v"(b));
      OP8(X)
#undef X
    } else if constexpr (K == 11) {
#define X(r) { uint64_t t; asm volatile("v_cmp_gt_u64_e64 %0, %1, %2" : "=s"(t) : "v"(a##r), "v"(b)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 12) {
#define X(r) asm volatile("v_rcp_f64 %0, %0" : "+v"(r));
      OP8(X)
#undef X
    } else if constexpr (K == 13) {
#define X(r) asm volatile("v_floor_f64 %0, %0" : "+v"(r));
      OP8(X)
#undef X
    } else if constexpr (K == 14) {
#define X(r) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a##r) : "v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 15) {
#define X(r) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 16) {
#define X(r) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(r) : "v"(fb));
      OP8(X)
#undef X
    } else if constexpr (K == 17) {
#define X(r) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(r));
      OP8(X)
#undef X
    } else if constexpr (K == 18) {
#define X(r) asm volatile("v_rsq_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 20) {
#define X(r) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
      OP8(X)
#undef X
    } else if constexpr (K == 21) {
#define X(r) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 22) {
#define X(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 23) {
#define X(r) asm volatile("v_mov_b32 %0, %1" : "=v"(f##r) : "v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 24) {
#define X(r) asm volatile("s_mov_b64 vcc, %2\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(f##r) : "v"(fb), "s"(m) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 25) {
#define X(r) { uint64_t t; asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(t) : "v"(f##r), "v"(fb)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 26) {
#define X(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 27) {
#define X(r) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 28) {
#define X(r) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 29) {
#define X(r) { uint64_t t; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a##r), "=s"(t) : "v"(f##r), "v"(fb), "v"(a##r)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 30) {
#define X(r) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 31) {
#define X(r) { uint32_t t; asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(t) : "v"(f##r)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 32) {
#define X(r) asm volatile("v_fract_f64 %0, %0" : "+v"(a##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 33) {
#define X(r) asm volatile("v_rsq_f64 %0, %0" : "+v"(a##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 34) {
#define X(r) asm volatile("v_sqrt_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 35) {
#define X(r) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 36) {
#define X(r) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 37) {
#define X(r) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a##r) : "v"(b));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 38) {
#define X(r) { uint64_t t; asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(t) : "v"(f##r), "v"(fb)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 39) {
#define X(r) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 40) {
#define X(r) { asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "s"(m)); }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 41) {
#define X(r) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 42) {
#define X(r) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "s"((uint32_t)0x07060100u));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 43) {
#define X(r) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 44) {
#define X(r) asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 45) {
#define X(r) asm volatile("v_min_u32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 46) {
#define X(r) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 47) {
#define X(r) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 48) {
#define X(r) asm volatile("v_lshl_add_u32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 49) {
#define X(r) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 50) {
#define X(r) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 51) {
#define X(r) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 52) {
#define X(r) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 53) {
#define X(r) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 54) {
#define X(r) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 55) {
#define X(r) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 56) {
#define X(r) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 57) {
#define X(r) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(f##r) : "v"(fb), "v"(fc));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 58) {
#define X(r) asm volatile("v_max_u32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 59) {
#define X(r) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 60) {
#define X(r) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 61) {
#define X(r) asm volatile("v_and_b32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 62) {
#define X(r) asm volatile("v_or_b32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 63) {
#define X(r) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 64) {
#define X(r) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 65) {
#define X(r) asm volatile("v_max_i32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 66) {
#define X(r) asm volatile("v_lshlrev_b32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 67) {
#define X(r) asm volatile("v_ashrrev_i32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 68) {
#define X(r) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 69) {
#define X(r) asm volatile("v_max_f32 %0, %0, %1" : "+v"(f##r) : "v"(fb));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 70) {
#define X(r) asm volatile("v_not_b32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 71) {
#define X(r) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 72) {
#define X(r) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 73) {
#define X(r) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 74) {
#define X(r) asm volatile("v_fract_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 75) {
#define X(r) asm volatile("v_floor_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 76) {
#define X(r) asm volatile("v_trunc_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 77) {
#define X(r) asm volatile("v_rndne_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 78) {
#define X(r) asm volatile("v_cvt_f16_f32 %0, %0" : "+v"(f##r));
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 79) {
#define X(r) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 80) {
#define X(r) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 81) {
#define X(r) asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 82) {
#define X(r) asm volatile("v_sub_co_u32_e32 %0, vcc, %0, %1" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 83) {
#define X(r) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 84) {
#define X(r) asm volatile("v_lshlrev_b16 %0, %0, %1" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 85) {
#define X(r) asm volatile("v_max_i16 %0, %0, %1" : "+v"(f##r) : "v"(fb) : "vcc");
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    } else if constexpr (K == 19) {
#define X(r) { uint64_t t; asm volatile("v_cmp_class_f64_e64 %0, %1, %2" : "=s"(t) : "v"(a##r), "v"(f0)); s##r ^= t; }
      X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#undef X
    }
  }
}

template <int K>
__global__ __launch_bounds__(256) void k_rate(double* out, unsigned long long* clk, double seed) {
  double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
         a7 = a0 + 7, b = seed * 0.5, c = seed * 0.25;
  float f0 = (float)a0, f1 = (float)a1, f2 = (float)a2, f3 = (float)a3, f4 = (float)a4, f5 = (float)a5,
        f6 = (float)a6, f7 = (float)a7, fb = (float)b, fc = (float)c;
  uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0, m = 0x5555555555555555ull;
  const unsigned long long t0 = clock64(), w0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < kIters; i++)
    body<K>(a0, a1, a2, a3, a4, a5, a6, a7, b, c, fc, f0, f1, f2, f3, f4, f5, f6, f7, fb, s0, s1, s2, s3, s4, s5, s6, s7, m);
  const unsigned long long t1 = clock64(), w1 = wall_clock64();
  if ((threadIdx.x & 63) == 0) {
    clk[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
    clk[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = w1 - w0;
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + f0 + f1 + f2 + f3 + f4 + f5 + f6 +
                                        f7 + (double)(s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7);
}

struct Entry {
  const char* name;
  void (*k)(double*, unsigned long long*, double);
};

int main() {
  const Entry es[] = {
      {"v_add_f64", k_rate<0>},        {"v_mul_f64", k_rate<1>},         {"v_fma_f64", k_rate<2>},
      {"v_max_f64", k_rate<3>},        {"v_cmp_lt_f64", k_rate<4>},      {"v_mov_b64", k_rate<5>},
      {"v_cvt_f32_f64", k_rate<6>},    {"v_add_f32", k_rate<7>},         {"v_fma_f32", k_rate<8>},
      {"v_cndmask_b32", k_rate<9>},    {"v_lshl_add_u64", k_rate<10>},   {"v_cmp_gt_u64", k_rate<11>},
      {"v_rcp_f64", k_rate<12>},       {"v_floor_f64", k_rate<13>},      {"v_cvt_f64_u32", k_rate<14>},
      {"v_mul_lo_u32", k_rate<15>},    {"v_ldexp_f64", k_rate<16>},      {"v_lshlrev_b64", k_rate<17>},
      {"v_rsq_f32", k_rate<18>},       {"v_cmp_class_f64", k_rate<19>},  {"v_pk_fma_f32", k_rate<20>},
      {"v_mul_f32", k_rate<21>},       {"v_xor_b32", k_rate<22>},
      {"v_mov_b32", k_rate<23>}, {"v_cndmask_b32_vcc", k_rate<24>}, {"v_cmp_lt_f32", k_rate<25>}, {"v_add_u32", k_rate<26>}, {"v_lshrrev_b32", k_rate<27>}, {"v_bfe_u32", k_rate<28>}, {"v_mad_u64_u32", k_rate<29>}, {"v_min_f32", k_rate<30>}, {"v_readfirstlane_b32", k_rate<31>}, {"v_fract_f64", k_rate<32>}, {"v_rsq_f64", k_rate<33>}, {"v_sqrt_f32", k_rate<34>}, {"v_mul_hi_u32", k_rate<35>}, {"v_cvt_f32_u32", k_rate<36>}, {"v_min_f64", k_rate<37>}, {"v_cmp_eq_u32", k_rate<38>}, {"v_bitop3_b32", k_rate<39>}, {"v_cndmask_b32_e64_v", k_rate<40>},
      {"v_fma_mix_f32", k_rate<41>}, {"v_perm_b32", k_rate<42>}, {"v_max3_f32", k_rate<43>}, {"v_cvt_f32_ubyte1", k_rate<44>},
      {"v_min_u32", k_rate<45>}, {"v_and_or_b32", k_rate<46>},
      {"v_add3_u32", k_rate<47>}, {"v_lshl_add_u32", k_rate<48>}, {"v_lshl_or_b32", k_rate<49>}, {"v_or3_b32", k_rate<50>},
      {"v_max3_u32", k_rate<51>}, {"v_min3_f32", k_rate<52>}, {"v_med3_f32", k_rate<53>}, {"v_mad_u32_u24", k_rate<54>},
      {"v_bfi_b32", k_rate<55>}, {"v_alignbit_b32", k_rate<56>}, {"v_xad_u32", k_rate<57>}, {"v_max_u32", k_rate<58>},
      {"v_mul_u32_u24", k_rate<59>}, {"v_sub_u32", k_rate<60>}, {"v_and_b32", k_rate<61>}, {"v_or_b32", k_rate<62>},
      {"v_ldexp_f32", k_rate<63>}, {"v_sub_f32", k_rate<64>}, {"v_max_i32", k_rate<65>}, {"v_lshlrev_b32", k_rate<66>},
      {"v_ashrrev_i32", k_rate<67>}, {"v_mul_hi_u32_u24", k_rate<68>}, {"v_max_f32", k_rate<69>}, {"v_not_b32", k_rate<70>},
      {"v_cvt_f32_f16", k_rate<71>}, {"v_cvt_u32_f32", k_rate<72>}, {"v_cvt_i32_f32", k_rate<73>}, {"v_fract_f32", k_rate<74>},
      {"v_floor_f32", k_rate<75>}, {"v_trunc_f32", k_rate<76>}, {"v_rndne_f32", k_rate<77>}, {"v_cvt_f16_f32", k_rate<78>},
      {"v_cndmask_b32_e32", k_rate<79>}, {"v_add_co_u32", k_rate<80>}, {"v_addc_co_u32", k_rate<81>}, {"v_sub_co_u32", k_rate<82>}, {"v_mul_i32_i24", k_rate<83>}, {"v_lshlrev_b16", k_rate<84>}, {"v_max_i16", k_rate<85>},
  };
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int waves_per_simd = 8, blocks = ncu * waves_per_simd;  // 256 lanes = one wave per SIMD per block
  double* out;
  unsigned long long* clk;
  CHECK(hipMalloc(&out, sizeof(double) * blocks * 256));
  CHECK(hipMalloc(&clk, sizeof(unsigned long long) * blocks * 8));
  std::vector<unsigned long long> h(blocks * 8);
  int wall_khz = 0;
  CHECK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("{\"cus\": %d, \"waves_per_simd\": %d, \"instr_per_wave\": %d, \"ops\": {", ncu, waves_per_simd,
              kIters * kPerIter);
  for (size_t i = 0; i < sizeof(es) / sizeof(es[0]); i++) {
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {  // the first launch warms up
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(es[i].k, dim3(blocks), dim3(256), 0, 0, out, clk, 1.25);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    double c = 0, w = 0;
    for (size_t j = 0; j < h.size(); j += 2) c += (double)h[j], w += (double)h[j + 1];
    c /= (double)(h.size() / 2);
    w /= (double)(h.size() / 2);
    const double instr = (double)waves_per_simd * kIters * kPerIter;  // per SIMD
    const double ghz = c / (w / (wall_khz * 1e3)) / 1e9;                // shader clock from clock64 / wall clock
    // cycles per wave64 instruction per SIMD: from the shader clock inside the loop, and from the
    // kernel's event time at that clock
    std::printf("%s\"%s\": {\"cycles\": %.3f, \"cycles_event\": %.3f, \"ghz\": %.3f}", i ? ", " : "", es[i].name,
                c / instr, ms * 1e-3 * ghz * 1e9 / instr, ghz);
  }
  std::printf("}, \"unit\": \"shader-clock cycles per wave64 instruction per SIMD (8 waves/SIMD, 8 chains); ghz = clock64 rate against wall_clock64\", \"wall_khz\": %d}\n", wall_khz);
  CHECK(hipFree(out));
  CHECK(hipFree(clk));
  return 0;
}
