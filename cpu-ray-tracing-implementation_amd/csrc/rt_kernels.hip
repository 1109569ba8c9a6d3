// rt_kernels.hip -- wavefront path tracer for MI355X (gfx950) + the C ABI of include/rt_hip.h.
//
// The reference's per-pixel/per-sample loop (camera.h:154-172) and recursive
// ray_color (camera.h:193-241) become P path slots. Default schedule (k_persist):
// one launch of as many lanes as the chip holds resident, each keeping its path in
// registers and pulling work items from per-XCD dequeue heads. Wavefront schedule (segments_per_launch = K > 0): the slots'
// state lives in HBM as structure-of-arrays (16-byte records per slot, coalesced
// dwordx4 access) between launches:
//
//   k_init    first camera ray of every slot            (camera.h:244-251)
//   repeat:
//     k_step    every live slot advances up to K segments: closest hit
//               (camera.h:198, world.hit), then emission + scatter + mixture
//               pdf (camera.h:199-240), or finish the sample and regenerate the
//               next camera ray of the slot's work item (pixel, chunk of samples)
//     every kBatch rounds: k_count/k_scan/k_compact build the live-slot queue
//     (wave __ballot + block prefix sums) once half the pool has drained
//   k_resolve  per-pixel mean over the chunks, in chunk order (camera.h:169-170)
//
// Work item = (pixel, chunk of C consecutive samples); a wavefront slot s owns items
// s, s + P, s + 2P, ... Each sample's random numbers are keyed by
// (seed, global pixel, sample) so the image is bit-identical for any pool size,
// tiling or GPU count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_device.h"
#include "scene_compile.h"

using namespace rtd;

namespace {

constexpr int kBlock = 256;
// RT_BG_BLACK_SKIP (retired in round 6, always on): shade: no unit-sphere test for a miss against a solid black
// background
// RT_BG_SOLID_FAST (retired in round 6, always on): shade: nor against another solid background when |d| < 500 (the
// test always hits)
#ifndef RT_LINEAR_WAVES
#define RT_LINEAR_WAVES 6
#endif
// RT_SPHERE_REFINE (retired in round 6, always on): fp32 sphere hits: point and normal from an fp64 re-solve (shade)
// RT_COLD_LDS (retired in round 6, always on): the volume linear program: the cold path state in LDS (Path, LC)
// RT_COLD_LDS_F64 (retired in round 6, always on): the same for the fp64 volume program (round 4)
// RT_LINEAR_NORAD (retired in round 6, always on): the volume programs: emission added straight into the item's running
// sum (Path NORAD)
// RT_F64_TAIL (retired in round 6, always on): 1: fp64 renders use the fp32 item layout (bulk + tail items); 0: uniform
// items of 16
#ifndef RT_PERSIST_MODE  // 2: dynamic (per-XCD heads), 1: static striding (development A/B)
#define RT_PERSIST_MODE 2
#endif
#ifndef RT_STACK_WAVES  // 4: the LDS limit of the LDS-node BVH kernel (32.8 KB per block); C3 151 -> 129 ms vs 3
#define RT_STACK_WAVES 4
#endif
#ifndef RT_LINEAR_WAVES_F64  // fp64 linear programs: waves per SIMD the register budget is cut for (C5 fp64:
#define RT_LINEAR_WAVES_F64 3   // none (2 waves) 3,605 ms/frame, 3: 2,865, 4: 3,885)
#endif
#ifndef RT_STACK_WAVES_F64  // fp64 binary BVH with its nodes in HBM (C4 fp64: none (2 waves) 2,019 ms/frame, 3: 1,964,
#define RT_STACK_WAVES_F64 4  // 4: 1,704); with the nodes in LDS (C3 fp64) none: 260 ms, 3: 295, 4: 276
#endif
#ifndef RT_LINEAR_VOL_WAVES  // fp32 quad + volume linear program (C5), with slab-tested box() volumes: 1 (4 waves at
                             // 128 VGPRs) 1661 ms/frame, 5: 1567, 6: 2594 (spills); round 4 (cold state in LDS,
#define RT_LINEAR_VOL_WAVES 6  // radiance folded, table sin/cos): 5: 1,326, 6: 1,247
#endif
// RT_LIN_LLI (retired in round 6, always on): the volume program for lambertian + isotropic + light scenes (shade LL,
// LLI): C5 fp32 1,189 -> 1,124 ms/frame, fp64 2,358 -> 2,262 (r05y)
// the LLI volume program's fp32 form at 7 waves per SIMD (72 VGPRs + 36 B spilled; 79 VGPRs at 6): 1,124 -> 1,097
// ms/frame (r05y). 8 waves (64 VGPRs + 60 B spilled) was 1.6 % faster (r05v2; r06a 1,070 against 1,094 ms) but its
// scratch -- 60 B for each of 8,192 waves' 64 lanes, 31 MB, about the L2s' size -- went to memory: 78.6 GB of writes
// per launch (r06a PMC) against 2.2 GB at 7 waves, where the partial sums are ~1.2 GB. Round 6 keeps 7.
#ifndef RT_LINEAR_VOL_WAVES_LLI
#define RT_LINEAR_VOL_WAVES_LLI 7
#endif
#ifndef RT_LINEAR_VOL_WAVES_F64  // the fp64 volume program (round 4, cold state in LDS): 3 waves 2,672 ms/frame, 4: 2,400
#define RT_LINEAR_VOL_WAVES_F64 4
#endif
constexpr int kBatch = 16;           // extend/shade rounds between live-slot counts
constexpr int kSegShards = 256;      // segment counter shards
constexpr uint32_t kAutoPool32 = 1u << 21;
constexpr uint32_t kAutoPool64 = 1u << 19;
constexpr uint32_t kAutoChunk = 16;
// The automatic item sizes (rt_render_params.samples_per_item = 0); RT_ITEM_* in the environment
// override them for A/B runs (scripts/dev_tail.py)
static uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? (uint32_t)std::strtoul(v, nullptr, 10) : dflt;
}
static double env_f64(const char* name, double dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::strtod(v, nullptr) : dflt;
}
// Bulk items: 8 samples (32 for the flat program, whose samples are cheap); at most
// kMaxItemsPerPixel items per pixel in all (both sizes doubled until they fit), so a high-spp frame
// (C5: 3840x2160 at 4096 spp) keeps its item count under 2^31 and its partial sums bounded.
// Measured (ms/frame, full frame / one rank of eight, scripts/dev_tail.sh): C3 16 samples 62.5 /
// 12.0, 8 with the last half in items of 4 61.2 / 8.9; C2 32 uniform 23.9 / 3.59, 32 with the last
// eighth in items of 8 23.6 / 3.47, with the last quarter 23.7-23.9 / 3.38 (the one-GPU frame, the
// headline, is kept).
constexpr uint32_t kMaxItemsPerPixel = 256;
// items a frame should have at least (render(); RT_ITEMS_TARGET overrides). C1 (400x400, 64 spp), ms/frame
// by target (item size): fp64 none (16) 0.918, 1 M (8) 0.792, 2.5 M (4) 0.735, 5 M (2) 0.710; fp32 none
// (32 + tail items of 8) 0.661, 1 M 0.589, 2.5 M 0.525, 5 M 0.536. The BASELINE configs from C2 up have
// 40 M items or more and keep their sizes.
constexpr uint32_t kItemsTarget = 4000000;
// item partial sums of one pass at most (render(): a call needing more renders its chunks in passes)
constexpr uint64_t kPartialBudget = 2ull << 30;
constexpr uint32_t kMinAutoChunk = 2;
static uint32_t auto_chunk(bool flat) {
  return std::max(1u, flat ? env_u32("RT_ITEM_CHUNK_FLAT", 2 * kAutoChunk) : env_u32("RT_ITEM_CHUNK", kAutoChunk / 2));
}
static uint32_t auto_tail_chunk(bool flat) {
  return std::max(1u, flat ? env_u32("RT_ITEM_TAIL_CHUNK_FLAT", 8) : env_u32("RT_ITEM_TAIL_CHUNK", 4));
}
static double auto_tail_frac(bool flat) {
  return std::min(1.0, std::max(0.0, flat ? env_f64("RT_ITEM_TAIL_FRAC_FLAT", 0.125) : env_f64("RT_ITEM_TAIL_FRAC", 0.5)));
}
constexpr int kAutoSegments = 16;  // segments each slot advances per k_step launch
// persistent schedule: upper bound of the grid's lanes. The dynamic schedule (persist 2) cuts the
// grid to what the chip holds resident; the static one (persist 1) launches them all (~10x the
// resident lanes: blocks that start late balance the uneven per-lane work)
constexpr uint32_t kAutoPersistLanes = 1u << 22;

// dynamic persistent schedule (persist 2): items are handed out in batches of kQBatch; batch j of
// head h is batch number j * kHeads + h of the item space, so the heads interleave over the whole
// frame and a head that runs dry steals from the others. Against static striding (persist 1) the
// tail shrinks to one item: C2 28.6 -> 26.5 ms on one GPU, 4.07 -> 3.70 ms for one rank of eight.
constexpr uint32_t kHeads = 8;
constexpr uint32_t kHeadStride = 64;  // 256 B apart: one L2 line per head
constexpr uint32_t kQBatch = 64;
constexpr uint32_t kNoItem = 0xFFFFFFFFu;

template <class R>
struct alignas(4 * sizeof(R)) R4 {
  R x, y, z, w;
};

// Path state in HBM, one entry per slot, structure of arrays of 16-byte (fp32)
// or 32-byte (fp64) records so every access is a coalesced dwordx4:
//   O  origin, ray time            D  direction, bounce (-1: slot retired)
//   T  throughput                  L  radiance of the running sample
//   A  running sum of the item     S  key_pixel, key of the running sample, item, sample
//   X  the surface the ray leaves (entry, instance): self-intersection exclusion;
//      the pixel (x | y << 16) and the end of the sample range of the slot's item
// utility.h:46-52 random_in_unit_disk by rejection; attempt k draws dimensions kDimDisk + 2k
// and + 2k + 1 (far above the per-bounce dimensions); the origin after kDiskTries failures
// (probability (1 - pi/4)^64 ~ 1e-43). Same as the oracle.
constexpr uint32_t kDimDisk = 0x7FFF0000u, kDiskTries = 64;

template <class R>
struct Params {
  DevScene<R> sc;
  R4<R>* O;
  R4<R>* D;
  R4<R>* T;
  R4<R>* L;
  R4<R>* A;
  uint4* S;
  uint4* X;
  R* partial;              // per item: 3 sums
  const uint32_t* pixmap;  // local pixel -> its image position x | y << 16
  const uint32_t* queue;   // live slots, or null = slots [0, n)
  uint32_t n;
  uint32_t P, npix, n_items, chunk, spp, first_sample, W;
  // two item sizes: chunks [0, k_bulk) hold `chunk` samples, the later ones (the frame's last
  // items in dequeue order) `tail_chunk` <= chunk samples each
  uint32_t k_bulk, tail_chunk;
  // the render's chunks come in passes (render(): the partial sums of one pass fit a memory budget): this
  // launch's items are chunks [chunk0, chunk0 + n_items / npix) of every pixel
  uint32_t chunk0;
  uint64_t npix_m;  // item / npix = (item * npix_m) >> npix_k for every item < 2^31 (div_magic)
  uint32_t npix_k;
  int32_t max_depth;
  uint64_t seed;
  // camera rays are built in fp64 for both paths (fp32 rounds once), from CamDev in device
  // memory (scalar loads at the point of use)
  int32_t cam_mode;
  const CamDev* camx;
  unsigned long long* seg_shards;
  int32_t K;  // segments per launch
  // persistent mode (k_persist): one launch. 1: lanes stride over the items by P; 2 (default):
  // the grid is what the chip holds resident and lanes pull items from the per-XCD heads
  int32_t persist;
  uint32_t* heads;  // kHeads dequeue counters, kHeadStride words apart (persist 2)
  uint64_t seg_cap;  // a lane never needs more segments than this (its items * chunk * max_depth)
  uint32_t* fault;   // set when a lane hits seg_cap (internal error, reported by the host)
};

// The per-lane words of the path state that only sample and item boundaries touch (LC paths,
// below), in LDS as [word][lane]: 32-bit words, then the fp64 pixel base as [component][lane].
constexpr int kColdWords = 8, kColdDoubles = 3;
__device__ __forceinline__ uint32_t* cold_words() {
  __shared__ uint32_t w[kColdWords * kBlock];
  return w + threadIdx.x;
}
__device__ __forceinline__ double* cold_doubles() {
  __shared__ double w[kColdDoubles * kBlock];
  return w + threadIdx.x;
}
// the throughput of an LT path ([component][lane])
template <class R>
__device__ __forceinline__ R* cold_thr() {
  __shared__ R w[3 * kBlock];
  return w + threadIdx.x;
}
// the fp64 item sum of an LC path ([component][lane]; fp32 keeps it in three of the cold words)
__device__ __forceinline__ __attribute__((unused)) double* cold_acc64() {
  __shared__ double w[3 * kBlock];
  return w + threadIdx.x;
}

// One path's state. The fields a segment reads stay in registers; the cold ones -- the item's
// running sum, its pixel and RNG key, the sample counter and range, the fp64 camera base -- are
// registers too unless LC, where they live in the lane's LDS words (cold_words) so the trace and
// shade code of the persistent loop gets their 14 VGPRs.
// LEAN: the pixel key, the end of the item's sample range and the camera base are not kept at all but
// recomputed where they are used (ka_of, send_of, begin_sample): 8 fewer registers for kernels whose
// traversal state competes with them (the wide BVH kernels), at a few integer and fp64 operations per
// sample.
// NORAD: no radiance register either (shade adds emission straight into the item's running sum).
// LT: the throughput in the lane's LDS words too (cold_thr; the fp32 LLI volume kernel, whose 72-VGPR budget
// otherwise spills it to scratch every segment)
template <class R, bool LC = false, bool LEAN = false, bool NORAD = LEAN, bool LT = false>
struct Path {
  static constexpr bool kLean = LEAN;
  static constexpr bool kNoRad = NORAD;
  V<R> o, d, thr_, rad;
  R tm;
  int32_t bounce;
  uint32_t ks;
  uint32_t xe;
  int32_t xi;
  // cold state (register copies: unused when LC)
  V<R> acc_;
  uint32_t ka_, item_, sample_, send_, xy_;
  V<double> cb_;  // (dir00 + x du) + y dv of the item's pixel (pixel_base)
#ifdef RT_ITEM_CLOCKS
  uint64_t t0_;  // development: wall clock at the item's start
#endif
  enum { kAcc = 0, kKa = 3, kItem, kSample, kSend, kXy };
  __device__ __forceinline__ V<R> thr() const {
    if constexpr (LT) return mkv(cold_thr<R>()[0], cold_thr<R>()[kBlock], cold_thr<R>()[2 * kBlock]);
    else return thr_;
  }
  __device__ __forceinline__ void set_thr(V<R> v) {
    if constexpr (LT) {
      cold_thr<R>()[0] = v.x;
      cold_thr<R>()[kBlock] = v.y;
      cold_thr<R>()[2 * kBlock] = v.z;
    } else {
      thr_ = v;
    }
  }
  __device__ __forceinline__ static uint32_t& w(int k) { return cold_words()[k * kBlock]; }
  __device__ __forceinline__ V<R> acc() const {
    if constexpr (LC && sizeof(R) == 8) {
      return mkv(cold_acc64()[0], cold_acc64()[kBlock], cold_acc64()[2 * kBlock]);
    } else if constexpr (LC) {
      return mkv(__uint_as_float(w(kAcc)), __uint_as_float(w(kAcc + 1)), __uint_as_float(w(kAcc + 2)));
    } else {
      return acc_;
    }
  }
  __device__ __forceinline__ void set_acc(V<R> v) {
    if constexpr (LC && sizeof(R) == 8) {
      cold_acc64()[0] = v.x;
      cold_acc64()[kBlock] = v.y;
      cold_acc64()[2 * kBlock] = v.z;
    } else if constexpr (LC) {
      w(kAcc) = __float_as_uint(v.x);
      w(kAcc + 1) = __float_as_uint(v.y);
      w(kAcc + 2) = __float_as_uint(v.z);
    } else {
      acc_ = v;
    }
  }
#define RT_COLD_U32(name, K)                                                        \
  __device__ __forceinline__ uint32_t name() const {                                \
    if constexpr (LC) return w(K); else return name##_;                             \
  }                                                                                 \
  __device__ __forceinline__ void set_##name(uint32_t v) {                          \
    if constexpr (LC) w(K) = v; else name##_ = v;                                   \
  }
  RT_COLD_U32(ka, kKa)
  RT_COLD_U32(item, kItem)
  RT_COLD_U32(sample, kSample)
  RT_COLD_U32(send, kSend)
  RT_COLD_U32(xy, kXy)
#undef RT_COLD_U32
  __device__ __forceinline__ V<double> cb() const {
    if constexpr (LC) return mkv(cold_doubles()[0], cold_doubles()[kBlock], cold_doubles()[2 * kBlock]);
    else return cb_;
  }
  __device__ __forceinline__ void set_cb(V<double> v) {
    if constexpr (LC) {
      cold_doubles()[0] = v.x;
      cold_doubles()[kBlock] = v.y;
      cold_doubles()[2 * kBlock] = v.z;
    } else {
      cb_ = v;
    }
  }
};
static_assert(Path<float>::kXy < kColdWords, "cold words");

// The pixel's part of the perspective camera ray, (dir00 + x du) + y dv (camera.h:246-250): the
// same for every sample of a work item, so it is computed once per item (and once per k_step
// launch), not once per sample. Same operations in the same order: bit-identical.
template <class R, class PS>
__device__ __forceinline__ void pixel_base(const Params<R>& p, PS& s, uint32_t xy) {
  if constexpr (!PS::kLean) {
    const double x = double(xy & 0xFFFFu), y = double(xy >> 16);
    s.set_cb((ld_here(&p.camx->dir00) + x * ld_here(&p.camx->du)) + y * ld_here(&p.camx->dv));
  }
}

template <class R>
__device__ __forceinline__ void load_path(const Params<R>& p, uint32_t slot, R4<R> Dv, Path<R>& s) {
  R4<R> Ov = p.O[slot], Tv = p.T[slot], Lv = p.L[slot], Av = p.A[slot];
  uint4 S = p.S[slot];
  uint4 X = p.X[slot];
  s.o = mkv(Ov.x, Ov.y, Ov.z);
  s.tm = Ov.w;
  s.d = mkv(Dv.x, Dv.y, Dv.z);
  s.bounce = (int32_t)Dv.w;
  s.set_thr(mkv(Tv.x, Tv.y, Tv.z));
  s.rad = mkv(Lv.x, Lv.y, Lv.z);
  s.set_acc(mkv(Av.x, Av.y, Av.z));
  s.set_ka(S.x);
  s.ks = S.y;
  s.set_item(S.z);
  s.set_sample(S.w);
  s.xe = X.x;
  s.xi = (int32_t)X.y;
  s.set_xy(X.z);
  s.set_send(X.w);
  pixel_base(p, s, X.z);
}

template <class R>
__device__ __forceinline__ void store_path(const Params<R>& p, uint32_t slot, const Path<R>& s) {
  p.D[slot] = {s.d.x, s.d.y, s.d.z, R(s.bounce)};
  if (s.bounce < 0) return;
  p.O[slot] = {s.o.x, s.o.y, s.o.z, s.tm};
  const V<R> thr = s.thr();
  p.T[slot] = {thr.x, thr.y, thr.z, R(0)};
  p.L[slot] = {s.rad.x, s.rad.y, s.rad.z, R(0)};
  const V<R> acc = s.acc();
  p.A[slot] = {acc.x, acc.y, acc.z, R(0)};
  p.S[slot] = make_uint4(s.ka(), s.ks, s.item(), s.sample());
  p.X[slot] = make_uint4(s.xe, (uint32_t)s.xi, s.xy(), s.send());
}

// The wave's local queue [next, end) of the dynamic schedule, in LDS (two words per wave).
__device__ __forceinline__ uint32_t* wave_queue() {
  __shared__ uint32_t wq[2 * (kBlock / 64)];
  return wq + 2 * (threadIdx.x >> 6);
}

// A batch of kQBatch items for the calling lane's wave: the block's own head first (blocks b and
// b + 8 share an XCD, so a head's counter stays in one XCD's traffic), then the others. Returns the
// first item, or kNoItem once every head has run past the item space.
// (Round 6 measured two ways of shortening the frame's end at one rank of eight, C2 fp64: the last 1-4 x the
// grid's lanes of items handed out in batches of 8 instead of 64 -- 0.856 / 0.855 / 0.854 / 0.856 of linear
// at 8 emulated ranks for 0 / 1 / 2 / 4 x; batches of 1, 0.699 -- and a third item tier, the last 1/64 - 1/16 of
// every pixel's samples in items of 1-4, 0.858 - 0.868 against 0.860 - 0.862, within the spread, and +8 B of
// spill in the C5 fp32 kernel (r06a, r06b; profiles/r06b_ab_summary.txt). Neither is kept.)
__device__ __forceinline__ uint32_t grab_batch(uint32_t* heads, uint32_t n_items) {
  const uint32_t g = blockIdx.x & (kHeads - 1);
  for (uint32_t t = 0; t < kHeads; t++) {
    const uint32_t h = (g + t) & (kHeads - 1);
    const uint32_t j = atomicAdd(heads + h * kHeadStride, 1u);
    const uint64_t first = ((uint64_t)j * kHeads + h) * kQBatch;
    if (first < n_items) return (uint32_t)first;
  }
  return kNoItem;
}

// The next item of each calling lane (the lanes of the wave that finished an item in this
// call, in divergent code): consecutive items from the wave's queue, refilled one batch at a
// time by the lowest calling lane. Every value below is identical in the calling lanes.
// kNoItem: the frame is exhausted and the lane retires (queue state [kNoItem, kNoItem)).
template <class R>
__device__ __forceinline__ uint32_t next_item_dyn(const Params<R>& p) {
  uint32_t* wq = wave_queue();
  const uint64_t need = __ballot(1);
  const uint32_t lane = __lane_id();
  const uint32_t k = (uint32_t)__popcll(need);
  const uint32_t r = (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
  const uint32_t leader = (uint32_t)__ffsll((unsigned long long)need) - 1;
  uint32_t qn = __hip_atomic_load(wq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  uint32_t qe = __hip_atomic_load(wq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  uint32_t item = kNoItem, off = 0;
  for (;;) {
    const uint32_t rem = qe - qn;
    if (r >= off && r - off < rem) item = qn + (r - off);
    const uint32_t take = min(rem, k - off);
    qn += take;
    off += take;
    if (off >= k || qe == kNoItem) break;  // served, or the wave already found every head dry
    uint32_t b = kNoItem;
    if (lane == leader) b = grab_batch(p.heads, p.n_items);
    b = __shfl(b, (int)leader);
    if (b == kNoItem) {  // remember it: a dry scan stalls the wave for kHeads atomics
      qn = qe = kNoItem;
      break;
    }
    qn = b;
    qe = min(b + kQBatch, p.n_items);
  }
  if (lane == leader) {
    __hip_atomic_store(wq, qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_store(wq + 1, qe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  return item;
}

// An item's first sample and the end of its sample range: bulk items of p.chunk samples, then tail
// items of p.tail_chunk (the item layout, render()). `lchunk`: the item's chunk within this pass (item =
// lchunk * npix + the pixel's index); the layout is decided by the frame's chunk, lchunk + chunk0.
template <class R>
__device__ __forceinline__ void item_range(const Params<R>& p, uint32_t item, uint32_t& lchunk, uint32_t& first,
                                           uint32_t& end) {
  lchunk = (uint32_t)(((uint64_t)item * p.npix_m) >> p.npix_k);
  const uint32_t chunk = lchunk + p.chunk0;
  // fp64 items are uniform (the host never gives them a tail): compiled out, the select costs
  // the fp64 Cornell kernel 10 VGPRs, 3 -> 2 waves per SIMD (C2 f64 5.22 -> 4.08 Gsamples/s)
  const bool bulk = chunk < p.k_bulk;
  first = bulk ? chunk * p.chunk : p.k_bulk * p.chunk + (chunk - p.k_bulk) * p.tail_chunk;
  end = min(first + (bulk ? p.chunk : p.tail_chunk), p.spp);
}
// the pixel's RNG key and the end of the item's samples: kept, or (LEAN) recomputed
template <class R, class PS>
__device__ __forceinline__ uint32_t ka_of(const Params<R>& p, const PS& s) {
  if constexpr (PS::kLean) {
    const uint32_t xy = s.xy();
    return key_pixel(p.seed, (xy >> 16) * p.W + (xy & 0xFFFFu));
  } else {
    return s.ka();
  }
}
template <class R, class PS>
__device__ __forceinline__ uint32_t send_of(const Params<R>& p, const PS& s) {
  if constexpr (PS::kLean) {
    uint32_t chunk, first, end;
    item_range(p, s.item(), chunk, first, end);
    return end;
  } else {
    return s.send();
  }
}

// A new work item for the slot: its pixel and that pixel's RNG key.
#ifdef RT_ITEM_CLOCKS
// development build (scripts/dev_item_clocks.py): each item's duration in wall-clock ticks (100 MHz), by item
__device__ uint32_t* g_item_clk;
#endif
template <class R, class PS>
__device__ __forceinline__ void begin_item(const Params<R>& p, PS& s, uint32_t item) {
#ifdef RT_ITEM_CLOCKS
  s.t0_ = wall_clock64();
#endif
  uint32_t lchunk, first, end;
  item_range(p, item, lchunk, first, end);
  const uint32_t xy = p.pixmap[item - lchunk * p.npix];
  s.set_item(item);
  s.set_sample(first);
  s.set_xy(xy);
  if constexpr (!PS::kLean) {
    s.set_send(end);
    s.set_ka(key_pixel(p.seed, (xy >> 16) * p.W + (xy & 0xFFFFu)));
  }
  pixel_base(p, s, xy);
}

// camera::generate_ray for the orthonormal, fisheye and lens models (camera.h:252-290), reading
// its fields from device memory. Only the CAMX kernel instantiations contain it, so the
// perspective kernels' registers are not shaped by it.
RT_EXT_FN void camera_ray(const CamDev* cp, uint32_t ks, uint32_t x, uint32_t y, double ox,
                                        double oy, V<double>& o, V<double>& d, double& tm) {
  const int32_t mode = ld_uniform(&cp->mode, 0);
  const V<double> du = ld_uniform(&cp->du, 0), dv = ld_uniform(&cp->dv, 0);
  o = ld_uniform(&cp->pos, 0);
  if (mode == RT_CAM_ORTHONORMAL) {  // camera.h:252-258
    const V<double> q = (ld_uniform(&cp->pos00, 0) + double(x) * du) + double(y) * dv;
    o = (q + ox * du) + oy * dv;
    d = ld_uniform(&cp->dir, 0);
    tm = to_unit<double>(draw_u32(ks, 2));
  } else if (mode == RT_CAM_LENS) {  // camera.h:276-283, 287-290
    d = ((((ld_uniform(&cp->pos00, 0) + double(x) * du) + double(y) * dv) + ox * du) + oy * dv) +
        ld_uniform(&cp->fdir, 0);
    double px = 0, py = 0;
    for (uint32_t k = 0; k < kDiskTries; k++) {
      const double ax = -1 + 2 * to_unit<double>(draw_u32(ks, kDimDisk + 2 * k));
      const double ay = -1 + 2 * to_unit<double>(draw_u32(ks, kDimDisk + 2 * k + 1));
      if (ax * ax + ay * ay + 0.0 * 0.0 < 1) {
        px = ax;
        py = ay;
        break;
      }
    }
    o = o + (px * ld_uniform(&cp->disk_u, 0) + py * ld_uniform(&cp->disk_v, 0));
    d = d - o;
    tm = 0;  // ray(origin, direction): time 0, no draw
  } else {  // fisheye (camera.h:259-275)
    const V<double> dir = ld_uniform(&cp->dir, 0);
    d = ((ld_uniform(&cp->dir00, 0) + double(x) * du) + double(y) * dv + ox * du) + oy * dv;
    const V<double> w = d - dir;
    const double r = sqrt(w.x * w.x + w.y * w.y + w.z * w.z);
    const double theta = asin(r / ld_uniform(&cp->focal, 0));
    const V<double> v1 = unit(dir), v2 = unit(d);
    const double st = sin(theta);
    const double b = sqrt(st * st / (1 - dot(v1, v2) * dot(v1, v2)));
    const double a = cos(theta) - b * dot(v1, v2);
    d = a * v1 + b * v2;
    tm = to_unit<double>(draw_u32(ks, 2));
  }
}

// camera::generate_ray, perspective mode (camera.h:244-251,293): sample s.sample of the slot's pixel
template <class R, bool CAMX, class PS>
__device__ __forceinline__ void begin_sample(const Params<R>& p, PS& s) {
  s.ks = key_path(ka_of(p, s), key_sample(p.seed, p.first_sample + s.sample()));
  // In fp64 for both paths: fp32 gets the correctly rounded ray, a few ulp less error on every
  // camera ray, which otherwise shows up as paths crossing a checker line or edge differently.
  const double ox = to_unit<double>(draw_u32(s.ks, 0)) - 0.5;  // sample_square (camera.h:293)
  const double oy = to_unit<double>(draw_u32(s.ks, 1)) - 0.5;
  V<double> o = ld_here(&p.camx->pos), d;
  double tm;
  if (!CAMX || p.cam_mode == RT_CAM_PERSPECTIVE) {  // camera.h:245-251
    const V<double> du = ld_here(&p.camx->du), dv = ld_here(&p.camx->dv);
    if constexpr (!PS::kLean) {
      d = (s.cb() + ox * du) + oy * dv;
    } else {  // the same operations in the same order as pixel_base + the above: bit-identical
      const uint32_t xy = s.xy(), x = xy & 0xFFFFu, y = xy >> 16;
      d = ((ld_here(&p.camx->dir00) + double(x) * du) + double(y) * dv + ox * du) + oy * dv;
    }
    tm = to_unit<double>(draw_u32(s.ks, 2));
  } else if constexpr (CAMX) {
    const uint32_t xy = s.xy();
    camera_ray(p.camx, s.ks, xy & 0xFFFFu, xy >> 16, ox, oy, o, d, tm);
  }
  s.o = mkv(R(o.x), R(o.y), R(o.z));
  s.d = mkv(R(d.x), R(d.y), R(d.z));
  s.tm = R(tm);
  s.bounce = 0;
  s.set_thr(mkv(R(1), R(1), R(1)));
  if constexpr (!PS::kNoRad) s.rad = mkv(R(0), R(0), R(0));
  s.xe = kNoHit;
  s.xi = -1;
}


template <class R, bool CAMX>
__global__ __launch_bounds__(kBlock) void k_init(Params<R> p) {
  uint32_t slot = blockIdx.x * kBlock + threadIdx.x;
  if (slot >= p.P) return;
  Path<R> s;
  s.set_acc(mkv(R(0), R(0), R(0)));
  if (slot >= p.n_items) {
    s.d = mkv(R(0), R(0), R(0));
    s.bounce = -1;
  } else {
    begin_item(p, s, slot);
    begin_sample<R, CAMX>(p, s);
  }
  store_path(p, slot, s);
}

// camera::ray_color for one segment (camera.h:193-241), iteratively: given the
// closest hit (t, e, inst) of s's ray, add emission, scatter (or finish the
// sample and regenerate the slot's next camera ray). Returns false once the slot
// has no work left.
// FLAT: the hit comes from the flat program (trace_flat): a quad whose outward normal (+-e_A)
// and material are packed in nm, so no primitive or instance record is read.
// MOVING = false: the kernel's scene has no moving sphere (the wide kernels without WK_MOVING), so the
// ray time is not read here. A LEAN path has no radiance register: emission goes straight into the
// item's running sum (the same terms, added one by one instead of per sample: a rounding-level
// regrouping of the pixel's sum).
// MLDS: `mats` is the kernel's LDS copy of the materials (FlatTrav tables), read with ds_read (a generic
// pointer that may be LDS or global compiled to flat loads, which wait on both counters).
// LL ("lambertian + light", round 5): the scene's materials are lambertian and diffuse_light with solid
// textures (the background's too), and the light an axis-aligned quad (the Cornell configs; host-checked,
// launch_step): the material is one LDS record lm[mat] = (colour, is_light), and the texture, metal,
// dielectric, gloss, isotropic and no-light code is compiled out.
// NL ("no light", round 5): the materials are lambertian, metal and dielectric (solid and checker textures)
// and there is no importance-sampling light (RTOW, C3; host-checked): the emission, gloss, isotropic and
// light-mixture code is compiled out.
// LLI (with LL): isotropic phase materials too (the lm record's w is 2; C5's smoke volumes)
template <class R, bool CAMX, bool FLAT = false, bool MOVING = true, bool MLDS = false, bool LL = false,
          bool NL = false, bool LLI = false, class PS>
__device__ bool shade(const Params<R>& p, PS& s, R t, uint32_t e, int32_t inst, uint32_t nm = 0,
                      const Material<R>* mats = nullptr, const R4<R>* lm = nullptr) {
  const DevScene<R>& sc = p.sc;
  constexpr bool kMixSel = RT_MIX_SELECT == 2 || (RT_MIX_SELECT == 1 && FLAT);
  V<R> add = mkv(R(0), R(0), R(0));
  bool has_add = false, done = false;
  V<R> new_o = s.o, new_d = s.d;
  const V<R> o = s.o, d = s.d;

  if (e == kNoHit) {  // camera::miss (camera.h:180-190)
#ifdef RT_DEBUG_TRACE
    printf("[dev] bounce %d o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) miss\n", s.bounce, (double)o.x, (double)o.y,
           (double)o.z, (double)d.x, (double)d.y, (double)d.z);
#endif
    // a solid black background (the Cornell configs' solid_color::black) adds thr * 0: the unit-sphere test
    // that decides whether it is sampled (camera.h:183-187) is skipped (a wave-uniform test of the record)
    const Texture<R>* bgt = sc.background >= 0 ? sc.texs + sc.background : nullptr;
    const bool bg_black = bgt != nullptr && ld_here(&bgt->kind) == T_SOLID &&
                          ld_here(&bgt->c0[0]) == R(0) && ld_here(&bgt->c0[1]) == R(0) && ld_here(&bgt->c0[2]) == R(0);
    // any other solid background: the unit sphere about the ray's origin has the root t = 1/|d|, inside
    // [0.001, inf) for |d| < 1000, and a solid colour does not depend on where it is hit -- so for |d| < 500
    // the colour is added without the test (RT_BG_SOLID_FAST; RTOW's sky, C3)
    // (0 < |d|^2: a zero direction has a = 0 in sphere.h:48-62, a NaN root and no hit -- nothing is added)
    const R dd2 = dot(d, d);
    const bool bg_solid = bgt != nullptr && !bg_black && ld_here(&bgt->kind) == T_SOLID &&
                          dd2 < R(250000) && dd2 > R(0);
    if (bg_solid) {
      add = s.thr() * mkv(ld_here(&bgt->c0[0]), ld_here(&bgt->c0[1]), ld_here(&bgt->c0[2]));
      has_add = true;
    } else if (sc.background >= 0 && !bg_black) {
      R tb;
      if (sphere_roots<R>(o.x, o.y, o.z, d.x, d.y, d.z, o.x, o.y, o.z, R(1), R(0.001), Num<R>::inf(), false, tb)) {
        double bu = 0, bv = 0;
        if constexpr (CAMX) sphere_uv(tb * d, bu, bv);  // the unit sphere about the origin (camera.h:184-187)
        add = s.thr() * tex_sample<R, CAMX>(sc, sc.texs[sc.background], o + tb * d, bu, bv);
        has_add = true;
      }
    }
    done = true;
  } else {
    uint32_t ty = etype(e), idx = epay(e);
    V<R> pw, n;
    bool front;
    int32_t mat;
    double hu = 0, hv = 0;  // hit_record u, v (EXT kernels: picture textures); 0 where the reference leaves them stale
    bool unit_n = true;  // false: a moving sphere's normal, (p - 0) / r (sphere.h:69), is not a unit vector
    [[maybe_unused]] uint32_t fA = 0;  // FLAT: n = fs e_fA
    [[maybe_unused]] R fs = R(1);
    if constexpr (FLAT) {  // quad.h:47-50 with n = +-e_A (translate leaves it alone, hittable.h:75-82)
      // outward = sg e_A (sg = -1 when bit 31 is set); hit_record::set_face_normal (hittable.h:26-29):
      // dot(d, outward) < 0 is exactly sg d_A < 0, and n = front ? outward : -outward, whose zero
      // components are -0 on a back face, as the negation gives them
      const uint32_t A = (nm >> 28) & 3u;
      const bool neg = (nm >> 31) != 0;
      const R dA = A == 0 ? d.x : (A == 1 ? d.y : d.z);
      mat = (int32_t)(nm & kNmMat);
      pw = o + t * d;
      front = neg ? dA > R(0) : dA < R(0);
      fA = A;
      fs = front != neg ? R(1) : R(-1);
      const R z = front ? R(0) : -R(0);
      n = mkv(A == 0 ? fs : z, A == 1 ? fs : z, A == 2 ? fs : z);
    } else if (ty == E_VOLUME) {  // volumne.h:40-44
      pw = o + t * d;
      n = mkv(R(1), R(0), R(0));
      front = true;
      mat = sc.vols[idx].phase_mat;
    } else {
      V<R> oo = o, dd = d;
      const Instance<R>* in = nullptr;
      if (inst >= 0) in = &sc.insts[inst];
      // fp32, planar primitives: instances are rigid, so the hit is o + t d in world space and
      // only the object-space normal needs rotating out (fp64 keeps the reference's
      // object-space point, hittable.h:75-82, 125-149)
      const bool world_space = sizeof(R) == 4 && ty != E_SPHERE && !CAMX;
      if (in && !world_space) chain_in(*in, oo, dd);
      V<R> po = oo + t * dd;
      V<R> outward;
      if (ty == E_QUAD) {
        const Quad<R>& q = sc.quads[idx];
        outward = ld3(q.n);
        mat = q.mat;
        if constexpr (CAMX) {  // quad.h:47-62: u, v = alpha, beta
          const V<R> rel = po - ld3(q.q);
          hu = (double)dot(rel, ld3(q.a));
          hv = (double)dot(rel, ld3(q.b));
        }
      } else if (ty == E_SPHERE) {  // sphere.h:69 (center_ member; (0,0,0) for moving spheres)
        const Sphere<R>& sp = sc.spheres[idx];
        unit_n = !MOVING || !sp.moving;
        if constexpr (sizeof(R) == 8) {
          outward = (po - ld3(sp.cn)) / sp.r;
        } else {
          // The hit refined in fp64 from the fp32 ray: one Newton step on the quadratic
          // g(t) = a t^2 + 2 b t + c from the fp32 root (which is ~1e-7 relative off: ~1e-6 along
          // the ray for t ~ 10, tilting a small sphere's normal by ~1e-5 -- enough for a chain of
          // mirror / glass bounces to leave the fp64 path a few times per million segments),
          // then the point and normal (sphere.h:67-69) from the refined root. A step that does
          // not land near the fp32 root (a grazing double root) keeps it.
          double cx = sp.c1[0], cy = sp.c1[1], cz = sp.c1[2];  // sphere.h:83 (a static sphere: dc = 0)
          if (!unit_n) {
            cx += (double)s.tm * sp.dc[0];
            cy += (double)s.tm * sp.dc[1];
            cz += (double)s.tm * sp.dc[2];
          }
          // g(t0) = |o + t0 d - c|^2 - r^2 needs fp64 (it cancels); the step g / g' is tiny next
          // to t0, so g' = 2 d.(o + t0 d - c) and the quotient are fp32
          const double ox = oo.x, oy = oo.y, oz = oo.z, dx = dd.x, dy = dd.y, dz = dd.z, t0 = t, rr = sp.r;
          const double qx = (ox + t0 * dx) - cx, qy = (oy + t0 * dy) - cy, qz = (oz + t0 * dz) - cz;
          const double g = (qx * qx + qy * qy + qz * qz) - rr * rr;
          const float gp = 2.0f * ((float)qx * dd.x + (float)qy * dd.y + (float)qz * dd.z);
          float step = fdiv((float)g, gp);
          if (!(fabsf(step) <= 1e-4f * fabsf(t))) step = 0.0f;
          const double td = t0 - (double)step;
          const double px = ox + td * dx, py = oy + td * dy, pz = oz + td * dz;
          po = mkv((float)px, (float)py, (float)pz);
          outward = mkv((float)(px - sp.cn[0]), (float)(py - sp.cn[1]), (float)(pz - sp.cn[2])) * fdiv(R(1), sp.r);
          // big spheres (the RTOW ground, r = 1000) in particular: o + t*d in fp32 is off the surface
          // by ~1e-7 absolute, enough to flip the sign of y near the top of the ground (y = 0 under the
          // glass sphere) and with it the checker parity (texture.h:51-55)
        }
        mat = sp.mat;
        if constexpr (CAMX) sphere_uv(outward, hu, hv);  // sphere.h:70
      } else {
        const Tri<R>& tr = sc.tris[idx];
        outward = ld3(tr.n);
        mat = tr.mat;
      }
      if (world_space) {
        if (in)
          for (int q = in->nops - 1; q >= 0; q--) outward = op_out(in->op[q], outward, false);
        front = dot(dd, outward) < R(0);  // hit_record::set_face_normal (hittable.h:26-29)
        n = front ? outward : -outward;
        pw = po;
      } else {
        front = dot(dd, outward) < R(0);  // hit_record::set_face_normal (hittable.h:26-29)
        n = front ? outward : -outward;
        pw = po;
        if (in) {
          for (int q = in->nops - 1; q >= 0; q--) {
            pw = op_out(in->op[q], pw, true);
            n = op_out(in->op[q], n, false);
          }
        }
      }
    }
#ifdef RT_DEBUG_TRACE  // development build (scripts/dev_sample_trace.py): one line per segment
    printf("[dev] bounce %d o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) t=%.9g p=(%.9g %.9g %.9g) n=(%.9g %.9g %.9g) "
           "front=%d mat=%d ty=%u idx=%u\n", s.bounce, (double)o.x, (double)o.y, (double)o.z, (double)d.x, (double)d.y,
           (double)d.z, (double)t, (double)pw.x, (double)pw.y, (double)pw.z, (double)n.x, (double)n.y, (double)n.z,
           (int)front, sc.mats[mat].kind, ty, idx);
#endif
    using LMat = const __attribute__((address_space(3))) Material<R>;
    using LRec = const __attribute__((address_space(3))) R4<R>;
    const Material<R>& m = MLDS ? *(const Material<R>*)((LMat*)mats + mat) : sc.mats[mat];
    V<R> col{};
    bool is_light;
    [[maybe_unused]] bool ll_iso = false;
    if constexpr (LL) {
      LRec* mc = (LRec*)lm + mat;
      col = mkv(mc->x, mc->y, mc->z);
      const R w = mc->w;
      is_light = w == R(1);
      if constexpr (LLI) ll_iso = w == R(2);
    } else {
      is_light = !NL && m.kind == M_DIFFUSE_LIGHT;
    }
    if (is_light) {  // material.h:211-215; no scatter
      if (front) {
        add = s.thr() * (LL ? col : tex_sample<R, CAMX>(sc, m.tx, pw, hu, hv));
        has_add = true;
      }
      done = true;
    } else {
      V<R> att = LL ? col : tex_sample<R, CAMX>(sc, m.tx, pw, hu, hv);
      const uint32_t bounce = (uint32_t)s.bounce;
      uint32_t js = 0;
      auto U = [&]() { return to_unit<R>(draw_u32(s.ks, dim_scatter(bounce, js++))); };
      // NL (lambertian / metal / dielectric, no light): the scatter draws are pure functions of (path key,
      // dimension), and lambertian's cosine sample and metal's fuzz sample each need sin/cos(2 pi u) of one of the
      // first two draws -- so both draws and one sincos are computed by every lane before the material branches,
      // which then hold no trigonometry (the same operations on the same values: bit-identical)
      [[maybe_unused]] R nl_u1 = R(0), nl_u2 = R(0), nl_sp = R(0), nl_cp = R(0);
      constexpr bool kNlTrig = NL;  // C3 fp32 48.16 -> 47.60 ms/frame, fp64 64.70 -> 64.09 (r06b)
      if constexpr (kNlTrig) {
        nl_u1 = to_unit<R>(draw_u32(s.ks, dim_scatter(bounce, 0)));
        nl_u2 = to_unit<R>(draw_u32(s.ks, dim_scatter(bounce, 1)));
        sincos2pi(m.kind == M_METAL ? nl_u2 : nl_u1, nl_sp, nl_cp);  // on_sphere: phi = 2 pi u2; cosine: 2 pi u1
      }
      if (!LL && m.kind == M_METAL) {  // material.h:85-92
        V<R> dir = unit(reflect(d, n));
        if constexpr (kNlTrig) {
          new_d = dir + m.fuzz * unit(on_sphere_sc(nl_u1, nl_sp, nl_cp));
        } else {
          R u1 = U();
          R u2 = U();
          new_d = dir + m.fuzz * unit(on_sphere(u1, u2));
        }
        s.set_thr(s.thr() * att);
      } else if (!LL && m.kind == M_DIELECTRIC) {  // material.h:113-131
        R ri = front ? fdiv(R(1), m.refr) : m.refr;
        V<R> ud = unit(d);
        R cos_t = fmin(dot(-ud, n), R(1));
        R sin_t = fsqrt(R(1) - cos_t * cos_t);
        bool cant = ri * sin_t > R(1);
        R r0 = fdiv(R(1) - ri, R(1) + ri);
        r0 = r0 * r0;
        if (cant || (r0 + (R(1) - r0) * pow5(R(1) - cos_t)) > (kNlTrig ? nl_u1 : U()))
          new_d = reflect(ud, n);
        else
          new_d = refract(ud, n, ri);
        s.set_thr(s.thr() * att);
      } else if (!LL && !NL && m.kind == M_GLOSS && to_unit<R>(draw_u32(s.ks, dim_scatter(bounce, js))) <= m.spec) {
        // gloss, specular branch (material.h:158-167): kDetermined, attenuation 1,
        // direction unit(lerp(smoothness, cosine-hemisphere sample about n, reflect(d_in, n)))
        js++;
        const Onb<R> b = FLAT ? make_onb_axis(n) : make_onb(n);
        const R r1 = U();
        const R r2 = U();
        const V<R> diffuse = onb_transform(b, cosine_dir(r1, r2));
        const R tt = m.smooth;
        new_d = unit((R(1) - tt) * diffuse + tt * reflect(d, n));
      } else {  // lambertian (material.h:62-72) / isotropic (material.h:193-200) / gloss diffuse: kRandom
        if (!LL && !NL && m.kind == M_GLOSS) js++;  // the specular-choice draw above (material.h:161)
        const bool iso = LL ? (LLI && ll_iso) : (!NL && m.kind == M_ISOTROPIC);
        const R iso_pdf = R(1) / (R(4) * Num<R>::pi());
        Onb<R> b;
        if (!FLAT && !iso) b = make_onb(n);
        // FLAT: n = fs e_A, so make_onb_axis(n) is a signed permutation (b.y = n; A = 0: b.x = -e_z,
        // b.z = -fs e_y; A = 1, 2: b.x = -e_x, b.z = -fs e_z / fs e_y) and onb_transform(b, v) is
        // exact: (fs v.y, -fs v.z, -v.x), (-v.x, fs v.y, -fs v.z), (-v.x, fs v.z, fs v.y) -- the same
        // values without the cross products and the nine multiply-adds (signed zeros aside, which no
        // later test can tell apart); dot(u, n) is fs u_A
        auto cos_dir = [&](R u1, R u2) -> V<R> {
          const V<R> v = cosine_dir(u1, u2);
          if constexpr (FLAT) {
            const R sy = fs * v.y, sz = fs * v.z;
            return fA == 0 ? mkv(sy, -sz, -v.x) : (fA == 1 ? mkv(-v.x, sy, -sz) : mkv(-v.x, sz, sy));
          } else {
            return onb_transform(b, v);
          }
        };
        auto cos_n = [&](V<R> u) -> R {  // dot(u, n) (onb.h's w = n)
          if constexpr (FLAT) return fs * (fA == 0 ? u.x : (fA == 1 ? u.y : u.z));
          return dot(u, b.y);
        };
        const Light<R>* Lt = sc.light;  // read at the point of use (light_pdf, light_random)
        R pv = R(1);
        V<R> dir;
        // no light (camera.h:217-226): the direction is drawn from the material's own pdf, the one
        // p_scattered returns (cosine for lambertian, material.h:62-80; uniform for isotropic,
        // material.h:193-205), so (attenuation * p_scattered) / pdf_value is the attenuation: the two
        // pdfs (equal up to rounding) are not evaluated (C3 fp32 52.49 -> 52.17 ms/frame, fp64 75.8 ->
        // 73.0). Not for a moving sphere: p_scattered takes the cosine against its non-unit normal,
        // the pdf against the unit one, and the ratio |n| is the reference's (quirk kept)
        bool own_pdf = false;
        if (NL || (!LL && ld_here(&Lt->kind) == L_NONE)) {
          if constexpr (kNlTrig) {  // NL has no isotropic material
            dir = onb_transform(b, cosine_dir_sc(nl_u2, nl_sp, nl_cp));
          } else {
            R u1 = U();
            R u2 = U();
            dir = iso ? unit(on_sphere(u1, u2)) : cos_dir(u1, u2);
          }
          own_pdf = iso || unit_n;
          if (!own_pdf) pv = fmax(R(0), div_pi(cos_n(unit(dir))));
        } else {  // dual_pdf(hittable_pdf(light), material pdf) (camera.h:227-239, pdf.h:48-61)
          R c = U();
          R u1 = U();
          R u2 = U();
          const bool from_light = c < R(0.5);
          if constexpr (kMixSel) {  // both generators for every lane, one select (no divergent branch)
            const V<R> dl = light_random(Lt, pw, u1, u2);
            const V<R> dc = iso ? unit(on_sphere(u1, u2)) : cos_dir(u1, u2);
            dir = from_light ? dl : dc;
          } else if (from_light) {
            dir = light_random(Lt, pw, u1, u2);
          } else if constexpr (LLI) {  // (C5 fp64 2,200 -> 2,185 ms/frame, fp32 1,094 -> 1,091, r06c)
            // the isotropic (on_sphere: phi = 2 pi u2) and lambertian (cosine: phi = 2 pi u1) lanes share one sincos
            R sp, cp;
            sincos2pi(iso ? u2 : u1, sp, cp);
            dir = iso ? unit(on_sphere_sc(u1, sp, cp)) : onb_transform(b, cosine_dir_sc(u2, sp, cp));
          } else {
            dir = iso ? unit(on_sphere(u1, u2)) : cos_dir(u1, u2);
          }
          R mp = iso ? iso_pdf : fmax(R(0), div_pi(cos_n(unit(dir))));
          pv = R(0.5) * light_pdf<R, kMixSel>(Lt, pw, dir, from_light) + R(0.5) * mp;
        }
        if (own_pdf) {
          s.set_thr(s.thr() * att);
        } else {
          R ps;
          if (iso) {
            ps = iso_pdf;
          } else {
            R c = FLAT ? cos_n(unit(dir)) : dot(n, unit(dir));
            ps = c < R(0) ? R(0) : div_pi(c);
          }
          if constexpr (sizeof(R) == 8)
            s.set_thr(s.thr() * ((att * ps) / pv));  // camera.h:238 grouping on the parity path
          else  // a zero mixture pdf (the reference's 0/0 = NaN) ends the path
            s.set_thr(pv > R(0) ? s.thr() * (att * fdiv(ps, pv)) : mkv(R(0), R(0), R(0)));
        }
        new_d = dir;
      }
      new_o = pw;
      if (s.bounce + 1 >= p.max_depth) done = true;  // ray_color(.., 0) returns 0 (camera.h:194)
      {
        const V<R> thr = s.thr();
        if (thr.x == R(0) && thr.y == R(0) && thr.z == R(0)) done = true;
      }
    }
  }
  if (has_add) {
    if constexpr (PS::kNoRad)
      s.set_acc(s.acc() + add);
    else
      s.rad = s.rad + add;
  }
  if (!done) {
    s.o = new_o;
    s.d = new_d;
    s.bounce += 1;
    s.xe = e;
    s.xi = inst;
    return true;
  }
  // the sample is finished (camera.h:167): add it to the item's running sum
  RT_WIDE_STAT(8);
  V<R> acc = s.acc();
  if constexpr (!PS::kNoRad) acc = acc + s.rad;
  const uint32_t sample = s.sample() + 1;
  s.set_sample(sample);
  if (sample < send_of(p, s)) {
    s.set_acc(acc);
  } else {
    const uint32_t item = s.item();
#ifdef RT_ITEM_CLOCKS
    if (g_item_clk) g_item_clk[item] = (uint32_t)(wall_clock64() - s.t0_);
#endif
    R* dst = p.partial + 3ull * item;
    dst[0] = acc.x;
    dst[1] = acc.y;
    dst[2] = acc.z;
    s.set_acc(mkv(R(0), R(0), R(0)));
    const uint32_t nx = p.persist == 2 ? next_item_dyn(p) : (item + p.P < p.n_items ? item + p.P : kNoItem);
    if (nx == kNoItem) {
      s.bounce = -1;
      return false;
    }
    begin_item(p, s, nx);
  }
  // (round 5: regenerating the finished lanes of a wave in batches -- a lane waiting idle until 16 or 32 of
  // its wave's lanes had finished -- was slower, C2 fp64 28.33 -> 28.46 / 29.95 ms/frame, r05e: the lanes a
  // wait idles in trace and shade cost more than the regeneration's 41 % lane use)
  begin_sample<R, CAMX>(p, s);
  return true;
}

// ------------------------------------------------------------------ the fused wavefront step
// Each launch advances every live slot by up to K segments: closest hit
// (extend, camera.h:198), then shade. Traversal: the wave-uniform linear
// program (small scenes) or the BVH stack machine with a per-lane LDS stack.
// LLI: a lambertian + isotropic + light scene (shade LL, LLI; C5's Cornell box with smoke volumes)
template <class R, bool SPH, bool TRI, bool VOL, bool LLI = false>
struct LinearTrav {
  static constexpr bool kLL = LLI;
  static constexpr bool kLinLL = LLI;
  static constexpr uint32_t kLdsMats = 16;
  static constexpr int kStack = 0;
  // waves per SIMD the register budget is cut for (occupancy hides the shading loads); the
  // lean quad-only program fits 96 VGPRs with a small spill, the others would spill heavily
  static constexpr int kWaves = sizeof(R) != 4 ? (VOL ? RT_LINEAR_VOL_WAVES_F64 : RT_LINEAR_WAVES_F64)
                                 : (!SPH && !TRI && !VOL) ? RT_LINEAR_WAVES
                                 : (!SPH && !TRI && VOL)  ? (LLI ? RT_LINEAR_VOL_WAVES_LLI : RT_LINEAR_VOL_WAVES)
                                                          : 1;
  static constexpr int kLdsNodes = 0;
  static constexpr bool kFlat = false;
  static constexpr bool kWide = false;
  // the volume program's registers (C5: 23 -> 6 VGPRs spilled at 96, 1563 -> 1498 ms/frame)
  static constexpr bool kTablesLds = false;
  static constexpr bool kLean = false;  // (LLI lean: 7 waves 1,094 -> 1,117 ms/frame; 8 waves 48 B spilled, r06a)
  static constexpr bool kNoRad = VOL;
  static constexpr bool kColdLds = VOL;
  static constexpr bool kThrLds = VOL && LLI && sizeof(R) == 4;  // (Path LT: C5 fp32 1,091 -> 1,072 ms/frame, r06d)
  template <class PS>
  __device__ __forceinline__ static void run(const DevScene<R>& sc, const Node<R>*, const PS& s, Keys k,
                                             uint32_t*, R& t, uint32_t& e, int32_t& i, uint32_t&) {
    trace_linear<R, SPH, TRI, VOL>(sc, s.o, s.d, s.tm, s.xe, s.xi, k, (uint32_t)s.bounce, t, e, i);
  }
};
// The flat program (quad/box scenes such as every Cornell config): rt_device.h trace_flat.
#ifndef RT_FLAT_WAVES
#define RT_FLAT_WAVES 8
#endif
// RT_F64_COLD_LDS (retired in round 6, always on): fp64 flat program: the cold path state (item sum, pixel, keys,
// camera base) in LDS
// RT_FLAT_LDS (retired in round 6, always on): flat program (persistent kernels): records and materials copied into LDS
#ifndef RT_FLAT_WAVES_F64_LL  // the same for the lambertian + light kernel
#define RT_FLAT_WAVES_F64_LL 7  // C2 fp64: 5 waves 28.90 ms/frame, 6: 28.08 (r05c; the general kernel at 5: 31.28);
                                // 7 (72 VGPRs + 32 B spilled, from 80): 27.94 -> 27.79 (r05w7); 8 does not fit
#endif
// RT_FLAT_LL (retired in round 6, always on): flat program: a kernel for lambertian + light scenes (shade LL)
// RT_FLAT_NORAD (retired in round 6, always on): flat program: emission added straight into the item's running sum
// (Path NORAD)
#ifndef RT_FLAT_WAVES_F64  // fp64 flat program: waves per SIMD the register budget is cut for (1: none)
#define RT_FLAT_WAVES_F64 5
#endif
template <class R, bool TLDS = false, bool LL = false>
struct FlatTrav {
  static constexpr bool kLinLL = false;
  static constexpr bool kTablesLds = TLDS;  // persistent kernel: Tables in LDS (fill, run_lds)
  static constexpr bool kLL = LL;           // lambertian + light scene (shade LL; the lm table)
  static constexpr int kStack = 0;
  static constexpr int kWaves = sizeof(R) == 4 ? RT_FLAT_WAVES : (LL ? RT_FLAT_WAVES_F64_LL : RT_FLAT_WAVES_F64);
  static constexpr int kLdsNodes = 0;
  static constexpr bool kFlat = true;
  static constexpr bool kWide = false;
  // fp32: 72 -> 64 VGPRs, but C2 23.5 -> 24.1 ms/frame; fp64: see RT_F64_COLD_LDS
  static constexpr bool kLean = false;
  static constexpr bool kNoRad = true;  // 6 VGPRs in fp64 (its item sum is in LDS)
  static constexpr bool kColdLds = sizeof(R) == 8;
  static constexpr bool kThrLds = false;
  template <class PS>
  __device__ __forceinline__ static void run(const DevScene<R>& sc, const Node<R>*, const PS& s, Keys, uint32_t*,
                                             R& t, uint32_t& e, int32_t& i, uint32_t& nm) {
    trace_flat<R>(sc, s.o, s.d, s.xe, s.xi, t, e, i, nm, sc.flatq, sc.flatb);
  }
  // the scene's small tables copied into LDS (persistent kernel, RT_FLAT_LDS): the hit's record and
  // material are then LDS reads instead of dependent global loads
  // (the LL kernel's tables are smaller, so a 256-lane block's LDS -- tables plus the fp64 cold path state,
  // ~27 KB with the general sizes -- leaves room for 6 blocks per CU)
  static constexpr uint32_t kLdsQuads = LL ? 16 : 64, kLdsBoxes = LL ? 8 : 16, kLdsMats = LL ? 16 : 32;
  struct Tables {
    FlatQuadT<R> q[kLdsQuads];
    FlatBoxT<R> b[kLdsBoxes];
    Material<R> m[LL ? 1 : kLdsMats];
    R4<R> lm[LL ? kLdsMats : 1];  // LL: (solid colour, 1 for diffuse_light)
  };
  __host__ __device__ __forceinline__ static bool tables_fit(const DevScene<R>& sc) {
    return sc.n_flatq[0] + sc.n_flatq[1] + sc.n_flatq[2] <= kLdsQuads && sc.n_flatb <= kLdsBoxes &&
           sc.n_mats <= kLdsMats;
  }
  __device__ __forceinline__ static void fill(const DevScene<R>& sc, Tables& tb) {
    const uint32_t nq = sc.n_flatq[0] + sc.n_flatq[1] + sc.n_flatq[2];
    for (uint32_t j = threadIdx.x; j < nq; j += kBlock) tb.q[j] = sc.flatq[j];
    for (uint32_t j = threadIdx.x; j < sc.n_flatb; j += kBlock) tb.b[j] = sc.flatb[j];
    for (uint32_t j = threadIdx.x; j < sc.n_mats; j += kBlock) {
      if constexpr (LL) {
        const Material<R>& m = sc.mats[j];
        tb.lm[j] = R4<R>{m.tx.c0[0], m.tx.c0[1], m.tx.c0[2], m.kind == M_DIFFUSE_LIGHT ? R(1) : R(0)};
      } else {
        tb.m[j] = sc.mats[j];
      }
    }
  }
  template <class PS>
  __device__ __forceinline__ static void run_lds(const DevScene<R>& sc, const Tables& tb, const PS& s, R& t,
                                                 uint32_t& e, int32_t& i, uint32_t& nm) {
    trace_flat<R>(sc, s.o, s.d, s.xe, s.xi, t, e, i, nm, tb.q, tb.b);
  }
};
// LDSN: the scene's BVH nodes (at most kLdsNodeMax) are copied into LDS at kernel start, so
// every traversal step reads LDS instead of waiting on the memory hierarchy (RTOW: 117 nodes)
constexpr uint32_t kLdsNodeMax = 256;
template <class R, int STACK, bool LDSN = false>
struct StackTrav {
  static constexpr bool kLL = false, kLinLL = false;
  static constexpr int kStack = STACK;
  static constexpr int kLdsNodes = LDSN ? (int)kLdsNodeMax : 0;
  static constexpr int kWaves = sizeof(R) == 4 ? RT_STACK_WAVES : (LDSN ? 1 : RT_STACK_WAVES_F64);  // occupancy over a small spill
  static constexpr bool kFlat = false;
  static constexpr bool kWide = false;
  static constexpr bool kTablesLds = false;
  static constexpr bool kLean = false;
  static constexpr bool kNoRad = false;
  static constexpr bool kColdLds = false;  // its LDS holds the traversal stacks
  static constexpr bool kThrLds = false;
  template <class PS>
  __device__ __forceinline__ static void run(const DevScene<R>& sc, const Node<R>* nodes, const PS& s, Keys k,
                                             uint32_t* stk, R& t, uint32_t& e, int32_t& i, uint32_t&) {
    trace<R, STACK, kBlock>(sc, LDSN ? nodes : sc.nodes, s.o, s.d, s.tm, s.xe, s.xi, k, (uint32_t)s.bounce, s.xy(),
                            stk, t, e, i);
  }
};

// The wide BVH (fp32, rt_device.h trace_wide). LDSN: the whole tree -- nodes and primitive
// words -- is copied into the block's dynamic LDS at kernel start; the per-lane stack follows it
// ([depth][lane], conflict-free). Otherwise nodes and primitives are read from global memory and
// only the stack is in LDS. Dynamic LDS is sized from the compiled scene (wide_lds_bytes).
#ifndef RT_WIDE_WAVES  // LDS-resident tree (C3: 4 waves 93.6 ms, 5: 86.2, 6: 83.0; with leaves of 6 spheres the
#define RT_WIDE_WAVES 7  // block needs ~21 KB, so 7 fit a CU: 64.0 -> 62.2 despite 22 spilled VGPRs; 8: 67.8)
#endif
#ifndef RT_WIDE_WAVES_GLOBAL  // tree in HBM, 32-bit stack in LDS (C4 stand-in: 4 waves 519 ms, 5: 462; with the
// speculative traversal 5: 424, 6: 412.5 -- 7 blocks of 24 KB stacks do not fit the 160 KB LDS)
#define RT_WIDE_WAVES_GLOBAL 8  // round 5, with 12 LDS stack entries and 55 top nodes in LDS (wide_lds_stack)
#endif
// RT_WIDE_TRIQUAD (retired in round 6, always on): a kernel for triangle + quad scenes (else the all-kinds kernel): C4
// 358.9 -> 353.8 ms
// RT_PARAM_RELOAD (retired in round 6, always on): flat / linear / binary-BVH loops: parameters reloaded per segment
// RT_WIDE_RELOAD (retired in round 6, always on): round 4 (lean state): C3 fp32 51.9 -> 51.1 ms/frame, fp64 71.3 ->
// 70.7, C4 neutral
#ifndef RT_SHADE_BATCH  // < 64: a wave stops traversing to shade once this many of its lanes have finished
#define RT_SHADE_BATCH 48  // (LDS-resident tree, C3 fp32 ms/frame: never 57.06, 48: 52.57, 52: 52.58, 56: 52.81, 60: 53.57; fp64 81.3 -> 75.8)
#endif
#ifndef RT_SHADE_BATCH_GLOBAL  // the same for trees in HBM (speculative traversal): C4 stand-in 413.6 ms/frame
#define RT_SHADE_BATCH_GLOBAL 48  // never pausing, 415.2 / 370.8 / 363.8 / 362.5 / 368.4 / 379.6 at 16/32/40/48/56/60
#endif
#ifndef RT_WIDE_WAVES_F64  // fp64 rays over the wide tree (round 3), tree in LDS (C3 fp64, ms/frame: 2 or 3 waves
#define RT_WIDE_WAVES_F64 4  // 99, 4 waves 90.2)
#endif
#ifndef RT_WIDE_WAVES_GLOBAL_F64  // tree in HBM (C4 fp64: 3 waves 599.8, 4: 555.0, 5: 567.3)
#define RT_WIDE_WAVES_GLOBAL_F64 4
#endif
#ifndef RT_WIDE_WAVES_GLOBAL_F64_LL  // the LL form (116 VGPRs at 4 waves): C4 fp64 at 4 waves 522.4 ms/frame, 5: 490.6
#define RT_WIDE_WAVES_GLOBAL_F64_LL 5  // (r05g; the general kernel at 4: 526.7)
#endif
#ifndef RT_WIDE_WAVES_F64_NL  // the NL form over an LDS tree, fp64 (116 VGPRs at 4 waves)
#define RT_WIDE_WAVES_F64_NL 5  // C3 fp64 at 4 waves 69.07 ms/frame, 5: 65.41 (r05q; the general kernel at 4: 70.23)
#endif
// RT_WIDE_NL (retired in round 6, always on): a wide kernel for sphere scenes without a light (shade NL)
// RT_WIDE_LL (retired in round 6, always on): a wide kernel for lambertian + light triangle/quad scenes (shade LL)
// RT_WIDE_LEAN (retired in round 6, always on): the wide kernels keep the lean path state (Path LEAN)
// LL: a lambertian + light scene (shade LL; the material table `Lm` in static LDS)
template <class R, bool SPH, bool TRI, bool QUAD, bool MOV, bool LDSN, bool LL = false, bool NL = false>
struct WideTrav {
  static constexpr bool kLL = LL;
  static constexpr bool kLinLL = false;
  static constexpr bool kNL = NL;  // no light (shade NL)
  static constexpr uint32_t kLdsMats = 16;
  static constexpr int kStack = 0;
  static constexpr int kLdsNodes = 0;
  static constexpr int kWaves = sizeof(R) == 4 ? (LDSN ? RT_WIDE_WAVES : RT_WIDE_WAVES_GLOBAL)
                                               : (LDSN ? (NL ? RT_WIDE_WAVES_F64_NL : RT_WIDE_WAVES_F64)
                                                       : (LL ? RT_WIDE_WAVES_GLOBAL_F64_LL : RT_WIDE_WAVES_GLOBAL_F64));
  static constexpr bool kFlat = false;
  static constexpr bool kWide = true;
  static constexpr bool kColdLds = false;  // its LDS holds the tree and the stacks
  // (Path LT) the fp64 LL kernel over a tree in HBM (C4): its throughput in LDS, 6 KB a block, for which its LDS stack
  // keeps 18 entries instead of 24: 339.2 -> 331.8 ms/frame, writes 16.4 -> 9.4 GB per launch (r06d). The fp64 NL
  // kernel over an LDS tree (C3) lost with it: 63.55 -> 68.08 ms/frame
  static constexpr bool kThrLds = sizeof(R) == 8 && !LDSN && LL;
  static constexpr bool kTablesLds = false;
  static constexpr bool kLean = true;  // registers for the traversal (fewer spills)
  static constexpr bool kNoRad = true;
  static constexpr bool kMoving = MOV;
  using StackT = WStackT<LDSN>;
  using WW = typename WWord<R>::T;
  // LDS layout: [nodes, kWNodeLdsStride each][primitive words][stack: entries x kBlock of StackT]
  __host__ __device__ static uint32_t stack_offset(uint32_t n_wnodes, uint32_t n_words) {
    return LDSN ? n_wnodes * kWNodeLdsStride + n_words * (uint32_t)sizeof(WW) : 0u;
  }
  // a tree in HBM, fp32 rays (RT_WIDE_TOP): [stack][the first wide_top nodes, WNode layout]
  static constexpr bool kTop = !LDSN && sizeof(R) == 4;
  static constexpr bool kTopH = !LDSN && sizeof(R) == 8;
  __host__ __device__ static uint32_t top_offset(uint32_t wide_stack) {
    return (wide_stack < wide_lds_stack<R>() ? wide_stack : wide_lds_stack<R>()) * kBlock * 4u;
  }
  __host__ __device__ static uint32_t root(const DevScene<R>& sc) {
    return LDSN ? wide_code16(sc.wroot) : sc.wroot;
  }
  __device__ __forceinline__ static StackT* fill(const DevScene<R>& sc, uint4* lds) {
    unsigned char* base = (unsigned char*)lds;
    if constexpr (LDSN) {
      const uint4* gn = (const uint4*)sc.wnodes;  // 8 words of 16 B per node, the last one padding
      for (uint32_t j = threadIdx.x; j < sc.n_wnodes * 7u; j += kBlock) {
        const uint32_t nd = j / 7u, f = j - nd * 7u;
        uint4 v = gn[nd * 8u + f];
        if (f == 6)  // four 16-bit codes in the first 8 bytes (trace_wide)
          v = make_uint4(wide_code16(v.x) | wide_code16(v.y) << 16, wide_code16(v.z) | wide_code16(v.w) << 16, 0u, 0u);
        *(uint4*)(base + nd * kWNodeLdsStride + f * 16u) = v;
      }
      uint4* pw = (uint4*)(base + sc.n_wnodes * kWNodeLdsStride);
      const uint4* gp = (const uint4*)sc.wprims;
      const uint32_t n16 = sc.n_wprim_words * (uint32_t)(sizeof(WW) / 16);
      for (uint32_t j = threadIdx.x; j < n16; j += kBlock) pw[j] = gp[j];
      __syncthreads();
    }
    if constexpr (kTop) {
      uint4* dst = (uint4*)(base + top_offset(sc.wide_stack));
      const uint4* gn = (const uint4*)sc.wnodes;
      const uint32_t ntop = min(sc.wide_top, (uint32_t)RT_WIDE_TOP_N);
      constexpr uint32_t kRows = kWTopStride / 16u;  // 7: the pad row of WNode is not copied
      for (uint32_t j = threadIdx.x; j < ntop * kRows; j += kBlock) {
        const uint32_t nd = j / kRows, r = j - nd * kRows;
        dst[j] = gn[nd * 8u + r];
      }
      __syncthreads();
    } else if constexpr (kTopH) {  // fp64 rays: the fp16 form, 5 words per node
      uint4* dst = (uint4*)(base + top_offset(sc.wide_stack));
      const uint4* gn = (const uint4*)sc.wnodesh;
      const uint32_t ntop = min(sc.wide_top, (uint32_t)RT_WIDE_TOP_N_F64);
      for (uint32_t j = threadIdx.x; j < ntop * 5u; j += kBlock) dst[j] = gn[j];
      __syncthreads();
    }
    return (StackT*)(base + stack_offset(sc.n_wnodes, sc.n_wprim_words));
  }
  // Advance the ray of s (false: paused, see trace_wide)
  template <class PS>
  __device__ __forceinline__ static bool steps(const DevScene<R>& sc, const Node<R>* lds, const PS& s, StackT* stk,
                                               WideRayT<R>& ry) {
    const unsigned char* base = (const unsigned char*)lds;
    // LDSN: the whole tree at the base; kTop: the copy of the tree's first levels after the stack
    return trace_wide<R, SPH, TRI, QUAD, MOV, LDSN, kBlock, LDSN ? RT_SHADE_BATCH : RT_SHADE_BATCH_GLOBAL>(
        sc, (kTop || kTopH) ? base + top_offset(sc.wide_stack) : base, (const WW*)(base + sc.n_wnodes * kWNodeLdsStride), s.o,
        s.d, s.tm, s.xe, stk, ry);
  }
};

template <int N>
struct Lds {
  uint32_t v[N];
};
template <>
struct Lds<0> {
  uint32_t v[1];
};

#ifdef RT_SECTION_CLOCKS
__device__ unsigned long long g_section_clocks[4];  // trace, shade, store, lanes
#endif

template <class R, class Trav, bool CAMX>
__device__ __forceinline__ void step_body(const Params<R>& p) {
  __shared__ Lds<Trav::kStack * kBlock> stk;
  __shared__ uint32_t wave_cnt[kBlock / 64];
  __shared__ Node<R> lds_nodes[Trav::kLdsNodes > 0 ? Trav::kLdsNodes : 1];
  if constexpr (Trav::kLdsNodes > 0) {
    for (uint32_t j = threadIdx.x; j < p.sc.n_nodes; j += kBlock) lds_nodes[j] = p.sc.nodes[j];
    __syncthreads();
  }
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  uint32_t slot = 0, segs = 0;
  bool active = i < p.n;
  R4<R> Dv{};
  if (active) {
    slot = p.queue ? p.queue[i] : i;
    Dv = p.D[slot];
    active = Dv.w >= R(0);
  }
  if (active) {
    Path<R> s;
    load_path(p, slot, Dv, s);
#ifdef RT_SECTION_CLOCKS
    uint64_t c_trace = 0, c_shade = 0;
#endif
#pragma unroll 1
    for (int k = 0; k < p.K; k++) {
      R t;
      uint32_t e, nm = 0;
      int32_t inst;
#ifdef RT_SECTION_CLOCKS
      const uint64_t c0 = clock64();
#endif
      Trav::run(p.sc, lds_nodes, s, Keys{s.ks}, stk.v + threadIdx.x, t, e, inst, nm);
      segs++;
#ifdef RT_SECTION_CLOCKS
      const uint64_t c1 = clock64();
      const bool more = shade<R, CAMX, Trav::kFlat>(p, s, t, e, inst, nm);
      const uint64_t c2 = clock64();
      c_trace += c1 - c0;
      c_shade += c2 - c1;
      if (!more) break;
#else
      if (!shade<R, CAMX, Trav::kFlat>(p, s, t, e, inst, nm)) break;
#endif
    }
#ifdef RT_SECTION_CLOCKS
    const uint64_t c3 = clock64();
#endif
    store_path(p, slot, s);
#ifdef RT_SECTION_CLOCKS
    // development build: shader-clock cycles per section, summed over lanes (divide by the lane count)
    atomicAdd(&g_section_clocks[0], (unsigned long long)c_trace);
    atomicAdd(&g_section_clocks[1], (unsigned long long)c_shade);
    atomicAdd(&g_section_clocks[2], (unsigned long long)(clock64() - c3));
    atomicAdd(&g_section_clocks[3], 1ull);
#endif
  }
  // segments traced: wave sums, one atomic per block
  for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off);
  if ((threadIdx.x & 63) == 0) wave_cnt[threadIdx.x >> 6] = segs;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
    if (c) atomicAdd(&p.seg_shards[blockIdx.x % kSegShards], (unsigned long long)c);
  }
}

// Persistent form of the same loop (the default schedule): the grid is what the chip holds
// resident, every lane keeps its path state in registers for the whole render. Dynamic
// (persist 2): shade's path regeneration pulls the next item from the wave's queue, refilled a
// batch at a time from the per-XCD heads (one returning atomic per 64 items; per-lane atomics on
// one counter for the whole chip serialised across the 8 XCDs' L2s: measured 6x slower on C2).
// Static (persist 1): lanes walk items lane, lane + P, ... (P = grid lanes). No state goes
// through HBM between segments, there is no launch per K segments and no live-slot compaction.
// Trav::Tables for the flat program, an empty stand-in for the others
template <class R, class Trav, bool = Trav::kTablesLds>
struct FlatTables {
  struct T {};
};
template <class R, class Trav>
struct FlatTables<R, Trav, true> {
  using T = typename Trav::Tables;
};
template <class R, class Trav, bool CAMX>
__device__ __forceinline__ void persist_body(const Params<R>& p) {
  __shared__ Lds<Trav::kStack * kBlock> stk;
  __shared__ uint32_t wave_cnt[kBlock / 64];
  __shared__ Node<R> lds_nodes[Trav::kLdsNodes > 0 ? Trav::kLdsNodes : 1];
  if constexpr (Trav::kLdsNodes > 0) {
    for (uint32_t j = threadIdx.x; j < p.sc.n_nodes; j += kBlock) lds_nodes[j] = p.sc.nodes[j];
    __syncthreads();
  }
  uint32_t* stk_lane = stk.v + threadIdx.x;
  const Node<R>* trav_nodes = lds_nodes;
  [[maybe_unused]] void* wstk = nullptr;  // the wide traversal's lane stack (uint16 or uint32 entries)
#ifdef RT_SECTION_CLOCKS
  if (threadIdx.x < 10) wide_stats_lds()[threadIdx.x] = 0;
  __syncthreads();
#endif
  if constexpr (Trav::kWide) {
    extern __shared__ uint4 dyn_lds[];
    wstk = Trav::fill(p.sc, dyn_lds) + threadIdx.x;
    trav_nodes = (const Node<R>*)dyn_lds;
  }
  [[maybe_unused]] const typename FlatTables<R, Trav>::T* flat_tb = nullptr;
  if constexpr (Trav::kTablesLds) {  // the host launches this kernel only when the tables fit
    __shared__ typename FlatTables<R, Trav>::T tb;
    Trav::fill(p.sc, tb);
    __syncthreads();
    flat_tb = &tb;
  }
  // the wide and linear LL kernels: the materials as (colour, kind) records in LDS, kind 0 lambertian, 1
  // diffuse_light, 2 isotropic (shade LL, LLI)
  [[maybe_unused]] const R4<R>* wlm = nullptr;
  if constexpr (Trav::kWide || Trav::kLinLL) {
    if constexpr (Trav::kLL) {
      __shared__ R4<R> wlm_tab[Trav::kLdsMats];
      for (uint32_t j = threadIdx.x; j < p.sc.n_mats; j += kBlock) {
        const Material<R>& m = p.sc.mats[j];
        wlm_tab[j] = R4<R>{m.tx.c0[0], m.tx.c0[1], m.tx.c0[2],
                           m.kind == M_DIFFUSE_LIGHT ? R(1) : (m.kind == M_ISOTROPIC ? R(2) : R(0))};
      }
      __syncthreads();
      wlm = wlm_tab;
    }
  }
  uint32_t item0 = blockIdx.x * kBlock + threadIdx.x;
  if (p.persist == 2) {
    if ((threadIdx.x & 63) == 0) {
      __hip_atomic_store(wave_queue(), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      __hip_atomic_store(wave_queue() + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    item0 = next_item_dyn(p);
  }
  uint64_t segs = 0;
  if (item0 < p.n_items) {
    Path<R, Trav::kColdLds, Trav::kLean, Trav::kNoRad, Trav::kThrLds> s;
    s.set_acc(mkv(R(0), R(0), R(0)));
    begin_item(p, s, item0);
    begin_sample<R, CAMX>(p, s);
    if constexpr (Trav::kWide) {
      // resumable traversal: a ray paused with the wave's laggards carries on after the others shade
      using StackT = typename Trav::StackT;
      const uint32_t root = Trav::root(p.sc);
      WideRayT<R> ry{root, 0, Num<R>::inf(), kNoHit, 1u};
      using KP = const __attribute__((address_space(4))) Params<R>*;
      const KP kp0 = (KP)__builtin_amdgcn_kernarg_segment_ptr();
#pragma unroll 1
      for (;;) {
        KP kp = kp0;
        asm volatile("" : "+s"(kp));
        const Params<R>& q = *(const Params<R>*)kp;
#ifdef RT_SECTION_CLOCKS
        const uint64_t c0 = clock64();
        const bool fin = Trav::steps(q.sc, trav_nodes, s, (StackT*)wstk, ry);
        if (__lane_id() == (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1)
          atomicAdd(wide_stats_lds() + 6, (unsigned long long)(clock64() - c0));
        if (!fin) continue;
#else
        if (!Trav::steps(q.sc, trav_nodes, s, (StackT*)wstk, ry)) continue;
#endif
        if (++segs > q.seg_cap) {  // cannot happen: every segment advances a bounce-capped path
          atomicOr(q.fault, 1u);
          break;
        }
        const R t = ry.tmax;
        const uint32_t e = ry.e;
        ry = WideRayT<R>{root, 0, Num<R>::inf(), kNoHit, 1u};
#ifdef RT_SECTION_CLOCKS
        RT_WIDE_STAT(4);
        const uint64_t c1 = clock64();
        const bool more = shade<R, CAMX, false, Trav::kMoving, Trav::kLL, Trav::kLL, Trav::kNL>(q, s, t, e, -1, 0, nullptr, wlm);
        if (__lane_id() == (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1)
          atomicAdd(wide_stats_lds() + 7, (unsigned long long)(clock64() - c1));
        if (!more) break;
#else
        if (!shade<R, CAMX, false, Trav::kMoving, Trav::kLL, Trav::kLL, Trav::kNL>(q, s, t, e, -1, 0, nullptr, wlm)) break;
#endif
      }
    } else if constexpr (Trav::kTablesLds) {
      // the flat program with its records and materials in LDS (Trav::Tables); the parameters are
      // reloaded per segment as below
      using KP = const __attribute__((address_space(4))) Params<R>*;
      const KP kp0 = (KP)__builtin_amdgcn_kernarg_segment_ptr();
#pragma unroll 1
      for (;;) {
        KP kp = kp0;
        asm volatile("" : "+s"(kp));
        const Params<R>& q = *(const Params<R>*)kp;
        R t;
        uint32_t e, nm = 0;
        int32_t inst;
        Trav::run_lds(q.sc, *flat_tb, s, t, e, inst, nm);
        if (++segs > q.seg_cap) {  // cannot happen: every segment advances a bounce-capped path
          atomicOr(q.fault, 1u);
          break;
        }
        if (!shade<R, CAMX, true, true, true, Trav::kLL>(q, s, t, e, inst, nm, flat_tb->m, flat_tb->lm)) break;
      }
    } else {
      // The parameters are read from the kernarg segment afresh each segment (the asm hides
      // the pointer from loop-invariant hoisting): hoisted, they outgrow the SGPR file and spill
      // into VGPR lanes, one v_readlane per use (C2 flat program: 73 SGPR spills -> 0, 24.9 ->
      // 23.9 ms/frame; scalar loads hit the constant cache)
      using KP = const __attribute__((address_space(4))) Params<R>*;
      const KP kp0 = (KP)__builtin_amdgcn_kernarg_segment_ptr();
#pragma unroll 1
      for (;;) {
        KP kp = kp0;
        asm volatile("" : "+s"(kp));
        const Params<R>& q = *(const Params<R>*)kp;
        R t;
        uint32_t e, nm = 0;
        int32_t inst;
#ifdef RT_SECTION_CLOCKS
        RT_WIDE_STAT(0);
        const uint64_t c0 = clock64();
#endif
        Trav::run(q.sc, trav_nodes, s, Keys{s.ks}, stk_lane, t, e, inst, nm);
        if (++segs > q.seg_cap) {  // cannot happen: every segment advances a bounce-capped path
          atomicOr(q.fault, 1u);
          break;
        }
#ifdef RT_SECTION_CLOCKS
        const uint64_t c1 = clock64();
        const bool more = shade<R, CAMX, Trav::kFlat, true, Trav::kLinLL, Trav::kLinLL, false, Trav::kLinLL>(
            q, s, t, e, inst, nm, nullptr, wlm);
        if (__lane_id() == (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1) {
          atomicAdd(wide_stats_lds() + 6, (unsigned long long)(c1 - c0));
          atomicAdd(wide_stats_lds() + 7, (unsigned long long)(clock64() - c1));
        }
        if (!more) break;
#else
        if (!shade<R, CAMX, Trav::kFlat, true, Trav::kLinLL, Trav::kLinLL, false, Trav::kLinLL>(q, s, t, e, inst, nm,
                                                                                            nullptr, wlm))
          break;
#endif
      }
    }
  }
  uint32_t sg = (uint32_t)segs;
  for (int off = 32; off > 0; off >>= 1) sg += __shfl_xor(sg, off);
  if ((threadIdx.x & 63) == 0) wave_cnt[threadIdx.x >> 6] = sg;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t c = (uint64_t)wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
    if (c) atomicAdd(&p.seg_shards[blockIdx.x % kSegShards], (unsigned long long)c);
  }
#ifdef RT_SECTION_CLOCKS
  if (threadIdx.x < 10) atomicAdd(&g_wide_stats[threadIdx.x], wide_stats_lds()[threadIdx.x]);
#endif
}
template <class R, class Trav, bool CAMX>
__global__ __launch_bounds__(kBlock) void k_persist(Params<R> p) {
  persist_body<R, Trav, CAMX>(p);
}
// CAMX kernels (non-perspective cameras, picture and procedural textures) take RT_CAMX_WAVES (fp32) and
// RT_CAMX_WAVES_F64 waves per SIMD. Round 4 left them unbudgeted: ~290 registers, 1 wave per SIMD. With the
// heavy code as calls (RT_EXT_FN) the §8(f) configs, ms/frame at 1 wave (round 4) / 2 / 3 / 4 waves (r05f,
// r05g): fisheye f64 14.8 / 11.0 / 13.5 / 16.2, f32 14.2 / 10.7 / 8.6 / 8.8; earth f64 10.5 / 6.6 / 8.9 /
// 11.1, f32 9.9 / 6.2 / 4.9 / 4.8; perlin f64 148 / 81 / 70 / 79, f32 128 / 69 / 50 / 43. The fp64 linear
// programs need ~144 registers without any CAMX code, so 4 waves spills there.
#ifndef RT_CAMX_WAVES
#define RT_CAMX_WAVES 4
#endif
#ifndef RT_CAMX_WAVES_F64
#define RT_CAMX_WAVES_F64 2
#endif
#define RT_CAMX_W(R) (sizeof(R) == 8 ? RT_CAMX_WAVES_F64 : RT_CAMX_WAVES)
template <class R, class Trav, bool CAMX>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(CAMX ? RT_CAMX_W(R) : Trav::kWaves))) void k_persist_occ(
    Params<R> p) {
  persist_body<R, Trav, CAMX>(p);
}

// The kernel; k_step_occ is the same body with the register budget cut for Trav::kWaves
// waves per SIMD (only where that does not spill much, see LinearTrav::kWaves).
// CAMX ("extended"): a non-perspective camera (camera_ray) or procedural textures (noise.h); the
// base kernels, which every BASELINE config except the noise scenes uses, contain neither.
template <class R, class Trav, bool CAMX>
__global__ __launch_bounds__(kBlock) void k_step(Params<R> p) {
  step_body<R, Trav, CAMX>(p);
}
template <class R, class Trav, bool CAMX>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(CAMX ? RT_CAMX_W(R) : Trav::kWaves))) void k_step_occ(Params<R> p) {
  step_body<R, Trav, CAMX>(p);
}

// ------------------------------------------------------------------ live-slot compaction
__device__ __forceinline__ bool slot_alive(const void* Dp, int prec, uint32_t slot) {
  if (prec == RT_PREC_F32) return reinterpret_cast<const R4<float>*>(Dp)[slot].w >= 0.f;
  return reinterpret_cast<const R4<double>*>(Dp)[slot].w >= 0.0;
}

__global__ __launch_bounds__(kBlock) void k_count(const void* Dp, int prec, const uint32_t* queue, uint32_t n,
                                                  uint32_t* blk) {
  __shared__ uint32_t wc[kBlock / 64];
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  bool alive = false;
  if (i < n) alive = slot_alive(Dp, prec, queue ? queue[i] : i);
  unsigned long long m = __ballot(alive);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (uint32_t)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) blk[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

// exclusive scan of the per-block counts (one workgroup), total in *total
__global__ __launch_bounds__(1024) void k_scan(uint32_t* blk, uint32_t nb, uint32_t* total) {
  __shared__ uint32_t part[1024];
  uint32_t per = (nb + 1023) / 1024;
  uint32_t b = threadIdx.x * per, e = min(nb, b + per);
  uint32_t s = 0;
  for (uint32_t j = b; j < e; j++) s += blk[j];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (uint32_t j = b; j < e; j++) {
    uint32_t c = blk[j];
    blk[j] = run;
    run += c;
  }
  if (threadIdx.x == 1023) *total = part[1023];
}

__global__ __launch_bounds__(kBlock) void k_compact(const void* Dp, int prec, const uint32_t* queue, uint32_t n,
                                                    const uint32_t* blk_off, uint32_t* out) {
  __shared__ uint32_t wc[kBlock / 64];
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  uint32_t slot = 0;
  bool alive = false;
  if (i < n) {
    slot = queue ? queue[i] : i;
    alive = slot_alive(Dp, prec, slot);
  }
  unsigned long long m = __ballot(alive);
  int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t base = blk_off[blockIdx.x];
  for (int w = 0; w < wave; w++) base += wc[w];
  if (alive) {
    unsigned long long below = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
    out[base + (uint32_t)__popcll(below)] = slot;
  }
}

// ------------------------------------------------------------------ resolve (camera.h:169-170)
// A render in passes (render()): pass k adds its chunks to the running sums that the earlier passes left in
// `out` (first: from 0), in chunk order, and the last pass divides -- the same additions in the same order as
// one pass over every chunk, so the image does not depend on the pass split.
template <class R>
__global__ __launch_bounds__(kBlock) void k_resolve(const R* partial, uint32_t npix, uint32_t nchunks, uint32_t spp,
                                                    R* out, int first, int last) {
  uint32_t px = blockIdx.x * kBlock + threadIdx.x;
  if (px >= npix) return;
  R s0 = 0, s1 = 0, s2 = 0;
  if (!first) {
    s0 = out[3ull * px];
    s1 = out[3ull * px + 1];
    s2 = out[3ull * px + 2];
  }
  for (uint32_t c = 0; c < nchunks; c++) {
    const R* q = partial + 3ull * ((uint64_t)c * npix + px);
    s0 += q[0];
    s1 += q[1];
    s2 += q[2];
  }
  if (last) {
    R inv = R(spp);
    s0 = s0 / inv;
    s1 = s1 / inv;
    s2 = s2 / inv;
  }
  out[3ull * px] = s0;
  out[3ull * px + 1] = s1;
  out[3ull * px + 2] = s2;
}

template <class R>
__global__ void k_zero(R* out, uint64_t n) {
  uint64_t i = blockIdx.x * (uint64_t)kBlock + threadIdx.x;
  if (i < n) out[i] = R(0);
}

// The pixel map (tiles packed in order, row-major inside each tile, camera.h:154-158's pixel
// loop per tile) built on the device from the tile list: tl[t] = {x0, y0, width, first packed
// pixel}; pixel i belongs to the last tile whose first pixel is <= i.
__global__ __launch_bounds__(kBlock) void k_pixmap(const uint4* tl, uint32_t ntiles, uint32_t npix, uint32_t* pixmap) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= npix) return;
  uint32_t lo = 0, hi = ntiles - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (tl[mid].w <= i) lo = mid;
    else hi = mid - 1;
  }
  const uint4 t = tl[lo];
  const uint32_t k = i - t.w, y = k / t.z, x = k - y * t.z;
  pixmap[i] = (t.x + x) | (t.y + y) << 16;
}

// camera.h:137-141, 246, 253, 278-279 evaluated in double exactly as the reference orders them
CamDev make_view(const rt_camera_desc* c) {
  CamDev v{};
  v.mode = c->mode;
  double du[3], dv[3], dir00[3], pos00[3];
  for (int k = 0; k < 3; k++) {
    du[k] = (c->right[k] * c->viewport_width) / (double)c->image_width;
    dv[k] = (c->up[k] * -c->viewport_height) / (double)c->image_height;
  }
  for (int k = 0; k < 3; k++) {
    double a = c->dir[k] * c->focal_length;
    double b = c->right[k] * (c->viewport_width / 2.0);
    double u = c->up[k] * (c->viewport_height / 2.0);
    double e = (du[k] + dv[k]) * 0.5;
    dir00[k] = ((a - b) + u) + e;
    pos00[k] = ((c->pos[k] - b) + u) + e;
  }
  v.pos = {c->pos[0], c->pos[1], c->pos[2]};
  v.du = {du[0], du[1], du[2]};
  v.dv = {dv[0], dv[1], dv[2]};
  v.dir00 = {dir00[0], dir00[1], dir00[2]};
  v.pos00 = {pos00[0], pos00[1], pos00[2]};
  v.dir = {c->dir[0], c->dir[1], c->dir[2]};
  v.fdir = {c->focus_dist * c->dir[0], c->focus_dist * c->dir[1], c->focus_dist * c->dir[2]};
  v.disk_u = {c->defocus_u[0], c->defocus_u[1], c->defocus_u[2]};
  v.disk_v = {c->defocus_v[0], c->defocus_v[1], c->defocus_v[2]};
  v.focal = c->focal_length;
  return v;
}

template <class R>
V<R> tov(const double* a) {
  return {(R)a[0], (R)a[1], (R)a[2]};
}

}  // namespace

// ====================================================================== host side

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};

struct rt_context {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  CompiledScene scene;
  bool has_scene = false;
  DevBuf scene32, scene64;
  DevBuf state, partial, pixmap, queue0, queue1, blk, out_tmp, counters, camx, heads, tiles;
  DevBuf wide_spill;  // the wide traversal's stack entries past wide_lds_stack (deep trees in HBM)
  CamDev cam_host;  // source of camx (kept alive for the async copy)
  uint32_t* total_host = nullptr;  // pinned: [0] live slots, [1] fault word, [16..] segment counter shards
  uint64_t samples = 0;
  rt_counters last{};  // host-known totals since rt_reset_counters; segments and step_ms settle in settle()
  int timing = 0;
  std::vector<hipEvent_t> events;
  // asynchronous renders (device output): what rt_stats / rt_reset_counters / a host-output render
  // settle with one sync -- the stream, the timing events recorded since the last settle
  hipStream_t pend_stream = nullptr;
  bool pending = false;
  size_t ev_used = 0;
  DevBuf fault;  // sticky internal-error word of the persistent kernel (zeroed by rt_reset_counters)
  // inputs kept on the device while they do not change between calls
  std::vector<uint4> tiles_dev;  // the tile list k_pixmap last expanded into pixmap
  void* pixmap_for = nullptr;    // pixmap buffer that expansion went to
  uint32_t pixmap_npix = 0;      // pixels it expanded: a tile entry {x0, y0, width, first} does not
                                 // hold the height, so the last tile can change with the list equal
  CamDev cam_dev{};              // the camera view in camx
  bool cam_valid = false;
  // the compiled scene is copied into scene32 / scene64 by the first render after rt_scene_upload,
  // on that render's stream: a copy made on another stream is not guaranteed visible to the kernels
  // of the render stream (their launch need not invalidate the L2 lines of the previous scene)
  bool scene_dirty32 = false, scene_dirty64 = false;
};

namespace {

std::mutex g_err_mu;
std::string g_create_err;

rt_status set_err(rt_context* c, rt_status s, const std::string& m) {
  if (c) {
    c->err = m;
  } else {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_create_err = m;
  }
  return s;
}

#define RT_HIP(ctx, call)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return set_err((ctx), RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Grow a context buffer. The only work that can still read the old buffer is this context's
// outstanding device-output render (host-output renders return finished, and a render on another
// stream waits for pend_stream first): wait for that stream, not for the whole device.
rt_status ensure(rt_context* c, DevBuf& b, size_t bytes) {
  if (b.ptr && b.bytes >= bytes) return RT_OK;
  if (b.ptr) {
    if (c->pending) RT_HIP(c, hipStreamSynchronize(c->pend_stream));
    RT_HIP(c, hipFree(b.ptr));
    b.ptr = nullptr;
    b.bytes = 0;
  }
  size_t want = std::max<size_t>(bytes, 256);
  hipError_t e = hipMalloc(&b.ptr, want);
  if (e != hipSuccess) {
    b.ptr = nullptr;
    (void)hipGetLastError();
    return set_err(c, RT_ERR_OUT_OF_MEMORY,
                   "hipMalloc(" + std::to_string(want) + " bytes): " + hipGetErrorString(e));
  }
  b.bytes = want;
  return RT_OK;
}

hipEvent_t take_event(rt_context* c, size_t idx) {
  while (c->events.size() <= idx) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->events.push_back(e);
  }
  return c->events[idx];
}

// Wait for the context's outstanding renders and fold their device-side results into c->last:
// the cumulative segment count, the kernel time of the timing events, the fault word.
rt_status settle(rt_context* c) {
  if (!c->pending) return RT_OK;
  c->pending = false;
  RT_HIP(c, hipStreamSynchronize(c->pend_stream));
  unsigned long long* shards = (unsigned long long*)(c->total_host + 16);
  RT_HIP(c, hipMemcpy(shards, c->counters.ptr, sizeof(unsigned long long) * kSegShards, hipMemcpyDeviceToHost));
  uint64_t segs = 0;
  for (int k = 0; k < kSegShards; k++) segs += shards[k];
  c->last.segments = segs;
  double ms = 0;
  for (size_t k = 0; k + 1 < c->ev_used; k += 2) {
    float a = 0;
    RT_HIP(c, hipEventElapsedTime(&a, c->events[k], c->events[k + 1]));
    ms += a;
  }
  c->ev_used = 0;
  c->last.step_ms += ms;
  uint32_t fault = 0;
  if (c->fault.ptr) RT_HIP(c, hipMemcpy(&fault, c->fault.ptr, 4, hipMemcpyDeviceToHost));
  if (fault) return set_err(c, RT_ERR_HIP, "a path did not finish (internal error)");
  return RT_OK;
}

// Division by a launch constant d >= 1 as a multiply (Granlund-Montgomery): with
// k = 32 + ceil(log2 d) and m = floor(2^k / d) + 1, (n * m) >> k == n / d for every n < 2^31
// (m d - 2^k <= d, so the error n (m d - 2^k) / 2^k stays below 1/d; n m < 2^64).
void div_magic(uint32_t d, uint64_t& m, uint32_t& k) {
  uint32_t l = 0;
  while ((1ull << l) < d) l++;
  k = 32 + l;
  m = (uint64_t)((((unsigned __int128)1) << k) / d) + 1;
}

template <class R>
DevScene<R> dev_scene(const SceneHeader& h, void* base) {
  auto at = [&](uint64_t off) { return (const unsigned char*)base + off; };
  DevScene<R> s{};
  s.quads = (const Quad<R>*)at(h.off_quads);
  s.spheres = (const Sphere<R>*)at(h.off_spheres);
  s.tris = (const Tri<R>*)at(h.off_tris);
  s.insts = (const Instance<R>*)at(h.off_instances);
  s.vols = (const Volume<R>*)at(h.off_volumes);
  s.nodes = (const Node<R>*)at(h.off_nodes);
  s.refs = (const uint32_t*)at(h.off_refs);
  s.mats = (const Material<R>*)at(h.off_mats);
  s.texs = (const Texture<R>*)at(h.off_texs);
  s.light = (const Light<R>*)at(h.off_light);
  s.lin = (const LinRec<R>*)at(h.off_linear);
  s.n_linear = h.n_linear;
  s.has_flat = (int32_t)h.has_flat;
  s.flatq = (const FlatQuadT<R>*)at(h.off_flat_quad);
  s.flatb = (const FlatBoxT<R>*)at(h.off_flat_box);
  for (int a = 0; a < 3; a++) s.n_flatq[a] = h.n_flat_quad[a];
  s.n_flatb = h.n_flat_box;
  s.n_mats = h.n_mats;
  s.root = h.root;
  s.background = h.background;
  s.has_volumes = h.has_volumes;
  s.n_nodes = h.n_nodes;
  s.texdata = (const double*)at(h.off_texdata);
  s.images = (const uint8_t*)at(h.off_images);
  s.has_procedural = h.n_texdata > 0 || h.has_cell_noise;
  s.has_wide = (int32_t)h.has_wide;
  s.wnodes = (const WNode*)at(h.off_wnodes);
  s.wprims = (const typename WWord<R>::T*)at(h.off_wprims);
  s.n_wnodes = h.n_wnodes;
  s.n_wprim_words = h.n_wprim_words;
  s.wroot = h.wroot;
  s.wide_stack = h.wide_stack;
  s.wide_kinds = h.wide_kinds;
  s.wide_big = h.wide_big;
  s.wide_top = h.wide_top;
  s.wnodesh = h.has_wnodesh ? (const WNodeH*)at(h.off_wnodesh) : nullptr;
  s.quads64 = h.has_quads64 ? (const Quad<double>*)at(h.off_quads64) : nullptr;
  return s;
}

// Resident blocks of one kernel on one device (occupancy query x CU count), cached per (kernel,
// device): every persistent kernel has its own register budget, so one kernel's grid must not
// size another's. Guarded: contexts on different host threads launch concurrently.
std::mutex g_occ_mu;
std::map<std::tuple<const void*, int, size_t>, uint32_t> g_occ;

uint32_t resident_blocks(const void* kern, int dev, size_t lds) {
  std::lock_guard<std::mutex> lk(g_occ_mu);
  auto it = g_occ.find({kern, dev, lds});
  if (it != g_occ.end()) return it->second;
  int n = 0, b = 0;
  uint32_t r = 0;  // unknown: keep the host's grid
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, kBlock, lds) == hipSuccess && b > 0 && n > 0)
    r = (uint32_t)(b * n);
  g_occ[{kern, dev, lds}] = r;
  return r;
}

// lanes of the last persistent launch on this host thread (rt_counters.grid_lanes)
thread_local uint64_t t_grid_lanes = 0;

template <class KernelT, class R>
void launch_one(KernelT kern, Params<R> p, uint32_t grid, hipStream_t st, size_t lds = 0) {
  if (p.persist == 2) {  // as many blocks as the chip holds resident; lanes pull items
    int dev = 0;
    const uint32_t res = hipGetDevice(&dev) == hipSuccess ? resident_blocks((const void*)kern, dev, lds) : 0;
    if (res > 0) grid = std::min<uint32_t>(grid, res);
    p.P = grid * kBlock;
    p.seg_cap = (uint64_t)p.n_items * p.chunk * (uint64_t)p.max_depth + 1;
  } else if (p.persist) {  // the lanes stride over the items by the grid's lane count
    p.P = grid * kBlock;
    p.seg_cap = ((uint64_t)p.n_items + p.P - 1) / p.P * p.chunk * (uint64_t)p.max_depth + 1;
  }
  if (p.persist) t_grid_lanes = (uint64_t)grid * kBlock;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, st, p);
}

// Dynamic LDS of a wide-BVH launch: the whole tree when it fits the budget (LDSN), else the stack only.
constexpr size_t kWideLdsBudget = 40u << 10;  // bytes per 256-lane block: 4 blocks per CU of 160 KiB
// The fp32 kernel over a tree in HBM runs RT_WIDE_WAVES_GLOBAL blocks per CU only if that many blocks' LDS -- the
// stack entries kept in LDS, the top of the tree and the small static tables -- fit the CU's 160 KiB. A knob
// combination over it does not fail: the occupancy query quietly launches fewer blocks (the round-5 sweep's "24 /
// 21 / 6" point ran at 5 blocks per CU), so it is refused here.
static_assert(((size_t)RT_WIDE_LDS_STACK * kBlock * 4u + (size_t)RT_WIDE_TOP_N * kWTopStride + 1024u) *
                      RT_WIDE_WAVES_GLOBAL <= (160u << 10),
              "RT_WIDE_LDS_STACK / RT_WIDE_TOP_N do not fit RT_WIDE_WAVES_GLOBAL blocks per CU");
// the same for the fp64 LL kernel over a tree in HBM at RT_WIDE_WAVES_GLOBAL_F64_LL blocks per CU: its LDS stack
// entries, the fp16 top nodes and the lanes' throughput (Path LT)
static_assert(((size_t)RT_WIDE_LDS_STACK_F64 * kBlock * 4u + (size_t)RT_WIDE_TOP_N_F64 * sizeof(WNodeH) +
               3u * kBlock * sizeof(double) + 1024u) *
                      RT_WIDE_WAVES_GLOBAL_F64_LL <= (160u << 10),
              "RT_WIDE_LDS_STACK_F64 / RT_WIDE_TOP_N_F64 do not fit RT_WIDE_WAVES_GLOBAL_F64_LL blocks per CU");
static_assert(RT_WIDE_TOP_N <= kWideTopMax && RT_WIDE_TOP_N_F64 <= kWideTopMax,
              "the scene compiler orders at most kWideTopMax top nodes first");
template <class R>
inline size_t wide_lds_bytes(const DevScene<R>& sc, bool ldsn) {
  // an LDS tree: every entry in LDS, uint16; a tree in HBM: up to wide_lds_stack uint32 entries (the rest spill)
  const size_t stack = ldsn ? (size_t)sc.wide_stack * kBlock * 2u
                            : (size_t)std::min<uint32_t>(sc.wide_stack, wide_lds_stack<R>()) * kBlock * 4u;
  // fp32 rays over a tree in HBM: the copy of its first levels (RT_WIDE_TOP)
  const size_t top = (!ldsn && sizeof(R) == 4)
                         ? (size_t)std::min<uint32_t>(sc.wide_top, RT_WIDE_TOP_N) * kWTopStride
                     : (!ldsn && sizeof(R) == 8)
                         ? (size_t)std::min<uint32_t>(sc.wide_top, RT_WIDE_TOP_N_F64) * sizeof(WNodeH) : 0u;
  return (ldsn ? (size_t)sc.n_wnodes * kWNodeLdsStride + (size_t)sc.n_wprim_words * sizeof(typename WWord<R>::T) : 0u) +
         stack + top;
}
template <class R, bool SPH, bool TRI, bool QUAD, bool MOV, bool LL = false, bool NL = false>
void launch_wide_k(const Params<R>& p, uint32_t grid, hipStream_t st) {
  const size_t full = wide_lds_bytes(p.sc, true);
  const uint32_t spill_grid = p.sc.wide_spill ? std::min<uint32_t>(grid, p.sc.spill_lanes / kBlock) : grid;
  // LDS-resident trees use 16-bit child codes (wide_code16): node offset (index x 9) < 2^15, first word < 2^12
  if (full <= kWideLdsBudget && p.sc.n_wnodes * kWNodeLdsUnits < 0x8000u && p.sc.n_wprim_words <= 0x1000u) {
    launch_one(k_persist_occ<R, WideTrav<R, SPH, TRI, QUAD, MOV, true, LL, NL>, false>, p, grid, st, full);
    return;
  }
  // the spill area holds spill_lanes lanes: never launch more (the resident grid is below it)
  launch_one(k_persist_occ<R, WideTrav<R, SPH, TRI, QUAD, MOV, false, LL, NL>, false>, p, spill_grid, st,
             wide_lds_bytes(p.sc, false));
}
// Kernel for the primitive kinds of the scene: spheres only (RTOW), triangles only or triangles and
// quads (meshes, the C4 stand-in with its light), or all.
template <class R>
inline void launch_wide(const Params<R>& p, bool ll, bool nl, uint32_t grid, hipStream_t st) {
  const uint32_t k = p.sc.wide_kinds;
  if (k == WK_SPHERE && nl)  // RTOW (C3)
    launch_wide_k<R, true, false, false, false, false, true>(p, grid, st);
  else if (k == WK_SPHERE)
    launch_wide_k<R, true, false, false, false>(p, grid, st);
  else if (k == WK_TRI)
    launch_wide_k<R, false, true, false, false>(p, grid, st);
  else if (k == (WK_TRI | WK_QUAD) && ll && p.sc.n_mats <= 16)
    launch_wide_k<R, false, true, true, false, true>(p, grid, st);  // ... lambertian + light (the C4 stand-in)
  else if (k == (WK_TRI | WK_QUAD))  // a mesh under a quad light
    launch_wide_k<R, false, true, true, false>(p, grid, st);
  else
    launch_wide_k<R, true, true, true, true>(p, grid, st);
}
template <class R, class Trav>
void launch_k(const Params<R>& p, uint32_t grid, hipStream_t st) {
  const bool camx = p.cam_mode != RT_CAM_PERSPECTIVE || p.sc.has_procedural;
  // the flat program only runs perspective renders without procedural textures (kernel_family): no CAMX form
  if (camx && !Trav::kFlat) {
    if constexpr (!Trav::kFlat) {
      if (p.persist)
        launch_one(k_persist_occ<R, Trav, true>, p, grid, st);
      else
        launch_one(k_step_occ<R, Trav, true>, p, grid, st);
    }
    return;
  }
  if (p.persist) {
    if constexpr (Trav::kWaves > 1)
      launch_one(k_persist_occ<R, Trav, false>, p, grid, st);
    else
      launch_one(k_persist<R, Trav, false>, p, grid, st);
  } else {
    if constexpr (Trav::kWaves > 1)
      launch_one(k_step_occ<R, Trav, false>, p, grid, st);
    else
      launch_one(k_step<R, Trav, false>, p, grid, st);
  }
}

// The kernel family a render takes, decided on the host from the compiled scene, the camera model, the
// schedule and the traversal order (launch_step launches it).
enum KernelFamily { KF_FLAT, KF_LIN_QUAD, KF_LIN_VOL, KF_LIN_SPH, KF_LIN_ALL, KF_WIDE, KF_STACK };
KernelFamily kernel_family(const SceneHeader& h, int32_t cam_mode, bool persist, bool ordered) {
  const bool persp = cam_mode == RT_CAM_PERSPECTIVE, procedural = h.n_texdata > 0 || h.has_cell_noise;
  const bool sph = h.n_spheres > 0, tri = h.n_tris > 0, vol = h.has_volumes != 0;
  // the flat program (world-space quads and boxes, fp32 and fp64); the extended kernels keep the linear one
  if (!ordered && h.has_flat && persp && !procedural) return KF_FLAT;
  if (h.n_linear > 0) {
    if (!sph && !tri) return vol ? KF_LIN_VOL : KF_LIN_QUAD;
    return (sph && !tri && !vol) ? KF_LIN_SPH : KF_LIN_ALL;
  }
  // the wide BVH (persistent schedule, base kernels; fp64 rays since round 3)
  if (!ordered && h.has_wide && persist && persp && !procedural) return KF_WIDE;
  return KF_STACK;
}
const char* family_name(KernelFamily f) {
  static const char* n[] = {"flat program", "linear program (quads)", "linear program (quads + volumes)",
                            "linear program (spheres)", "linear program (all kinds)", "wide BVH", "binary BVH"};
  return n[f];
}
// RT_DEV_ONLY (development builds for register/spill iteration, scripts/kernel_usage.py): instantiate one
// kernel family only -- 1 the flat program, 2 the wide BVH, 3 the quad + volume linear program. 0:
// everything. A render (and rt_scene_check) that needs a family such a build omits fails with
// RT_ERR_UNSUPPORTED instead of launching nothing.
#ifndef RT_DEV_ONLY
#define RT_DEV_ONLY 0
#endif
constexpr bool family_built(KernelFamily f) {
  return RT_DEV_ONLY == 0 || (RT_DEV_ONLY == 1 && f == KF_FLAT) || (RT_DEV_ONLY == 2 && f == KF_WIDE) ||
         (RT_DEV_ONLY == 3 && f == KF_LIN_VOL);
}
// a lambertian + diffuse_light scene with solid textures (a background too) and an axis-aligned quad light (the
// Cornell configs): the flat kernel's LL form (shade LL)
bool lamb_light_scene(const SceneHeader& h) {
  const uint32_t ok_m = (1u << M_LAMBERTIAN) | (1u << M_DIFFUSE_LIGHT);
  return (h.mat_kinds & ~ok_m) == 0 && (h.tex_kinds & ~(1u << T_SOLID)) == 0 && h.light_kind == L_QUAD &&
         h.light_aligned != 0;
}
// no light, lambertian / metal / dielectric materials with solid or checker textures (RTOW): shade NL
bool no_light_scene(const SceneHeader& h) {
  const uint32_t ok_m = (1u << M_LAMBERTIAN) | (1u << M_METAL) | (1u << M_DIELECTRIC);
  return (h.mat_kinds & ~ok_m) == 0 && (h.tex_kinds & ~((1u << T_SOLID) | (1u << T_CHECKER))) == 0 &&
         h.light_kind == L_NONE;
}
// lambertian, isotropic and diffuse_light materials with solid textures and an axis-aligned quad light (C5)
bool lamb_iso_light_scene(const SceneHeader& h) {
  const uint32_t ok_m = (1u << M_LAMBERTIAN) | (1u << M_DIFFUSE_LIGHT) | (1u << M_ISOTROPIC);
  return (h.mat_kinds & ~ok_m) == 0 && (h.tex_kinds & ~(1u << T_SOLID)) == 0 && h.light_kind == L_QUAD &&
         h.light_aligned != 0;
}
template <class R>
void launch_step(const Params<R>& p, KernelFamily fam, bool ll, bool nl, bool lli, int stack, uint32_t grid,
                 hipStream_t st) {
  switch (fam) {
    case KF_FLAT:
      if constexpr (family_built(KF_FLAT)) {
        if (p.persist && FlatTrav<R, true>::tables_fit(p.sc)) {
          if (ll && FlatTrav<R, true, true>::tables_fit(p.sc))
            launch_k<R, FlatTrav<R, true, true>>(p, grid, st);
          else
            launch_k<R, FlatTrav<R, true>>(p, grid, st);
        } else {
          launch_k<R, FlatTrav<R>>(p, grid, st);
        }
      }
      return;
    case KF_LIN_QUAD:
      if constexpr (family_built(KF_LIN_QUAD)) launch_k<R, LinearTrav<R, false, false, false>>(p, grid, st);
      return;
    case KF_LIN_VOL:
      if constexpr (family_built(KF_LIN_VOL)) {
        // lambertian + isotropic + light (C5), persistent schedule only: the LLI form's shade and LDS material table
        // are persist_body's; step_body (segments_per_launch > 0) shades with the general program, which its
        // register budget would squeeze
        if (lli && p.persist && p.sc.n_mats <= 16)
          launch_k<R, LinearTrav<R, false, false, true, true>>(p, grid, st);
        else
          launch_k<R, LinearTrav<R, false, false, true>>(p, grid, st);
      }
      return;
    case KF_LIN_SPH:
      if constexpr (family_built(KF_LIN_SPH)) launch_k<R, LinearTrav<R, true, false, false>>(p, grid, st);
      return;
    case KF_LIN_ALL:
      if constexpr (family_built(KF_LIN_ALL)) launch_k<R, LinearTrav<R, true, true, true>>(p, grid, st);
      return;
    case KF_WIDE:
      if constexpr (family_built(KF_WIDE)) launch_wide(p, ll, nl, grid, st);
      return;
    case KF_STACK:
      if constexpr (family_built(KF_STACK)) {
        if constexpr (sizeof(R) == 4) {  // nodes in LDS: fp32 only
          if (p.sc.n_nodes <= kLdsNodeMax && stack <= 16) {
            launch_k<R, StackTrav<R, 16, true>>(p, grid, st);
            return;
          }
        }
        if (stack <= 8)
          launch_k<R, StackTrav<R, 8>>(p, grid, st);
        else if (stack <= 16)
          launch_k<R, StackTrav<R, 16>>(p, grid, st);
        else
          launch_k<R, StackTrav<R, kStackDepth>>(p, grid, st);
      }
      return;
  }
}

template <class R>
rt_status render(rt_context* c, const rt_camera_desc* cam, const rt_render_params* prm, const rt_tile* tiles,
                 int32_t ntiles, void* out, int32_t out_dev, hipStream_t st) {
  const bool f64 = sizeof(R) == 8;
  const CompiledScene& cs = c->scene;
  const SceneHeader& hdr = f64 ? cs.hdr64 : cs.hdr;
  void* sbase = f64 ? c->scene64.ptr : c->scene32.ptr;
  bool& dirty = f64 ? c->scene_dirty64 : c->scene_dirty32;
  auto t0 = std::chrono::steady_clock::now();
  // A device-output render still pending on another stream reads the context's shared buffers
  // (pixmap, tiles, camx, heads, partial): wait for it before this call writes any of them.
  if (c->pending && c->pend_stream != st) RT_HIP(c, hipStreamSynchronize(c->pend_stream));
  if (dirty) {  // the scene uploaded since the last render of this precision, stream-ordered before its kernels
    const std::vector<unsigned char>& blob = f64 ? cs.blob64 : cs.blob32;
    RT_HIP(c, hipMemcpyAsync(sbase, blob.data(), blob.size(), hipMemcpyHostToDevice, st));
    dirty = false;
    // outstanding from here on, whatever this call does next (an empty tile list or max_depth <= 0
    // launches nothing that reads the scene): a later render on another stream waits for st
    c->pending = true;
    c->pend_stream = st;
  }

  // pixel map: tiles packed in order, row-major inside each tile (expanded by k_pixmap)
  std::vector<uint4> tl;
  tl.reserve(ntiles);
  uint64_t npix64 = 0;
  for (int t = 0; t < ntiles; t++) {
    if (tiles[t].width == 0 || tiles[t].height == 0) continue;
    tl.push_back(make_uint4((uint32_t)tiles[t].x0, (uint32_t)tiles[t].y0, (uint32_t)tiles[t].width, (uint32_t)npix64));
    npix64 += (uint64_t)tiles[t].width * (uint64_t)tiles[t].height;
  }
  if (npix64 >= (1ull << 31)) return set_err(c, RT_ERR_INVALID_ARGUMENT, "too many pixels in one call");
  const uint32_t npix = (uint32_t)npix64;
  if (npix == 0) return RT_OK;
  const size_t out_elems = 3ull * npix;
  rt_status s;
  void* dout = out;
  if (!out_dev) {
    if ((s = ensure(c, c->out_tmp, out_elems * sizeof(R))) != RT_OK) return s;
    dout = c->out_tmp.ptr;
  }

  if (prm->max_depth <= 0) {  // ray_color(r, 0) is black for every sample (camera.h:194-195)
    hipLaunchKernelGGL(k_zero<R>, dim3((unsigned)((out_elems + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       (R*)dout, (uint64_t)out_elems);
  } else {
    const uint32_t spp = (uint32_t)prm->spp;
    // the flat program's items are cheaper per sample, so its default items are twice as long
    // (fewer item ends, dequeues and partial-sum stores; C2: 23.9 -> 23.5 ms/frame)
    const bool flat_prog = hdr.has_flat && prm->traversal != RT_TRAV_ORDERED &&
                           make_view(cam).mode == RT_CAM_PERSPECTIVE && !(hdr.n_texdata > 0 || hdr.has_cell_noise);
    uint32_t chunk0 = prm->samples_per_item > 0 ? std::min<uint32_t>((uint32_t)prm->samples_per_item, spp)
                                               : std::min<uint32_t>(auto_chunk(flat_prog), spp);
    // a small frame (C1: 160,000 px x 64 spp is ~2 items of 16 per resident lane) takes smaller items, so
    // the lanes that finish early find work while the last items run: the automatic size is halved until
    // the whole frame has kItemsTarget items (the full image's pixels, not this call's tiles: the layout,
    // and so the image, is the same for any tiling or rank count)
    if (prm->samples_per_item <= 0) {
      const uint64_t target = env_u32("RT_ITEMS_TARGET", kItemsTarget);
      const uint64_t full = (uint64_t)cam->image_width * (uint64_t)cam->image_height;
      while (chunk0 > kMinAutoChunk && full * ((spp + chunk0 - 1) / chunk0) < target) chunk0 /= 2;
    }
    // The frame's last items are short (auto item size only): a lane that takes a long item just
    // before the queue runs dry keeps its wave resident while the others idle, and a small frame
    // (one rank of eight) has few items per lane. The last tail_samples of every pixel come in
    // items of tail_chunk samples; both depend on spp alone, so the image is the same for any
    // tiling or rank count.
    uint32_t chunk = chunk0, tail_chunk = chunk0, k_bulk = (spp + chunk0 - 1) / chunk0, nchunks = k_bulk;
    if (prm->samples_per_item <= 0) {  // (fp64 too since round 3: round 2 kept uniform items of 16 for it)
      const uint32_t ts = std::min<uint32_t>(spp, (uint32_t)((double)spp * auto_tail_frac(flat_prog) + 0.5));
      tail_chunk = std::min(chunk, auto_tail_chunk(flat_prog));
      for (;;) {
        k_bulk = (spp - ts) / chunk;  // bulk items cover [0, k_bulk * chunk)
        nchunks = k_bulk + (spp - k_bulk * chunk + tail_chunk - 1) / tail_chunk;
        if (nchunks <= kMaxItemsPerPixel || chunk >= spp) break;
        chunk = std::min(spp, 2 * chunk);
        tail_chunk = std::min(chunk, 2 * tail_chunk);
      }
    }
    // Passes: the item partial sums of a call are 3 R per (pixel, chunk) -- C5 fp64 (3840 x 2160 at 4096 spp,
    // 192 chunks) would need 38 GB. The chunks come in passes of `cpp` chunks whose partial sums fit
    // kPartialBudget (and whose items fit 32 bits); every pass is one launch, and its resolve adds its chunks
    // to the running per-pixel sums in chunk order (k_resolve), so the image is the same for any split.
    const uint64_t budget = (uint64_t)env_f64("RT_PARTIAL_BUDGET", (double)kPartialBudget);
    const uint64_t per_chunk = 3ull * sizeof(R) * npix;
    const uint32_t cpp = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>({(uint64_t)nchunks, budget / per_chunk, ((1ull << 31) - 1) / npix}));
    const uint32_t n_items = npix * cpp;  // items of the largest pass
    // the default schedule is persistent (k_persist); an explicit segments_per_launch selects the
    // launch-per-K-segments wavefront with HBM path state and live-slot compaction
    const bool persist = prm->segments_per_launch <= 0;
    const KernelFamily fam = kernel_family(hdr, cam->mode, persist, prm->traversal == RT_TRAV_ORDERED);
    if (!family_built(fam))
      return set_err(c, RT_ERR_UNSUPPORTED, std::string("this build (RT_DEV_ONLY) has no ") + family_name(fam) + " kernels");
    const bool ll = lamb_light_scene(hdr), nl = no_light_scene(hdr), lli = lamb_iso_light_scene(hdr);
    uint32_t P = prm->pool_slots > 0 ? (uint32_t)prm->pool_slots
                 : persist       ? kAutoPersistLanes
                                 : (f64 ? kAutoPool64 : kAutoPool32);
    P = std::max<uint32_t>(1, std::min(P, n_items));
    const uint32_t nblk_max = (P + kBlock - 1) / kBlock;

    // path state: 5 R4 arrays (O, D, T, L, A) + uint4 keys (S) + uint4 exclusion/pixel (X), each P long
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t r4 = al(sizeof(R4<R>) * (size_t)P), sb = al(16 * (size_t)P), xb = al(16 * (size_t)P);
    if (!persist) {
      if ((s = ensure(c, c->state, 5 * r4 + sb + xb)) != RT_OK) return s;
      if ((s = ensure(c, c->queue0, 4ull * P)) != RT_OK) return s;
      if ((s = ensure(c, c->queue1, 4ull * P)) != RT_OK) return s;
    }
    if ((s = ensure(c, c->partial, 3ull * n_items * sizeof(R))) != RT_OK) return s;
    c->last.passes += (nchunks + cpp - 1) / cpp;
    c->last.partial_bytes = 3ull * n_items * sizeof(R);
    const size_t pixmap_bytes = c->pixmap.bytes;
    if ((s = ensure(c, c->pixmap, 4ull * npix)) != RT_OK) return s;
    if (c->pixmap.bytes != pixmap_bytes) c->tiles_dev.clear();  // reallocated: the old map is gone
    if ((s = ensure(c, c->blk, 4ull * (nblk_max + 2))) != RT_OK) return s;
    const bool same_tiles = c->pixmap_for == c->pixmap.ptr && c->pixmap_npix == npix && c->tiles_dev.size() == tl.size() &&
                            std::memcmp(c->tiles_dev.data(), tl.data(), sizeof(uint4) * tl.size()) == 0;
    if (!same_tiles) {  // the pixel map of an unchanged tile list is still in pixmap
      if ((s = ensure(c, c->tiles, sizeof(uint4) * tl.size())) != RT_OK) return s;
      c->tiles_dev = tl;  // the copy's source outlives this call
      c->pixmap_for = c->pixmap.ptr;
      c->pixmap_npix = npix;
      RT_HIP(c, hipMemcpyAsync(c->tiles.ptr, c->tiles_dev.data(), sizeof(uint4) * tl.size(), hipMemcpyHostToDevice,
                               st));
      hipLaunchKernelGGL(k_pixmap, dim3((npix + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                         (const uint4*)c->tiles.ptr, (uint32_t)tl.size(), npix, (uint32_t*)c->pixmap.ptr);
    }

    unsigned char* sp = (unsigned char*)c->state.ptr;
    Params<R> p{};
    p.sc = dev_scene<R>(hdr, sbase);
    const uint32_t wide_need = hdr.wide_stack;
    constexpr uint32_t kWideLdsStack = wide_lds_stack<R>();
    if (hdr.has_wide && wide_need > kWideLdsStack) {
      // a deep wide tree: a spill area of (need - kWideLdsStack) entries for every lane the chip can hold
      int ncu = 0;
      RT_HIP(c, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
      const uint32_t lanes = (uint32_t)std::max(ncu, 1) * 2048u;  // 32 waves of 64 per CU at most
      if ((s = ensure(c, c->wide_spill, 4ull * (wide_need - kWideLdsStack) * lanes)) != RT_OK) return s;
      p.sc.wide_spill = (uint32_t*)c->wide_spill.ptr;
      p.sc.spill_lanes = lanes;
    }
    if (prm->traversal == RT_TRAV_ORDERED) p.sc.has_flat = p.sc.has_wide = 0;
    p.sc.cam64 = nullptr;  // set with the camera below (perspective only)
    p.O = (R4<R>*)sp;
    p.D = (R4<R>*)(sp + r4);
    p.T = (R4<R>*)(sp + 2 * r4);
    p.L = (R4<R>*)(sp + 3 * r4);
    p.A = (R4<R>*)(sp + 4 * r4);
    p.S = (uint4*)(sp + 5 * r4);
    p.X = (uint4*)(sp + 5 * r4 + sb);
    p.partial = (R*)c->partial.ptr;
    p.pixmap = (const uint32_t*)c->pixmap.ptr;
    p.queue = nullptr;
    p.n = P;
    p.P = P;
    p.npix = npix;
    div_magic(npix, p.npix_m, p.npix_k);
    p.n_items = n_items;
    p.chunk = chunk;
    p.k_bulk = k_bulk;
    p.tail_chunk = tail_chunk;
    p.spp = spp;
    p.first_sample = (uint32_t)std::max(0, prm->first_sample);
    p.W = (uint32_t)cam->image_width;
    p.max_depth = prm->max_depth;
    p.seed = prm->seed;
    c->cam_host = make_view(cam);
    if ((s = ensure(c, c->camx, sizeof(CamDev))) != RT_OK) return s;
    if (!c->cam_valid || std::memcmp(&c->cam_dev, &c->cam_host, sizeof(CamDev)) != 0) {
      RT_HIP(c, hipMemcpyAsync(c->camx.ptr, &c->cam_host, sizeof(CamDev), hipMemcpyHostToDevice, st));
      c->cam_dev = c->cam_host;
      c->cam_valid = true;
    }
    p.cam_mode = c->cam_host.mode;
    p.camx = (const CamDev*)c->camx.ptr;
    if (p.cam_mode == RT_CAM_PERSPECTIVE) p.sc.cam64 = p.camx;
    p.seg_shards = (unsigned long long*)c->counters.ptr;
    const int K = prm->segments_per_launch > 0 ? std::min(prm->segments_per_launch, 64) : kAutoSegments;
    p.K = K;
    uint64_t launches = 0, iters = 0;
    size_t ev = 0;
    if (c->timing && c->ev_used > 4096 && (s = settle(c)) != RT_OK) return s;  // bound the pending events
    const size_t ev0 = c->ev_used;
    if (persist) {
      if ((s = ensure(c, c->fault, 4)) != RT_OK) return s;
      p.persist = RT_PERSIST_MODE;
      p.fault = (uint32_t*)c->fault.ptr;
      if ((s = ensure(c, c->heads, 4ull * kHeads * kHeadStride)) != RT_OK) return s;
      p.heads = (uint32_t*)c->heads.ptr;
    }
    for (uint32_t c0 = 0; c0 < nchunks; c0 += cpp) {  // the passes (one for every BASELINE config but C5)
      const uint32_t pc = std::min(cpp, nchunks - c0);
      p.chunk0 = c0;
      p.n_items = npix * pc;
      if (persist) {
        // one launch of P lanes (pool_slots, or kAutoPersistLanes)
        RT_HIP(c, hipMemsetAsync(c->heads.ptr, 0, 4ull * kHeads * kHeadStride, st));
        const uint32_t grid = nblk_max;
        if (c->timing) {
          hipEvent_t e0 = take_event(c, ev0 + ev), e1 = take_event(c, ev0 + ev + 1);
          if (!e0 || !e1) return set_err(c, RT_ERR_HIP, "hipEventCreate failed");
          RT_HIP(c, hipEventRecord(e0, st));
          launch_step<R>(p, fam, ll, nl, lli, cs.stack_need, grid, st);
          RT_HIP(c, hipEventRecord(e1, st));
          ev += 2;
        } else {
          launch_step<R>(p, fam, ll, nl, lli, cs.stack_need, grid, st);
        }
        RT_HIP(c, hipGetLastError());
        c->last.grid_lanes = t_grid_lanes;
        launches++;
        iters++;
        // a fault is reported by the settle after this call (rt_stats, or a host-output render)
      } else {
        p.queue = nullptr;
        p.n = P;
        if (p.cam_mode != RT_CAM_PERSPECTIVE || p.sc.has_procedural)
          hipLaunchKernelGGL((k_init<R, true>), dim3(nblk_max), dim3(kBlock), 0, st, p);
        else
          hipLaunchKernelGGL((k_init<R, false>), dim3(nblk_max), dim3(kBlock), 0, st, p);
        launches++;
        uint32_t* qbuf[2] = {(uint32_t*)c->queue0.ptr, (uint32_t*)c->queue1.ptr};
        int qsel = 0;
        uint32_t* blk = (uint32_t*)c->blk.ptr;
        uint32_t* d_total = blk + nblk_max + 1;
        // every slot finishes within (items per slot) * chunk * max_depth segments; anything longer is a bug
        const uint64_t iter_cap =
            iters + (((uint64_t)(p.n_items + P - 1) / P) * chunk * (uint64_t)prm->max_depth + K - 1) / K + 4 * kBatch;
        for (;;) {
          if (iters > iter_cap) return set_err(c, RT_ERR_HIP, "wavefront did not drain (internal error)");
          const uint32_t grid = (p.n + kBlock - 1) / kBlock;
          for (int b = 0; b < kBatch; b++) {
            if (c->timing) {
              hipEvent_t e0 = take_event(c, ev0 + ev), e1 = take_event(c, ev0 + ev + 1);
              if (!e0 || !e1) return set_err(c, RT_ERR_HIP, "hipEventCreate failed");
              RT_HIP(c, hipEventRecord(e0, st));
              launch_step<R>(p, fam, ll, nl, lli, cs.stack_need, grid, st);
              RT_HIP(c, hipEventRecord(e1, st));
              ev += 2;
            } else {
              launch_step<R>(p, fam, ll, nl, lli, cs.stack_need, grid, st);
            }
            launches++;
            iters++;
          }
          RT_HIP(c, hipGetLastError());
          // live-slot count; compact into a queue once half the pool has finished
          hipLaunchKernelGGL(k_count, dim3(grid), dim3(kBlock), 0, st, (const void*)p.D, (int)f64, p.queue, p.n, blk);
          hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, blk, grid, d_total);
          launches += 2;
          RT_HIP(c, hipMemcpyAsync(c->total_host, d_total, 4, hipMemcpyDeviceToHost, st));
          RT_HIP(c, hipStreamSynchronize(st));
          uint32_t alive = *c->total_host;
          if (alive == 0) break;
          if (p.queue || alive * 2 <= p.P) {
            uint32_t* nq = qbuf[qsel];
            qsel ^= 1;
            hipLaunchKernelGGL(k_compact, dim3(grid), dim3(kBlock), 0, st, (const void*)p.D, (int)f64, p.queue, p.n,
                               (const uint32_t*)blk, nq);
            launches++;
            p.queue = nq;
            p.n = alive;
          }
        }
      }
      hipLaunchKernelGGL(k_resolve<R>, dim3((npix + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                         (const R*)c->partial.ptr, npix, pc, spp, (R*)dout, (int)(c0 == 0),
                         (int)(c0 + pc >= nchunks));
      launches++;
      RT_HIP(c, hipGetLastError());
    }
    // device output: nothing waits here -- the segment counters (cumulative on the device), the
    // timing events and the fault word are settled by rt_stats, rt_reset_counters or a host-output call
    c->ev_used = ev0 + ev;
    c->pending = true;
    c->pend_stream = st;
    c->last.samples += (uint64_t)npix * spp;
    c->last.iterations += iters;
    c->last.launches += launches;
  }
  if (!out_dev) {
    RT_HIP(c, hipMemcpyAsync(out, dout, out_elems * sizeof(R), hipMemcpyDeviceToHost, st));
    RT_HIP(c, hipStreamSynchronize(st));
    if ((s = settle(c)) != RT_OK) return s;
  }
  c->last.last_render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RT_OK;
}

}  // namespace

// ====================================================================== C ABI

extern "C" {

int32_t rt_abi_version(void) { return RT_ABI_VERSION; }

#define RT_STR2(x) #x
#define RT_STR(x) RT_STR2(x)
const char* rt_build_info(void) {
  return "dev_only=" RT_STR(RT_DEV_ONLY) " wide_top_n=" RT_STR(RT_WIDE_TOP_N) " wide_lds_stack=" RT_STR(RT_WIDE_LDS_STACK) " wide_waves_global=" RT_STR(RT_WIDE_WAVES_GLOBAL)
#ifdef RT_SECTION_CLOCKS
      " sections=1"
#endif
#ifdef RT_DEBUG_TRACE
      " trace=1"
#endif
#ifdef RT_PRECISE_F32
      " precise_f32=1"
#endif
      ;
}
#undef RT_STR
#undef RT_STR2

namespace {
// g_sincos_tab (rt_device.h sincos2pi, fp64): (sin, cos)(2 pi j / 1024) in long double, rounded once,
// copied to the device of the calling thread (every context's device; module globals are per device)
hipError_t sincos_table_init() {
  static double2 tab[kSinCosTab];
  static std::once_flag once;
  std::call_once(once, [] {
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int j = 0; j < kSinCosTab; j++) {
      const long double a = 2.0L * pi * (long double)j / (long double)kSinCosTab;
      tab[j] = make_double2((double)sinl(a), (double)cosl(a));
    }
  });
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sincos_tab), tab, sizeof(tab));
}
}  // namespace

rt_status rt_context_create(int32_t device, rt_context** out) {
  if (!out) return set_err(nullptr, RT_ERR_INVALID_ARGUMENT, "out is null");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    (void)hipGetLastError();
    return set_err(nullptr, RT_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  }
  if (device < 0 || device >= n) return set_err(nullptr, RT_ERR_INVALID_ARGUMENT, "device index out of range");
  if ((e = hipSetDevice(device)) != hipSuccess) return set_err(nullptr, RT_ERR_HIP, hipGetErrorString(e));
  if ((e = sincos_table_init()) != hipSuccess)
    return set_err(nullptr, RT_ERR_HIP, std::string("sin/cos table: ") + hipGetErrorString(e));
  auto* c = new rt_context;
  c->device = device;
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
    delete c;
    return set_err(nullptr, RT_ERR_HIP, hipGetErrorString(e));
  }
  if ((e = hipHostMalloc((void**)&c->total_host, 64 + 8 * kSegShards, hipHostMallocDefault)) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return set_err(nullptr, RT_ERR_HIP, hipGetErrorString(e));
  }
  if (ensure(c, c->counters, sizeof(unsigned long long) * kSegShards) != RT_OK || ensure(c, c->fault, 4) != RT_OK ||
      hipMemset(c->counters.ptr, 0, sizeof(unsigned long long) * kSegShards) != hipSuccess ||
      hipMemset(c->fault.ptr, 0, 4) != hipSuccess) {
    std::string m = c->err;
    rt_context_destroy(c);
    return set_err(nullptr, RT_ERR_OUT_OF_MEMORY, m);
  }
  *out = c;
  return RT_OK;
}

void rt_context_destroy(rt_context* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  // an outstanding device-output render still reads the buffers freed below (its fault word is
  // dropped with the context: nobody is left to report it to)
  if (c->pending) (void)hipStreamSynchronize(c->pend_stream);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->scene32, &c->scene64, &c->state, &c->partial, &c->pixmap, &c->queue0, &c->queue1, &c->blk, &c->wide_spill,
                    &c->out_tmp, &c->counters, &c->camx, &c->heads, &c->tiles, &c->fault})
    if (b->ptr) (void)hipFree(b->ptr);
  for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
  if (c->total_host) (void)hipHostFree(c->total_host);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* rt_last_error(const rt_context* c) {
  if (c) return c->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_create_err.c_str();
}

rt_status rt_scene_upload(rt_context* c, const rt_scene_desc* desc) {
  if (!c || !desc) return set_err(c, RT_ERR_INVALID_ARGUMENT, "null context or descriptor");
  RT_HIP(c, hipSetDevice(c->device));
  CompiledScene cs;
  std::string err;
  rt_status s = compile_scene(desc, &cs, &err);
  if (s != RT_OK) return set_err(c, s, err);
  // renders still pending on any stream read the current scene buffers
  if (c->pending) RT_HIP(c, hipStreamSynchronize(c->pend_stream));
  if ((s = ensure(c, c->scene32, cs.blob32.size())) != RT_OK) return s;
  if ((s = ensure(c, c->scene64, cs.blob64.size())) != RT_OK) return s;
  c->scene = std::move(cs);  // copied to the device by the next render, on its stream (render<R>)
  c->scene_dirty32 = c->scene_dirty64 = true;
  c->has_scene = true;
  return RT_OK;
}

rt_status rt_scene_check(const rt_scene_desc* desc, rt_scene_info* info, char* err, int32_t errlen) {
  CompiledScene cs;
  std::string m;
  rt_status s = desc ? compile_scene(desc, &cs, &m) : RT_ERR_INVALID_ARGUMENT;
  if (!desc) m = "null descriptor";
  if (s == RT_OK) {  // the kernels a perspective render on the default (persistent) schedule would take
    const KernelFamily fam = kernel_family(cs.hdr, RT_CAM_PERSPECTIVE, true, false);
    if (!family_built(fam)) {
      s = RT_ERR_UNSUPPORTED;
      m = std::string("this build (RT_DEV_ONLY) has no ") + family_name(fam) + " kernels";
    }
  }
  if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", m.c_str());
  if (s == RT_OK && info) {
    const SceneHeader& h = cs.hdr;
    info->quads = cs.desc_quads;
    info->flat_quads = cs.flat_quads;
    info->flat_boxes = cs.flat_boxes;
    info->wide_nodes = cs.hdr.has_wide ? (int32_t)cs.hdr.n_wnodes : 0;
    info->wide_stack = cs.hdr.has_wide ? (int32_t)cs.hdr.wide_stack : 0;
    info->wide_kinds = cs.hdr.has_wide ? (int32_t)cs.hdr.wide_kinds : 0;
    info->wide_prim_words = cs.hdr.has_wide ? (int32_t)cs.hdr.n_wprim_words : 0;
    info->wide_big = cs.hdr.has_wide ? (int32_t)cs.hdr.wide_big : 0;
    info->spheres = (int32_t)h.n_spheres;
    info->triangles = (int32_t)h.n_tris;
    info->instances = h.num_instances;
    info->volumes = (int32_t)h.n_volumes;
    info->bvh_nodes = (int32_t)h.n_nodes;
    info->linear_ops = (int32_t)h.n_linear;
    info->stack_need = cs.stack_need;
    info->bytes_f32 = cs.blob32.size();
    info->bytes_f64 = cs.blob64.size();
  }
  return s;
}

rt_status rt_render_tiles(rt_context* c, const rt_camera_desc* cam, const rt_render_params* prm, const rt_tile* tiles,
                          int32_t ntiles, void* out_rgb, int32_t out_is_device, void* stream) {
  if (!c) return set_err(nullptr, RT_ERR_INVALID_ARGUMENT, "null context");
  if (!cam || !prm || (!tiles && ntiles > 0) || ntiles < 0 || (!out_rgb && ntiles > 0))
    return set_err(c, RT_ERR_INVALID_ARGUMENT, "null argument");
  if (!c->has_scene) return set_err(c, RT_ERR_NO_SCENE, "rt_scene_upload has not succeeded on this context");
  if (cam->mode < RT_CAM_PERSPECTIVE || cam->mode > RT_CAM_LENS)
    return set_err(c, RT_ERR_INVALID_ARGUMENT, "unknown camera mode");
  if (cam->image_width <= 0 || cam->image_height <= 0) return set_err(c, RT_ERR_INVALID_ARGUMENT, "empty image");
  if (cam->image_width > 65535 || cam->image_height > 65535)  // pixel positions are packed x | y << 16
    return set_err(c, RT_ERR_INVALID_ARGUMENT, "image wider or taller than 65535 pixels");
  if (prm->spp <= 0) return set_err(c, RT_ERR_INVALID_ARGUMENT, "spp must be positive");
  if (prm->precision != RT_PREC_F32 && prm->precision != RT_PREC_F64)
    return set_err(c, RT_ERR_INVALID_ARGUMENT, "unknown precision");
  for (int t = 0; t < ntiles; t++) {
    const rt_tile& tl = tiles[t];
    if (tl.x0 < 0 || tl.y0 < 0 || tl.width < 0 || tl.height < 0 || tl.x0 + tl.width > cam->image_width ||
        tl.y0 + tl.height > cam->image_height)
      return set_err(c, RT_ERR_INVALID_ARGUMENT, "tile " + std::to_string(t) + " outside the image");
  }
  RT_HIP(c, hipSetDevice(c->device));
  // Device output: NULL is the HIP null stream (torch's default stream), so work the caller queues
  // after this call on that stream -- a clone, a gather -- is ordered after the render. Host output
  // (the call returns the finished image): NULL is the context's own non-blocking stream, so contexts
  // driven from different host threads do not serialise on the null stream.
  hipStream_t st = (stream == nullptr && !out_is_device) ? c->stream : (hipStream_t)stream;
  try {
    if (prm->precision == RT_PREC_F64) return render<double>(c, cam, prm, tiles, ntiles, out_rgb, out_is_device, st);
    return render<float>(c, cam, prm, tiles, ntiles, out_rgb, out_is_device, st);
  } catch (const std::bad_alloc&) {
    return set_err(c, RT_ERR_OUT_OF_MEMORY, "out of host memory");
  } catch (const std::exception& e) {
    return set_err(c, RT_ERR_INVALID_ARGUMENT, e.what());
  }
}

rt_status rt_stats(rt_context* c, rt_counters* out) {
  if (!c || !out) return set_err(c, RT_ERR_INVALID_ARGUMENT, "null argument");
  RT_HIP(c, hipSetDevice(c->device));
  const rt_status s = settle(c);
  *out = c->last;
  return s;
}

rt_status rt_reset_counters(rt_context* c) {
  if (!c) return set_err(nullptr, RT_ERR_INVALID_ARGUMENT, "null context");
  RT_HIP(c, hipSetDevice(c->device));
  const rt_status s = settle(c);  // nothing of this context is outstanding after it
  RT_HIP(c, hipMemsetAsync(c->counters.ptr, 0, sizeof(unsigned long long) * kSegShards, c->stream));
  if (c->fault.ptr) RT_HIP(c, hipMemsetAsync(c->fault.ptr, 0, 4, c->stream));
  RT_HIP(c, hipStreamSynchronize(c->stream));
  c->last = rt_counters{};
  return s;
}

rt_status rt_set_timing(rt_context* c, int32_t enable) {
  if (!c) return set_err(nullptr, RT_ERR_INVALID_ARGUMENT, "null context");
  c->timing = enable ? 1 : 0;
  return RT_OK;
}

#ifdef RT_ITEM_CLOCKS
// development build only (scripts/dev_item_clocks.py): where the persistent kernels write item durations
int rt_dev_set_item_clocks(void* dev_ptr) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_item_clk), &dev_ptr, sizeof(void*)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef RT_SECTION_CLOCKS
// development build only (scripts/dev_sections.py): read and clear the section clocks
int rt_dev_section_clocks(unsigned long long out[7]) {
  const unsigned long long z[4] = {0, 0, 0, 0};
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_section_clocks), sizeof(unsigned long long) * 4);
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 4, HIP_SYMBOL(rtd::g_trace_totals), sizeof(unsigned long long) * 3);
  // each symbol is cleared with its own size (g_section_clocks: 4 entries, g_trace_totals: 3)
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_section_clocks), z, sizeof(unsigned long long) * 4);
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(rtd::g_trace_totals), z, sizeof(unsigned long long) * 3);
  return e == hipSuccess ? 0 : -1;
}
// the wide kernels' wave-level counts (rt_device.h g_wide_stats), read and cleared
void rt_dev_wide_stats(unsigned long long out[10]) {
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(rtd::g_wide_stats), sizeof(unsigned long long) * 10);
  unsigned long long z[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(rtd::g_wide_stats), z, sizeof(z));
}
#endif

uint32_t rt_rng_u32(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t dim) {
  return draw_u32(key_path(key_pixel(seed, pixel), key_sample(seed, sample)), dim);
}

}  // extern "C"
