// rt_multi.hip -- the multi-GPU driver of include/rt_hip.h (rt_multi_*).
//
// The reference parallelises camera::render over image rows with
// std::for_each(std::execution::par_unseq) (camera.h:154-172). Here the framebuffer is cut
// into tiles dealt round-robin over the GPUs of one node: every device
// has its own rt_context (scene replicated, KB-sized) and renders its tiles into a padded
// buffer on its own stream; one ncclGather (RCCL, single-process communicator from
// ncclCommInitAll) collects the buffers on the first device, where k_unpack scatters them into
// the linear framebuffer that is copied to the host. Renders of all devices are queued before
// the gather, so the GPUs work concurrently; the gather is ordered after each device's render
// by its stream.
//
// RCCL is loaded with dlopen when a communicator is first needed, so single-GPU users of
// librt_hip.so never map it. A device list that repeats a device cannot form a communicator
// (RCCL refuses duplicate GPUs): those ranks gather with device copies, which lets the
// multi-rank plan and unpack run on a one-GPU box.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"

namespace {

constexpr int kUnpackBlock = 256;
constexpr uint32_t kPad = 0xFFFFFFFFu;

// gathered[i] (rank-major: rank r's packed pixel j at r * maxpix + j) -> fb[gidx[i]]
template <class R>
__global__ __launch_bounds__(kUnpackBlock) void k_unpack(const R* gathered, const uint32_t* gidx, uint64_t n, R* fb) {
  const uint64_t i = blockIdx.x * (uint64_t)kUnpackBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = gidx[i];
  if (g == kPad) return;
  fb[3ull * g] = gathered[3 * i];
  fb[3ull * g + 1] = gathered[3 * i + 1];
  fb[3ull * g + 2] = gathered[3 * i + 2];
}

// The RCCL entry points this driver uses (rccl.h), resolved from librccl.so.1.
struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
  std::string err;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("cannot load RCCL: ") + (e ? e : "?");
      return;
    }
    r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.init_all && r.destroy && r.gather && r.group_start && r.group_end && r.error_string;
    if (!r.ok) r.err = "librccl lacks ncclCommInitAll / ncclGather / ncclGroupStart";
  });
  return r;
}

std::mutex g_multi_err_mu;
std::string g_multi_create_err;
std::atomic<uint64_t> g_comm_inits{0};  // ncclCommInitAll calls (rt_multi_comm_inits)

}  // namespace

struct rt_multi {
  std::vector<int32_t> devs;
  std::vector<rt_context*> ctx;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> done;  // per rank: its render (and, copy gather, its buffer) is complete
  bool use_rccl = false;
  std::vector<ncclComm_t> comms;
  std::string err;
  // per rank send buffers on its device; rank 0 renders in place into recv's first segment
  std::vector<void*> send;
  std::vector<size_t> send_bytes;
  void* recv = nullptr;  // n * maxpix * 3 elements on devs[0]
  size_t recv_bytes = 0;
  void* fb = nullptr;  // W * H * 3 elements on devs[0]
  size_t fb_bytes = 0;
  uint32_t* gidx = nullptr;  // n * maxpix global pixel indices (kPad for padding) on devs[0]
  size_t gidx_bytes = 0;
  int32_t plan_w = -1, plan_h = -1, plan_ts = -1;
  hipEvent_t g0 = nullptr, g1 = nullptr;  // gather + unpack timing on devs[0]
  double gather_ms = 0;
};

namespace {

rt_status merr(rt_multi* m, rt_status s, const std::string& msg) {
  if (m) {
    m->err = msg;
  } else {
    std::lock_guard<std::mutex> lk(g_multi_err_mu);
    g_multi_create_err = msg;
  }
  return s;
}

#define MHIP(m, call)                                                                         \
  do {                                                                                        \
    hipError_t e_ = (call);                                                                   \
    if (e_ != hipSuccess) return merr((m), RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define MNCCL(m, call)                                                                                 \
  do {                                                                                                 \
    ncclResult_t r_ = (call);                                                                          \
    if (r_ != ncclSuccess) return merr((m), RT_ERR_HIP, std::string(#call) + ": " + rccl().error_string(r_)); \
  } while (0)

// tiles of one rank: all tiles row-major over the image, every ndev-th from `rank`
std::vector<rt_tile> plan_rank(int32_t W, int32_t H, int32_t n, int32_t ts, int32_t rank) {
  std::vector<rt_tile> out;
  int64_t k = 0;
  for (int32_t y = 0; y < H; y += ts)
    for (int32_t x = 0; x < W; x += ts, k++)
      if (k % n == rank) out.push_back({x, y, std::min(ts, W - x), std::min(ts, H - y)});
  return out;
}

// Grow a buffer on device `dev`. rt_multi_render returns with every rank's stream drained, so only
// the streams of this rt_multi on that device can still hold work touching it: wait for those, not
// for the whole device (other contexts on it keep running).
rt_status ensure_dev(rt_multi* m, int dev, void*& p, size_t& have, size_t want) {
  if (p && have >= want) return RT_OK;
  MHIP(m, hipSetDevice(dev));
  if (p) {
    for (size_t r = 0; r < m->devs.size(); r++)
      if (m->devs[r] == dev && m->streams[r]) MHIP(m, hipStreamSynchronize(m->streams[r]));
    MHIP(m, hipFree(p));
    p = nullptr;
    have = 0;
  }
  want = std::max<size_t>(want, 256);
  if (hipMalloc(&p, want) != hipSuccess) {
    p = nullptr;
    (void)hipGetLastError();
    return merr(m, RT_ERR_OUT_OF_MEMORY, "hipMalloc(" + std::to_string(want) + ") on device " + std::to_string(dev));
  }
  have = want;
  return RT_OK;
}

}  // namespace

extern "C" {

int32_t rt_multi_plan(int32_t width, int32_t height, int32_t ndev, int32_t tile_size, int32_t rank,
                      rt_tile* tiles_out, int32_t cap) {
  if (width <= 0 || height <= 0 || ndev <= 0 || rank < 0 || rank >= ndev || cap < 0) return -1;
  const int32_t ts = tile_size > 0 ? tile_size : 16;
  const std::vector<rt_tile> t = plan_rank(width, height, ndev, ts, rank);
  if (tiles_out)
    for (int32_t i = 0; i < (int32_t)t.size() && i < cap; i++) tiles_out[i] = t[i];
  return (int32_t)t.size();
}

const char* rt_multi_last_error(const rt_multi* m) {
  if (m) return m->err.c_str();
  std::lock_guard<std::mutex> lk(g_multi_err_mu);
  return g_multi_create_err.c_str();
}

int32_t rt_multi_uses_rccl(const rt_multi* m) { return m && m->use_rccl ? 1 : 0; }

uint64_t rt_multi_comm_inits(void) { return g_comm_inits.load(); }

void rt_multi_destroy(rt_multi* m) {
  if (!m) return;
  for (size_t r = 0; r < m->devs.size(); r++) {
    (void)hipSetDevice(m->devs[r]);
    if (r < m->streams.size() && m->streams[r]) (void)hipStreamSynchronize(m->streams[r]);
  }
  for (ncclComm_t c : m->comms)
    if (c) (void)rccl().destroy(c);
  for (size_t r = 0; r < m->devs.size(); r++) {
    (void)hipSetDevice(m->devs[r]);
    if (r > 0 && r < m->send.size() && m->send[r]) (void)hipFree(m->send[r]);
    if (r < m->done.size() && m->done[r]) (void)hipEventDestroy(m->done[r]);
    if (r < m->streams.size() && m->streams[r]) (void)hipStreamDestroy(m->streams[r]);
    if (r < m->ctx.size() && m->ctx[r]) rt_context_destroy(m->ctx[r]);
  }
  if (!m->devs.empty()) {
    (void)hipSetDevice(m->devs[0]);
    for (void* p : {m->recv, m->fb, (void*)m->gidx})
      if (p) (void)hipFree(p);
    if (m->g0) (void)hipEventDestroy(m->g0);
    if (m->g1) (void)hipEventDestroy(m->g1);
  }
  delete m;
}

rt_status rt_multi_create(const int32_t* devices, int32_t ndev, rt_multi** out) {
  if (!out || !devices || ndev <= 0) return merr(nullptr, RT_ERR_INVALID_ARGUMENT, "null argument or ndev <= 0");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    (void)hipGetLastError();
    return merr(nullptr, RT_ERR_NO_DEVICE, "no HIP device");
  }
  for (int32_t r = 0; r < ndev; r++)
    if (devices[r] < 0 || devices[r] >= count)
      return merr(nullptr, RT_ERR_INVALID_ARGUMENT, "device " + std::to_string(devices[r]) + " out of range");
  auto* m = new rt_multi;
  m->devs.assign(devices, devices + ndev);
  m->ctx.assign(ndev, nullptr);
  m->streams.assign(ndev, nullptr);
  m->done.assign(ndev, nullptr);
  m->send.assign(ndev, nullptr);
  m->send_bytes.assign(ndev, 0);
  auto fail = [&](rt_status s, const std::string& msg) {
    rt_multi_destroy(m);
    return merr(nullptr, s, msg);
  };
  for (int32_t r = 0; r < ndev; r++) {
    if (rt_context_create(m->devs[r], &m->ctx[r]) != RT_OK) return fail(RT_ERR_HIP, rt_last_error(nullptr));
    if (hipSetDevice(m->devs[r]) != hipSuccess ||
        hipStreamCreateWithFlags(&m->streams[r], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&m->done[r], hipEventDisableTiming) != hipSuccess)
      return fail(RT_ERR_HIP, "stream/event creation failed on device " + std::to_string(m->devs[r]));
  }
  if (hipSetDevice(m->devs[0]) != hipSuccess || hipEventCreate(&m->g0) != hipSuccess ||
      hipEventCreate(&m->g1) != hipSuccess)
    return fail(RT_ERR_HIP, "event creation failed");
  const bool distinct = std::set<int32_t>(m->devs.begin(), m->devs.end()).size() == m->devs.size();
  if (distinct) {
    const Rccl& R = rccl();
    if (!R.ok) return fail(RT_ERR_UNSUPPORTED, R.err);
    m->comms.assign(ndev, nullptr);
    const ncclResult_t nr = R.init_all(m->comms.data(), ndev, m->devs.data());
    g_comm_inits.fetch_add(1);
    if (nr != ncclSuccess) {
      m->comms.clear();
      return fail(RT_ERR_HIP, std::string("ncclCommInitAll: ") + R.error_string(nr));
    }
    m->use_rccl = true;
  }
  *out = m;
  return RT_OK;
}

rt_status rt_multi_scene_upload(rt_multi* m, const rt_scene_desc* desc) {
  if (!m || !desc) return merr(m, RT_ERR_INVALID_ARGUMENT, "null argument");
  for (size_t r = 0; r < m->ctx.size(); r++) {
    const rt_status s = rt_scene_upload(m->ctx[r], desc);
    if (s != RT_OK) return merr(m, s, "rank " + std::to_string(r) + ": " + rt_last_error(m->ctx[r]));
  }
  return RT_OK;
}

rt_status rt_multi_render(rt_multi* m, const rt_camera_desc* cam, const rt_render_params* prm, int32_t tile_size,
                          void* out_rgb) {
  if (!m || !cam || !prm || !out_rgb) return merr(m, RT_ERR_INVALID_ARGUMENT, "null argument");
  if (prm->precision != RT_PREC_F32 && prm->precision != RT_PREC_F64)
    return merr(m, RT_ERR_INVALID_ARGUMENT, "unknown precision");
  const int32_t W = cam->image_width, H = cam->image_height, n = (int32_t)m->devs.size();
  if (W <= 0 || H <= 0) return merr(m, RT_ERR_INVALID_ARGUMENT, "empty image");
  const int32_t ts = tile_size > 0 ? tile_size : 16;
  const bool f64 = prm->precision == RT_PREC_F64;
  const size_t elem = f64 ? sizeof(double) : sizeof(float);

  std::vector<std::vector<rt_tile>> tiles(n);
  uint64_t maxpix = 1;
  for (int32_t r = 0; r < n; r++) {
    tiles[r] = plan_rank(W, H, n, ts, r);
    uint64_t c = 0;
    for (const rt_tile& t : tiles[r]) c += (uint64_t)t.width * t.height;
    maxpix = std::max(maxpix, c);
  }
  const uint64_t nslots = (uint64_t)n * maxpix;
  rt_status s;
  if ((s = ensure_dev(m, m->devs[0], m->recv, m->recv_bytes, nslots * 3 * elem)) != RT_OK) return s;
  if ((s = ensure_dev(m, m->devs[0], m->fb, m->fb_bytes, (size_t)W * H * 3 * elem)) != RT_OK) return s;
  if (m->plan_w != W || m->plan_h != H || m->plan_ts != ts || m->gidx_bytes < nslots * 4) {
    // where every gathered pixel goes (tiles packed in order, row-major inside a tile)
    std::vector<uint32_t> g(nslots, kPad);
    for (int32_t r = 0; r < n; r++) {
      uint64_t j = (uint64_t)r * maxpix;
      for (const rt_tile& t : tiles[r])
        for (int32_t y = t.y0; y < t.y0 + t.height; y++)
          for (int32_t x = t.x0; x < t.x0 + t.width; x++) g[j++] = (uint32_t)((uint64_t)y * W + x);
    }
    void* gp = m->gidx;
    if ((s = ensure_dev(m, m->devs[0], gp, m->gidx_bytes, nslots * 4)) != RT_OK) return s;
    m->gidx = (uint32_t*)gp;
    MHIP(m, hipSetDevice(m->devs[0]));
    MHIP(m, hipMemcpy(m->gidx, g.data(), nslots * 4, hipMemcpyHostToDevice));
    m->plan_w = W;
    m->plan_h = H;
    m->plan_ts = ts;
  }
  // every rank's render, queued on its own stream (asynchronous: device output)
  for (int32_t r = 0; r < n; r++) {
    void* dst;
    if (r == 0) {
      dst = m->recv;  // in place: ncclGather's root segment 0
    } else {
      if ((s = ensure_dev(m, m->devs[r], m->send[r], m->send_bytes[r], maxpix * 3 * elem)) != RT_OK) return s;
      dst = m->send[r];
    }
    MHIP(m, hipSetDevice(m->devs[r]));
    s = rt_render_tiles(m->ctx[r], cam, prm, tiles[r].data(), (int32_t)tiles[r].size(), dst, 1, m->streams[r]);
    if (s != RT_OK) return merr(m, s, "rank " + std::to_string(r) + ": " + rt_last_error(m->ctx[r]));
  }
  MHIP(m, hipSetDevice(m->devs[0]));
  MHIP(m, hipEventRecord(m->g0, m->streams[0]));
  const size_t count = (size_t)maxpix * 3;
  if (m->use_rccl) {
    const Rccl& R = rccl();
    MNCCL(m, R.group_start());
    for (int32_t r = 0; r < n; r++) {
      const void* sb = r == 0 ? m->recv : m->send[r];
      MNCCL(m, R.gather(sb, r == 0 ? m->recv : nullptr, count, f64 ? ncclFloat64 : ncclFloat32, 0, m->comms[r],
                        m->streams[r]));
    }
    MNCCL(m, R.group_end());
  } else {
    for (int32_t r = 1; r < n; r++) {
      MHIP(m, hipSetDevice(m->devs[r]));
      MHIP(m, hipEventRecord(m->done[r], m->streams[r]));
      MHIP(m, hipSetDevice(m->devs[0]));
      MHIP(m, hipStreamWaitEvent(m->streams[0], m->done[r], 0));
      MHIP(m, hipMemcpyPeerAsync((char*)m->recv + (size_t)r * count * elem, m->devs[0], m->send[r], m->devs[r],
                                 count * elem, m->streams[0]));
    }
  }
  MHIP(m, hipSetDevice(m->devs[0]));
  const unsigned blocks = (unsigned)((nslots + kUnpackBlock - 1) / kUnpackBlock);
  if (f64)
    hipLaunchKernelGGL(k_unpack<double>, dim3(blocks), dim3(kUnpackBlock), 0, m->streams[0], (const double*)m->recv,
                       (const uint32_t*)m->gidx, nslots, (double*)m->fb);
  else
    hipLaunchKernelGGL(k_unpack<float>, dim3(blocks), dim3(kUnpackBlock), 0, m->streams[0], (const float*)m->recv,
                       (const uint32_t*)m->gidx, nslots, (float*)m->fb);
  MHIP(m, hipGetLastError());
  MHIP(m, hipEventRecord(m->g1, m->streams[0]));
  MHIP(m, hipMemcpyAsync(out_rgb, m->fb, (size_t)W * H * 3 * elem, hipMemcpyDeviceToHost, m->streams[0]));
  MHIP(m, hipStreamSynchronize(m->streams[0]));
  float ms = 0;
  MHIP(m, hipEventElapsedTime(&ms, m->g0, m->g1));
  m->gather_ms = ms;
  // settle every rank: waits for its stream and reports a device-side fault of its render
  for (int32_t r = 0; r < n; r++) {
    rt_counters c{};
    if ((s = rt_stats(m->ctx[r], &c)) != RT_OK)
      return merr(m, s, "rank " + std::to_string(r) + ": " + rt_last_error(m->ctx[r]));
  }
  return RT_OK;
}

rt_status rt_multi_stats(rt_multi* m, int32_t rank, rt_counters* out) {
  if (!m || !out || rank < 0 || rank >= (int32_t)m->ctx.size())
    return merr(m, RT_ERR_INVALID_ARGUMENT, "null argument or rank out of range");
  const rt_status s = rt_stats(m->ctx[rank], out);
  if (s != RT_OK) return merr(m, s, rt_last_error(m->ctx[rank]));
  out->aux_ms = rank == 0 ? m->gather_ms : 0.0;
  return RT_OK;
}

}  // extern "C"
