// smax_runtime.cpp -- host runtime behind the host-table entry points of
// include/gt_smax_hip.h (gt_smax_hip_enumerate / _to_buffer), the drop-in
// replacement of gt_esa_bottomup driving the smax visitor
// (src/match/esa-bottomup.c:116-273, src/match/esa_visitor_rep.h:46-51).
//
// One call: validate the borrowed .lcp/.llv/.bwt tables, split the suffix
// rows [1, N) into num_gpus shards, and give each used
// device one host thread that
//   1. stages its shards' tables into HBM through the device's persistent
//      pinned ring (threaded host fill overlapping the DMA); the .bwt bytes
//      are packed to their bit planes during the fill (0.5 B/row over PCIe
//      and in HBM instead of 1 B/row), so no pass over byte BWT is left for
//      the device;
//   2. creates and runs each shard's plan (K1 -> K1b + block sums -> K3, see
//      smax_kernels.hip) on the device's stream;
//   3. exchanges the 152-byte boundary records: an RCCL all-gather over the
//      used devices (ncclAllGather on a communicator the library creates
//      with ncclCommInitAll, cached for the process), or device-to-device
//      copies when one device holds every shard; then the device stitch
//      (smax_stitch_kernel) appends each shard's cross-shard interval;
//   4. copies its shards' records to the caller's triple array at their
//      global offsets (pinned ring, threaded conversion to (lcp, lb, rb)).
// Callbacks then run on the calling thread in ascending lb, as the
// reference's single-threaded traversal calls them.
//
// Device memory (tables, plan buffers) comes from a per-device caching
// allocator and pinned staging buffers live for the process, so repeated
// calls do not pay hipMalloc/hipHostMalloc of multi-GB buffers per call (a
// freed block is reused only after its device has finished the work queued
// before the free, smax_dev_free);
// gt_smax_release_cache() returns everything (GT_SMAX_NO_CACHE=1: free
// before return).
#include <dlfcn.h>
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gt_smax_hip.h"
#include "smax_internal.h"

namespace {

void seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
  if (errbuf == NULL || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

std::string hipmsg(const char *what, hipError_t e) {
  char b[256];
  snprintf(b, sizeof b, "%s: %s", what, hipGetErrorString(e));
  return b;
}

bool env_on(const char *name) {
  const char *v = getenv(name);
  return v != NULL && *v && strcmp(v, "0") != 0;
}

// ------------------------------------------------------------ device cache

}  // namespace

// helper threads' own plans (warm_kernels) keep out of the call's phase list
static thread_local bool t_phase_mute = false;

// A freed block's fence: events recorded on the streams whose work may still
// use it (or the whole device); the allocation that hands the block out
// again waits for them once.  Reference-counted by the blocks holding it.
struct SmaxFence {
  int device = -1;
  bool whole_device = false;
  std::vector<hipEvent_t> ev;
  std::atomic<int> refs{1};
  std::mutex mu;
  bool waited = false;
  hipError_t result = hipSuccess;
  hipError_t wait() {   // on any thread; restores its device
    std::lock_guard<std::mutex> g(mu);
    if (waited) return result;
    int cur = -1;
    (void) hipGetDevice(&cur);
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess && whole_device) e = hipDeviceSynchronize();
    for (size_t i = 0; e == hipSuccess && i < ev.size(); i++) e = hipEventSynchronize(ev[i]);
    if (cur >= 0) (void) hipSetDevice(cur);
    result = e;
    waited = true;
    return e;
  }
  ~SmaxFence() {
    int cur = -1;
    (void) hipGetDevice(&cur);
    (void) hipSetDevice(device);
    for (hipEvent_t e : ev) (void) hipEventDestroy(e);
    if (cur >= 0) (void) hipSetDevice(cur);
  }
};

namespace {

struct IdleBlock {
  void *ptr;
  SmaxFence *fence;   // null: no work pending on it
};

void fence_unref(SmaxFence *f) {
  if (f != nullptr && f->refs.fetch_sub(1) == 1) delete f;
}

struct Pool {
  std::mutex mu;
  std::unordered_map<void *, std::pair<int, size_t>> live;   // ptr -> (device, bytes)
  std::multimap<std::pair<int, size_t>, IdleBlock> idle;     // (device, bytes) -> block
};
Pool &pool() {
  static Pool *p = new Pool;   // never destroyed: frees may come from atexit paths
  return *p;
}

size_t round_block(size_t bytes) {
  if (bytes == 0) return 256;
  if (bytes < (1u << 20)) return (bytes + 255) & ~(size_t) 255;
  return (bytes + (2u << 20) - 1) & ~(size_t) ((2u << 20) - 1);
}

void release_idle(int device) {   // pool.mu held
  Pool &P = pool();
  int cur = -1;
  (void) hipGetDevice(&cur);
  for (auto it = P.idle.begin(); it != P.idle.end();) {
    if (device >= 0 && it->first.first != device) { ++it; continue; }
    (void) hipSetDevice(it->first.first);
    if (it->second.fence) (void) it->second.fence->wait();
    (void) hipFree(it->second.ptr);
    fence_unref(it->second.fence);
    it = P.idle.erase(it);
  }
  if (cur >= 0) (void) hipSetDevice(cur);
}

// ------------------------------------------------------------ timing

// ------------------------------------------------------------ per device

// pinned staging chunk (bytes): 16 MiB, GT_SMAX_STAGE_MB overrides.  A
// first call waits for the ring's chunks to be pinned (~4-5 GB/s): at C3 its
// median over five fresh processes was 0.137 s with 16 MiB chunks against
// 0.170 s with 64, the warm second call the same (0.096 / 0.097 s,
// profiles/s7/stage_mb_sweep_c3.txt)
uint64_t stage_bytes() {
  static const uint64_t b = [] {
    const char *v = getenv("GT_SMAX_STAGE_MB");
    const uint64_t mb = v ? strtoull(v, NULL, 0) : 16;
    return (mb < 1 ? 1 : mb > 1024 ? 1024 : mb) << 20;
  }();
  return b;
}
#define kStage stage_bytes()

// pinned chunks in the H2D ring: 3 (with the interleaved upload the planes'
// CPU-bound fill overlaps two queued LCP chunks; warm h2d of the C3 tables
// 76-79 ms against 83+ with 2, profiles/r04o/e2e_ring_sweep_c3.json),
// GT_SMAX_RING (2..4) overrides
constexpr int kRingMax = 4;
int ring_depth() {
  static const int r = [] {
    const char *v = getenv("GT_SMAX_RING");
    const long d = v ? strtol(v, NULL, 0) : 3;
    return (int) (d < 2 ? 2 : d > kRingMax ? kRingMax : d);
  }();
  return r;
}

struct DevCtx {
  int device = -1;
  std::mutex mu;                 // one call at a time uses the ring
  hipStream_t stream = nullptr;
  void *pin[kRingMax] = {};
  hipEvent_t ev[kRingMax] = {};
  // chunk 0 is pinned with the context, the others one after another on a
  // helper thread while the first chunks fill and drain (a first call pays
  // one chunk's pinning up front); chunk_ready(c, i) waits for chunk i,
  // ring_ready for all of them.  (Pinning beside the stream creation, one
  // thread per chunk, made the context 45-68 ms instead of 24-36:
  // profiles/r04o/e2e_ring_sweep_c3.json)
  std::promise<hipError_t> pinned[kRingMax];
  std::shared_future<hipError_t> pin_done[kRingMax];
  // every kernel of a plan launched once in this process (warm_kernels)
  std::atomic<bool> kernels_warm{false};
};

hipError_t chunk_ready(DevCtx *c, int i) {
  return c->pin_done[i].valid() ? c->pin_done[i].get() : hipSuccess;
}
hipError_t ring_ready(DevCtx *c) {
  hipError_t e = hipSuccess;
  for (int i = 0; i < ring_depth(); i++) {
    const hipError_t r = chunk_ready(c, i);
    if (e == hipSuccess) e = r;
  }
  return e;
}
// A chunk whose pinning failed (pinned-memory pressure) shrinks the ring to
// the chunks pinned before it instead of failing every later transfer on
// the device: chunk 0 is pinned with the context, the helper stops at its
// first failure, so the usable chunks are always a prefix.
bool chunk_usable(DevCtx *c, int i) { return chunk_ready(c, i) == hipSuccess && c->pin[i] != nullptr; }
// ring slot of the k-th chunk of an upload: the first R chunks take fresh
// slots as their pinning completes (R drops to the pinned prefix on a
// failure), later ones wait for the slot's previous DMA
hipError_t ring_slot(DevCtx *c, uint64_t k, uint64_t &R, int *slot) {
  if (k < R) {
    if (chunk_usable(c, (int) k)) {
      *slot = (int) k;
      return hipSuccess;
    }
    R = k;   // >= 1
  }
  *slot = (int) (k % R);
  return hipEventSynchronize(c->ev[*slot]);
}
// download buffers: 2 (chunk k+1's DMA beside chunk k's copy-out), 1 when
// the second chunk could not be pinned
int d2h_buffers(DevCtx *c, uint64_t nch) {
  if (nch <= 1 || ring_depth() < 2) return 1;
  return chunk_usable(c, 1) ? 2 : 1;
}

std::mutex g_ctx_mu;
std::map<int, DevCtx *> g_ctx;

hipError_t ctx_get(int device, DevCtx **out) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  auto it = g_ctx.find(device);
  if (it != g_ctx.end()) { *out = it->second; return hipSuccess; }
  DevCtx *c = new DevCtx;
  c->device = device;
  double tc = smax_phase_clock();
  hipError_t e = hipSetDevice(device);
  smax_phase_mark(" ctx.device", &tc);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  for (int i = 0; i < ring_depth() && e == hipSuccess; i++)
    e = hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming);
  smax_phase_mark(" ctx.stream", &tc);
  if (e == hipSuccess) e = hipHostMalloc(&c->pin[0], kStage, hipHostMallocDefault);
  smax_phase_mark(" ctx.pin0", &tc);
  if (e == hipSuccess) {
    for (int i = 1; i < ring_depth(); i++) c->pin_done[i] = c->pinned[i].get_future().share();
    std::thread([c, device] {
      hipError_t r = hipSetDevice(device);
      // GT_SMAX_PIN_FAIL_AT=i: chunk i and later report a pinning failure
      // (tests: the ring degrades instead of failing the device)
      const char *fa = getenv("GT_SMAX_PIN_FAIL_AT");
      const int fail_at = fa ? (int) strtol(fa, NULL, 0) : kRingMax;
      for (int i = 1; i < ring_depth(); i++) {
        if (r == hipSuccess && i >= fail_at) r = hipErrorOutOfMemory;
        if (r == hipSuccess) r = hipHostMalloc(&c->pin[i], kStage, hipHostMallocDefault);
        if (r != hipSuccess) c->pin[i] = nullptr;
        c->pinned[i].set_value(r);
      }
    }).detach();
  }
  if (e != hipSuccess) {
    (void) ring_ready(c);   // the helper may still write pin[]
    for (int i = 0; i < kRingMax; i++) {
      if (c->pin[i]) (void) hipHostFree(c->pin[i]);
      if (c->ev[i]) (void) hipEventDestroy(c->ev[i]);
    }
    if (c->stream) (void) hipStreamDestroy(c->stream);
    delete c;
    return e;
  }
  g_ctx[device] = c;
  *out = c;
  return hipSuccess;
}

// Persistent worker threads for the staging fills and copy-outs: a call
// runs one fill per 64 MiB chunk, and spawning its helpers each time cost
// ~11 thread creations per chunk (hundreds per call).  Workers are created on
// first use and live for the process; several device threads may submit at
// once (each par_for waits for its own tasks only).
class WorkPool {
 public:
  static WorkPool &get() {
    static WorkPool *p = new WorkPool;   // never destroyed: no join at exit
    return *p;
  }
  void ensure(unsigned n) {
    std::lock_guard<std::mutex> g(mu_);
    while (workers_ < n) {
      std::thread([this] { loop(); }).detach();
      workers_++;
    }
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  unsigned workers_ = 0;
};

// f(lo, hi) over [0, n) on nt threads (the calling thread takes the first
// part, pool workers the others)
template <typename F>
void par_for(uint64_t n, unsigned nt, F f) {
  if (nt <= 1 || n < (1u << 10)) { f(0, n); return; }
  static std::atomic<unsigned> active{0};
  struct Active {
    Active() { active++; }
    ~Active() { active--; }
  } in_flight;
  WorkPool &P = WorkPool::get();
  P.ensure(std::min((nt - 1) * active.load(), 64u));   // enough for every concurrent caller
  std::mutex mu;
  std::condition_variable cv;
  unsigned left = nt - 1;
  for (unsigned t = 1; t < nt; t++)
    P.submit([&, t] {
      f(n * t / nt, n * (t + 1) / nt);
      std::lock_guard<std::mutex> g(mu);
      if (--left == 0) cv.notify_one();
    });
  f(0, n / nt);
  std::unique_lock<std::mutex> g(mu);
  cv.wait(g, [&] { return left == 0; });
}

// CPUs this process may actually run on: the cgroup's CPU quota
// (/sys/fs/cgroup/cpu.max, "quota period"; v1: cpu.cfs_quota_us /
// cpu.cfs_period_us) and the affinity mask, not hardware_concurrency()
// (256 on the GPU box, whose cgroup allows 16)
unsigned usable_cpus() {
  static const unsigned n = [] {
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) hw = std::max(1, CPU_COUNT(&set));
    double quota = -1.0;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = "";
      long per = 0;
      if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
        quota = strtod(q, NULL) / (double) per;
      fclose(f);
    } else if (FILE *f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
      long q = -1, per = 0;
      if (fscanf(f1, "%ld", &q) == 1 && q > 0)
        if (FILE *f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
          if (fscanf(f2, "%ld", &per) == 1 && per > 0) quota = (double) q / (double) per;
          fclose(f2);
        }
      fclose(f1);
    }
    if (quota > 0) hw = std::min(hw, std::max(1u, (unsigned) (quota + 0.5)));
    return hw;
  }();
  return n;
}

// Staging threads per device thread of a call over ndev devices.  One
// device: 12 (h2d of the C3 tables 92-95 ms with 8, 83-88 ms with 12 or 16,
// 124 ms with 4: profiles/r03zt/e2e_threads.txt).  Several devices fill
// their rings at once, so they share the CPUs the cgroup allows
// (usable_cpus): 16 on the GPU box -> 2 per device at 8 devices, where
// 12 x 2 / 8 = 3 each had oversubscribed the quota 24 : 16.
// GT_SMAX_COPY_THREADS: the total over all devices.
unsigned copy_threads(int ndev) {
  const char *v = getenv("GT_SMAX_COPY_THREADS");
  const unsigned nd = (unsigned) std::max(1, ndev);
  const unsigned cpus = usable_cpus();
  unsigned total = v ? (unsigned) strtoul(v, NULL, 0) : 0u;
  if (total == 0) total = nd == 1 ? std::min(12u, cpus) : cpus;
  return std::min(16u, std::max(1u, total / nd));
}

// Host -> device through the context's ring of pinned chunks: fill(off, n,
// buf) writes destination bytes [off, off+n) into buf (on nt threads) while
// the DMA engine drains the others.  fill returns false to abort (*aborted).
template <typename Fill>
hipError_t stage_h2d(DevCtx *c, void *dst, uint64_t len, unsigned nt, Fill fill,
                     bool *aborted) {
  hipError_t e = hipSuccess;
  if (aborted) *aborted = false;
  uint64_t R = (uint64_t) ring_depth();
  for (uint64_t off = 0, k = 0; e == hipSuccess && off < len; off += kStage, k++) {
    int b;
    const uint64_t n = std::min(kStage, len - off);
    if ((e = ring_slot(c, k, R, &b)) != hipSuccess) break;
    char *buf = (char *) c->pin[b];
    std::atomic<bool> ok{true};
    // split at 64-byte units (whole packed groups for the BWT fill)
    const uint64_t units = (n + 63) / 64;
    par_for(units, nt, [&, buf, off](uint64_t ulo, uint64_t uhi) {
      const uint64_t lo = ulo * 64, hi = std::min(n, uhi * 64);
      if (lo < hi && !fill(off + lo, hi - lo, buf + lo)) ok = false;
    });
    if (!ok) {
      if (aborted) *aborted = true;
      break;
    }
    e = hipMemcpyAsync((char *) dst + off, buf, n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipEventRecord(c->ev[b], c->stream);
  }
  hipError_t e2 = hipStreamSynchronize(c->stream);   // the ring is free again on return
  return e == hipSuccess ? e2 : e;
}

// Several uploads through one pass of the ring, their chunks interleaved in
// proportion to their sizes (each next chunk from the least advanced
// segment): a segment whose fill is CPU-bound (the BWT plane packing reads
// 16 source bytes per 4 staged) then fills while the DMA engine drains the
// chunks of a copy-bound one (the LCP bytes) queued before it, instead of
// the two running one after the other.  A segment whose fill returns false
// stops (*aborted set; the others go on); without `aborted` that fails the
// upload.
struct StageSeg {
  void *dst;
  uint64_t len;
  std::function<bool(uint64_t, uint64_t, char *)> fill;
  bool *aborted;
  uint64_t done;
  bool stop;
};

hipError_t stage_h2d_multi(DevCtx *c, std::vector<StageSeg> &segs, unsigned nt) {
  hipError_t e = hipSuccess;
  uint64_t R = (uint64_t) ring_depth();
  // GT_SMAX_TIMING: where the pass waits -- for a ring slot (its DMA, or a
  // chunk still being pinned) or in the fills; the first chunks apart
  static const bool timing = env_on("GT_SMAX_TIMING");
  double t_wait = 0, t_fill = 0, t_wait4 = 0, t_fill4 = 0, tq = timing ? smax_phase_clock() : 0;
  for (auto &sg : segs) {
    sg.done = 0;
    sg.stop = false;
    if (sg.aborted) *sg.aborted = false;
  }
  for (uint64_t k = 0; e == hipSuccess; k++) {
    int pick = -1;
    double best = 2.0;
    for (size_t i = 0; i < segs.size(); i++) {
      const StageSeg &sg = segs[i];
      if (sg.stop || sg.done >= sg.len) continue;
      const double f = (double) sg.done / (double) sg.len;
      if (f < best) {
        best = f;
        pick = (int) i;
      }
    }
    if (pick < 0) break;
    StageSeg &sg = segs[(size_t) pick];
    int b;
    const uint64_t off = sg.done, n = std::min(kStage, sg.len - off);
    if ((e = ring_slot(c, k, R, &b)) != hipSuccess) break;
    if (timing) {
      const double t = smax_phase_clock();
      t_wait += t - tq;
      if (k < 4) t_wait4 += t - tq;
      tq = t;
    }
    char *buf = (char *) c->pin[b];
    std::atomic<bool> ok{true};
    const uint64_t units = (n + 63) / 64;   // 64-byte units (whole packed groups)
    par_for(units, nt, [&, buf, off](uint64_t ulo, uint64_t uhi) {
      const uint64_t lo = ulo * 64, hi = std::min(n, uhi * 64);
      if (lo < hi && !sg.fill(off + lo, hi - lo, buf + lo)) ok = false;
    });
    if (timing) {
      const double t = smax_phase_clock();
      t_fill += t - tq;
      if (k < 4) t_fill4 += t - tq;
      tq = t;
    }
    if (!ok) {
      sg.stop = true;
      if (sg.aborted) {
        *sg.aborted = true;
        continue;   // slot b stays free; its last DMA was waited for above
      }
      e = hipErrorInvalidValue;
      break;
    }
    e = hipMemcpyAsync((char *) sg.dst + off, buf, n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipEventRecord(c->ev[b], c->stream);
    sg.done += n;
  }
  hipError_t e2 = hipStreamSynchronize(c->stream);
  if (timing) {
    const double t = smax_phase_clock();
    fprintf(stderr, "[gt_smax timing]  h2d.waits   %8.2f ms (first 4 chunks %.2f)\n", t_wait * 1e3,
            t_wait4 * 1e3);
    fprintf(stderr, "[gt_smax timing]  h2d.fills   %8.2f ms (first 4 chunks %.2f)\n", t_fill * 1e3,
            t_fill4 * 1e3);
    fprintf(stderr, "[gt_smax timing]  h2d.drain   %8.2f ms\n", (t - tq) * 1e3);
  }
  return e == hipSuccess ? e2 : e;
}

// packed groups [g0, g1) of bwt[0 .. len) (layout: GT_SMAX_PK_GROUPS in
// include/gt_smax_hip.h) as their code planes (low 32 bits of a group) in
// out32, or whole groups in out64; the groups holding a special row are
// appended to *spec as (group << 16 | special mask) when out32 is used.
// False when a symbol in [4, 254) is seen.
bool pack_bits(const uint8_t *bwt, uint64_t len, uint64_t g0, uint64_t g1, uint64_t *out64,
               uint32_t *out32, std::vector<uint64_t> *spec, std::mutex *smu) {
  const __m128i k3 = _mm_set1_epi8(3), k254 = _mm_set1_epi8((char) 254), z = _mm_setzero_si128();
  __m128i bad = z;
  bool badscalar = false;
  std::vector<uint64_t> mine;
  for (uint64_t gi = g0; gi < g1; gi++) {
    const int64_t r0 = ((int64_t) gi - 1) * 16;
    uint64_t w = 0;
    if (r0 >= 0 && (uint64_t) r0 + 16 <= len) {
      const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i *>(bwt + r0));
      const __m128i sp = _mm_cmpeq_epi8(_mm_max_epu8(v, k254), v);            // v >= 254
      const __m128i gt3 = _mm_andnot_si128(_mm_cmpeq_epi8(_mm_subs_epu8(v, k3), z),
                                           _mm_set1_epi8((char) 0xff));      // v > 3
      bad = _mm_or_si128(bad, _mm_andnot_si128(sp, gt3));
      const uint32_t spm = (uint32_t) _mm_movemask_epi8(sp);
      const uint32_t lo = (uint32_t) _mm_movemask_epi8(_mm_slli_epi64(v, 7)) & ~spm;   // bit 0
      const uint32_t hi = (uint32_t) _mm_movemask_epi8(_mm_slli_epi64(v, 6)) & ~spm;   // bit 1
      w = (uint64_t) lo | ((uint64_t) hi << 16) | ((uint64_t) spm << 32);
    } else {
      for (int q = 0; q < 16; q++) {
        const int64_t r = r0 + q;
        if (r < 0 || (uint64_t) r >= len) continue;
        const uint32_t b = bwt[r];
        if (b >= 254) w |= 1ull << (32 + q);
        else {
          if (b > 3) badscalar = true;
          w |= (uint64_t) (b & 1u) << q | (uint64_t) ((b >> 1) & 1u) << (16 + q);
        }
      }
    }
    if (out64 != nullptr) {
      out64[gi - g0] = w;
    } else {
      out32[gi - g0] = (uint32_t) w;
      if (w >> 32) mine.push_back(gi << 16 | (w >> 32));
    }
  }
  if (!mine.empty()) {
    std::lock_guard<std::mutex> g(*smu);
    spec->insert(spec->end(), mine.begin(), mine.end());
  }
  return !badscalar && _mm_movemask_epi8(bad) == 0;
}

bool pack_groups(const uint8_t *bwt, uint64_t len, uint64_t g0, uint64_t g1, uint64_t *out) {
  return pack_bits(bwt, len, g0, g1, out, nullptr, nullptr, nullptr);
}

// device records -> host (lcp, lb, rb) triples through the pinned ring: the
// DMA of chunk k+1 overlaps the threaded conversion of chunk k
hipError_t d2h_triples(DevCtx *c, uint64_t *dst, const GtSmaxRecord *dev, uint64_t cnt,
                       unsigned nt) {
  const uint64_t CH = kStage / sizeof (GtSmaxRecord);
  const uint64_t nch = (cnt + CH - 1) / CH;
  const uint64_t nb = (uint64_t) d2h_buffers(c, nch);
  hipError_t e = hipSuccess;
  auto issue = [&](uint64_t j) {
    const uint64_t n = std::min(CH, cnt - j * CH);
    hipError_t r = hipMemcpyAsync(c->pin[j % nb], dev + j * CH, sizeof (GtSmaxRecord) * n,
                                  hipMemcpyDeviceToHost, c->stream);
    return r == hipSuccess ? hipEventRecord(c->ev[j % nb], c->stream) : r;
  };
  if (nch > 0) e = issue(0);
  for (uint64_t k = 0; e == hipSuccess && k < nch; k++) {
    if (nb > 1 && k + 1 < nch && (e = issue(k + 1)) != hipSuccess) break;
    if ((e = hipEventSynchronize(c->ev[k % nb])) != hipSuccess) break;
    const GtSmaxRecord *h = (const GtSmaxRecord *) c->pin[k % nb];
    uint64_t *t0 = dst + 3 * k * CH;
    par_for(std::min(CH, cnt - k * CH), nt, [=](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; i++) {
        t0[3 * i] = h[i].lcp;
        t0[3 * i + 1] = h[i].lb;
        t0[3 * i + 2] = h[i].lb + h[i].width - 1;
      }
    });
    // chunk k+2 reuses this buffer: issued only after this conversion
    if (nb == 1 && k + 1 < nch && (e = issue(k + 1)) != hipSuccess) break;
  }
  hipError_t e2 = hipStreamSynchronize(c->stream);
  return e == hipSuccess ? e2 : e;
}

// device bytes -> host through the pinned ring (chunk k+1's DMA overlaps the
// threaded copy-out of chunk k)
hipError_t d2h_bytes(DevCtx *c, void *dst, const void *dev, uint64_t bytes, unsigned nt) {
  const uint64_t nch = (bytes + kStage - 1) / kStage;
  const uint64_t nb = (uint64_t) d2h_buffers(c, nch);
  hipError_t e = hipSuccess;
  auto issue = [&](uint64_t j) {
    const uint64_t n = std::min(kStage, bytes - j * kStage);
    hipError_t r = hipMemcpyAsync(c->pin[j % nb], (const char *) dev + j * kStage, n,
                                  hipMemcpyDeviceToHost, c->stream);
    return r == hipSuccess ? hipEventRecord(c->ev[j % nb], c->stream) : r;
  };
  if (nch > 0) e = issue(0);
  for (uint64_t k = 0; e == hipSuccess && k < nch; k++) {
    if (nb > 1 && k + 1 < nch && (e = issue(k + 1)) != hipSuccess) break;
    if ((e = hipEventSynchronize(c->ev[k % nb])) != hipSuccess) break;
    const char *h = (const char *) c->pin[k % nb];
    char *t0 = (char *) dst + k * kStage;
    const uint64_t n = std::min(kStage, bytes - k * kStage);
    par_for((n + 4095) / 4096, nt, [=](uint64_t lo, uint64_t hi) {
      const uint64_t a = lo * 4096, b = std::min(n, hi * 4096);
      if (a < b) memcpy(t0 + a, h + a, b - a);
    });
    if (nb == 1 && k + 1 < nch && (e = issue(k + 1)) != hipSuccess) break;
  }
  hipError_t e2 = hipStreamSynchronize(c->stream);
  return e == hipSuccess ? e2 : e;
}

// ------------------------------------------------------------ RCCL

struct Rccl {
  bool tried = false, ok = false;
  void *h = nullptr;
  decltype(&ncclCommInitAll) init = nullptr;
  decltype(&ncclAllGather) allgather = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  std::vector<int> devs;              // device set of the cached communicators
  std::vector<ncclComm_t> comms;
};
std::mutex g_rccl_mu;
Rccl g_rccl;

// Loads RCCL (the library torch already mapped, if any) on first use.
bool rccl_load(std::string *err) {
  if (g_rccl.tried) {
    if (!g_rccl.ok) *err = "RCCL is not available";
    return g_rccl.ok;
  }
  g_rccl.tried = true;
  const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
  for (const char *n : names)
    if ((g_rccl.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
  if (g_rccl.h == nullptr) { *err = std::string("dlopen librccl: ") + dlerror(); return false; }
  g_rccl.init = (decltype(g_rccl.init)) dlsym(g_rccl.h, "ncclCommInitAll");
  g_rccl.allgather = (decltype(g_rccl.allgather)) dlsym(g_rccl.h, "ncclAllGather");
  g_rccl.errstr = (decltype(g_rccl.errstr)) dlsym(g_rccl.h, "ncclGetErrorString");
  g_rccl.destroy = (decltype(g_rccl.destroy)) dlsym(g_rccl.h, "ncclCommDestroy");
  g_rccl.ok = g_rccl.init && g_rccl.allgather && g_rccl.errstr && g_rccl.destroy;
  if (!g_rccl.ok) *err = "librccl lacks ncclCommInitAll/ncclAllGather";
  return g_rccl.ok;
}

// communicators over devs (one rank per device, rank = position), cached
bool rccl_comms(const std::vector<int> &devs, std::string *err) {
  if (!rccl_load(err)) return false;
  if (g_rccl.devs == devs && !g_rccl.comms.empty()) return true;
  for (ncclComm_t c : g_rccl.comms) (void) g_rccl.destroy(c);
  g_rccl.comms.assign(devs.size(), nullptr);
  g_rccl.devs.clear();
  ncclResult_t r = g_rccl.init(g_rccl.comms.data(), (int) devs.size(), devs.data());
  if (r != ncclSuccess) {
    *err = std::string("ncclCommInitAll: ") + g_rccl.errstr(r);
    g_rccl.comms.clear();
    return false;
  }
  g_rccl.devs = devs;
  return true;
}

// ------------------------------------------------------------ validation

int validate_input(const GtSmaxInput *in, char *errbuf, size_t errlen) {
  if (in == NULL || in->lcptab == NULL || in->bwttab == NULL) {
    seterr(errbuf, errlen, "missing lcptab or bwttab");
    return -1;
  }
  if (in->numllv > 0 && in->llvtab == NULL) {
    seterr(errbuf, errlen, "missing llvtab");
    return -1;
  }
  if (in->nonspecials > in->totallength) {
    seterr(errbuf, errlen, "nonspecials (%lu) exceeds totallength (%lu)",
           (unsigned long) in->nonspecials, (unsigned long) in->totallength);
    return -1;
  }
  return 0;
}

// The .llv scan of the validation (positions ascending, inside the text, on
// a 255 LCP byte): runs beside the staged upload (no device work starts
// before it has passed, run_call's phase 1 waits for it before planning).
int validate_llv(const GtSmaxInput *in, std::string *msg) {
  std::mutex mu;
  uint64_t first = UINT64_MAX;
  par_for(in->numllv, std::max(1u, copy_threads(1) / 3), [&, in](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; i++) {
      if (in->llvtab[i].position > in->totallength ||
          (i > 0 && in->llvtab[i].position <= in->llvtab[i - 1].position) ||
          in->lcptab[in->llvtab[i].position] != 255) {
        std::lock_guard<std::mutex> g(mu);
        first = std::min(first, i);
        break;
      }
    }
  });
  if (first != UINT64_MAX) {
    char b[96];
    snprintf(b, sizeof b, "inconsistent .llv entry %lu", (unsigned long) first);
    *msg = b;
    return -1;
  }
  return 0;
}

uint64_t llv_lower(const GtSmaxInput *in, uint64_t g) {
  uint64_t lo = 0, hi = in->numllv;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (in->llvtab[mid].position < g) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------ one call

struct Shard {
  uint64_t begin, end, base, len, lo, hi;
  GtSmaxDevShard sh;
  void *lcp = nullptr, *bwt = nullptr, *llv = nullptr;   // pool blocks (tables padded)
  GtSmaxPlan *plan = nullptr;
  uint64_t count = 0, offset = 0;
};

struct Call {
  const GtSmaxInput *in;
  unsigned minlen;
  int nshards = 0, ndev = 0;
  bool rccl = false;
  std::vector<int> devs;          // device ordinal of each used device slot
  std::vector<int> first;         // shards [first[d], first[d+1]) on device slot d
  std::vector<Shard> sh;
  std::vector<std::string> err;   // per device slot
  std::atomic<bool> failed{false};
  // phase barrier between the device threads (before the collective)
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t *trip = nullptr;
  unsigned nt = 1;
  double t0 = 0;
  // the .llv validation running beside the upload (validate_llv); every
  // device thread waits for it before it creates a plan
  std::shared_future<int> valid;
  std::string valid_msg;
};

// all device threads meet here; returns false if any of them failed
bool call_barrier(Call *C) {
  std::unique_lock<std::mutex> g(C->mu);
  if (++C->arrived == C->ndev) C->cv.notify_all();
  else C->cv.wait(g, [C] { return C->arrived == C->ndev; });
  return !C->failed.load();
}

void fail_dev(Call *C, int d, const std::string &m) {
  if (C->err[d].empty()) C->err[d] = m;
  C->failed = true;
}

#define DCHK(call)                                              \
  do {                                                          \
    hipError_t e_ = (call);                                     \
    if (e_ != hipSuccess) { fail_dev(C, d, hipmsg(#call, e_)); goto out; } \
  } while (0)

hipError_t alloc_table(void **raw, uint64_t bytes) {
  hipError_t e = smax_dev_alloc(raw, bytes + GT_SMAX_PAD_FRONT + GT_SMAX_PAD_BACK);
  if (e != hipSuccess) return e;
  char *p = (char *) *raw;
  e = hipMemset(p, 0, GT_SMAX_PAD_FRONT);
  if (e == hipSuccess) e = hipMemset(p + GT_SMAX_PAD_FRONT + bytes, 0, GT_SMAX_PAD_BACK);
  return e;
}

// Phase 1 of device slot d: upload, plan, run, exchange, stitch, counts.
void warm_kernels(int dev, hipStream_t st);

void device_phase1(Call *C, int d) {
  const GtSmaxInput *in = C->in;
  DevCtx *c = nullptr;
  char eb[512] = "";
  bool voted = false;
  const int dev = C->devs[d];
  const int s0 = C->first[d], s1 = C->first[d + 1], kmax = C->first[1] - C->first[0];
  void *send = nullptr, *recv = nullptr, *all = nullptr;
  double tc = smax_phase_clock();
  DCHK(hipSetDevice(dev));
  DCHK(ctx_get(dev, &c));
  if (d == 0) smax_phase_mark("ctx", &tc);   // stream + pinned ring (first call per device)
  {
    std::lock_guard<std::mutex> g(c->mu);
    double tp = smax_phase_clock(), th = tp;   // th: the upload's parts
    for (int s = s0; s < s1; s++) {
      Shard &S = C->sh[s];
      // the plan's buffers into the device cache (and the code object
      // loaded) on a helper thread while this thread stages the tables: a
      // first call otherwise pays ~30 ms of cold allocations in plan creation
      std::thread reserve;
      hipError_t reserve_err = hipSuccess;
      struct JoinT {
        std::thread &t;
        ~JoinT() { if (t.joinable()) t.join(); }
      } join_reserve{reserve};
      // the tables' device buffers first (the BWT as its code planes, 4 B per
      // 16 rows, plus the u64 groups the device rebuilds from them)
      const uint64_t ng = GT_SMAX_PK_GROUPS(S.len);
      const uint8_t *bsrc = in->bwttab + S.base;
      const uint64_t blen = S.len;
      bool nondna = env_on("GT_SMAX_BYTE_BWT");
      void *planes = nullptr;
      // the LCP table's zero pads travel with its bytes in the upload (no
      // memset kernels ahead of the first DMA: in a fresh process the first
      // fill launch cost tens of ms before the ring started)
      DCHK(smax_dev_alloc(&S.lcp, SMAX_TABLE_SHIFT + S.len + GT_SMAX_PAD_FRONT + GT_SMAX_PAD_BACK));
      if (!nondna) DCHK(smax_dev_alloc(&planes, sizeof (uint32_t) * ng));
      DCHK(smax_dev_alloc(&S.llv, sizeof (GtSmaxLlv) * (S.hi - S.lo + 1)));
      if (d == 0) smax_phase_mark(" h2d.alloc", &th);
      {
        // the plan's own buffers into the cache beside the upload
        GtSmaxDevShard g;
        memset(&g, 0, sizeof g);
        g.numllv = S.hi - S.lo;
        g.base = S.base;
        g.local_len = S.len;
        g.begin = S.begin;
        g.end = S.end;
        g.nonspecials = in->nonspecials;
        g.device = dev;
        // the u64 groups are first written after the ring: allocated here
        // (a cold allocation costs ~5 ms per GB), then every plan kernel's
        // first launch in the process and the null stream plan creation
        // uses (~10 ms in a fresh process, profiles/s5/bench_c3.json)
        const bool want_groups = !nondna;
        reserve = std::thread([g, dev, c, want_groups, ng, &S, &reserve_err] {
          // after the ring's chunks are pinned (beside the pinning, the
          // first chunks waited 22-27 ms instead of 8: profiles/s5/)
          // (a chunk that failed to pin is the ring's concern, not an error)
          (void) ring_ready(c);
          hipError_t e = hipSetDevice(dev);
          if (e == hipSuccess && want_groups) e = smax_dev_alloc(&S.bwt, sizeof (uint64_t) * ng);
          reserve_err = e;
          if (e != hipSuccess) return;
          (void) smax_plan_reserve(&g, 0);
          t_phase_mute = true;
          if (!c->kernels_warm.exchange(true)) warm_kernels(dev, nullptr);
        });
      }
      {
        // one pass of the ring over the LCP bytes, the BWT planes (packed
        // during the fill; a non-DNA alphabet stops that segment and the
        // bytes are staged after) and the .llv entries
        std::vector<uint64_t> spec;
        std::mutex smu;
        const char *lsrc = (const char *) in->lcptab + S.base;
        std::vector<StageSeg> segs;
        const uint64_t llen = S.len;
        segs.push_back({(char *) S.lcp + SMAX_TABLE_SHIFT, GT_SMAX_PAD_FRONT + S.len + GT_SMAX_PAD_BACK,
                        [lsrc, llen](uint64_t off, uint64_t n, char *buf) {
                          // [0, PAD_FRONT) zeros, the table, then PAD_BACK zeros
                          const uint64_t t0 = GT_SMAX_PAD_FRONT, t1 = t0 + llen;
                          const uint64_t a = std::max(off, t0), b = std::min(off + n, t1);
                          if (off < t0) memset(buf, 0, std::min(off + n, t0) - off);
                          if (a < b) memcpy(buf + (a - off), lsrc + (a - t0), b - a);
                          if (off + n > t1) {
                            const uint64_t z = std::max(off, t1);
                            memset(buf + (z - off), 0, off + n - z);
                          }
                          return true;
                        }, nullptr, 0, false});
        if (!nondna)
          segs.push_back({planes, sizeof (uint32_t) * ng,
                          [bsrc, blen, &spec, &smu](uint64_t off, uint64_t n, char *buf) {
                            return pack_bits(bsrc, blen, off / 4, (off + n) / 4, nullptr,
                                             (uint32_t *) buf, &spec, &smu);
                          }, &nondna, 0, false});
        if (S.hi > S.lo) {
          const char *vsrc = (const char *) (in->llvtab + S.lo);
          segs.push_back({S.llv, sizeof (GtSmaxLlv) * (S.hi - S.lo),
                          [vsrc](uint64_t off, uint64_t n, char *buf) {
                            memcpy(buf, vsrc + off, n);
                            return true;
                          }, nullptr, 0, false});
        }
        hipError_t pe = stage_h2d_multi(c, segs, C->nt);
        if (d == 0) smax_phase_mark(" h2d.ring", &th);
        if (reserve.joinable()) reserve.join();
        if (pe == hipSuccess) pe = reserve_err;
        if (d == 0) smax_phase_mark(" h2d.helper", &th);
        void *dspec = nullptr;
        if (pe == hipSuccess && !nondna && !spec.empty()) {
          pe = smax_dev_alloc(&dspec, sizeof (uint64_t) * spec.size());
          if (pe == hipSuccess)
            pe = hipMemcpyAsync(dspec, spec.data(), sizeof (uint64_t) * spec.size(),
                                hipMemcpyHostToDevice, c->stream);
        }
        if (pe == hipSuccess && !nondna)
          pe = smax_groups_from_planes((uint64_t *) S.bwt, (const uint32_t *) planes, ng,
                                       (const uint64_t *) dspec, spec.size(), c->stream);
        {
          // unconditionally: on an error above, work enqueued before it may
          // still read dspec / planes, which go back to the cache here
          const hipError_t se = hipStreamSynchronize(c->stream);
          if (pe == hipSuccess) pe = se;
        }
        smax_dev_free(dspec);
        smax_dev_free(planes);
        DCHK(pe);
        S.sh.bwtpk_dev = nondna ? nullptr : (const uint64_t *) S.bwt;
      }
      if (nondna) {
        smax_dev_free(S.bwt);
        S.bwt = nullptr;
        DCHK(alloc_table(&S.bwt, S.len));
        DCHK(stage_h2d(c, (char *) S.bwt + GT_SMAX_PAD_FRONT, S.len, C->nt,
                       [bsrc](uint64_t off, uint64_t n, char *buf) {
                         memcpy(buf, bsrc + off, n);
                         return true;
                       }, nullptr));
        S.sh.bwt_dev = (const uint8_t *) S.bwt + GT_SMAX_PAD_FRONT;
      }
      S.sh.lcp_dev = (const uint8_t *) S.lcp + SMAX_TABLE_SHIFT + GT_SMAX_PAD_FRONT;
      S.sh.llv_dev = (const GtSmaxLlv *) S.llv;
      S.sh.numllv = S.hi - S.lo;
      S.sh.base = S.base;
      S.sh.local_len = S.len;
      S.sh.begin = S.begin;
      S.sh.end = S.end;
      S.sh.nonspecials = in->nonspecials;
      S.sh.device = dev;
      if (d == 0) smax_phase_mark(s == s0 ? "h2d" : "h2d(next)", &tp);
      if (C->valid.valid() && C->valid.get() != 0) {   // no kernel over unvalidated tables
        fail_dev(C, d, C->valid_msg);
        goto out;
      }
      if (gt_smax_plan_create(&S.plan, &S.sh, C->minlen, 0, eb, sizeof eb)) {
        fail_dev(C, d, eb);
        goto out;
      }
      if (d == 0) smax_phase_mark("plan", &tp);
      if (gt_smax_plan_run(S.plan, c->stream)) { fail_dev(C, d, "plan run failed"); goto out; }
    }
    DCHK(hipStreamSynchronize(c->stream));
    for (int s = s0; s < s1; s++) {
      Shard &S = C->sh[s];
      const uint32_t eb2 = gt_smax_plan_error_bits(S.plan);
      if (eb2 != 0) {
        snprintf(eb, sizeof eb, "inconsistent index: %s%s",
                 (eb2 & 1u) ? "a .lcp byte 255 without its .llv entry " : "",
                 (eb2 & 2u) ? "a table read outside the shard" : "");
        fail_dev(C, d, eb);
        goto out;
      }
      DCHK(hipMemcpy(&S.count, gt_smax_plan_count_dev(S.plan), sizeof (uint64_t),
                     hipMemcpyDeviceToHost));
      if (S.count + 1 > gt_smax_plan_capacity(S.plan)) {   // + 1: a stitched interval
        gt_smax_plan_delete(S.plan);
        S.plan = nullptr;
        if (gt_smax_plan_create(&S.plan, &S.sh, C->minlen, S.count + 16, eb, sizeof eb)) {
          fail_dev(C, d, eb);
          goto out;
        }
        if (gt_smax_plan_run(S.plan, c->stream)) { fail_dev(C, d, "plan run failed"); goto out; }
        DCHK(hipStreamSynchronize(c->stream));
      }
    }
    if (d == 0) smax_phase_mark("run", &tp);
    // ---- boundary exchange: device slot d's records at
    // send[0 .. s1-s0), all slots gathered to recv[slot * kmax ..], then laid
    // out in shard order in all[]
    const size_t B = sizeof (GtSmaxBoundary);
    DCHK(smax_dev_alloc(&send, B * kmax));
    DCHK(smax_dev_alloc(&recv, B * kmax * C->ndev));
    DCHK(smax_dev_alloc(&all, B * C->nshards));
    DCHK(hipMemsetAsync(send, 0, B * kmax, c->stream));
    for (int s = s0; s < s1; s++)
      if (gt_smax_plan_copy_boundary(C->sh[s].plan, (char *) send + B * (s - s0), c->stream)) {
        fail_dev(C, d, "boundary copy failed");
        goto out;
      }
    voted = true;
    if (!call_barrier(C)) goto out;          // every slot's plans ran: collective is safe
    if (C->rccl) {
      ncclResult_t r = g_rccl.allgather(send, recv, B * kmax, ncclUint8, g_rccl.comms[d], c->stream);
      if (r != ncclSuccess) {
        fail_dev(C, d, std::string("ncclAllGather: ") + g_rccl.errstr(r));
        goto out;
      }
    } else {
      DCHK(hipMemcpyAsync(recv, send, B * kmax, hipMemcpyDeviceToDevice, c->stream));
    }
    for (int e = 0; e < C->ndev; e++) {
      const int n = C->first[e + 1] - C->first[e];
      if (n > 0)
        DCHK(hipMemcpyAsync((char *) all + B * C->first[e], (char *) recv + B * kmax * e, B * n,
                            hipMemcpyDeviceToDevice, c->stream));
    }
    for (int s = s0; s < s1; s++)
      if (gt_smax_plan_stitch(C->sh[s].plan, (const GtSmaxBoundary *) all, C->nshards, s,
                              c->stream)) {
        fail_dev(C, d, "stitch failed");
        goto out;
      }
    for (int s = s0; s < s1; s++)
      DCHK(hipMemcpyAsync(&C->sh[s].count, gt_smax_plan_count_dev(C->sh[s].plan),
                          sizeof (uint64_t), hipMemcpyDeviceToHost, c->stream));
    DCHK(hipStreamSynchronize(c->stream));
    if (d == 0) smax_phase_mark("exchange", &tp);
  }
out:
  if (!voted) call_barrier(C);   // a failed slot still meets the others (no collective then)
  // a failed slot may leave work queued on its stream: done before the
  // exchange buffers go back to the cache
  if (c != nullptr) (void) hipStreamSynchronize(c->stream);
  smax_dev_free(send);
  smax_dev_free(recv);
  smax_dev_free(all);
}

// Phase 2 of device slot d: its shards' records -> triples at their offsets.
void device_phase2(Call *C, int d) {
  DevCtx *c = nullptr;
  const int dev = C->devs[d];
  DCHK(hipSetDevice(dev));
  DCHK(ctx_get(dev, &c));
  {
    std::lock_guard<std::mutex> g(c->mu);
    for (int s = C->first[d]; s < C->first[d + 1]; s++) {
      Shard &S = C->sh[s];
      if (S.count > 0)
        DCHK(d2h_triples(c, C->trip + 3 * S.offset, gt_smax_plan_records(S.plan), S.count, C->nt));
    }
  }
out:
  return;
}

template <typename F>
void on_devices(Call *C, F f) {
  if (C->ndev == 1) { f(C, 0); return; }
  std::vector<std::thread> th;
  for (int d = 0; d < C->ndev; d++) th.emplace_back(f, C, d);
  for (auto &t : th) t.join();
}

// ------------------------------------------------------------ warm-up

// gt_smax_hip_prepare: a first call's fixed costs on a helper thread ahead of
// it -- the HIP runtime and device contexts (stream, pinned ring), the
// staging workers, the code object, and the tables' and plans' device
// buffers at the sizes of the announced index in the device cache.  A fresh
// process's first call otherwise pays them inside the call (bench.py's
// cold legs: the first stream alone 20-160 ms, profiles/s5/cold_probe.txt).
// Every host entry waits for it (prepare_wait) before touching a device.
struct Prep {
  std::mutex mu;
  std::thread t;
  ~Prep() {   // at exit: never leave the helper inside the HIP runtime
    if (t.joinable()) t.join();
  }
};
Prep &prep() {
  static Prep p;
  return p;
}
void prepare_wait() {
  Prep &P = prep();
  std::lock_guard<std::mutex> g(P.mu);
  if (P.t.joinable()) P.t.join();
}

// shards [first[d], first[d+1]) on device slot d: contiguous blocks, the
// first slots one larger (run_call and the warm-up agree on it)
std::vector<int> shard_blocks(int nshards, int ndev) {
  std::vector<int> first(ndev + 1, 0);
  for (int d = 0; d < ndev; d++)
    first[d + 1] = first[d] + nshards / ndev + (d < nshards % ndev ? 1 : 0);
  return first;
}

// One plan over a 64 Ki-row all-zero index on stream st: the first plan in a
// process pays ~10 ms in its .llv index phase (the null stream plan creation
// uses for its memsets and copies, and the kernels' first launches:
// profiles/s5/bench_c3.json, llv_index 10-11 ms in a first call, 1 ms after)
void warm_kernels(int dev, hipStream_t st) {
  const uint64_t len = 1u << 16, ng = GT_SMAX_PK_GROUPS(len);
  const uint64_t lbytes = len + GT_SMAX_PAD_FRONT + GT_SMAX_PAD_BACK;
  void *lcp = nullptr, *grp = nullptr, *pl = nullptr, *llv = nullptr;
  hipError_t e = smax_dev_alloc(&lcp, lbytes);
  if (e == hipSuccess) e = smax_dev_alloc(&grp, sizeof (uint64_t) * ng);
  if (e == hipSuccess) e = smax_dev_alloc(&pl, sizeof (uint32_t) * ng);
  if (e == hipSuccess) e = smax_dev_alloc(&llv, sizeof (GtSmaxLlv));
  if (e == hipSuccess) e = hipMemsetAsync(lcp, 0, lbytes, st);
  if (e == hipSuccess) e = hipMemsetAsync(pl, 0, sizeof (uint32_t) * ng, st);
  if (e == hipSuccess)
    e = smax_groups_from_planes((uint64_t *) grp, (const uint32_t *) pl, ng, nullptr, 0, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) {
    GtSmaxDevShard g;
    memset(&g, 0, sizeof g);
    g.lcp_dev = (const uint8_t *) lcp + GT_SMAX_PAD_FRONT;
    g.bwtpk_dev = (const uint64_t *) grp;
    g.llv_dev = (const GtSmaxLlv *) llv;
    g.base = 0;
    g.local_len = len;
    g.begin = 1;
    g.end = len - 1;
    g.nonspecials = len - 1;
    g.device = dev;
    GtSmaxPlan *plan = nullptr;
    char eb[256];
    if (gt_smax_plan_create(&plan, &g, 20, 0, eb, sizeof eb) == 0) {
      (void) gt_smax_plan_run(plan, st);
      (void) hipStreamSynchronize(st);
      gt_smax_plan_delete(plan);
    }
  }
  (void) hipStreamSynchronize(st);
  for (void *p : {lcp, grp, pl, llv}) smax_dev_free(p);
}

// the stream's first copies in each direction set up their DMA path: one
// small copy out of every pinned chunk, one back; then the kernels
void warm_pass(DevCtx *c, int dev) {
  void *buf = nullptr;
  const uint64_t n = std::min<uint64_t>(kStage, 1u << 16);
  hipError_t e = smax_dev_alloc(&buf, n);
  for (int i = 0; i < ring_depth() && e == hipSuccess; i++)
    if (chunk_usable(c, i)) e = hipMemcpyAsync(buf, c->pin[i], n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(c->pin[0], buf, 4096, hipMemcpyDeviceToHost, c->stream);
  (void) hipStreamSynchronize(c->stream);
  smax_dev_free(buf);
  if (!c->kernels_warm.exchange(true)) warm_kernels(dev, c->stream);
}

void prepare_run(uint64_t n, uint64_t N, int num_gpus) {
  const int avail = gt_smax_device_count();
  if (avail <= 0 || N < 2 || n + 1 < N) return;
  int nshards = std::max(1, num_gpus);
  if ((uint64_t) nshards > N - 1) nshards = (int) (N - 1);
  const int ndev = std::min(nshards, avail);
  const std::vector<int> first = shard_blocks(nshards, ndev);
  // the staging workers (created on first use)
  par_for(1u << 12, copy_threads(ndev), [](uint64_t, uint64_t) {});
  std::vector<std::thread> th;
  for (int d = 0; d < ndev; d++)
    th.emplace_back([&first, d, nshards, N] {
      // devices 0 .. ndev-1: a fresh process's calling thread is on device 0
      if (hipSetDevice(d) != hipSuccess) return;
      DevCtx *c = nullptr;
      if (ctx_get(d, &c) != hipSuccess) return;
      (void) ring_ready(c);
      {
        std::lock_guard<std::mutex> g(c->mu);   // the ring's chunks
        warm_pass(c, d);
      }
      for (int s = first[d]; s < first[d + 1]; s++) {
        GtSmaxDevShard g;
        memset(&g, 0, sizeof g);
        g.begin = 1 + (N - 1) * (uint64_t) s / (uint64_t) nshards;
        g.end = 1 + (N - 1) * (uint64_t) (s + 1) / (uint64_t) nshards;
        g.base = g.begin - 1;
        g.local_len = g.end - g.base + 1;
        g.nonspecials = N;
        g.device = d;
        const uint64_t ng = GT_SMAX_PK_GROUPS(g.local_len);
        void *b[3] = {};
        hipError_t e = smax_dev_alloc(&b[0], SMAX_TABLE_SHIFT + g.local_len + GT_SMAX_PAD_FRONT +
                                             GT_SMAX_PAD_BACK);
        if (e == hipSuccess) e = smax_dev_alloc(&b[1], sizeof (uint64_t) * ng);
        if (e == hipSuccess) e = smax_dev_alloc(&b[2], sizeof (uint32_t) * ng);
        if (e == hipSuccess) (void) smax_plan_reserve(&g, 0);
        for (void *p : b) smax_dev_free(p);   // no work was enqueued on them
      }
    });
  for (auto &t : th) t.join();
}

int run_call(const GtSmaxInput *in, unsigned minlen, int num_gpus, uint64_t **trip_out,
             uint64_t *count_out, char *errbuf, size_t errlen) {
  prepare_wait();
  Call C;
  // the .llv scan overlaps the staged upload; its future is waited for by
  // every device thread before planning, and on every return path here
  C.valid = std::async(std::launch::async, [in, &C] { return validate_llv(in, &C.valid_msg); }).share();
  struct Join {
    std::shared_future<int> &f;
    ~Join() { if (f.valid()) f.wait(); }
  } join{C.valid};
  const uint64_t N = in->nonspecials;
  const int avail = gt_smax_device_count();
  *trip_out = NULL;
  *count_out = 0;
  if (avail <= 0) {
    seterr(errbuf, errlen, "no HIP device available");
    return -1;
  }
  if (N < 2) {
    if (C.valid.get() != 0) {
      seterr(errbuf, errlen, "%s", C.valid_msg.c_str());
      return -1;
    }
    *trip_out = (uint64_t *) malloc(sizeof (uint64_t));
    return *trip_out ? 0 : -1;
  }
  C.in = in;
  C.minlen = minlen;
  C.nshards = std::max(1, num_gpus);
  if ((uint64_t) C.nshards > N - 1) C.nshards = (int) (N - 1);
  C.ndev = std::min(C.nshards, avail);
  {
    // the calling thread's device first, then the next ones (wrapping)
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur < 0 || cur >= avail) cur = 0;
    for (int d = 0; d < C.ndev; d++) C.devs.push_back((cur + d) % avail);
  }
  // contiguous shard blocks per device slot, the first slots one larger
  C.first = shard_blocks(C.nshards, C.ndev);
  C.err.assign(C.ndev, std::string());
  C.nt = copy_threads(C.ndev);
  if (env_on("GT_SMAX_TIMING"))
    fprintf(stderr, "[gt_smax timing] staging    %d device(s) x %u fill threads (usable CPUs %u), "
            "%d shard(s)\n", C.ndev, C.nt, usable_cpus(), C.nshards);
  C.sh.resize(C.nshards);
  for (int s = 0; s < C.nshards; s++) {
    Shard &S = C.sh[s];
    memset(&S.sh, 0, sizeof S.sh);
    S.begin = 1 + (N - 1) * (uint64_t) s / (uint64_t) C.nshards;
    S.end = 1 + (N - 1) * (uint64_t) (s + 1) / (uint64_t) C.nshards;
    S.base = S.begin - 1;
    S.len = S.end - S.base + 1;               // LCP[base .. end], BWT[base .. end]
    S.lo = llv_lower(in, S.base);
    S.hi = llv_lower(in, S.base + S.len);
    // the searches run over a .llv that is validated beside the upload: with
    // positions out of order hi can fall below lo (the call then fails with
    // the validation's message, not with an underflowed allocation size)
    if (S.hi < S.lo) S.hi = S.lo;
  }
  C.rccl = C.ndev > 1 || env_on("GT_SMAX_FORCE_RCCL");
  if (C.rccl) {
    std::lock_guard<std::mutex> g(g_rccl_mu);
    std::string m;
    if (!rccl_comms(C.devs, &m)) {
      seterr(errbuf, errlen, "%s", m.c_str());
      return -1;
    }
  }
  int rc = -1;
  std::unique_lock<std::mutex> rl(g_rccl_mu, std::defer_lock);
  if (C.rccl) rl.lock();   // one call at a time on the cached communicators
  on_devices(&C, device_phase1);
  if (!C.failed) {
    uint64_t total = 0;
    double tt = smax_phase_clock();
    for (auto &S : C.sh) { S.offset = total; total += S.count; }
    C.trip = (uint64_t *) malloc(sizeof (uint64_t) * 3 * (total + 1));
    if (C.trip != NULL) {
      // the converting threads first-touch every page of the fresh buffer:
      // ask for transparent huge pages over its 2 MiB-aligned interior
      // (one fault per 2 MiB instead of per 4 KiB; advice only, the buffer
      // stays an ordinary malloc block for gt_smax_free)
      const uintptr_t a0 = ((uintptr_t) C.trip + (2u << 20) - 1) & ~(uintptr_t) ((2u << 20) - 1);
      const uintptr_t a1 = ((uintptr_t) C.trip + sizeof (uint64_t) * 3 * (total + 1)) &
                           ~(uintptr_t) ((2u << 20) - 1);
      if (a1 > a0) (void) madvise((void *) a0, a1 - a0, MADV_HUGEPAGE);
    }
    smax_phase_mark("triples_alloc", &tt);
    if (C.trip == NULL) {
      seterr(errbuf, errlen, "out of memory for %lu intervals", (unsigned long) total);
    } else {
      double tp = smax_phase_clock();
      on_devices(&C, device_phase2);
      smax_phase_mark("d2h+triples", &tp);
      if (!C.failed) {
        *trip_out = C.trip;
        *count_out = total;
        C.trip = NULL;
        rc = 0;
      }
    }
  }
  // a table the validation rejected explains any device-side failure too
  if (rc != 0 && C.valid.valid() && C.valid.get() != 0) seterr(errbuf, errlen, "%s", C.valid_msg.c_str());
  if (rc != 0 && (errbuf == NULL || errlen == 0 || errbuf[0] == 0))
    for (auto &m : C.err)
      if (!m.empty()) { seterr(errbuf, errlen, "%s", m.c_str()); break; }
  free(C.trip);
  double tr = smax_phase_clock();
  // every table was used on its device context's stream (uploads, plans):
  // after those streams (idle already unless a slot failed) the blocks
  // return to the cache
  for (int d : C.devs) {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    auto it = g_ctx.find(d);
    if (it != g_ctx.end() && hipSetDevice(d) == hipSuccess) (void) hipStreamSynchronize(it->second->stream);
  }
  for (auto &S : C.sh) {
    if (S.plan) gt_smax_plan_delete(S.plan);
    smax_dev_free(S.lcp);
    smax_dev_free(S.bwt);
    smax_dev_free(S.llv);
  }
  if (env_on("GT_SMAX_NO_CACHE")) gt_smax_release_cache();
  smax_phase_mark("release", &tr);
  return rc;
}

}  // namespace

// ============================================================ internal API

hipError_t smax_dev_alloc(void **ptr, size_t bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const size_t sz = round_block(bytes);
  Pool &P = pool();
  for (;;) {
    IdleBlock b{nullptr, nullptr};
    std::pair<int, size_t> key;
    {
      std::lock_guard<std::mutex> g(P.mu);
      // reuse an idle block of this device of at most twice the size
      auto it = P.idle.lower_bound({dev, sz});
      if (it != P.idle.end() && it->first.first == dev && it->first.second <= 2 * sz) {
        b = it->second;
        key = it->first;
        P.idle.erase(it);
      }
    }
    if (b.ptr == nullptr) break;
    // the work still using the block (its fence) first; a fence that
    // reports an error (a faulted kernel) retires the block
    const hipError_t fe = b.fence ? b.fence->wait() : hipSuccess;
    fence_unref(b.fence);
    if (fe != hipSuccess) {
      (void) hipGetLastError();
      (void) hipFree(b.ptr);
      continue;
    }
    std::lock_guard<std::mutex> g(P.mu);
    *ptr = b.ptr;
    P.live[b.ptr] = key;
    return hipSuccess;
  }
  e = hipMalloc(ptr, sz);
  if (e == hipErrorOutOfMemory) {   // give the cached blocks back and retry
    (void) hipGetLastError();
    {
      std::lock_guard<std::mutex> g(P.mu);
      release_idle(dev);
    }
    e = hipMalloc(ptr, sz);
  }
  if (e != hipSuccess) { *ptr = nullptr; return e; }
  std::lock_guard<std::mutex> g(P.mu);
  P.live[*ptr] = {dev, sz};
  return hipSuccess;
}

namespace {
void dev_free_impl(void *ptr, SmaxFence *fence) {
  if (ptr == nullptr) return;
  Pool &P = pool();
  std::pair<int, size_t> key;
  {
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.live.find(ptr);
    if (it == P.live.end()) return;
    key = it->second;
    P.live.erase(it);
  }
  static const bool nocache = env_on("GT_SMAX_NO_CACHE");
  if (nocache) {
    // hipFree waits for the device's work itself
    int cur = -1;
    (void) hipGetDevice(&cur);
    (void) hipSetDevice(key.first);
    (void) hipFree(ptr);
    if (cur >= 0) (void) hipSetDevice(cur);
    return;
  }
  if (fence) fence->refs.fetch_add(1);
  std::lock_guard<std::mutex> g(P.mu);
  P.idle.insert({key, IdleBlock{ptr, fence}});
}
}  // namespace

void smax_dev_free(void *ptr) { dev_free_impl(ptr, nullptr); }

void smax_dev_free_fenced(void *ptr, SmaxFence *fence) { dev_free_impl(ptr, fence); }

SmaxFence *smax_fence_create(const hipStream_t *streams, int nstreams) {
  SmaxFence *f = new SmaxFence;
  (void) hipGetDevice(&f->device);
  if (nstreams < 0) {
    f->whole_device = true;
    return f;
  }
  for (int i = 0; i < nstreams; i++) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(e, streams[i]) != hipSuccess) {
      (void) hipGetLastError();
      if (e) (void) hipEventDestroy(e);
      f->whole_device = true;   // could not fence the stream: wait for everything
      continue;
    }
    f->ev.push_back(e);
  }
  return f;
}

SmaxFence *smax_fence_adopt(const hipEvent_t *events, int nevents, bool whole_device) {
  SmaxFence *f = new SmaxFence;
  (void) hipGetDevice(&f->device);
  f->whole_device = whole_device;
  for (int i = 0; i < nevents; i++) f->ev.push_back(events[i]);
  return f;
}

void smax_fence_release(SmaxFence *fence) { fence_unref(fence); }

void smax_marks_init(SmaxStreamMarks *m) {
  m->n = 0;
  m->overflow = false;
}

void smax_marks_record(SmaxStreamMarks *m, hipStream_t s) {
  int i = 0;
  while (i < m->n && m->s[i] != s) i++;
  if (i == m->n) {
    if (m->n == SMAX_MARK_STREAMS ||
        hipEventCreateWithFlags(&m->ev[i], hipEventDisableTiming) != hipSuccess) {
      (void) hipGetLastError();
      m->overflow = true;
      return;
    }
    m->s[i] = s;
    m->n++;
  }
  if (hipEventRecord(m->ev[i], s) != hipSuccess) {
    (void) hipGetLastError();
    m->overflow = true;
  }
}

hipError_t smax_marks_sync(SmaxStreamMarks *m) {
  if (m->overflow) return hipDeviceSynchronize();
  for (int i = 0; i < m->n; i++) {
    const hipError_t e = hipEventSynchronize(m->ev[i]);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t smax_marks_wait(SmaxStreamMarks *m, hipStream_t s) {
  if (m->overflow) return hipDeviceSynchronize();
  for (int i = 0; i < m->n; i++) {
    if (m->s[i] == s) continue;          // stream order already
    const hipError_t e = hipStreamWaitEvent(s, m->ev[i], 0);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

SmaxFence *smax_marks_fence(SmaxStreamMarks *m) {
  SmaxFence *f = smax_fence_adopt(m->ev, m->n, m->overflow);
  smax_marks_init(m);
  return f;
}

double smax_phase_clock() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void smax_phase_mark(const char *what, double *t) {
  static const bool on = env_on("GT_SMAX_TIMING");
  const double now = smax_phase_clock();
  if (on && !t_phase_mute) fprintf(stderr, "[gt_smax timing] %-12s %8.2f ms\n", what, (now - *t) * 1e3);
  *t = now;
}

hipError_t smax_d2h_triples(uint64_t *dst, const GtSmaxRecord *dev, uint64_t cnt, void *stream) {
  (void) stream;   // callers synchronised the plan's work already
  int d = 0;
  DevCtx *c = nullptr;
  hipError_t e = hipGetDevice(&d);
  if (e == hipSuccess) e = ctx_get(d, &c);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(c->mu);
  return d2h_triples(c, dst, dev, cnt, copy_threads(1));
}

hipError_t smax_stage_upload(void *dst, const void *src, uint64_t bytes) {
  int d = 0;
  DevCtx *c = nullptr;
  hipError_t e = hipGetDevice(&d);
  if (e == hipSuccess) e = ctx_get(d, &c);
  if (e != hipSuccess || bytes == 0) return e;
  std::lock_guard<std::mutex> g(c->mu);
  const char *s = (const char *) src;
  return stage_h2d(c, dst, bytes, copy_threads(1),
                   [s](uint64_t off, uint64_t n, char *buf) {
                     memcpy(buf, s + off, n);
                     return true;
                   }, nullptr);
}

hipError_t smax_stage_download(void *dst, const void *src, uint64_t bytes) {
  int d = 0;
  DevCtx *c = nullptr;
  hipError_t e = hipGetDevice(&d);
  if (e == hipSuccess) e = ctx_get(d, &c);
  if (e != hipSuccess || bytes == 0) return e;
  std::lock_guard<std::mutex> g(c->mu);
  return d2h_bytes(c, dst, src, bytes, copy_threads(1));
}

// ============================================================ C-ABI

extern "C" int gt_smax_pack_bwt(const uint8_t *bwt, uint64_t len, uint64_t *pk) {
  std::atomic<bool> ok{true};
  par_for(GT_SMAX_PK_GROUPS(len), copy_threads(1), [&](uint64_t lo, uint64_t hi) {
    if (!pack_groups(bwt, len, lo, hi, pk + lo)) ok = false;
  });
  return ok ? 0 : 1;
}

extern "C" int gt_smax_hip_prepare(uint64_t totallength, uint64_t nonspecials, int num_gpus) {
  prepare_wait();   // one warm-up at a time
  Prep &P = prep();
  std::lock_guard<std::mutex> g(P.mu);
  try {
    P.t = std::thread([=] { prepare_run(totallength, nonspecials, num_gpus); });
  } catch (...) {
    return -1;
  }
  return 0;
}

extern "C" void gt_smax_release_cache(void) {
  prepare_wait();
  {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    release_idle(-1);
  }
}

extern "C" int gt_smax_hip_enumerate_to_buffer(const GtSmaxInput *in, unsigned int minlen,
                                               int num_gpus, uint64_t **lcp_lb_rb,
                                               uint64_t *count, char *errbuf, size_t errlen) {
  double tv = smax_phase_clock();
  SmaxDeviceGuard keep;   // the device threads set their own; the caller's is restored
  if (errbuf && errlen) errbuf[0] = 0;
  if (validate_input(in, errbuf, errlen)) return -1;
  smax_phase_mark("validate", &tv);
  if (minlen == 0) {
    seterr(errbuf, errlen, "minlen must be >= 1");
    return -1;
  }
  return run_call(in, minlen, num_gpus, lcp_lb_rb, count, errbuf, errlen);
}

extern "C" int gt_smax_hip_enumerate(const GtSmaxInput *in, unsigned int minlen, int num_gpus,
                                     GtSmaxIntervalFunc cb, void *data, char *errbuf,
                                     size_t errlen) {
  uint64_t *trip = NULL, count = 0;
  if (cb == NULL) {
    seterr(errbuf, errlen, "no interval callback");
    return -1;
  }
  if (gt_smax_hip_enumerate_to_buffer(in, minlen, num_gpus, &trip, &count, errbuf, errlen))
    return -1;
  for (uint64_t i = 0; i < count; i++) {
    if (cb(data, trip[3 * i], trip[3 * i + 1], trip[3 * i + 2]) != 0) {
      seterr(errbuf, errlen, "interval callback failed at interval %lu", (unsigned long) i);
      free(trip);
      return -1;
    }
  }
  free(trip);
  return 0;
}
