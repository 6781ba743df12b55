// Node pipeline (sg_node_*): one host process drives every GPU of the node for one partitioned query.
//
// The reference runs a partitioned query in one JVM: PartitionStreamReceiver.receive looks each event's key up and
// hands it to that key's cloned runtime (C/partition/PartitionStreamReceiver.java:80-281, PartitionRuntime.java:
// 255-308); the matches reach QueryCallback.receive in one ordered stream (C/query/output/callback/
// QueryCallback.java:52-85).  Here the same contract is met by a pipeline over chunks of the host batch.
//
// G > 1 GPUs with the device key dictionary (every partitioned query without playback timers): the GPU-side shard
// exchange (x_loop below).  Each GPU uploads a contiguous slice of the caller's rows, shards them on the device,
// exchanges rows with the other GPUs (peer copies), runs its shard, sends each match to the GPU that owns its trigger's
// slice, and that GPU merges by trigger and copies straight into the caller's columns -- the host does no per-row or
// per-match work.
//
// One GPU, or queries whose playback timers need every row's clock on every shard (host key dictionary):
//   route    host thread pool: raw partition-key values -> first-seen dense ids -> shard (GPU) + per-shard id
//            (router.h); with G > 1 every chunk's rows are scattered, in arrival order, into per-shard pinned
//            staging (clock rows fan out to every shard), keeping each row's global event index on the host
//   upload   one copy thread per GPU: the shard's rows of chunk j go to HBM while chunk j-1 computes
//   compute  one thread per GPU: sg_push_view over the chunk (state carried between chunks = one stream)
//   deliver  the same thread: the chunk's matches are transposed on the GPU into SoA columns and copied back into
//            the shard's pinned ring while the next chunk computes
//   merge    (G > 1) host thread pool: chunk j's shard streams merged into the node's delivery order by (global
//            trigger, phase, global dense key) -- timer passes fan out to every shard; G = 1: the GPU delivers
//            straight into the caller's columns.
//
// Every stage of chunk j overlaps the other stages of chunks j-1 and j+1 (ring depth NODE_RING on the host,
// two device slots per GPU); no stage blocks another except through those rings.  A handle (sg_handle) is
// single-threaded: each is only ever driven by its shard's compute thread (and its copy thread's stream).
// Host threads come from process-wide pools (host_pool, pipeline_threads): no thread is started per node or push.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "keydict.h"
#include "router.h"
#include "sg_engine.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct sg_handle {   // (api.hip's definition)
  SgHandle h;
};

namespace {

const int NODE_RING = 3;   // host route/staging slots (chunk j reuses slot j % 3 once chunk j-3 is uploaded+merged)
const int MAX_GPUS = 16;

// non-temporal store of a 1/4/8-byte value (movnti for 4/8 bytes; a byte goes through the cache): host columns
// written once and read next by a DMA or by the caller skip the read-for-ownership of their lines
template <class V>
inline void nt_store(V* p, V v) {
  if constexpr (sizeof(V) == 4 || sizeof(V) == 8) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// (used by the host fill of trigger-row columns; A/B runs of streaming stores in the G > 1 host scatter and merge,
// profiles/r04/node_nt_ab.log, were inside the host stages' own run-to-run spread)
template <int BIT, class V>
inline void put(V* p, V v) {
  if (BIT == 1) nt_store(p, v);
  else *p = v;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Process-wide thread pool shared by every node: parallel_for(n, fn) runs fn(0..n-1) on the workers and the caller
// and returns when all are done.  Several coordinator threads may submit at once (their tasks interleave).  Workers
// live as long as the process (glibc gives each new thread a malloc arena of its own, kept after the thread exits:
// threads started per node or per push would keep adding arenas); grow() adds workers up to the largest host_threads
// a node asked for.
struct Pool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::function<void()>> q;
  void grow(int n) {
    std::lock_guard<std::mutex> lk(mu);
    while ((int)th.size() < n) {
      th.emplace_back([this] {
        while (true) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk2(mu);
            cv.wait(lk2, [&] { return !q.empty(); });
            f = std::move(q.back());
            q.pop_back();
          }
          f();
        }
      });
      th.back().detach();
    }
  }
  // Completion state of one parallel_for, shared by the submitter and every queued closure: the worker that finishes
  // the last task decrements and notifies under the mutex, and the closures own the state, so the submitter may
  // return (and its stack frame die) the moment it observes left == 0.
  struct Join {
    std::mutex m;
    std::condition_variable cv;
    int left = 0;
    std::exception_ptr err;
  };
  template <class F>
  void parallel_for(int n, F&& fn) {
    if (n <= 0) return;
    auto js = std::make_shared<Join>();
    js->left = n;
    // `fn` is only touched before this task's decrement, while the submitter is still waiting for it
    auto run = [js, &fn](int i) {
      std::exception_ptr e;
      try {
        fn(i);
      } catch (...) {
        e = std::current_exception();
      }
      std::lock_guard<std::mutex> lk(js->m);
      if (e && !js->err) js->err = e;
      if (--js->left == 0) js->cv.notify_all();
    };
    {
      std::lock_guard<std::mutex> lk(mu);
      for (int i = n - 1; i >= 1; --i) q.push_back([run, i] { run(i); });
    }
    cv.notify_all();
    run(0);
    // help with queued work while waiting (a submitter never idles behind its own tasks)
    while (true) {
      {
        std::lock_guard<std::mutex> lk(js->m);
        if (js->left == 0) break;
      }
      std::function<void()> f;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (!q.empty()) {
          f = std::move(q.back());
          q.pop_back();
        }
      }
      if (f) {
        f();
        continue;
      }
      std::unique_lock<std::mutex> lk(js->m);
      js->cv.wait_for(lk, std::chrono::milliseconds(1), [&] { return js->left == 0; });
    }
    if (js->err) std::rethrow_exception(js->err);
  }
};

Pool& host_pool() {
  static Pool* p = new Pool();   // (never destroyed: its detached workers outlive static destruction)
  return *p;
}

// Process-wide pipeline threads: a node push runs its per-GPU loops as tasks on parked threads, starting a new thread
// only when every one is busy -- the thread count stays at the largest number of loops that ran at once.
struct Task {
  std::function<void()> fn;
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  void join() {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return done; });
  }
};
struct ThreadCache {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::shared_ptr<Task>> q;
  int idle = 0;
  std::shared_ptr<Task> run(std::function<void()> fn) {
    auto t = std::make_shared<Task>();
    t->fn = std::move(fn);
    std::lock_guard<std::mutex> lk(mu);
    q.push_back(t);
    if ((int)q.size() > idle) {
      std::thread([this] { loop(); }).detach();
    } else {
      cv.notify_one();
    }
    return t;
  }
  void loop() {
    while (true) {
      std::shared_ptr<Task> t;
      {
        std::unique_lock<std::mutex> lk(mu);
        ++idle;
        cv.wait(lk, [&] { return !q.empty(); });
        --idle;
        t = q.front();
        q.erase(q.begin());
      }
      t->fn();
      {
        std::lock_guard<std::mutex> lk(t->m);
        t->done = true;
      }
      t->cv.notify_all();
    }
  }
};
ThreadCache& pipeline_threads() {
  static ThreadCache* c = new ThreadCache();   // (never destroyed, like host_pool)
  return *c;
}

// Pinned host buffer (hipHostMalloc), grow-only.
struct Pinned {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) hipHostFree(p);
    p = nullptr;
    bytes = 0;
    if (hipHostMalloc(&p, b ? b : 1, hipHostMallocDefault) != hipSuccess) throw SgError(SG_EHIP, "hipHostMalloc (node)");
    bytes = b;
  }
  ~Pinned() {
    if (p) hipHostFree(p);
  }
  template <class T> T* as() const { return (T*)p; }
};

// =====================================================================================================================
// GPU-side shard exchange (G > 1 with the device dictionary: every partitioned query without playback timers).
//
// The host only hands out contiguous row slices: GPU g uploads rows [lo + n*g/G, lo + n*(g+1)/G) of chunk j straight
// from the caller's columns.  On the device:
//   shard    k_xcount: each row's shard mix64(raw key) mod G (PartitionStreamReceiver.receive routes a row to its key's
//            runtime, C/partition/PartitionStreamReceiver.java:177-221) and per-block counts per shard; one scan;
//            k_xscatter: a stable counting scatter into a send buffer grouped by shard, arrival order kept, with each
//            row's global event index
//   exchange the G x G pieces go to their shard's receive slot (hipMemcpyPeerAsync when the GPUs differ, plain D2D
//            copies when shards share a device): rows, not state -- per-key state never moves (PartitionRuntime.java:
//            255-308 keeps one runtime per key)
//   compute  shard s dictionary-encodes its rows (keydict.hip) and runs them with their global indices as triggers
//   return   its matches, in delivery order, are cut by trigger slice (k_xbounds) and sent to the slice's GPU
//   merge    GPU g merges the G runs it receives -- every trigger's matches come from its key's shard, so the merge
//            is a placement by trigger (k_xmark + scan + k_xplace) -- and copies the merged columns straight into the
//            caller's columns at its offset (the host adds up G match counts per chunk).
// Host work is per chunk (counts, offsets, events), never per row or per match.  Rows of stream -1 (clock-only) are
// dropped: without playback timers they change no runtime.
// =====================================================================================================================
constexpr int XB_ROWS = 2048;   // rows per block of the shard count / scatter (8 per thread)

__device__ __forceinline__ uint64_t xmix64(uint64_t x) {   // (router.h sgr::mix64)
  x += 0x9E3779B97F4A7C15ull;
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

struct XCols {   // one row set's device columns
  int64_t* ts;
  int64_t* raw;
  int32_t* stream;
  uint64_t* gidx;
  void* col[SG_MAX_COLS];
  uint8_t* nul[SG_MAX_COLS];
};
struct XSpec {
  int32_t ncols;
  int32_t width[SG_MAX_COLS];   // 0: column not moved
  int32_t nul[SG_MAX_COLS];
  int32_t stream;
};

__global__ void __launch_bounds__(256) k_xcount(const int64_t* __restrict__ raw, const int32_t* __restrict__ stream,
                                                int64_t n, uint32_t G, uint8_t* __restrict__ shard,
                                                uint32_t* __restrict__ bcnt, uint32_t nblk) {
  __shared__ uint32_t c[MAX_GPUS];
  const uint32_t t = threadIdx.x, b = blockIdx.x;
  if (t < MAX_GPUS) c[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)b * XB_ROWS;
#pragma unroll
  for (int k = 0; k < XB_ROWS / 256; ++k) {
    const int64_t i = base + k * 256 + t;
    if (i >= n) break;
    const bool clock = stream && stream[i] < 0;
    const uint32_t s = clock ? 0xffu : (uint32_t)(xmix64((uint64_t)raw[i]) % G);
    shard[i] = (uint8_t)s;
    if (!clock) atomicAdd(&c[s], 1u);
  }
  __syncthreads();
  if (t < G) bcnt[(size_t)t * nblk + b] = c[t];
}

// per shard s: the start of its rows in the send buffer (boff[s * nblk]); [G] = rows sent
__global__ void k_xstarts(const uint32_t* __restrict__ boff, uint32_t nblk, uint32_t G, uint32_t* __restrict__ out) {
  const uint32_t s = threadIdx.x;
  if (s <= G) out[s] = boff[(size_t)s * nblk];
}

__global__ void __launch_bounds__(256) k_xscatter(XCols in, XCols out, XSpec sp, int64_t n, uint64_t gbase,
                                                  const uint8_t* __restrict__ shard, const uint32_t* __restrict__ boff,
                                                  uint32_t nblk, uint32_t G) {
  __shared__ uint32_t cur[MAX_GPUS];
  __shared__ uint32_t wc[4][MAX_GPUS];
  const uint32_t t = threadIdx.x, b = blockIdx.x, w = t >> 6, lane = t & 63;
  if (t < G) cur[t] = boff[(size_t)t * nblk + b];
  if (t < 4 * MAX_GPUS) wc[t / MAX_GPUS][t % MAX_GPUS] = 0;
  __syncthreads();
  uint32_t nb = 0;
  while ((1u << nb) < G) ++nb;
  const int64_t base = (int64_t)b * XB_ROWS;
  for (int k = 0; k < XB_ROWS / 256; ++k) {   // 256 rows per step, in arrival order
    const int64_t i = base + k * 256 + t;
    const uint32_t s = i < n ? shard[i] : 0xffu;
    const bool keep = s != 0xffu;
    // lanes of the wave with the same shard: rank among them and their count
    uint64_t m = __ballot(keep);
    for (uint32_t q = 0; q < nb; ++q) {
      const bool bit = (s >> q) & 1u;
      const uint64_t bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (keep && rank == 0) wc[w][s] = (uint32_t)__popcll(m);
    __syncthreads();
    if (keep) {
      uint32_t pos = cur[s] + rank;
      for (uint32_t q = 0; q < w; ++q) pos += wc[q][s];
      out.ts[pos] = in.ts[i];
      out.raw[pos] = in.raw[i];
      out.gidx[pos] = gbase + (uint64_t)i;
      if (sp.stream) out.stream[pos] = in.stream[i];
      for (int c = 0; c < sp.ncols; ++c) {
        if (sp.width[c] == 8) ((int64_t*)out.col[c])[pos] = ((const int64_t*)in.col[c])[i];
        else if (sp.width[c] == 4) ((int32_t*)out.col[c])[pos] = ((const int32_t*)in.col[c])[i];
        if (sp.nul[c]) out.nul[c][pos] = in.nul[c][i];
      }
    }
    __syncthreads();
    if (t < G) {
      cur[t] += wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t];
      wc[0][t] = wc[1][t] = wc[2][t] = wc[3][t] = 0;
    }
    __syncthreads();
    (void)lane;
  }
}

struct XSlices {
  uint64_t lo[MAX_GPUS + 1];   // global index of each slice's first row; [G] = the chunk's end
};
// matches of one shard (delivery order: triggers non-decreasing) -> the first match of each slice
__global__ void k_xbounds(const uint64_t* __restrict__ trig, int64_t k, XSlices sl, uint32_t G, int64_t* __restrict__ out) {
  const uint32_t g = threadIdx.x;
  if (g > G) return;
  int64_t a = 0, e = k;
  const uint64_t x = sl.lo[g];
  while (a < e) {
    const int64_t mid = a + (e - a) / 2;
    if (trig[mid] < x) a = mid + 1;
    else e = mid;
  }
  out[g] = a;
}

__global__ void k_xmapkeys(int32_t* __restrict__ key, int64_t k, const int32_t* __restrict__ l2g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < k && key[i] >= 0) key[i] = l2g[key[i]];
}

__global__ void k_xgather_u64(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t m,
                              uint64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) dst[i] = src[idx[i]];
}

struct XRuns {
  int64_t off[MAX_GPUS + 1];   // run r = merge-input rows [off[r], off[r + 1])
};
// merge input (G runs, each ordered by trigger; a trigger's matches all in one run): per trigger row of the slice, the
// length of its segment and where it starts
__global__ void k_xmark(const uint64_t* __restrict__ trig, int64_t M, XRuns runs, uint32_t G, uint64_t slo,
                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ seg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  uint32_t r = 0;
  while (r + 1 < G && runs.off[r + 1] <= i) ++r;
  const uint64_t x = trig[i];
  if (i > runs.off[r] && trig[i - 1] == x) return;
  int64_t e = i + 1;
  while (e < runs.off[r + 1] && trig[e] == x) ++e;
  cnt[x - slo] = (uint32_t)(e - i);
  seg[x - slo] = (uint32_t)i;
}

struct XLay {   // one SoA match layout (ColLayout offsets from a base)
  char* base;
  size_t off_trig, off_ts, off_key, off_grp, off_col[SG_MAX_SELECT], off_nul[SG_MAX_SELECT];
};
struct XWant {
  int32_t ts, key, grp, ns;
  int32_t width[SG_MAX_SELECT];   // 0: column not delivered
  int32_t nul[SG_MAX_SELECT];
};
__device__ __forceinline__ void xcopy_row(const XLay& a, int64_t i, const XLay& b, int64_t o, const XWant& w) {
  ((uint64_t*)(b.base + b.off_trig))[o] = ((const uint64_t*)(a.base + a.off_trig))[i];
  if (w.ts) ((int64_t*)(b.base + b.off_ts))[o] = ((const int64_t*)(a.base + a.off_ts))[i];
  if (w.key) ((int32_t*)(b.base + b.off_key))[o] = ((const int32_t*)(a.base + a.off_key))[i];
  if (w.grp) ((uint32_t*)(b.base + b.off_grp))[o] = ((const uint32_t*)(a.base + a.off_grp))[i];
  for (int c = 0; c < w.ns; ++c) {
    if (w.width[c] == 8) ((int64_t*)(b.base + b.off_col[c]))[o] = ((const int64_t*)(a.base + a.off_col[c]))[i];
    else if (w.width[c] == 4) ((int32_t*)(b.base + b.off_col[c]))[o] = ((const int32_t*)(a.base + a.off_col[c]))[i];
    if (w.nul[c]) ((uint8_t*)(b.base + b.off_nul[c]))[o] = ((const uint8_t*)(a.base + a.off_nul[c]))[i];
  }
}
__global__ void k_xplace(XLay in, int64_t M, uint64_t slo, const uint32_t* __restrict__ off,
                         const uint32_t* __restrict__ seg, XLay out, XWant w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint64_t t = ((const uint64_t*)(in.base + in.off_trig))[i] - slo;
  xcopy_row(in, i, out, (int64_t)off[t] + (i - (int64_t)seg[t]), w);
}

// ---- host side of the exchange ---------------------------------------------------------------------------------
struct XBuf {   // device buffer, grow-only (the caller makes sure no queued work still reads the old one)
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    bytes = 0;
    HIPCHK(hipMalloc(&p, b ? b : 1));
    bytes = b;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T* as() const { return (T*)p; }
};

struct XRows {   // columns of up to `cap` rows in one allocation
  XBuf buf;
  int64_t cap = 0;
  XCols c;
};

void xrows_layout(XRows& r, int64_t cap, const XSpec& sp, bool gidx) {
  cap = std::max(cap, r.cap);
  auto sz = [&](size_t w) { return ((w * (size_t)cap + 255) / 256) * 256; };
  size_t bytes = 2 * sz(8) + (gidx ? sz(8) : 0) + (sp.stream ? sz(4) : 0);
  for (int c = 0; c < sp.ncols; ++c) bytes += (sp.width[c] ? sz((size_t)sp.width[c]) : 0) + (sp.nul[c] ? sz(1) : 0);
  r.buf.ensure(bytes);
  r.cap = cap;
  char* q = r.buf.as<char>();
  memset(&r.c, 0, sizeof(r.c));
  auto take = [&](size_t w) { char* x = q; q += sz(w); return x; };
  r.c.ts = (int64_t*)take(8);
  r.c.raw = (int64_t*)take(8);
  if (gidx) r.c.gidx = (uint64_t*)take(8);
  if (sp.stream) r.c.stream = (int32_t*)take(4);
  for (int c = 0; c < sp.ncols; ++c) {
    if (sp.width[c]) r.c.col[c] = take((size_t)sp.width[c]);
    if (sp.nul[c]) r.c.nul[c] = (uint8_t*)take(1);
  }
}

struct XGpu {
  XRows in[2], send[2];
  XBuf shard, bcnt, boff, scan_tmp, starts, bounds, mcnt, mseg, moff, mscan_tmp, l2g, nfg;
  XBuf min[2], mo[2];
  int64_t min_cap[2] = {0, 0}, mo_cap[2] = {0, 0};
  int64_t l2g_n = 0;
  Pinned hstarts[2], hbounds, hnf;
  hipStream_t xs = nullptr;
  hipEvent_t ev_in[2] = {}, ev_scat[2] = {}, ev_sent[2] = {}, ev_rfree[2] = {}, ev_osent[2] = {}, ev_mfree[2] = {},
             ev_d2h[2] = {};
  bool init = false;
  void release() {
    for (int p = 0; p < 2; ++p) {
      in[p].buf.release();
      send[p].buf.release();
      in[p].cap = send[p].cap = 0;
      min[p].release();
      mo[p].release();
      min_cap[p] = mo_cap[p] = 0;
    }
    for (XBuf* b : {&shard, &bcnt, &boff, &scan_tmp, &starts, &bounds, &mcnt, &mseg, &moff, &mscan_tmp, &l2g, &nfg})
      b->release();
    l2g_n = 0;
    if (xs) hipStreamDestroy(xs);
    xs = nullptr;
    for (hipEvent_t* e : {ev_in, ev_scat, ev_sent, ev_rfree, ev_osent, ev_mfree, ev_d2h})
      for (int p = 0; p < 2; ++p) {
        if (e[p]) hipEventDestroy(e[p]);
        e[p] = nullptr;
      }
    init = false;
  }
};

}  // namespace

// One shard's rows of one chunk, in arrival order (host staging, G > 1).
struct NodeStage {
  Pinned ts, ts32, key, stream, gidx;   // (ts32: the chunk's timestamps as 32-bit offsets from its minimum)
  Pinned col[SG_MAX_COLS], nul[SG_MAX_COLS];
};

// One shard's delivered matches (pinned ring of M rows, G > 1).
struct NodeRing {
  int64_t M = 0;
  Pinned trig, ts, key, grp;
  Pinned col[SG_MAX_SELECT], nul[SG_MAX_SELECT];
};

struct sg_node {
  int G = 1;
  int dev[MAX_GPUS] = {};
  sg_nfa_desc desc;
  sg_options opt;
  sg_handle* h[MAX_GPUS] = {};
  sg_router* router = nullptr;
  int threads = 16;
  int64_t chunk_rows = 0;
  Pool* pool = nullptr;
  std::string err;
  sg_node_stats st;
  int64_t local_rows[MAX_GPUS] = {};   // rows each shard has seen (its local event index space)
  int64_t next_index = 0;
  bool broken = false;
  bool no_fill = false;
  bool no_ts32 = false;              // testing: timestamps always travel as 8 bytes              // testing: ship every column back instead of filling trigger-row columns on the host
  // per-GPU device-side ingress slots and copy stream
  hipStream_t cp[MAX_GPUS] = {};
  hipEvent_t ev_copied[MAX_GPUS][2] = {}, ev_used[MAX_GPUS][2] = {};
  SlotPtrs dslot[MAX_GPUS][2];       // device ingress slots (resolved once, before the pipeline's threads start)
  // host staging: route slot per chunk (G = 1: the routed key column; G > 1: per-shard rows)
  Pinned keyslot[NODE_RING];
  Pinned tsslot[NODE_RING];          // G = 1: the chunk's timestamps as 32-bit offsets
  int32_t* dts32[MAX_GPUS][2] = {};  // device slots of the 32-bit offsets
  int64_t dts32_rows = 0;
  std::vector<int32_t> dense_tmp[NODE_RING];
  NodeStage stage[NODE_RING][MAX_GPUS];
  NodeRing ring[MAX_GPUS];
  // key dictionary: the host router (sg_router) or one device dictionary per GPU (keydict.h)
  int key_dict_mode = 0;             // 0 auto, 1 host, 2 device (sg_node_set_key_dict)
  int ddict = -1;                    // decided at the first push of a stream: 1 device, 0 host
  KeyDict kd[MAX_GPUS];
  int64_t* draw[MAX_GPUS][2] = {};   // device raw-key slots
  int64_t draw_rows = 0;
  std::vector<int32_t> l2g[MAX_GPUS];   // G > 1, device mode: shard-local id -> node-wide first-seen id
  XGpu x[MAX_GPUS];                  // G > 1, device mode: the GPU-side shard exchange's buffers, streams, events
  int64_t g_keys = 0;
};

namespace {

// What every shard delivers: the caller's columns plus, for the merge, trigger (always) and phase / key when two
// shards can produce matches for the same trigger (timer passes fan out to every shard).  Columns the host can read
// from the trigger row itself are not shipped back over PCIe at all (`fill`): for the closed form `every A -> B[..]`
// the output timestamp is the trigger's (StateEvent.timestamp is set by the event that completed the match,
// C/query/input/stream/state/StreamPostStateProcessor.java:53-72) and every B.attr projection is the trigger row's
// attribute (QuerySelector.processNoGroupBy, C/query/selector/QuerySelector.java:125-163) -- the host selector copies
// them from the caller's pinned input columns by global trigger index.
struct Want {
  bool ts, key, grp, col[SG_MAX_SELECT], nul[SG_MAX_SELECT];
  int ns;
  int width[SG_MAX_SELECT];
  bool fill_ts;                 // out->ts from the trigger row's ts (host)
  int fill_col[SG_MAX_SELECT];  // >= 0: out->cols[k] (and nulls[k]) from batch column fill_col[k] at the trigger row
  bool any_fill;
};

Want want_of(const sg_node& nd, const sg_node_batch& b, const sg_match_columns* out, bool allow_fill) {
  Want w;
  memset(&w, 0, sizeof(w));
  const sg_nfa_desc& d = nd.desc;
  w.ns = d.n_out > 0 ? d.n_out : d.n_select;
  const bool tie = nd.G > 1 && d.shape != SG_SHAPE_EVERY_NEXT_CMP;
  const bool closed = allow_fill && d.shape == SG_SHAPE_EVERY_NEXT_CMP && d.n_out == 0 && !nd.no_fill;
  const int b_state = d.shape_args[1];
  w.ts = out->ts != nullptr;
  w.fill_ts = closed && w.ts;
  if (w.fill_ts) w.ts = false;
  w.key = out->key != nullptr || tie;
  w.grp = out->group != nullptr || tie;
  for (int k = 0; k < w.ns; ++k) {
    w.col[k] = out->cols[k] != nullptr;
    w.nul[k] = out->nulls[k] != nullptr;
    w.width[k] = sg_col_width(d.n_out > 0 ? d.out_type[k] : d.sel_type[k]);
    w.fill_col[k] = -1;
    if (!closed || (!w.col[k] && !w.nul[k])) continue;
    const int c = d.ret_col[d.sel_ret[k]];
    const bool single = d.sel_index[k] == 0 || d.sel_index[k] == -1;
    if (d.sel_state[k] == b_state && single && d.sel_type[k] == d.col_type[c] && b.cols && b.cols[c] &&
        true) {
      w.fill_col[k] = c;
      w.col[k] = w.nul[k] = false;
    }
  }
  w.any_fill = w.fill_ts;
  for (int k = 0; k < w.ns; ++k) w.any_fill |= w.fill_col[k] >= 0;
  return w;
}

// Host selector for the trigger-row columns of output rows [o0, o1): trig[] holds their global trigger indices.
inline void fill_row(const sg_node_batch& b, const sg_nfa_desc& d, const Want& w, const sg_match_columns* out,
                     int64_t o, uint64_t trig) {
  const int64_t t = (int64_t)(trig - b.base_index);
  if (w.fill_ts) put<1>(&out->ts[o], b.ts[t]);
  for (int k = 0; k < w.ns; ++k) {
    const int c = w.fill_col[k];
    if (c < 0) continue;
    if (out->cols[k]) {
      if (w.width[k] == 8) put<1>(&((int64_t*)out->cols[k])[o], ((const int64_t*)b.cols[c])[t]);
      else put<1>(&((int32_t*)out->cols[k])[o], ((const int32_t*)b.cols[c])[t]);
    }
    if (out->nulls[k]) out->nulls[k][o] = (b.nulls && b.nulls[c]) ? b.nulls[c][t] : 0;
  }
  (void)d;
}

// Pipeline state of one sg_node_push call.
struct Run {
  sg_node& nd;
  const sg_node_batch& b;
  const sg_match_columns* out;
  int64_t cap;
  Want w;
  int64_t nch = 0, C = 0;
  std::mutex mu;
  std::condition_variable cv;
  bool failed = false;
  int fail_code = 0;
  std::string fail_msg;
  int64_t routed = 0;                        // chunks routed (staging complete)
  int64_t uploaded[MAX_GPUS] = {};           // chunks whose H2D completed, per shard
  int64_t issued[MAX_GPUS] = {};             // chunks whose H2D was issued (ev_copied recorded)
  int64_t used[MAX_GPUS] = {};               // chunks whose compute was issued (ev_used recorded)
  int64_t delivered[MAX_GPUS] = {};          // chunks whose matches are in host memory
  int64_t merged = 0;                        // chunks merged (G > 1)
  std::vector<int64_t> dlv_end[MAX_GPUS];    // ring position after chunk j
  int64_t ring_tail[MAX_GPUS] = {};          // rows of the ring the merge has consumed
  int64_t out_rows = 0;                      // rows written to the caller's columns
  // per (chunk, shard): rows, key bound and local index of row 0 (fixed when the chunk is routed)
  std::vector<int64_t> rows_of, lbase_of;
  std::vector<int32_t> kb_of;
  // per chunk: timestamps travel as 32-bit offsets from ts_base_of[j] when the chunk spans less than 2^31 ms
  std::vector<int64_t> ts_base_of;
  std::vector<uint8_t> ts32_of;
  double t_route = 0, t_merge = 0, t_gpu[MAX_GPUS] = {};
  // GPU-side shard exchange (x_loop): per (chunk, GPU) send starts per shard and match bounds per slice (G + 1 each),
  // new keys' first global rows; per GPU the chunks past each step
  std::vector<int64_t> xst, xpc, xkbase;
  std::vector<std::vector<uint64_t>> xnf;
  int64_t xcounted[MAX_GPUS] = {}, xsent[MAX_GPUS] = {}, xused[MAX_GPUS] = {}, xnfp[MAX_GPUS] = {},
          xpieced[MAX_GPUS] = {}, xmready[MAX_GPUS] = {}, xosent[MAX_GPUS] = {};
  int64_t xids = 0;
  int64_t h2d_bytes = 0, d2h_bytes = 0;

  Run(sg_node& n, const sg_node_batch& bb, const sg_match_columns* o, int64_t c) : nd(n), b(bb), out(o), cap(c) {}

  void fail(int code, const std::string& m) {
    std::lock_guard<std::mutex> lk(mu);
    if (!failed) {
      failed = true;
      fail_code = code;
      fail_msg = m;
    }
    cv.notify_all();
  }
  // wait until pred() or failure; returns false on failure
  template <class P>
  bool wait(P pred) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return failed || pred(); });
    return !failed;
  }
  void publish(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      f();
    }
    cv.notify_all();
  }
  template <class F>
  void guarded(F&& f) {
    try {
      f();
    } catch (SgError& e) {
      fail(e.code, e.msg);
    } catch (std::exception& e) {
      fail(SG_EINVAL, e.what());
    }
  }
};

int64_t chunk_lo(const Run& r, int64_t j) { return std::min(r.b.n, j * r.C); }

// playback queries with timers (absence states) need every row's clock on every shard
bool need_clocks(const sg_nfa_desc& d) { return d.playback && d.n_sched > 0; }

// row lo + i starts a new timestamp (the first row of a thread's slice always counts: a repeated clock row at an
// unchanged time fires nothing)
inline bool is_clock_point(const Run& r, int64_t lo, int64_t slice_a, int64_t i) {
  return i == slice_a || r.b.ts[lo + i] != r.b.ts[lo + i - 1];
}

// Chunk j's timestamps as 32-bit offsets from its first row's when every row is within 2^31 ms of it (G = 1:
// written into the host slot in the same pass; G > 1: by the scatter).  Halves the timestamp column's PCIe bytes.
void ts_prepare(Run& r, int64_t j) {
  sg_node& nd = r.nd;
  const int slot = (int)(j % NODE_RING);
  const int64_t lo = chunk_lo(r, j), hi = chunk_lo(r, j + 1), n = hi - lo;
  r.ts32_of[j] = 0;
  if (n <= 0 || nd.no_ts32) return;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nd.threads, n / 65536 + 1));
  const int64_t* ts = r.b.ts + lo;
  const int64_t base = ts[0];
  int32_t* o = nd.G == 1 ? nd.tsslot[slot].as<int32_t>() : nullptr;
  std::atomic<bool> wide(false);
  nd.pool->parallel_for(T, [&](int t) {
    const int64_t a = n * t / T, e = n * (t + 1) / T;
    uint64_t bad = 0;
    if (o) {
      for (int64_t i = a; i < e; ++i) {
        const int64_t d = ts[i] - base;
        bad |= (uint64_t)(d + 0x80000000ll) >> 32;   // nonzero unless INT32_MIN <= d <= INT32_MAX
        o[i] = (int32_t)d;
      }
    } else {
      for (int64_t i = a; i < e; ++i) bad |= (uint64_t)(ts[i] - base + 0x80000000ll) >> 32;
    }
    if (bad) wide = true;
  });
  r.ts_base_of[j] = base;
  r.ts32_of[j] = wide ? 0 : 1;
}

// staged timestamp of shard row p of chunk j
inline void put_ts(const Run& r, NodeStage& S, int64_t j, int64_t p, int64_t ts) {
  if (r.ts32_of[j]) S.ts32.as<int32_t>()[p] = (int32_t)(ts - r.ts_base_of[j]);
  else S.ts.as<int64_t>()[p] = ts;
}

// ---- device-dictionary mode, one GPU: no key lookups on the host (G > 1: the GPU-side shard exchange, x_loop)
void route_chunk_dev(Run& r, int64_t j) {
  r.rows_of[j] = chunk_lo(r, j + 1) - chunk_lo(r, j);
}

// ---- route (+ scatter) of chunk j into host slot j % NODE_RING --------------------------------------------------
void route_chunk(Run& r, int64_t j) {
  ts_prepare(r, j);
  if (r.nd.ddict == 1) {
    route_chunk_dev(r, j);
    return;
  }
  sg_node& nd = r.nd;
  const sg_nfa_desc& d = nd.desc;
  const int slot = (int)(j % NODE_RING);
  const int64_t lo = chunk_lo(r, j), hi = chunk_lo(r, j + 1), n = hi - lo;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nd.threads, n / 65536 + 1));
  auto slice = [&](int t, int64_t& a, int64_t& e) {
    a = n * t / T;
    e = n * (t + 1) / T;
  };
  const int32_t* stream = r.b.stream ? r.b.stream + lo : nullptr;
  if (!d.partitioned) {   // one runtime: no keys (replicas only, G = 1)
    int32_t* kd = nd.keyslot[slot].as<int32_t>();
    nd.pool->parallel_for(T, [&](int t) {
      int64_t a, e;
      slice(t, a, e);
      memset(kd + a, 0, (size_t)(e - a) * 4);
    });
    r.rows_of[j] = n;
    r.kb_of[j] = 1;
    return;
  }
  sg_router* rt = nd.router;
  const int64_t* raw = r.b.raw_key + lo;
  int32_t* dense = nd.G == 1 ? nd.keyslot[slot].as<int32_t>() : nd.dense_tmp[slot].data();
  std::vector<sgr::SliceMiss> miss(T);
  const int G = nd.G;
  // playback timers (absence states) fire when the app's clock reaches a row's time, for every key
  // (TimestampGeneratorImpl.setCurrentTimestamp, C/util/timestamp/TimestampGeneratorImpl.java:106-125): every shard
  // gets a clock-only row at each new timestamp of a row it does not own, with that row's global index
  const bool clocks = G > 1 && need_clocks(d);
  std::vector<std::vector<int64_t>> cnt(T, std::vector<int64_t>(G, 0));
  // 1. lookups; hits are counted per shard
  nd.pool->parallel_for(T, [&](int t) {
    int64_t a, e;
    slice(t, a, e);
    sgr::lookup_slice(rt->dict, raw + a, e - a, dense + a, miss[t]);
    if (stream)   // clock-only rows (stream -1) carry no key: every shard sees them
      for (int64_t i = a; i < e; ++i)
        if (stream[i] < 0) dense[i] = -1;
    if (G > 1) {
      const int32_t* so = rt->shard_of.data();
      int64_t* c = cnt[t].data();
      int64_t bcast = 0;
      for (int64_t i = a; i < e; ++i) {
        const int32_t x = dense[i];
        if (x >= 0) ++c[so[x]];
        else if (x == -1) ++bcast;
        if (clocks && x != -1 && is_clock_point(r, lo, a, i)) ++bcast;   // (the owner's share is taken back below)
      }
      for (int s = 0; s < G; ++s) c[s] += bcast;
    }
  });
  // 2. new keys, first-seen order
  std::vector<std::vector<int32_t>> remap(T);
  bool any = false;
  for (int t = 0; t < T; ++t) {
    if (!miss[t].any) continue;
    any = true;
    remap[t].resize(miss[t].fresh.size());
    for (size_t q = 0; q < miss[t].fresh.size(); ++q) remap[t][q] = rt->add_key(miss[t].fresh[q]);
  }
  if (any)
    nd.pool->parallel_for(T, [&](int t) {
      if (!miss[t].any) return;
      int64_t a, e;
      slice(t, a, e);
      const int32_t* rm = remap[t].data();
      const int32_t* so = rt->shard_of.data();
      for (int64_t i = a; i < e; ++i) {
        const int32_t x = dense[i];
        if (x >= -1) continue;
        const int32_t id = rm[-x - 2];
        dense[i] = id;
        if (G > 1) ++cnt[t][so[id]];
      }
    });
  if (clocks)   // a clock point was counted for every shard: its owner gets the row itself instead
    nd.pool->parallel_for(T, [&](int t) {
      int64_t a, e;
      slice(t, a, e);
      const int32_t* so = rt->shard_of.data();
      for (int64_t i = a; i < e; ++i)
        if (dense[i] >= 0 && is_clock_point(r, lo, a, i)) --cnt[t][so[dense[i]]];
    });
  for (int s = 0; s < G; ++s) r.kb_of[j * G + s] = std::max<int32_t>(1, rt->shard_keys[s]);
  if (G == 1) {   // dense ids are the shard's ids; clock rows keep -1 (no key)
    r.rows_of[j] = n;
    return;
  }
  // 3. scatter into per-shard staging, arrival order kept
  std::vector<std::vector<int64_t>> off(T, std::vector<int64_t>(G, 0));
  for (int s = 0; s < G; ++s) {
    int64_t o = 0;
    for (int t = 0; t < T; ++t) {
      off[t][s] = o;
      o += cnt[t][s];
    }
    r.rows_of[j * G + s] = o;
  }
  const int nc = d.n_cols;
  int need[SG_MAX_COLS] = {};
  for (int k = 0; k < d.n_ret; ++k) need[d.ret_col[k]] = 1;
  const bool stage_stream = stream != nullptr || clocks;
  nd.pool->parallel_for(T, [&](int t) {
    int64_t a, e;
    slice(t, a, e);
    const int32_t* so = rt->shard_of.data();
    const int32_t* lc = rt->local_of.data();
    int64_t cur[MAX_GPUS];
    for (int s = 0; s < G; ++s) cur[s] = off[t][s];
    for (int64_t i = a; i < e; ++i) {
      const int32_t x = dense[i];
      const int own = x >= 0 ? so[x] : -1;
      const bool fan = x < 0 || (clocks && is_clock_point(r, lo, a, i));
      for (int s = 0; s < G; ++s) {
        if (s != own && !fan) continue;
        const bool clock = s != own;   // a clock-only row on a shard that does not own the row
        NodeStage& S = nd.stage[slot][s];
        const int64_t p = cur[s]++;
        put_ts(r, S, j, p, r.b.ts[lo + i]);
        S.key.as<int32_t>()[p] = clock ? -1 : lc[x];
        if (stage_stream) S.stream.as<int32_t>()[p] = clock ? -1 : (stream ? stream[i] : 0);
        S.gidx.as<uint64_t>()[p] = r.b.base_index + (uint64_t)(lo + i);
        if (clock) {
          for (int c = 0; c < nc; ++c) {
            if (!need[c] || !r.b.cols[c]) continue;
            if (sg_col_width(d.col_type[c]) == 8) S.col[c].as<int64_t>()[p] = 0;
            else S.col[c].as<int32_t>()[p] = 0;
            if (r.b.nulls && r.b.nulls[c]) S.nul[c].as<uint8_t>()[p] = 1;
          }
          continue;
        }
        for (int c = 0; c < nc; ++c) {
          if (!need[c] || !r.b.cols[c]) continue;
          if (sg_col_width(d.col_type[c]) == 8) S.col[c].as<int64_t>()[p] = ((const int64_t*)r.b.cols[c])[lo + i];
          else S.col[c].as<int32_t>()[p] = ((const int32_t*)r.b.cols[c])[lo + i];
          if (r.b.nulls && r.b.nulls[c]) S.nul[c].as<uint8_t>()[p] = r.b.nulls[c][lo + i];
        }
      }
    }
  });
}

// The sg_batch of shard s's rows of chunk j (host memory).
sg_batch shard_batch(Run& r, int64_t j, int s, const void** cols, const uint8_t** nuls) {
  sg_node& nd = r.nd;
  const sg_nfa_desc& d = nd.desc;
  const int slot = (int)(j % NODE_RING);
  sg_batch sb;
  memset(&sb, 0, sizeof(sb));
  sb.on_device = 0;
  sb.key_bound = r.kb_of[j * nd.G + s];
  sb.n = r.rows_of[j * nd.G + s];
  int need[SG_MAX_COLS] = {};
  for (int k = 0; k < d.n_ret; ++k) need[d.ret_col[k]] = 1;
  if (nd.G == 1) {
    const int64_t lo = chunk_lo(r, j);
    sb.base_index = r.b.base_index + (uint64_t)lo;
    sb.ts = r.ts32_of[j] ? nullptr : r.b.ts + lo;
    sb.stream = r.b.stream ? r.b.stream + lo : nullptr;
    sb.key = nd.ddict == 1 ? nullptr : nd.keyslot[slot].as<int32_t>();   // (device mode: raw keys go up instead)
    bool nul = false;
    for (int c = 0; c < d.n_cols; ++c) {
      cols[c] = (need[c] && r.b.cols[c]) ? (const char*)r.b.cols[c] + (size_t)sg_col_width(d.col_type[c]) * lo : nullptr;
      nuls[c] = (need[c] && r.b.nulls && r.b.nulls[c]) ? r.b.nulls[c] + lo : nullptr;
      nul |= nuls[c] != nullptr;
    }
    sb.cols = cols;
    sb.nulls = nul ? nuls : nullptr;
    return sb;
  }
  NodeStage& S = nd.stage[slot][s];
  sb.base_index = (uint64_t)r.lbase_of[j * nd.G + s];   // local index space: the host maps triggers back through gidx
  sb.ts = r.ts32_of[j] ? nullptr : S.ts.as<int64_t>();
  sb.stream = (r.b.stream || need_clocks(d)) ? S.stream.as<int32_t>() : nullptr;
  sb.key = nd.ddict == 1 ? nullptr : S.key.as<int32_t>();
  bool nul = false;
  for (int c = 0; c < d.n_cols; ++c) {
    cols[c] = (need[c] && r.b.cols[c]) ? S.col[c].p : nullptr;
    nuls[c] = (need[c] && r.b.nulls && r.b.nulls[c]) ? S.nul[c].as<uint8_t>() : nullptr;
    nul |= nuls[c] != nullptr;
  }
  sb.cols = cols;
  sb.nulls = nul ? nuls : nullptr;
  return sb;
}

// ---- per-GPU copy thread: H2D of shard s's rows, two device slots ------------------------------------------------
void copy_loop(Run& r, int s) {
  sg_node& nd = r.nd;
  r.guarded([&] {
    HIPCHK(hipSetDevice(nd.dev[s]));
    for (int64_t j = 0; j < r.nch; ++j) {
      if (!r.wait([&] { return r.routed > j && (j < 2 || r.used[s] >= j - 1); })) return;
      const int ds = (int)(j & 1);
      if (j >= 2) HIPCHK(hipStreamWaitEvent(nd.cp[s], nd.ev_used[s][ds], 0));   // device slot free again
      const void* cols[SG_MAX_COLS];
      const uint8_t* nuls[SG_MAX_COLS];
      sg_batch sb = shard_batch(r, j, s, cols, nuls);
      // (the slot's buffers were reserved for a whole chunk before the pipeline started: no workspace-map access
      // from this thread)
      if (sb.n > 0) sg_upload_to(nd.desc, nd.dslot[s][ds], &sb, 0, sb.n, nd.cp[s]);
      if (sb.n > 0 && r.ts32_of[j]) {
        const int32_t* t32 = nd.G == 1 ? nd.tsslot[j % NODE_RING].as<int32_t>() : nd.stage[j % NODE_RING][s].ts32.as<int32_t>();
        HIPCHK(hipMemcpyAsync(nd.dts32[s][ds], t32, 4 * (size_t)sb.n, hipMemcpyHostToDevice, nd.cp[s]));
      }
      if (sb.n > 0 && nd.ddict == 1) {
        const int64_t* rk = r.b.raw_key + chunk_lo(r, j);   // (device dictionary: one GPU here)
        HIPCHK(hipMemcpyAsync(nd.draw[s][ds], rk, 8 * (size_t)sb.n, hipMemcpyHostToDevice, nd.cp[s]));
      }
      HIPCHK(hipEventRecord(nd.ev_copied[s][ds], nd.cp[s]));
      r.publish([&] { r.issued[s] = j + 1; });
      HIPCHK(hipEventSynchronize(nd.ev_copied[s][ds]));
      int64_t bytes = (r.ts32_of[j] ? 4 : 8) * sb.n + (sb.stream ? 4 * sb.n : 0) + (nd.ddict == 1 ? 8 : 4) * sb.n;
      for (int c = 0; c < nd.desc.n_cols; ++c) {
        if (sb.cols[c]) bytes += (int64_t)sg_col_width(nd.desc.col_type[c]) * sb.n;
        if (sb.nulls && sb.nulls[c]) bytes += sb.n;
      }
      r.publish([&] { r.uploaded[s] = j + 1; r.h2d_bytes += bytes; });
    }
  });
}

// ---- per-GPU compute + deliver thread --------------------------------------------------------------------------
__global__ void k_ts_widen(const int32_t* __restrict__ d, int64_t base, int64_t n, int64_t* __restrict__ ts) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ts[i] = base + (int64_t)d[i];
}

struct Dst {   // where delivered rows go: the caller's columns (G = 1) or the shard's ring (G > 1)
  uint64_t* trig;
  int64_t* ts;
  int32_t* key;
  uint32_t* grp;
  void* col[SG_MAX_SELECT];
  uint8_t* nul[SG_MAX_SELECT];
  int64_t M;   // ring size (rows wrap at M); G = 1: no wrap
};

// transpose all pending matches of h into staging slot es and copy them to dst rows [pos, pos + k) (mod M)
void deliver(Run& r, SgHandle& h, const Dst& dst, int64_t pos, int64_t k, int es) {
  const sg_nfa_desc& d = h.desc;
  const Want& w = r.w;
  sg_egress_init(h);
  const ColLayout L = sg_col_layout(d, k);
  // (reserve_all sized both slots for a chunk's worth of matches; a larger chunk output grows the slot here, which
  // synchronises the device once)
  sg_stage_reserve(h, es, (int64_t)L.bytes);
  char* st = h.eg.stage[es];
  HIPCHK(hipStreamWaitEvent(h.stream, h.eg.done[es], 0));
  sg_launch_to_columns(k, h.out.rec, h.out.stride, L, st, h.stream);
  HIPCHK(hipEventRecord(h.eg.ready[es], h.stream));
  h.out.n = 0;   // all consumed (the next push writes after the transpose in stream order)
  HIPCHK(hipStreamWaitEvent(h.eg.d2h, h.eg.ready[es], 0));
  int64_t bytes = 0;
  // every D2H destination range checked on the host before it is issued: G = 1 rows [pos, pos + k) of the caller's
  // columns (capacity r.cap), G > 1 rows of the shard's ring of M rows (at most two pieces, each inside the ring)
  if (pos < 0 || k < 0 || (dst.M == 0 && pos + k > r.cap) || (dst.M > 0 && k > dst.M))
    throw SgError(SG_EINVAL, "internal: node delivery range [" + std::to_string(pos) + ", " + std::to_string(pos + k) +
                                 ") outside its destination");
  auto cp = [&](void* base, size_t off, size_t width) {
    if (!base) return;
    const int64_t p = dst.M ? pos % dst.M : pos;
    const int64_t first = dst.M ? std::min<int64_t>(k, dst.M - p) : k;
    if (p < 0 || first < 0 || (dst.M > 0 && (p + first > dst.M || k - first > dst.M)))
      throw SgError(SG_EINVAL, "internal: node ring delivery piece outside the ring");
    HIPCHK(hipMemcpyAsync((char*)base + width * (size_t)p, st + off, width * (size_t)first, hipMemcpyDeviceToHost, h.eg.d2h));
    if (first < k)
      HIPCHK(hipMemcpyAsync(base, st + off + width * (size_t)first, width * (size_t)(k - first), hipMemcpyDeviceToHost,
                            h.eg.d2h));
    bytes += (int64_t)(width * (size_t)k);
  };
  cp(dst.trig, L.off_trig, 8);
  if (w.ts) cp(dst.ts, L.off_ts, 8);
  if (w.key) cp(dst.key, L.off_key, 4);
  if (w.grp) cp(dst.grp, L.off_grp, 4);
  for (int c = 0; c < w.ns; ++c) {
    if (w.col[c]) cp(dst.col[c], L.off_col[c], (size_t)L.width[c]);
    if (w.nul[c]) cp(dst.nul[c], L.off_nul[c], 1);
  }
  HIPCHK(hipEventRecord(h.eg.done[es], h.eg.d2h));
  std::lock_guard<std::mutex> lk(r.mu);
  r.d2h_bytes += bytes;
}

void gpu_loop(Run& r, int s) {
  sg_node& nd = r.nd;
  SgHandle& h = nd.h[s]->h;
  r.guarded([&] {
    HIPCHK(hipSetDevice(nd.dev[s]));
    Dst dst;
    memset(&dst, 0, sizeof(dst));
    if (nd.G == 1) {
      dst.trig = r.out->trigger;
      dst.ts = r.out->ts;
      dst.key = r.out->key;
      dst.grp = r.out->group;
      for (int c = 0; c < r.w.ns; ++c) {
        dst.col[c] = r.out->cols[c];
        dst.nul[c] = r.out->nulls[c];
      }
      dst.M = 0;
    } else {
      NodeRing& R = nd.ring[s];
      dst.trig = R.trig.as<uint64_t>();
      dst.ts = R.ts.as<int64_t>();
      dst.key = R.key.as<int32_t>();
      dst.grp = R.grp.as<uint32_t>();
      for (int c = 0; c < r.w.ns; ++c) { dst.col[c] = R.col[c].p; dst.nul[c] = R.nul[c].as<uint8_t>(); }
      dst.M = R.M;
    }
    int64_t pos = 0;
    int es = 0;
    for (int64_t j = 0; j < r.nch; ++j) {
      if (!r.wait([&] { return r.issued[s] > j; })) return;
      const double t0 = now_ms();
      const int ds = (int)(j & 1);
      HIPCHK(hipStreamWaitEvent(h.stream, nd.ev_copied[s][ds], 0));
      const void* cols[SG_MAX_COLS];
      const uint8_t* nuls[SG_MAX_COLS];
      sg_batch sb = shard_batch(r, j, s, cols, nuls);
      int64_t k = 0;
      if (sb.n > 0) {
        // the device view of the slot the copy thread filled
        BatchView bv;
        memset(&bv, 0, sizeof(bv));
        bv.n = sb.n;
        bv.base_index = sb.base_index;
        bv.key_bound = sb.key_bound;
        const SlotPtrs& sp = nd.dslot[s][ds];
        bv.ts = (const int64_t*)sp.ts;
        bv.stream = sb.stream ? (const int32_t*)sp.stream : nullptr;
        bv.key = (const int32_t*)sp.key;
        bv.index = nullptr;
        if (r.ts32_of[j]) {   // widen the 32-bit offsets into the slot's timestamp column
          hipLaunchKernelGGL(k_ts_widen, dim3((unsigned)std::min<int64_t>((sb.n + 255) / 256, 8192)), dim3(256), 0,
                             h.stream, (const int32_t*)nd.dts32[s][ds], r.ts_base_of[j], sb.n, (int64_t*)sp.ts);
          HIPCHK(hipGetLastError());
        }
        if (nd.ddict == 1) {   // dictionary-encode the chunk's raw keys on this GPU
          kd_resolve(nd.kd[s], nd.draw[s][ds], bv.stream, sb.n, (int32_t*)sp.key, h.stream, nullptr);
          bv.key_bound = (int32_t)std::max<int64_t>(1, nd.kd[s].n_keys);
        }
        for (int c = 0; c < nd.desc.n_cols; ++c) {
          bv.cols.col[c] = sb.cols[c] ? sp.col[c] : nullptr;
          bv.cols.nul[c] = (sb.nulls && sb.nulls[c]) ? (const uint8_t*)sp.nul[c] : nullptr;
        }
        sg_push_view(h, bv, sb.n);
        k = h.out.n;
      }
      HIPCHK(hipEventRecord(nd.ev_used[s][ds], h.stream));
      r.publish([&] { r.used[s] = j + 1; });
      // the previous chunk's matches have landed: hand them to the merge before waiting for ring space
      if (j > 0) {
        HIPCHK(hipEventSynchronize(h.eg.done[es ^ 1]));
        r.publish([&] { r.delivered[s] = j; });
      }
      if (k > 0) {
        if (nd.G == 1) {
          if (pos + k > r.cap) throw SgError(SG_ECAPACITY, "node: more matches than the output capacity");
        } else {
          if (k > dst.M) throw SgError(SG_ECAPACITY, "node: one chunk's matches exceed the shard ring");
          if (!r.wait([&] { return pos + k - r.ring_tail[s] <= dst.M; })) return;
        }
        deliver(r, h, dst, pos, k, es);
        pos += k;
        es ^= 1;
      }
      r.publish([&] { r.dlv_end[s][j] = pos; });
      std::lock_guard<std::mutex> lk(r.mu);
      r.t_gpu[s] += now_ms() - t0;
    }
    if (h.eg.d2h) HIPCHK(hipStreamSynchronize(h.eg.d2h));
    r.publish([&] {
      r.delivered[s] = r.nch;
      if (nd.G == 1) r.out_rows = pos;
    });
  });
}

// ---- merge of chunk j (G > 1) ------------------------------------------------------------------------------------
void merge_chunk(Run& r, int64_t j) {
  sg_node& nd = r.nd;
  const int G = nd.G;
  const int slot = (int)(j % NODE_RING);
  const Want& w = r.w;
  int64_t a[MAX_GPUS], e[MAX_GPUS], total = 0;
  for (int s = 0; s < G; ++s) {
    a[s] = j ? r.dlv_end[s][j - 1] : 0;
    e[s] = r.dlv_end[s][j];
    total += e[s] - a[s];
  }
  if (r.out_rows + total > r.cap) throw SgError(SG_ECAPACITY, "node: more matches than the output capacity");
  if (total == 0) return;
  // global trigger of ring row p of shard s (its chunk-j local trigger mapped through the staged global indices)
  auto gtrig = [&](int s, int64_t p) -> uint64_t {
    const NodeRing& R = nd.ring[s];
    const uint64_t lt = R.trig.as<uint64_t>()[p % R.M];
    return nd.stage[slot][s].gidx.as<uint64_t>()[lt - (uint64_t)r.lbase_of[j * G + s]];
  };
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nd.threads, total / 131072 + 1));
  const int64_t lo = chunk_lo(r, j), hi = chunk_lo(r, j + 1);
  std::vector<std::vector<int64_t>> cut(T + 1, std::vector<int64_t>(G));
  for (int t = 0; t <= T; ++t)
    for (int s = 0; s < G; ++s) {
      if (t == 0) { cut[t][s] = a[s]; continue; }
      if (t == T) { cut[t][s] = e[s]; continue; }
      const uint64_t bound = r.b.base_index + (uint64_t)(lo + (hi - lo) * t / T);
      int64_t x = a[s], y = e[s];
      while (x < y) {
        const int64_t m = x + (y - x) / 2;
        if (gtrig(s, m) < bound) x = m + 1;
        else y = m;
      }
      cut[t][s] = x;
    }
  std::vector<int64_t> o0(T + 1, r.out_rows);
  for (int t = 0; t < T; ++t) {
    int64_t c = 0;
    for (int s = 0; s < G; ++s) c += cut[t + 1][s] - cut[t][s];
    o0[t + 1] = o0[t] + c;
  }
  const sg_router* rt = nd.router;
  nd.pool->parallel_for(T, [&](int t) {
    // per shard: rows left, ring slot of the head (wrapped by compare, not by division), the head's global trigger
    int64_t left[MAX_GPUS], q[MAX_GPUS];
    uint64_t head[MAX_GPUS];
    const uint64_t* trig[MAX_GPUS];
    const uint64_t* gidx[MAX_GPUS];
    uint64_t lbase[MAX_GPUS];
    for (int s = 0; s < G; ++s) {
      const NodeRing& R = nd.ring[s];
      left[s] = cut[t + 1][s] - cut[t][s];
      q[s] = cut[t][s] % R.M;
      trig[s] = R.trig.as<uint64_t>();
      gidx[s] = nd.stage[slot][s].gidx.as<uint64_t>();
      lbase[s] = (uint64_t)r.lbase_of[j * G + s];
      head[s] = left[s] > 0 ? gidx[s][trig[s][q[s]] - lbase[s]] : ~0ull;
    }
    const bool ties = w.grp;   // (a trigger on two shards: clock passes)
    auto gkey = [&](int s, int64_t p) -> int64_t {
      const int32_t lk = nd.ring[s].key.as<int32_t>()[p];
      if (lk < 0) return -1;
      return (int64_t)rt->l2d[s][lk];
    };
    for (int64_t o = o0[t]; o < o0[t + 1]; ++o) {
      int best = -1;
      for (int s = 0; s < G; ++s) {
        if (left[s] <= 0) continue;
        if (best < 0 || head[s] < head[best]) { best = s; continue; }
        if (ties && head[s] == head[best]) {   // same trigger on two shards: a clock pass -> (phase, key)
          const uint32_t pa = nd.ring[s].grp.as<uint32_t>()[q[s]] >> 24, pb = nd.ring[best].grp.as<uint32_t>()[q[best]] >> 24;
          if (pa < pb || (pa == pb && gkey(s, q[s]) < gkey(best, q[best]))) best = s;
        }
      }
      const int s = best;
      const NodeRing& R = nd.ring[s];
      const int64_t p = q[s];
      if (r.out->trigger) put<4>(&r.out->trigger[o], head[s]);
      if (w.ts) put<4>(&r.out->ts[o], R.ts.as<int64_t>()[p]);
      if (w.any_fill) fill_row(r.b, nd.desc, w, r.out, o, head[s]);
      if (r.out->key) put<4>(&r.out->key[o], (int32_t)gkey(s, p));
      if (r.out->group) put<4>(&r.out->group[o], R.grp.as<uint32_t>()[p]);
      for (int c = 0; c < w.ns; ++c) {
        if (w.col[c]) {
          if (w.width[c] == 8) put<4>(&((int64_t*)r.out->cols[c])[o], R.col[c].as<int64_t>()[p]);
          else put<4>(&((int32_t*)r.out->cols[c])[o], R.col[c].as<int32_t>()[p]);
        }
        if (w.nul[c]) r.out->nulls[c][o] = R.nul[c].as<uint8_t>()[p];
      }
      if (++q[s] == R.M) q[s] = 0;
      head[s] = --left[s] > 0 ? gidx[s][trig[s][q[s]] - lbase[s]] : ~0ull;
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);
  });
  r.out_rows += total;
}

// G = 1: the GPU delivers straight into the caller's columns; the trigger-row columns of chunk j are filled in once
// its triggers have landed (host thread pool, rows in parallel)
void fill_loop(Run& r) {
  sg_node& nd = r.nd;
  r.guarded([&] {
    for (int64_t j = 0; j < r.nch; ++j) {
      if (!r.wait([&] { return r.delivered[0] > j; })) return;
      const int64_t o0 = j ? r.dlv_end[0][j - 1] : 0, o1 = r.dlv_end[0][j];
      const double t0 = now_ms();
      const int64_t cnt = o1 - o0;
      if (cnt > 0) {
        const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nd.threads, cnt / 65536 + 1));
        nd.pool->parallel_for(T, [&](int t) {
          const int64_t a = o0 + cnt * t / T, e = o0 + cnt * (t + 1) / T;
          for (int64_t o = a; o < e; ++o) {
            fill_row(r.b, nd.desc, r.w, r.out, o, r.out->trigger[o]);
          }
          std::atomic_thread_fence(std::memory_order_seq_cst);
        });
      }
      r.publish([&] {
        r.merged = j + 1;
        r.t_merge += now_ms() - t0;
      });
    }
  });
}

void merge_loop(Run& r) {
  sg_node& nd = r.nd;
  r.guarded([&] {
    for (int64_t j = 0; j < r.nch; ++j) {
      if (!r.wait([&] {
            for (int s = 0; s < nd.G; ++s)
              if (r.delivered[s] <= j) return false;
            return true;
          }))
        return;
      const double t0 = now_ms();
      merge_chunk(r, j);
      r.publish([&] {
        for (int s = 0; s < nd.G; ++s) r.ring_tail[s] = r.dlv_end[s][j];
        r.merged = j + 1;
        r.t_merge += now_ms() - t0;
      });
    }
  });
}

// ---- GPU-side shard exchange: the per-push pipeline (G > 1, device dictionary) -----------------------------------
bool use_xchg(const sg_node& nd) { return nd.G > 1 && nd.ddict == 1; }

XSpec xspec_of(const sg_node& nd, const sg_node_batch& b) {
  const sg_nfa_desc& d = nd.desc;
  XSpec sp;
  memset(&sp, 0, sizeof(sp));
  sp.ncols = d.n_cols;
  sp.stream = b.stream ? 1 : 0;
  int need[SG_MAX_COLS] = {};
  for (int k = 0; k < d.n_ret; ++k) need[d.ret_col[k]] = 1;
  for (int c = 0; c < d.n_cols; ++c) {
    if (!need[c] || !b.cols || !b.cols[c]) continue;
    sp.width[c] = sg_col_width(d.col_type[c]);
    sp.nul[c] = (b.nulls && b.nulls[c]) ? 1 : 0;
  }
  return sp;
}

// one slice of chunk j: rows [a, e) of the caller's batch
void x_slice(const Run& r, int64_t j, int g, int64_t& a, int64_t& e) {
  const int64_t lo = chunk_lo(r, j), n = chunk_lo(r, j + 1) - lo;
  a = lo + n * g / r.nd.G;
  e = lo + n * (g + 1) / r.nd.G;
}

void xcopy(void* dst, int ddev, const void* src, int sdev, size_t bytes, hipStream_t st) {
  if (!bytes) return;
  if (ddev == sdev) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
  else HIPCHK(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, st));
}

// H2D of GPU g's slice of chunk j into its ingress slot j & 1 (copy stream)
void x_upload(Run& r, int g, int64_t j, const XSpec& sp) {
  sg_node& nd = r.nd;
  XGpu& X = nd.x[g];
  const int p = (int)(j & 1);
  int64_t a, e;
  x_slice(r, j, g, a, e);
  const int64_t n = e - a;
  if (j >= 2) HIPCHK(hipStreamWaitEvent(nd.cp[g], X.ev_scat[p], 0));   // the slot's last rows were scattered
  const XCols& c = X.in[p].c;
  int64_t bytes = 0;
  auto up = [&](void* dst, const void* src, size_t w) {
    if (!n) return;
    HIPCHK(hipMemcpyAsync(dst, (const char*)src + w * (size_t)a, w * (size_t)n, hipMemcpyHostToDevice, nd.cp[g]));
    bytes += (int64_t)(w * (size_t)n);
  };
  up(c.ts, r.b.ts, 8);
  up(c.raw, r.b.raw_key, 8);
  if (sp.stream) up(c.stream, r.b.stream, 4);
  for (int k = 0; k < sp.ncols; ++k) {
    if (sp.width[k]) up(c.col[k], r.b.cols[k], (size_t)sp.width[k]);
    if (sp.nul[k]) up(c.nul[k], r.b.nulls[k], 1);
  }
  HIPCHK(hipEventRecord(X.ev_in[p], nd.cp[g]));
  std::lock_guard<std::mutex> lk(r.mu);
  r.h2d_bytes += bytes;
}

XLay xlay(char* base, const ColLayout& L) {
  XLay x;
  x.base = base;
  x.off_trig = L.off_trig;
  x.off_ts = L.off_ts;
  x.off_key = L.off_key;
  x.off_grp = L.off_grp;
  for (int k = 0; k < SG_MAX_SELECT; ++k) {
    x.off_col[k] = k < L.ns ? L.off_col[k] : 0;
    x.off_nul[k] = k < L.ns ? L.off_nul[k] : 0;
  }
  return x;
}

XWant xwant(const Want& w, const ColLayout& L) {
  XWant x;
  memset(&x, 0, sizeof(x));
  x.ts = w.ts;
  x.key = w.key;
  x.grp = w.grp;
  x.ns = L.ns;
  for (int k = 0; k < L.ns; ++k) {
    x.width[k] = w.col[k] ? L.width[k] : 0;
    x.nul[k] = w.nul[k] ? 1 : 0;
  }
  return x;
}

// device buffers of every GPU for chunks of C rows (before the pipeline's threads start)
void x_reserve(Run& r, const XSpec& sp) {
  sg_node& nd = r.nd;
  const int G = nd.G;
  const int64_t C = r.C, S = C / G + 1;
  const int64_t nblk = (S + XB_ROWS - 1) / XB_ROWS;
  for (int g = 0; g < G; ++g) {
    XGpu& X = nd.x[g];
    SgHandle& h = nd.h[g]->h;
    HIPCHK(hipSetDevice(nd.dev[g]));
    if (!X.init) {
      HIPCHK(hipStreamCreateWithFlags(&X.xs, hipStreamNonBlocking));
      for (hipEvent_t* e : {X.ev_in, X.ev_scat, X.ev_sent, X.ev_rfree, X.ev_osent, X.ev_mfree, X.ev_d2h})
        for (int p = 0; p < 2; ++p) HIPCHK(hipEventCreateWithFlags(&e[p], hipEventDisableTiming));
      X.init = true;
    }
    for (int p = 0; p < 2; ++p) {
      xrows_layout(X.in[p], S, sp, false);
      xrows_layout(X.send[p], S, sp, true);
    }
    X.shard.ensure((size_t)S);
    X.bcnt.ensure(4 * (size_t)(G * nblk + 1));
    X.boff.ensure(4 * (size_t)(G * nblk + 1));
    X.starts.ensure(4 * (MAX_GPUS + 1));
    X.bounds.ensure(8 * (MAX_GPUS + 1));
    X.mcnt.ensure(4 * (size_t)(S + 1));
    X.mseg.ensure(4 * (size_t)(S + 1));
    X.moff.ensure(4 * (size_t)(S + 1));
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, X.bcnt.as<uint32_t>(), X.boff.as<uint32_t>(), (uint32_t)0,
                                   (size_t)(G * nblk + 1), rocprim::plus<uint32_t>(), h.stream));
    X.scan_tmp.ensure(tb);
    tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, X.mcnt.as<uint32_t>(), X.moff.as<uint32_t>(), (uint32_t)0, (size_t)(S + 1),
                                   rocprim::plus<uint32_t>(), h.stream));
    X.mscan_tmp.ensure(tb);
    for (int p = 0; p < 2; ++p) X.hstarts[p].ensure(8 * (MAX_GPUS + 1));
    X.hbounds.ensure(8 * (MAX_GPUS + 1));
    // receive slots: a shard may get every row of a chunk
    sg_batch sb;
    memset(&sb, 0, sizeof(sb));
    const void* cols[SG_MAX_COLS] = {};
    const uint8_t* nuls[SG_MAX_COLS] = {};
    static const char dummy[1] = {0};
    sb.ts = (const int64_t*)dummy;
    sb.key = (const int32_t*)dummy;
    sb.index = (const uint64_t*)dummy;
    sb.stream = sp.stream ? (const int32_t*)dummy : nullptr;
    bool nul = false;
    for (int c = 0; c < sp.ncols; ++c) {
      cols[c] = sp.width[c] ? dummy : nullptr;
      nuls[c] = sp.nul[c] ? (const uint8_t*)dummy : nullptr;
      nul |= nuls[c] != nullptr;
    }
    sb.cols = cols;
    sb.nulls = nul ? nuls : nullptr;
    for (int p = 0; p < 2; ++p) nd.dslot[g][p] = sg_reserve_slot(h, &sb, C, p);
    if (nd.draw_rows < C)
      for (int p = 0; p < 2; ++p) {
        if (nd.draw[g][p]) HIPCHK(hipFree(nd.draw[g][p]));
        nd.draw[g][p] = nullptr;
        HIPCHK(hipMalloc((void**)&nd.draw[g][p], (size_t)C * 8));
      }
    HIPCHK(hipStreamSynchronize(h.stream));
    sg_egress_init(h);
    const int64_t eb = (int64_t)sg_col_layout(h.desc, std::max<int64_t>(1, std::min<int64_t>(S, r.cap))).bytes;
    sg_stage_reserve(h, 0, eb);
    sg_stage_reserve(h, 1, eb);
  }
  nd.draw_rows = std::max(nd.draw_rows, C);
}

// merge input / output slot p of GPU g for m rows (waits for the slot's earlier users first)
void x_merge_room(sg_node& nd, int g, int p, int64_t m, bool out_slot) {
  XGpu& X = nd.x[g];
  int64_t& cap = out_slot ? X.mo_cap[p] : X.min_cap[p];
  if (m <= cap && cap > 0) return;
  const int64_t c = std::max<int64_t>({m + m / 4, 1024, cap});
  HIPCHK(hipEventSynchronize(out_slot ? X.ev_d2h[p] : X.ev_mfree[p]));
  (out_slot ? X.mo[p] : X.min[p]).ensure(sg_col_layout(nd.h[g]->h.desc, c).bytes);
  cap = c;
}

void x_loop(Run& r, int g, XSpec sp) {
  sg_node& nd = r.nd;
  XGpu& X = nd.x[g];
  SgHandle& h = nd.h[g]->h;
  const int G = nd.G;
  const sg_nfa_desc& d = nd.desc;
  const Want& w = r.w;
  auto all_gt = [&](const int64_t* v, int64_t j) {
    for (int q = 0; q < G; ++q)
      if (v[q] <= j) return false;
    return true;
  };
  r.guarded([&] {
    HIPCHK(hipSetDevice(nd.dev[g]));
    int64_t out_before = 0;   // matches of the chunks before this one, node-wide
    for (int64_t j = 0; j < r.nch; ++j) {
      const double t0 = now_ms();
      const int p = (int)(j & 1);
      if (j == 0) x_upload(r, g, 0, sp);
      if (j + 1 < r.nch) x_upload(r, g, j + 1, sp);   // (slot (j + 1) & 1 held chunk j - 1, scattered already)
      int64_t a, e;
      x_slice(r, j, g, a, e);
      const int64_t n = e - a;
      const int64_t nblk = (n + XB_ROWS - 1) / XB_ROWS;
      // ---- shard of every row, counts per (block, shard), send offsets
      HIPCHK(hipStreamWaitEvent(h.stream, X.ev_in[p], 0));
      uint32_t* hst = X.hstarts[p].as<uint32_t>();
      if (n > 0) {
        HIPCHK(hipMemsetAsync(X.bcnt.as<uint32_t>() + G * nblk, 0, 4, h.stream));
        hipLaunchKernelGGL(k_xcount, dim3((unsigned)nblk), dim3(256), 0, h.stream, X.in[p].c.raw, X.in[p].c.stream, n,
                           (uint32_t)G, X.shard.as<uint8_t>(), X.bcnt.as<uint32_t>(), (uint32_t)nblk);
        HIPCHK(hipGetLastError());
        size_t tb = X.scan_tmp.bytes;
        HIPCHK(rocprim::exclusive_scan(X.scan_tmp.p, tb, X.bcnt.as<uint32_t>(), X.boff.as<uint32_t>(), (uint32_t)0,
                                       (size_t)(G * nblk + 1), rocprim::plus<uint32_t>(), h.stream));
        hipLaunchKernelGGL(k_xstarts, dim3(1), dim3(64), 0, h.stream, X.boff.as<uint32_t>(), (uint32_t)nblk, (uint32_t)G,
                           X.starts.as<uint32_t>());
        HIPCHK(hipMemcpyAsync(hst, X.starts.p, 4 * (size_t)(G + 1), hipMemcpyDeviceToHost, h.stream));
        HIPCHK(hipStreamSynchronize(h.stream));
        hipLaunchKernelGGL(k_xscatter, dim3((unsigned)nblk), dim3(256), 0, h.stream, X.in[p].c, X.send[p].c, sp, n,
                           r.b.base_index + (uint64_t)a, X.shard.as<uint8_t>(), X.boff.as<uint32_t>(), (uint32_t)nblk,
                           (uint32_t)G);
        HIPCHK(hipGetLastError());
      } else {
        for (int s = 0; s <= G; ++s) hst[s] = 0;
      }
      HIPCHK(hipEventRecord(X.ev_scat[p], h.stream));
      r.publish([&] {
        for (int s = 0; s <= G; ++s) r.xst[(size_t)(j * G + g) * (G + 1) + s] = hst[s];
        r.xcounted[g] = j + 1;
      });
      // ---- rows to their shards: piece (g -> s) lands after the pieces of slices 0 .. g-1
      if (!r.wait([&] {
            if (!all_gt(r.xcounted, j)) return false;
            if (j < 2) return true;
            for (int s = 0; s < G; ++s)
              if (r.xused[s] < j - 1) return false;   // shard s consumed chunk j - 2 from its receive slot p
            return true;
          }))
        return;
      auto cnt_of = [&](int src, int s) {
        const int64_t* q = &r.xst[(size_t)(j * G + src) * (G + 1)];
        return q[s + 1] - q[s];
      };
      HIPCHK(hipStreamWaitEvent(X.xs, X.ev_scat[p], 0));
      for (int s = 0; s < G; ++s) {
        const int64_t c = cnt_of(g, s);
        if (!c) continue;
        int64_t ro = 0;
        for (int q = 0; q < g; ++q) ro += cnt_of(q, s);
        const int64_t so = r.xst[(size_t)(j * G + g) * (G + 1) + s];
        if (j >= 2) HIPCHK(hipStreamWaitEvent(X.xs, nd.x[s].ev_rfree[p], 0));
        const SlotPtrs& rs = nd.dslot[s][p];
        const XCols& sc = X.send[p].c;
        const int ds = nd.dev[s], dg = nd.dev[g];
        xcopy((int64_t*)rs.ts + ro, ds, sc.ts + so, dg, 8 * (size_t)c, X.xs);
        xcopy(nd.draw[s][p] + ro, ds, sc.raw + so, dg, 8 * (size_t)c, X.xs);
        xcopy((uint64_t*)rs.index + ro, ds, sc.gidx + so, dg, 8 * (size_t)c, X.xs);
        if (sp.stream) xcopy((int32_t*)rs.stream + ro, ds, sc.stream + so, dg, 4 * (size_t)c, X.xs);
        for (int k = 0; k < sp.ncols; ++k) {
          if (sp.width[k])
            xcopy((char*)rs.col[k] + (size_t)sp.width[k] * ro, ds, (const char*)sc.col[k] + (size_t)sp.width[k] * so, dg,
                  (size_t)sp.width[k] * c, X.xs);
          if (sp.nul[k]) xcopy((uint8_t*)rs.nul[k] + ro, ds, sc.nul[k] + so, dg, (size_t)c, X.xs);
        }
      }
      HIPCHK(hipEventRecord(X.ev_sent[p], X.xs));
      r.publish([&] { r.xsent[g] = j + 1; });
      // ---- shard g: its rows of chunk j, arrival order, global indices as triggers
      if (!r.wait([&] { return all_gt(r.xsent, j); })) return;
      int64_t ns = 0;
      for (int q = 0; q < G; ++q) {
        ns += cnt_of(q, g);
        HIPCHK(hipStreamWaitEvent(h.stream, nd.x[q].ev_sent[p], 0));
      }
      const SlotPtrs& sl = nd.dslot[g][p];
      int64_t kbefore = nd.kd[g].n_keys, mnew = 0;
      if (ns > 0) {
        mnew = kd_resolve(nd.kd[g], nd.draw[g][p], sp.stream ? (const int32_t*)sl.stream : nullptr, ns,
                          (int32_t*)sl.key, h.stream, nullptr);
        if (w.key && mnew > 0) {   // global first rows of the new keys (node-wide first-seen ids)
          X.nfg.ensure(8 * (size_t)mnew);
          X.hnf.ensure(8 * (size_t)mnew);
          hipLaunchKernelGGL(k_xgather_u64, dim3((unsigned)((mnew + 255) / 256)), dim3(256), 0, h.stream,
                             (const uint64_t*)sl.index, nd.kd[g].sfirst, mnew, X.nfg.as<uint64_t>());
          HIPCHK(hipGetLastError());
          HIPCHK(hipMemcpyAsync(X.hnf.p, X.nfg.p, 8 * (size_t)mnew, hipMemcpyDeviceToHost, h.stream));
          HIPCHK(hipStreamSynchronize(h.stream));
        }
        BatchView bv;
        memset(&bv, 0, sizeof(bv));
        bv.n = ns;
        bv.base_index = 0;
        bv.key_bound = (int32_t)std::max<int64_t>(1, nd.kd[g].n_keys);
        bv.ts = (const int64_t*)sl.ts;
        bv.stream = sp.stream ? (const int32_t*)sl.stream : nullptr;
        bv.key = (const int32_t*)sl.key;
        bv.index = (const uint64_t*)sl.index;
        for (int k = 0; k < sp.ncols; ++k) {
          bv.cols.col[k] = sp.width[k] ? sl.col[k] : nullptr;
          bv.cols.nul[k] = sp.nul[k] ? (const uint8_t*)sl.nul[k] : nullptr;
        }
        sg_push_view(h, bv, ns);
      }
      HIPCHK(hipEventRecord(X.ev_rfree[p], h.stream));
      r.publish([&] {
        r.xused[g] = j + 1;
        nd.local_rows[g] += ns;
        if (w.key) {
          r.xnf[(size_t)(j * G + g)].assign(X.hnf.as<uint64_t>(), X.hnf.as<uint64_t>() + (mnew > 0 ? mnew : 0));
          r.xkbase[(size_t)(j * G + g)] = kbefore;
          r.xnfp[g] = j + 1;
        }
      });
      // ---- node-wide first-seen key ids (only when the caller wants keys): the shards' new keys interleaved by
      // their first global row; GPU 0's thread assigns them for everyone
      if (w.key) {
        if (g == 0) {
          if (!r.wait([&] { return all_gt(r.xnfp, j); })) return;
          int64_t cur[MAX_GPUS] = {}, m[MAX_GPUS];
          for (int s = 0; s < G; ++s) {
            m[s] = (int64_t)r.xnf[(size_t)(j * G + s)].size();
            if (m[s] > 0) nd.l2g[s].resize((size_t)(r.xkbase[(size_t)(j * G + s)] + m[s]));
          }
          while (true) {
            int best = -1;
            for (int s = 0; s < G; ++s)
              if (cur[s] < m[s] && (best < 0 || r.xnf[(size_t)(j * G + s)][cur[s]] < r.xnf[(size_t)(j * G + best)][cur[best]]))
                best = s;
            if (best < 0) break;
            nd.l2g[best][(size_t)(r.xkbase[(size_t)(j * G + best)] + cur[best])] = (int32_t)nd.g_keys++;
            ++cur[best];
          }
          r.publish([&] { r.xids = j + 1; });
        }
        if (!r.wait([&] { return r.xids > j; })) return;
        const int64_t nk = (int64_t)nd.l2g[g].size();
        if (nk > X.l2g_n) {
          if ((size_t)nk * 4 > X.l2g.bytes) {
            HIPCHK(hipStreamSynchronize(h.stream));
            XBuf nb;
            nb.ensure((size_t)(nk + nk / 2 + 1024) * 4);
            if (X.l2g_n) HIPCHK(hipMemcpy(nb.p, X.l2g.p, 4 * (size_t)X.l2g_n, hipMemcpyDeviceToDevice));
            X.l2g.release();
            X.l2g = nb;
            nb.p = nullptr;
          }
          HIPCHK(hipMemcpyAsync(X.l2g.as<int32_t>() + X.l2g_n, nd.l2g[g].data() + X.l2g_n, 4 * (size_t)(nk - X.l2g_n),
                                hipMemcpyHostToDevice, h.stream));
          HIPCHK(hipStreamSynchronize(h.stream));
          X.l2g_n = nk;
        }
      }
      // ---- its matches -> SoA columns in egress slot p, cut by trigger slice
      const int64_t k = h.out.n;
      ColLayout L = sg_col_layout(d, std::max<int64_t>(k, 1));
      int64_t* hb = X.hbounds.as<int64_t>();
      if (k > 0) {
        sg_stage_reserve(h, p, (int64_t)L.bytes);
        HIPCHK(hipStreamWaitEvent(h.stream, h.eg.done[p], 0));
        sg_launch_to_columns(k, h.out.rec, h.out.stride, L, h.eg.stage[p], h.stream);
        h.out.n = 0;
        if (w.key)
          hipLaunchKernelGGL(k_xmapkeys, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, h.stream,
                             (int32_t*)(h.eg.stage[p] + L.off_key), k, X.l2g.as<int32_t>());
        XSlices xs;
        for (int q = 0; q <= G; ++q) {
          int64_t qa, qe;
          x_slice(r, j, q < G ? q : G - 1, qa, qe);
          xs.lo[q] = r.b.base_index + (uint64_t)(q < G ? qa : qe);
        }
        hipLaunchKernelGGL(k_xbounds, dim3(1), dim3(64), 0, h.stream, (const uint64_t*)(h.eg.stage[p] + L.off_trig), k, xs,
                           (uint32_t)G, X.bounds.as<int64_t>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(hb, X.bounds.p, 8 * (size_t)(G + 1), hipMemcpyDeviceToHost, h.stream));
        HIPCHK(hipEventRecord(h.eg.ready[p], h.stream));
        HIPCHK(hipStreamSynchronize(h.stream));
      } else {
        for (int q = 0; q <= G; ++q) hb[q] = 0;
      }
      r.publish([&] {
        for (int q = 0; q <= G; ++q) r.xpc[(size_t)(j * G + g) * (G + 1) + q] = hb[q];
        r.xpieced[g] = j + 1;
      });
      auto piece = [&](int s, int q) {
        const int64_t* b2 = &r.xpc[(size_t)(j * G + s) * (G + 1)];
        return b2[q + 1] - b2[q];
      };
      // ---- slice owner g: room for the matches of its triggers
      if (!r.wait([&] { return all_gt(r.xpieced, j); })) return;
      int64_t mg = 0, chunk_total = 0, before_g = 0;
      for (int s = 0; s < G; ++s) mg += piece(s, g);
      for (int q = 0; q < G; ++q)
        for (int s = 0; s < G; ++s) {
          chunk_total += piece(s, q);
          if (q < g) before_g += piece(s, q);
        }
      if (out_before + chunk_total > r.cap) throw SgError(SG_ECAPACITY, "node: more matches than the output capacity");
      if (mg > 0) x_merge_room(nd, g, p, mg, false);
      r.publish([&] { r.xmready[g] = j + 1; });
      // ---- shard g: piece (g -> q) into owner q's merge input after the pieces of shards 0 .. g-1
      if (!r.wait([&] { return all_gt(r.xmready, j); })) return;
      if (k > 0) {
        HIPCHK(hipStreamWaitEvent(X.xs, h.eg.ready[p], 0));
        for (int q = 0; q < G; ++q) {
          const int64_t c = piece(g, q);
          if (!c) continue;
          int64_t ro = 0;
          for (int s = 0; s < g; ++s) ro += piece(s, q);
          XGpu& Q = nd.x[q];
          if (j >= 2) HIPCHK(hipStreamWaitEvent(X.xs, Q.ev_mfree[p], 0));   // owner q merged chunk j - 2
          const ColLayout Lq = sg_col_layout(d, Q.min_cap[p]);
          char* dst = Q.min[p].as<char>();
          const char* src = h.eg.stage[p];
          const int64_t sr = r.xpc[(size_t)(j * G + g) * (G + 1) + q];
          const int dq = nd.dev[q], dg = nd.dev[g];
          auto col = [&](size_t doff, size_t soff, size_t wd) {
            xcopy(dst + doff + wd * (size_t)ro, dq, src + soff + wd * (size_t)sr, dg, wd * (size_t)c, X.xs);
          };
          col(Lq.off_trig, L.off_trig, 8);
          if (w.ts) col(Lq.off_ts, L.off_ts, 8);
          if (w.key) col(Lq.off_key, L.off_key, 4);
          if (w.grp) col(Lq.off_grp, L.off_grp, 4);
          for (int c2 = 0; c2 < L.ns; ++c2) {
            if (w.col[c2]) col(Lq.off_col[c2], L.off_col[c2], (size_t)L.width[c2]);
            if (w.nul[c2]) col(Lq.off_nul[c2], L.off_nul[c2], 1);
          }
        }
        HIPCHK(hipEventRecord(h.eg.done[p], X.xs));
      }
      HIPCHK(hipEventRecord(X.ev_osent[p], X.xs));
      r.publish([&] { r.xosent[g] = j + 1; });
      // ---- owner g: merge the G runs by trigger, then straight into the caller's columns
      if (!r.wait([&] { return all_gt(r.xosent, j); })) return;
      for (int q = 0; q < G; ++q) HIPCHK(hipStreamWaitEvent(h.stream, nd.x[q].ev_osent[p], 0));
      const int64_t o0 = out_before + before_g;
      if (mg > 0) {
        x_merge_room(nd, g, p, mg, true);
        int64_t sa, se;
        x_slice(r, j, g, sa, se);
        const int64_t nsl = se - sa;
        const uint64_t slo = r.b.base_index + (uint64_t)sa;
        XRuns runs;
        runs.off[0] = 0;
        for (int s = 0; s < G; ++s) runs.off[s + 1] = runs.off[s] + piece(s, g);
        HIPCHK(hipMemsetAsync(X.mcnt.p, 0, 4 * (size_t)(nsl + 1), h.stream));
        const ColLayout Li = sg_col_layout(d, X.min_cap[p]), Lo = sg_col_layout(d, X.mo_cap[p]);
        const XLay li = xlay(X.min[p].as<char>(), Li), lo = xlay(X.mo[p].as<char>(), Lo);
        hipLaunchKernelGGL(k_xmark, dim3((unsigned)((mg + 255) / 256)), dim3(256), 0, h.stream,
                           (const uint64_t*)(li.base + li.off_trig), mg, runs, (uint32_t)G, slo, X.mcnt.as<uint32_t>(),
                           X.mseg.as<uint32_t>());
        HIPCHK(hipGetLastError());
        size_t tb = X.mscan_tmp.bytes;
        HIPCHK(rocprim::exclusive_scan(X.mscan_tmp.p, tb, X.mcnt.as<uint32_t>(), X.moff.as<uint32_t>(), (uint32_t)0,
                                       (size_t)(nsl + 1), rocprim::plus<uint32_t>(), h.stream));
        HIPCHK(hipStreamWaitEvent(h.stream, X.ev_d2h[p], 0));   // the output slot's last copies are done
        hipLaunchKernelGGL(k_xplace, dim3((unsigned)((mg + 255) / 256)), dim3(256), 0, h.stream, li, mg, slo,
                           X.moff.as<uint32_t>(), X.mseg.as<uint32_t>(), lo, xwant(w, Lo));
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(X.ev_mfree[p], h.stream));
        HIPCHK(hipStreamWaitEvent(h.eg.d2h, X.ev_mfree[p], 0));
        int64_t bytes = 0;
        if (o0 < 0 || o0 + mg > r.cap)
          throw SgError(SG_EINVAL, "internal: exchange delivery rows [" + std::to_string(o0) + ", " +
                                       std::to_string(o0 + mg) + ") beyond the output capacity");
        auto down = [&](void* dst, size_t off, size_t wd) {
          if (!dst) return;
          HIPCHK(hipMemcpyAsync((char*)dst + wd * (size_t)o0, lo.base + off, wd * (size_t)mg, hipMemcpyDeviceToHost,
                                h.eg.d2h));
          bytes += (int64_t)(wd * (size_t)mg);
        };
        down(r.out->trigger, Lo.off_trig, 8);
        if (w.ts) down(r.out->ts, Lo.off_ts, 8);
        if (w.key) down(r.out->key, Lo.off_key, 4);
        if (w.grp) down(r.out->group, Lo.off_grp, 4);
        for (int c2 = 0; c2 < Lo.ns; ++c2) {
          if (w.col[c2]) down(r.out->cols[c2], Lo.off_col[c2], (size_t)Lo.width[c2]);
          if (w.nul[c2]) down(r.out->nulls[c2], Lo.off_nul[c2], 1);
        }
        HIPCHK(hipEventRecord(X.ev_d2h[p], h.eg.d2h));
        std::lock_guard<std::mutex> lk(r.mu);
        r.d2h_bytes += bytes;
      } else {
        HIPCHK(hipEventRecord(X.ev_mfree[p], h.stream));
      }
      out_before += chunk_total;
      r.publish([&] {
        r.t_gpu[g] += now_ms() - t0;
        if (g == 0) r.out_rows = out_before;
      });
    }
    HIPCHK(hipStreamSynchronize(h.stream));
    HIPCHK(hipStreamSynchronize(X.xs));
    HIPCHK(hipStreamSynchronize(h.eg.d2h));
  });
}

void reserve_all(Run& r) {
  sg_node& nd = r.nd;
  const sg_nfa_desc& d = nd.desc;
  const int64_t C = r.C;
  int need[SG_MAX_COLS] = {};
  for (int k = 0; k < d.n_ret; ++k) need[d.ret_col[k]] = 1;
  for (int q = 0; q < NODE_RING; ++q) {
    if (nd.G == 1) {
      nd.keyslot[q].ensure((size_t)C * 4);
      nd.tsslot[q].ensure((size_t)C * 4);
    }
    else {
      if ((int64_t)nd.dense_tmp[q].size() < C) nd.dense_tmp[q].resize((size_t)C);
      for (int s = 0; s < nd.G; ++s) {
        NodeStage& S = nd.stage[q][s];
        S.ts.ensure((size_t)C * 8);
        S.key.ensure((size_t)C * 4);
        S.gidx.ensure((size_t)C * 8);
        S.ts32.ensure((size_t)C * 4);
        if (r.b.stream || need_clocks(d)) S.stream.ensure((size_t)C * 4);
        for (int c = 0; c < d.n_cols; ++c) {
          if (!need[c] || !r.b.cols[c]) continue;
          S.col[c].ensure((size_t)C * sg_col_width(d.col_type[c]));
          if (r.b.nulls && r.b.nulls[c]) S.nul[c].ensure((size_t)C);
        }
      }
    }
  }
  // device slots of every GPU, sized for a whole chunk (no workspace growth inside the pipeline)
  for (int s = 0; s < nd.G; ++s) {
    SgHandle& h = nd.h[s]->h;
    HIPCHK(hipSetDevice(nd.dev[s]));
    sg_batch sb;
    memset(&sb, 0, sizeof(sb));
    const void* cols[SG_MAX_COLS] = {};
    const uint8_t* nuls[SG_MAX_COLS] = {};
    static const char dummy[1] = {0};
    sb.ts = (const int64_t*)dummy;
    sb.key = (const int32_t*)dummy;
    sb.stream = (r.b.stream || (nd.G > 1 && need_clocks(d))) ? (const int32_t*)dummy : nullptr;
    bool nul = false;
    for (int c = 0; c < d.n_cols; ++c) {
      cols[c] = (need[c] && r.b.cols[c]) ? dummy : nullptr;
      nuls[c] = (need[c] && r.b.nulls && r.b.nulls[c]) ? (const uint8_t*)dummy : nullptr;
      nul |= nuls[c] != nullptr;
    }
    sb.cols = cols;
    sb.nulls = nul ? nuls : nullptr;
    for (int ds = 0; ds < 2; ++ds) nd.dslot[s][ds] = sg_reserve_slot(h, &sb, C, ds);
    if (nd.dts32_rows < C)
      for (int ds = 0; ds < 2; ++ds) {
        if (nd.dts32[s][ds]) HIPCHK(hipFree(nd.dts32[s][ds]));
        nd.dts32[s][ds] = nullptr;
        HIPCHK(hipMalloc((void**)&nd.dts32[s][ds], (size_t)C * 4));
      }
    if (nd.ddict == 1 && nd.draw_rows < C)
      for (int ds = 0; ds < 2; ++ds) {
        if (nd.draw[s][ds]) HIPCHK(hipFree(nd.draw[s][ds]));
        nd.draw[s][ds] = nullptr;
        HIPCHK(hipMalloc((void**)&nd.draw[s][ds], (size_t)C * 8));
      }
    HIPCHK(hipStreamSynchronize(h.stream));
    sg_egress_init(h);
    // egress slots for one chunk's matches (the closed forms emit at most one match per e1 row, the lane routes rarely
    // more): no hipFree / hipMalloc -- a device-wide synchronisation -- inside the pipeline for such chunks
    const int64_t eb = (int64_t)sg_col_layout(h.desc, std::max<int64_t>(1, std::min<int64_t>(C, r.cap))).bytes;
    sg_stage_reserve(h, 0, eb);
    sg_stage_reserve(h, 1, eb);
  }
  if (nd.ddict == 1) nd.draw_rows = std::max(nd.draw_rows, C);
  nd.dts32_rows = std::max(nd.dts32_rows, C);
  // shard rings: room for two chunks' worth of matches per shard beyond the share of the output capacity
  if (nd.G > 1) {
    const int64_t M = std::max<int64_t>(1024, std::min<int64_t>(r.cap, r.cap / nd.G * 2 + 2 * C));
    for (int s = 0; s < nd.G; ++s) {
      NodeRing& R = nd.ring[s];
      R.M = M;
      R.trig.ensure((size_t)M * 8);
      if (r.w.ts) R.ts.ensure((size_t)M * 8);
      if (r.w.key) R.key.ensure((size_t)M * 4);
      if (r.w.grp) R.grp.ensure((size_t)M * 4);
      for (int c = 0; c < r.w.ns; ++c) {
        if (r.w.col[c]) R.col[c].ensure((size_t)M * r.w.width[c]);
        if (r.w.nul[c]) R.nul[c].ensure((size_t)M);
      }
    }
  }
}

// Auto key dictionary: keys are encoded on the GPUs whenever the query allows it (partitioned, no playback clocks).
// Measured on C2 (100M events, 10k keys, one GPU, profiles/r03/whole_node_*_dict.log): the host router's lookups were
// the pipeline's bound (route 50 ms of 58.7 ms per push) even with a cache-resident table, while raw 8-byte keys cost
// only 0.4 GB more H2D (route 13 ms, 48.8 ms per push); with 1M keys (C5) the host table is DRAM-bound as well.
void run_push(sg_node& nd, const sg_node_batch& b, const sg_match_columns* out, int64_t cap, int64_t* n_out) {
  if (nd.ddict < 0) {   // the first push of a stream fixes where keys are encoded
    const bool dev_ok = nd.desc.partitioned && !need_clocks(nd.desc);
    nd.ddict = (dev_ok && nd.key_dict_mode != 1) ? 1 : 0;
  }
  Run r(nd, b, out, cap);
  const bool xchg = use_xchg(nd);
  r.w = want_of(nd, b, out, !xchg);
  // default chunks: ~16 per push (short pipeline fill and drain), 4M..25M rows each
  r.C = nd.chunk_rows > 0 ? nd.chunk_rows
                          : std::max<int64_t>(1, std::min<int64_t>(b.n, std::max<int64_t>((int64_t)4 << 20,
                                                                   std::min<int64_t>((int64_t)25 << 20, (b.n + 15) / 16))));
  if (r.C >= (1ll << 30) - 1) throw SgError(SG_EINVAL, "node chunk too large (max 2^30-2 rows)");
  r.nch = (b.n + r.C - 1) / r.C;
  for (int s = 0; s < nd.G; ++s) r.dlv_end[s].assign((size_t)r.nch, 0);
  r.rows_of.assign((size_t)(r.nch * nd.G), 0);
  r.lbase_of.assign((size_t)(r.nch * nd.G), 0);
  r.kb_of.assign((size_t)(r.nch * nd.G), 1);
  r.ts_base_of.assign((size_t)r.nch, 0);
  r.ts32_of.assign((size_t)r.nch, 0);
  const double t0 = now_ms();
  std::vector<std::shared_ptr<Task>> th;
  ThreadCache& tc = pipeline_threads();
  double t1 = 0;
  if (xchg) {   // GPU-side shard exchange: one loop per GPU, no host route or merge
    const int G = nd.G;
    const XSpec sp = xspec_of(nd, b);
    r.xst.assign((size_t)(r.nch * G * (G + 1)), 0);
    r.xpc.assign((size_t)(r.nch * G * (G + 1)), 0);
    r.xkbase.assign((size_t)(r.nch * G), 0);
    r.xnf.assign((size_t)(r.nch * G), std::vector<uint64_t>());
    x_reserve(r, sp);
    t1 = now_ms();
    for (int s = 0; s < G; ++s) th.push_back(tc.run([&r, s, sp] { x_loop(r, s, sp); }));
  } else {
  reserve_all(r);
  t1 = now_ms();
  for (int s = 0; s < nd.G; ++s) {
    th.push_back(tc.run([&r, s] { copy_loop(r, s); }));
    th.push_back(tc.run([&r, s] { gpu_loop(r, s); }));
  }
  if (nd.G > 1) th.push_back(tc.run([&r] { merge_loop(r); }));
  else if (r.w.any_fill) th.push_back(tc.run([&r] { fill_loop(r); }));
  r.guarded([&] {
    for (int64_t j = 0; j < r.nch; ++j) {
      // slot j % NODE_RING is free once chunk j - NODE_RING is uploaded everywhere (and merged: its gidx)
      if (!r.wait([&] {
            if (j < NODE_RING) return true;
            for (int s = 0; s < nd.G; ++s)
              if (r.uploaded[s] <= j - NODE_RING) return false;
            return nd.G == 1 || r.merged > j - NODE_RING;
          }))
        return;
      const double ta = now_ms();
      route_chunk(r, j);
      for (int s = 0; s < nd.G; ++s) {
        r.lbase_of[j * nd.G + s] = nd.local_rows[s];
        nd.local_rows[s] += r.rows_of[j * nd.G + s];
      }
      r.publish([&] {
        r.routed = j + 1;
        r.t_route += now_ms() - ta;
      });
    }
  });
  }
  const double t_res = t1 - t0;
  for (auto& t : th) t->join();
  for (int s = 0; s < nd.G; ++s) {
    hipSetDevice(nd.dev[s]);
    hipStreamSynchronize(nd.h[s]->h.stream);
    hipStreamSynchronize(nd.cp[s]);
    if (nd.h[s]->h.eg.d2h) hipStreamSynchronize(nd.h[s]->h.eg.d2h);
    if (xchg && nd.x[s].xs) hipStreamSynchronize(nd.x[s].xs);   // (a failed exchange loop skips its own syncs)
  }
  if (r.failed) {
    nd.broken = true;
    throw SgError(r.fail_code, r.fail_msg);
  }
  const double t2 = now_ms();
  sg_node_stats& st = nd.st;
  st.total_ms = t2 - t1;
  st.reserve_ms = t_res;
  st.route_ms = r.t_route;
  st.merge_ms = r.t_merge;
  for (int s = 0; s < nd.G; ++s) st.gpu_ms[s] = r.t_gpu[s];
  st.rows = b.n;
  st.matches = r.out_rows;
  st.chunks = r.nch;
  st.chunk_rows = r.C;
  st.h2d_bytes = r.h2d_bytes;
  st.d2h_bytes = r.d2h_bytes;
  for (int s = 0; s < nd.G; ++s) st.shard_rows[s] = nd.local_rows[s];
  *n_out = r.out_rows;
}

void close_node(sg_node* nd) {
  for (int s = 0; s < nd->G; ++s) {
    hipSetDevice(nd->dev[s]);
    nd->x[s].release();
    kd_free(nd->kd[s]);
    for (int k = 0; k < 2; ++k) {
      if (nd->draw[s][k]) hipFree(nd->draw[s][k]);
      if (nd->dts32[s][k]) hipFree(nd->dts32[s][k]);
    }
    if (nd->h[s]) sg_close(nd->h[s]);
    if (nd->cp[s]) hipStreamDestroy(nd->cp[s]);
    for (int k = 0; k < 2; ++k) {
      if (nd->ev_copied[s][k]) hipEventDestroy(nd->ev_copied[s][k]);
      if (nd->ev_used[s][k]) hipEventDestroy(nd->ev_used[s][k]);
    }
  }
  if (nd->router) sg_router_close(nd->router);
  delete nd;
}

}  // namespace

extern "C" {

int sg_node_open(int n_gpus, const int* devices, const sg_nfa_desc* nfa, const sg_options* opt, int host_threads,
                 int64_t chunk_rows, sg_node** out) {
  if (!out || !nfa || n_gpus < 1 || n_gpus > MAX_GPUS || host_threads < 0 || chunk_rows < 0) return SG_EINVAL;
  *out = nullptr;
  if (!nfa->partitioned && n_gpus != 1) return SG_EUNSUPPORTED;   // one runtime: replicas only
  sg_node* nd = new sg_node();
  nd->G = n_gpus;
  nd->desc = *nfa;
  if (opt) nd->opt = *opt;
  else memset(&nd->opt, 0, sizeof(nd->opt));
  nd->opt.no_carry = 0;       // chunks are consecutive pushes of one stream
  nd->opt.ingress_rows = -1;  // (the node does its own chunking)
  nd->threads = host_threads ? host_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nd->chunk_rows = chunk_rows;
  nd->no_fill = getenv("SG_DEBUG_NODE_NO_FILL") != nullptr;   // (test hooks)
  nd->no_ts32 = getenv("SG_DEBUG_NODE_NO_TS32") != nullptr;
  memset(&nd->st, 0, sizeof(nd->st));
  int rc = SG_OK;
  for (int s = 0; s < n_gpus && rc == SG_OK; ++s) {
    nd->dev[s] = devices ? devices[s] : 0;
    rc = sg_open(nd->dev[s], &nd->desc, &nd->opt, &nd->h[s]);
    if (rc != SG_OK) {
      nd->err = nd->h[s] ? sg_last_error(nd->h[s]) : "sg_open failed";
      break;
    }
    if (hipSetDevice(nd->dev[s]) != hipSuccess || hipStreamCreateWithFlags(&nd->cp[s], hipStreamNonBlocking) != hipSuccess) {
      rc = SG_EHIP;
      nd->err = "node: stream creation failed";
      break;
    }
    for (int k = 0; k < 2 && rc == SG_OK; ++k)
      if (hipEventCreateWithFlags(&nd->ev_copied[s][k], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&nd->ev_used[s][k], hipEventDisableTiming) != hipSuccess) {
        rc = SG_EHIP;
        nd->err = "node: event creation failed";
      }
  }
  if (rc == SG_OK) rc = sg_router_open(n_gpus, nd->threads, &nd->router);
  for (int a = 0; a < n_gpus && rc == SG_OK; ++a)   // peer copies of the shard exchange (xGMI) where devices differ
    for (int b = 0; b < n_gpus; ++b) {
      if (nd->dev[a] == nd->dev[b]) continue;
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, nd->dev[a], nd->dev[b]) == hipSuccess && ok && hipSetDevice(nd->dev[a]) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(nd->dev[b], 0);   // (already enabled is fine; hipMemcpyPeerAsync works either way)
      (void)hipGetLastError();
    }
  if (rc == SG_OK) {
    nd->pool = &host_pool();
    nd->pool->grow(std::max(0, nd->threads - 1));
  }
  if (rc != SG_OK) {
    std::string e = nd->err;
    close_node(nd);
    (void)e;
    return rc;
  }
  *out = nd;
  return SG_OK;
}

int sg_node_push(sg_node* nd, const sg_node_batch* b, const sg_match_columns* out, int64_t cap, int64_t* n) {
  if (!nd || !b || !out || cap < 0) return SG_EINVAL;
  int64_t got = 0;
  try {
    if (nd->broken) throw SgError(SG_EINVAL, "node: a failed push left it inconsistent; call sg_node_reset");
    if (b->n < 0 || (b->n && !b->ts)) throw SgError(SG_EINVAL, "node batch without timestamps");
    if (nd->desc.partitioned && b->n && !b->raw_key) throw SgError(SG_EINVAL, "partitioned query without raw keys");
    if (!out->trigger) throw SgError(SG_EINVAL, "node delivery needs the trigger column");
    if (b->n == 0) {
      if (n) *n = 0;
      return SG_OK;
    }
    if (b->base_index != (uint64_t)nd->next_index && nd->next_index != 0)
      throw SgError(SG_EINVAL, "node batches must continue the stream's event index");
    run_push(*nd, *b, out, cap, &got);
    nd->next_index = (int64_t)(b->base_index + (uint64_t)b->n);
  } catch (SgError& e) {
    nd->err = e.msg;
    if (n) *n = got;
    return e.code;
  } catch (std::exception& e) {
    nd->err = e.what();
    nd->broken = true;
    return SG_EINVAL;
  }
  if (n) *n = got;
  return SG_OK;
}

int sg_node_reset(sg_node* nd) {
  if (!nd) return SG_EINVAL;
  int rc = SG_OK;
  for (int s = 0; s < nd->G; ++s) {
    const int x = sg_reset(nd->h[s]);
    if (x != SG_OK) rc = x;
    nd->local_rows[s] = 0;
    kd_reset(nd->kd[s]);
    nd->l2g[s].clear();
  }
  nd->g_keys = 0;
  nd->ddict = -1;
  if (nd->router) sg_router_close(nd->router);
  nd->router = nullptr;
  const int x = sg_router_open(nd->G, nd->threads, &nd->router);
  if (x != SG_OK) rc = x;
  nd->next_index = 0;
  nd->broken = rc != SG_OK;
  return rc;
}

int sg_node_stats_get(const sg_node* nd, sg_node_stats* st) {
  if (!nd || !st) return SG_EINVAL;
  *st = nd->st;
  return SG_OK;
}

int sg_node_keys(const sg_node* nd, int64_t* n_keys) {
  if (!nd || !n_keys) return SG_EINVAL;
  if (nd->ddict == 1) {
    *n_keys = 0;
    for (int s = 0; s < nd->G; ++s) *n_keys += nd->kd[s].n_keys;
    return SG_OK;
  }
  return sg_router_keys(nd->router, n_keys, -1, nullptr);
}

int sg_node_set_key_dict(sg_node* nd, int mode) {
  if (!nd || mode < 0 || mode > 2) return SG_EINVAL;
  if (nd->ddict >= 0) {
    nd->err = "node: the key dictionary is chosen at the first push of a stream (call before it or after sg_node_reset)";
    return SG_EINVAL;
  }
  if (mode == 2 && (!nd->desc.partitioned || need_clocks(nd->desc))) {
    nd->err = "node: the device dictionary needs a partitioned query without playback timers";
    return SG_EUNSUPPORTED;
  }
  nd->key_dict_mode = mode;
  return SG_OK;
}

int sg_node_close(sg_node* nd) {
  if (!nd) return SG_EINVAL;
  close_node(nd);
  return SG_OK;
}

const char* sg_node_last_error(const sg_node* nd) { return nd ? nd->err.c_str() : "null node"; }

}  // extern "C"
