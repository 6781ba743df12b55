// Node pipeline (sg_node_*): one host process drives every GPU of the node for one partitioned query.
//
// The reference runs a partitioned query in one JVM: PartitionStreamReceiver.receive looks each event's key up and
// hands it to that key's cloned runtime (C/partition/PartitionStreamReceiver.java:80-281, PartitionRuntime.java:
// 255-308); the matches reach QueryCallback.receive in one ordered stream (C/query/output/callback/
// QueryCallback.java:52-85).  Here the same contract is met by a pipeline over chunks of the host batch:
//
//   route    host thread pool: raw partition-key values -> first-seen dense ids -> shard (GPU) + per-shard id
//            (router.h); with G > 1 every chunk's rows are scattered, in arrival order, into per-shard pinned
//            staging (two passes: count per shard, then place), keeping each row's global event index on the host
//   upload   one copy thread per GPU: the shard's rows of chunk j go to HBM while chunk j-1 computes
//   compute  one thread per GPU: sg_push_view over the chunk (state carried between chunks = one stream)
//   deliver  the same thread: the chunk's matches are transposed on the GPU into SoA columns and copied back into
//            the shard's pinned ring while the next chunk computes
//   merge    (G > 1) host thread pool: chunk j's shard streams merged into the node's delivery order by (global
//            trigger, phase, global dense key) -- every trigger's matches come from its key's shard, so the merge
//            is a k-way interleave by trigger; G = 1: the GPU delivers straight into the caller's columns.
//
// Every stage of chunk j overlaps the other stages of chunks j-1 and j+1 (ring depth NODE_RING on the host,
// two device slots per GPU); no stage blocks another except through those rings.  A handle (sg_handle) is
// single-threaded: each is only ever driven by its shard's compute thread (and its copy thread's stream).
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
// where the node uses them (SG_NODE_NT bit mask, read once): 1 the host fill of trigger-row columns, 2 the G > 1
// scatter into shard staging, 4 the G > 1 merge's own column writes.  Default 1.  (A/B runs of the bits on one box,
// profiles/r04/node_nt_ab.log, were inside the host stages' own run-to-run spread of up to 2x.)
inline int nt_mode() {
  static const int m = [] {
    const char* e = getenv("SG_NODE_NT");
    return e ? atoi(e) : 1;
  }();
  return m;
}
template <int BIT, class V>
inline void put(V* p, V v) {
  if (nt_mode() & BIT) nt_store(p, v);
  else *p = v;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Fixed thread pool: parallel_for(n, fn) runs fn(0..n-1) on the workers and the caller and returns when all are
// done.  Several coordinator threads may submit at once (their tasks interleave).
struct Pool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::function<void()>> q;
  bool stop = false;
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i)
      th.emplace_back([this] {
        while (true) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || !q.empty(); });
            if (stop && q.empty()) return;
            f = std::move(q.back());
            q.pop_back();
          }
          f();
        }
      });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
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

}  // namespace

// One shard's rows of one chunk, in arrival order (host staging, G > 1).
struct NodeStage {
  Pinned ts, ts32, key, stream, gidx, raw;   // (ts32: the chunk's timestamps as 32-bit offsets from its minimum)   // (raw: device-dictionary mode, the key as received)
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
  int64_t g_keys = 0;
  // Row tags (one GPU, closed form): the e1 attribute the query only projects (e.g. `e1.id`) never crosses PCIe --
  // the GPU carries each row's event index mod 2^32 in its place (generated in HBM) and the host selector reads the
  // attribute of the e1 row the tag names from the caller's columns, or, for rows of earlier pushes the engine still
  // holds, from `hist` (kept at each push's end for exactly the carried rows' range).
  int tag_col = -1;
  int tag_cand = -1;                 // the query's tag column if it has one (tag_col: in use for this stream)
  bool tag_sel[SG_MAX_SELECT] = {};
  sg_nfa_desc edesc;                 // what the engine runs (the tag column as INT)
  Pinned tagbuf;
  int64_t hist_lo = 0, hist_n = 0;
  std::vector<int64_t> hist;
  std::vector<uint8_t> hist_nul;
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
  bool tag[SG_MAX_SELECT];      // e1.<tag column>: the GPU delivers the row tag (node tagbuf), the host the value
  int ns;
  int width[SG_MAX_SELECT];
  bool fill_ts;                 // out->ts from the trigger row's ts (host)
  int fill_col[SG_MAX_SELECT];  // >= 0: out->cols[k] (and nulls[k]) from batch column fill_col[k] at the trigger row
  bool any_fill;
};

Want want_of(const sg_node& nd, const sg_node_batch& b, const sg_match_columns* out) {
  Want w;
  memset(&w, 0, sizeof(w));
  const sg_nfa_desc& d = nd.desc;
  w.ns = d.n_out > 0 ? d.n_out : d.n_select;
  const bool tie = nd.G > 1 && d.shape != SG_SHAPE_EVERY_NEXT_CMP;
  const bool closed = d.shape == SG_SHAPE_EVERY_NEXT_CMP && d.n_out == 0 && !nd.no_fill;
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
  for (int k = 0; k < w.ns; ++k)
    if (nd.tag_sel[k] && (w.col[k] || w.nul[k])) {
      w.tag[k] = true;
      w.col[k] = true;   // (D2H of the tag into tagbuf)
      w.nul[k] = false;
    }
  w.any_fill = w.fill_ts;
  for (int k = 0; k < w.ns; ++k) w.any_fill |= w.fill_col[k] >= 0 || w.tag[k];
  return w;
}

// Host selector for the trigger-row columns of output rows [o0, o1): trig[] holds their global trigger indices.
inline void fill_row(const sg_node_batch& b, const sg_nfa_desc& d, const Want& w, const sg_match_columns* out,
                     int64_t o, uint64_t trig, const sg_node* nd = nullptr) {
  const int64_t t = (int64_t)(trig - b.base_index);
  if (nd && nd->tag_col >= 0) {   // e1's projected attribute through its row tag
    const int c = nd->tag_col;
    const int wc = sg_col_width(d.col_type[c]);
    for (int k = 0; k < w.ns; ++k) {
      if (!w.tag[k]) continue;
      const uint32_t tag = nd->tagbuf.as<uint32_t>()[o];
      const uint64_t g = trig - (uint64_t)(uint32_t)((uint32_t)trig - tag);   // e1 is at most 2^32 - 1 rows back
      int64_t v = 0;
      uint8_t nul = 0;
      if (g >= b.base_index) {
        const int64_t r = (int64_t)(g - b.base_index);
        v = wc == 8 ? ((const int64_t*)b.cols[c])[r] : (int64_t)((const int32_t*)b.cols[c])[r];
        nul = (b.nulls && b.nulls[c]) ? b.nulls[c][r] : 0;
      } else if ((int64_t)g >= nd->hist_lo && (int64_t)g < nd->hist_lo + nd->hist_n) {
        v = nd->hist[(size_t)((int64_t)g - nd->hist_lo)];
        nul = nd->hist_nul.empty() ? 0 : nd->hist_nul[(size_t)((int64_t)g - nd->hist_lo)];
      }
      if (out->cols[k]) {
        if (w.width[k] == 8) put<1>(&((int64_t*)out->cols[k])[o], v);
        else put<1>(&((int32_t*)out->cols[k])[o], (int32_t)v);
      }
      if (out->nulls[k]) out->nulls[k][o] = nul;
    }
  }
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
  // device-dictionary mode, per (chunk, shard): the shard's key count before the chunk and the first rows of the
  // keys the chunk introduced, in id order (G > 1: merged into node-wide first-seen ids)
  std::vector<int64_t> kbase_of;
  // per chunk: timestamps travel as 32-bit offsets from ts_base_of[j] when the chunk spans less than 2^31 ms
  std::vector<int64_t> ts_base_of;
  std::vector<uint8_t> ts32_of;
  std::vector<std::vector<uint32_t>> newf_of;
  std::vector<uint8_t> shard_tmp;            // device-dictionary route, G > 1: each row's shard (0xff: every shard)
  double t_route = 0, t_merge = 0, t_gpu[MAX_GPUS] = {};
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

// ---- device-dictionary mode: no key lookups on the host.  G = 1: nothing to do; G > 1: rows are scattered to
// shard mix64(raw key) mod G (rows of stream -1 reach every shard), each GPU dictionary-encodes its own keys --
// first-seen order inside a shard is the node's first-seen order restricted to it.
void route_chunk_dev(Run& r, int64_t j) {
  sg_node& nd = r.nd;
  const sg_nfa_desc& d = nd.desc;
  const int G = nd.G;
  const int slot = (int)(j % NODE_RING);
  const int64_t lo = chunk_lo(r, j), hi = chunk_lo(r, j + 1), n = hi - lo;
  if (G == 1) {
    r.rows_of[j] = n;
    return;
  }
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nd.threads, n / 65536 + 1));
  auto slice = [&](int t, int64_t& a, int64_t& e) {
    a = n * t / T;
    e = n * (t + 1) / T;
  };
  const int32_t* stream = r.b.stream ? r.b.stream + lo : nullptr;
  const int64_t* raw = r.b.raw_key + lo;
  auto shard = [&](int64_t i) -> int {
    return (stream && stream[i] < 0) ? -1 : (int)(sgr::mix64((uint64_t)raw[i]) % (uint64_t)G);
  };
  // pass 1: each row's shard (0xff: a clock-only row every shard gets) and the counts per (thread slice, shard)
  std::vector<uint8_t>& sh = r.shard_tmp;
  if ((int64_t)sh.size() < n) sh.resize((size_t)n);
  std::vector<std::vector<int64_t>> cnt(T, std::vector<int64_t>(G, 0));
  std::vector<int64_t> nbc(T, 0);
  nd.pool->parallel_for(T, [&](int t) {
    int64_t a, e;
    slice(t, a, e);
    int64_t* c = cnt[t].data();
    int64_t bcast = 0;
    for (int64_t i = a; i < e; ++i) {
      const int x = shard(i);
      sh[(size_t)i] = x >= 0 ? (uint8_t)x : (uint8_t)0xff;
      if (x >= 0) ++c[x];
      else ++bcast;
    }
    for (int q = 0; q < G; ++q) c[q] += bcast;
    nbc[t] = bcast;
  });
  std::vector<std::vector<int64_t>> off(T, std::vector<int64_t>(G, 0));
  for (int q = 0; q < G; ++q) {
    int64_t o = 0;
    for (int t = 0; t < T; ++t) {
      off[t][q] = o;
      o += cnt[t][q];
    }
    r.rows_of[j * G + q] = o;
  }
  const int nc = d.n_cols;
  int need[SG_MAX_COLS] = {};
  for (int k = 0; k < d.n_ret; ++k) need[d.ret_col[k]] = 1;
  const uint8_t* shp = sh.data();
  // pass 2: column by column, each a tight loop over the slice's rows into the G shard streams (arrival order kept)
  nd.pool->parallel_for(T, [&](int t) {
    int64_t a, e;
    slice(t, a, e);
    if (nbc[t]) {   // a slice with clock-only rows: row by row, those rows to every shard
      int64_t cur[MAX_GPUS];
      for (int q = 0; q < G; ++q) cur[q] = off[t][q];
      for (int64_t i = a; i < e; ++i) {
        const int own = shp[i] == 0xff ? -1 : (int)shp[i];
        for (int q = 0; q < G; ++q) {
          if (own >= 0 && q != own) continue;
          NodeStage& S = nd.stage[slot][q];
          const int64_t p = cur[q]++;
          put_ts(r, S, j, p, r.b.ts[lo + i]);
          S.raw.as<int64_t>()[p] = raw[i];
          if (stream) S.stream.as<int32_t>()[p] = stream[i];
          S.gidx.as<uint64_t>()[p] = r.b.base_index + (uint64_t)(lo + i);
          for (int c = 0; c < nc; ++c) {
            if (!need[c] || !r.b.cols[c]) continue;
            if (sg_col_width(d.col_type[c]) == 8) S.col[c].as<int64_t>()[p] = ((const int64_t*)r.b.cols[c])[lo + i];
            else S.col[c].as<int32_t>()[p] = ((const int32_t*)r.b.cols[c])[lo + i];
            if (r.b.nulls && r.b.nulls[c]) S.nul[c].as<uint8_t>()[p] = r.b.nulls[c][lo + i];
          }
        }
      }
      return;
    }
    auto scatter = [&](auto* const* dst, auto val) {
      int64_t cur[MAX_GPUS];
      for (int q = 0; q < G; ++q) cur[q] = off[t][q];
      for (int64_t i = a; i < e; ++i) {
        const int q = shp[i];
        put<2>(&dst[q][cur[q]++], val(i));
      }
    };
    const int64_t* ts = r.b.ts + lo;
    if (r.ts32_of[j]) {
      int32_t* dt[MAX_GPUS];
      for (int q = 0; q < G; ++q) dt[q] = nd.stage[slot][q].ts32.as<int32_t>();
      const int64_t tb = r.ts_base_of[j];
      scatter(dt, [&](int64_t i) { return (int32_t)(ts[i] - tb); });
    } else {
      int64_t* dt[MAX_GPUS];
      for (int q = 0; q < G; ++q) dt[q] = nd.stage[slot][q].ts.as<int64_t>();
      scatter(dt, [&](int64_t i) { return ts[i]; });
    }
    {
      int64_t* dr[MAX_GPUS];
      for (int q = 0; q < G; ++q) dr[q] = nd.stage[slot][q].raw.as<int64_t>();
      scatter(dr, [&](int64_t i) { return raw[i]; });
    }
    if (stream) {
      int32_t* ds[MAX_GPUS];
      for (int q = 0; q < G; ++q) ds[q] = nd.stage[slot][q].stream.as<int32_t>();
      scatter(ds, [&](int64_t i) { return stream[i]; });
    }
    {
      uint64_t* dg[MAX_GPUS];
      for (int q = 0; q < G; ++q) dg[q] = nd.stage[slot][q].gidx.as<uint64_t>();
      const uint64_t gb = r.b.base_index + (uint64_t)lo;
      scatter(dg, [&](int64_t i) { return gb + (uint64_t)i; });
    }
    for (int c = 0; c < nc; ++c) {
      if (!need[c] || !r.b.cols[c]) continue;
      if (sg_col_width(d.col_type[c]) == 8) {
        int64_t* dc[MAX_GPUS];
        for (int q = 0; q < G; ++q) dc[q] = nd.stage[slot][q].col[c].as<int64_t>();
        const int64_t* sc = (const int64_t*)r.b.cols[c] + lo;
        scatter(dc, [&](int64_t i) { return sc[i]; });
      } else {
        int32_t* dc[MAX_GPUS];
        for (int q = 0; q < G; ++q) dc[q] = nd.stage[slot][q].col[c].as<int32_t>();
        const int32_t* sc = (const int32_t*)r.b.cols[c] + lo;
        scatter(dc, [&](int64_t i) { return sc[i]; });
      }
      if (r.b.nulls && r.b.nulls[c]) {
        uint8_t* dn[MAX_GPUS];
        for (int q = 0; q < G; ++q) dn[q] = nd.stage[slot][q].nul[c].as<uint8_t>();
        const uint8_t* sn = r.b.nulls[c] + lo;
        scatter(dn, [&](int64_t i) { return sn[i]; });
      }
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);   // (streaming stores drained before the chunk is published)
  });
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
      if (c == nd.tag_col) cols[c] = nuls[c] = nullptr;   // (tags are made in HBM)
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
        const int64_t* rk = nd.G == 1 ? r.b.raw_key + chunk_lo(r, j) : nd.stage[j % NODE_RING][s].raw.as<int64_t>();
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
__global__ void k_row_tags(uint32_t base, int64_t n, uint32_t* __restrict__ tag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    tag[i] = base + (uint32_t)i;
}

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
  auto cp = [&](void* base, size_t off, size_t width) {
    if (!base) return;
    const int64_t p = dst.M ? pos % dst.M : pos;
    const int64_t first = dst.M ? std::min<int64_t>(k, dst.M - p) : k;
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
        dst.col[c] = r.w.tag[c] ? nd.tagbuf.p : r.out->cols[c];
        dst.nul[c] = r.w.tag[c] ? nullptr : r.out->nulls[c];
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
        if (nd.tag_col >= 0) {   // row tags: event index mod 2^32, in place of the projected-only column
          hipLaunchKernelGGL(k_row_tags, dim3((unsigned)std::min<int64_t>((sb.n + 255) / 256, 8192)), dim3(256), 0,
                             h.stream, (uint32_t)(sb.base_index), sb.n, (uint32_t*)sp.col[nd.tag_col]);
          HIPCHK(hipGetLastError());
        }
        if (r.ts32_of[j]) {   // widen the 32-bit offsets into the slot's timestamp column
          hipLaunchKernelGGL(k_ts_widen, dim3((unsigned)std::min<int64_t>((sb.n + 255) / 256, 8192)), dim3(256), 0,
                             h.stream, (const int32_t*)nd.dts32[s][ds], r.ts_base_of[j], sb.n, (int64_t*)sp.ts);
          HIPCHK(hipGetLastError());
        }
        if (nd.ddict == 1) {   // dictionary-encode the chunk's raw keys on this GPU
          const int64_t before = nd.kd[s].n_keys;
          std::vector<uint32_t> nf;
          kd_resolve(nd.kd[s], nd.draw[s][ds], bv.stream, sb.n, (int32_t*)sp.key, h.stream, nd.G > 1 ? &nf : nullptr);
          bv.key_bound = (int32_t)std::max<int64_t>(1, nd.kd[s].n_keys);
          r.publish([&] {
            r.kbase_of[j * nd.G + s] = before;
            r.newf_of[j * nd.G + s].swap(nf);
          });
        }
        for (int c = 0; c < nd.desc.n_cols; ++c) {
          bv.cols.col[c] = (sb.cols[c] || c == nd.tag_col) ? sp.col[c] : nullptr;
          bv.cols.nul[c] = (sb.nulls && sb.nulls[c] && c != nd.tag_col) ? (const uint8_t*)sp.nul[c] : nullptr;
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
  if (nd.ddict == 1) {
    // node-wide first-seen ids of the keys chunk j introduced: every shard's new keys are in first-row order, so a
    // k-way merge by global first row interleaves them
    int64_t cur[MAX_GPUS] = {}, m[MAX_GPUS];
    for (int s = 0; s < G; ++s) {
      m[s] = (int64_t)r.newf_of[j * G + s].size();
      if (m[s] > 0) nd.l2g[s].resize((size_t)(r.kbase_of[j * G + s] + m[s]));   // (kbase_of is unset without rows)
    }
    auto gfirst = [&](int s, int64_t q) { return nd.stage[slot][s].gidx.as<uint64_t>()[r.newf_of[j * G + s][q]]; };
    while (true) {
      int best = -1;
      for (int s = 0; s < G; ++s)
        if (cur[s] < m[s] && (best < 0 || gfirst(s, cur[s]) < gfirst(best, cur[best]))) best = s;
      if (best < 0) break;
      nd.l2g[best][r.kbase_of[j * G + best] + cur[best]] = (int32_t)nd.g_keys++;
      ++cur[best];
    }
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
      return nd.ddict == 1 ? (int64_t)nd.l2g[s][lk] : (int64_t)rt->l2d[s][lk];
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
          const int tc = nd.tag_col;
          const bool pf = tc >= 0 && r.b.cols[tc];
          const int wc = pf ? sg_col_width(nd.desc.col_type[tc]) : 8;
          const uint32_t* tags = nd.tagbuf.as<uint32_t>();
          constexpr int64_t D = 32;   // e1 rows are scattered over the last `within`: keep 32 of their lines in flight
          for (int64_t o = a; o < e; ++o) {
            if (pf && o + D < e) {
              const uint64_t tr = r.out->trigger[o + D];
              const uint64_t g = tr - (uint64_t)(uint32_t)((uint32_t)tr - tags[o + D]);
              if (g >= r.b.base_index) __builtin_prefetch((const char*)r.b.cols[tc] + (size_t)wc * (g - r.b.base_index));
            }
            fill_row(r.b, nd.desc, r.w, r.out, o, r.out->trigger[o], &nd);
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
        if (nd.ddict == 1) S.raw.ensure((size_t)C * 8);
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
  if (nd.tag_col >= 0) nd.tagbuf.ensure((size_t)std::max<int64_t>(r.cap, 1) * 4);
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

void keep_history(sg_node& nd, const sg_node_batch& b);

// Switch the row tags on or off for a new stream: the GPU handles are reopened with the tag column as INT (or as the
// query declares it).
void set_tags(sg_node& nd, bool on) {
  if ((nd.tag_col >= 0) == on) return;
  const sg_nfa_desc* dd = &nd.desc;
  nd.edesc = nd.desc;
  for (int k = 0; k < SG_MAX_SELECT; ++k) nd.tag_sel[k] = false;
  if (on) {
    const int c = nd.tag_cand;
    nd.edesc.col_type[c] = SG_T_INT;
    for (int k = 0; k < nd.desc.n_ret; ++k)
      if (nd.desc.ret_col[k] == c) nd.edesc.ret_type[k] = SG_T_INT;
    for (int k = 0; k < nd.desc.n_select; ++k)
      if (nd.desc.ret_col[nd.desc.sel_ret[k]] == c) {
        nd.edesc.sel_type[k] = SG_T_INT;
        nd.tag_sel[k] = nd.desc.sel_state[k] == nd.desc.shape_args[0];
      }
    dd = &nd.edesc;
  }
  for (int s = 0; s < nd.G; ++s) {
    HIPCHK(hipSetDevice(nd.dev[s]));
    if (nd.h[s]) sg_close(nd.h[s]);
    nd.h[s] = nullptr;
    const int rc = sg_open(nd.dev[s], dd, &nd.opt, &nd.h[s]);
    if (rc != SG_OK) throw SgError(rc, "node: reopening the GPU handle failed");
  }
  nd.tag_col = on ? nd.tag_cand : -1;
  nd.hist_n = 0;
}

// Auto key dictionary: keys are encoded on the GPUs whenever the query allows it (partitioned, no playback clocks).
// Measured on C2 (100M events, 10k keys, one GPU, profiles/r03/whole_node_*_dict.log): the host router's lookups were
// the pipeline's bound (route 50 ms of 58.7 ms per push) even with a cache-resident table, while raw 8-byte keys cost
// only 0.4 GB more H2D (route 13 ms, 48.8 ms per push); with 1M keys (C5) the host table is DRAM-bound as well.
void run_push(sg_node& nd, const sg_node_batch& b, const sg_match_columns* out, int64_t cap, int64_t* n_out) {
  if (nd.ddict < 0) {   // the first push of a stream fixes where keys are encoded, and whether rows carry tags
    const bool dev_ok = nd.desc.partitioned && !need_clocks(nd.desc);
    nd.ddict = (dev_ok && nd.key_dict_mode != 1) ? 1 : 0;
    // tags save PCIe bytes at the price of host selector work (random e1 reads): opt-in, SG_NODE_TAGS=1
    const char* e = getenv("SG_NODE_TAGS");
    const bool want = nd.tag_cand >= 0 && e && e[0] == '1';   // (measured: the host's e1 gathers cost more than
                                                               // the PCIe bytes they save on this pool's hosts)
    set_tags(nd, want);
  }
  Run r(nd, b, out, cap);
  r.w = want_of(nd, b, out);
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
  r.kbase_of.assign((size_t)(r.nch * nd.G), 0);
  r.ts_base_of.assign((size_t)r.nch, 0);
  r.ts32_of.assign((size_t)r.nch, 0);
  r.newf_of.assign((size_t)(r.nch * nd.G), std::vector<uint32_t>());
  const double t0 = now_ms();
  reserve_all(r);
  const double t_res = now_ms() - t0;
  // local index bases of each shard's rows per chunk are fixed as chunks are routed
  std::vector<std::thread> th;
  for (int s = 0; s < nd.G; ++s) {
    th.emplace_back(copy_loop, std::ref(r), s);
    th.emplace_back(gpu_loop, std::ref(r), s);
  }
  if (nd.G > 1) th.emplace_back(merge_loop, std::ref(r));
  else if (r.w.any_fill) th.emplace_back(fill_loop, std::ref(r));
  const double t1 = now_ms();
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
  for (auto& t : th) t.join();
  for (int s = 0; s < nd.G; ++s) {
    hipSetDevice(nd.dev[s]);
    hipStreamSynchronize(nd.h[s]->h.stream);
    hipStreamSynchronize(nd.cp[s]);
    if (nd.h[s]->h.eg.d2h) hipStreamSynchronize(nd.h[s]->h.eg.d2h);
  }
  if (r.failed) {
    nd.broken = true;
    throw SgError(r.fail_code, r.fail_msg);
  }
  if (nd.tag_col >= 0) keep_history(nd, b);
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
  delete nd->pool;
  delete nd;
}

// The tag column of a closed-form query: the one batch column e1 contributes to the select besides the compared value
// (LONG / INT), read by no predicate -- or -1.
int tag_column(const sg_nfa_desc& d) {
  if (d.shape != SG_SHAPE_EVERY_NEXT_CMP || d.n_out != 0) return -1;
  const int a_state = d.shape_args[0];
  const int val_a = d.ret_col[d.shape_args[4]], val_b = d.ret_col[d.shape_args[3]];
  int c = -1;
  for (int k = 0; k < d.n_select; ++k) {
    if (d.sel_state[k] != a_state) continue;
    const int col = d.ret_col[d.sel_ret[k]];
    if (col == val_a) continue;
    if (d.sel_index[k] != 0 && d.sel_index[k] != -1) return -1;
    if (c >= 0 && c != col) return -1;
    c = col;
  }
  if (c < 0 || c == val_b || (d.col_type[c] != SG_T_LONG && d.col_type[c] != SG_T_INT)) return -1;
  auto reads = [&](int off, int len) {   // does a postfix program read column c?
    for (int pc = off; pc < off + len;) {
      const int64_t op = d.code[pc];
      if (op == SG_OP_VAR) {
        if (d.ret_col[d.code[pc + 3]] == c) return true;
        pc += 5;
      } else if (op == SG_OP_CONST || op == SG_OP_CMP || op == SG_OP_MATH) {
        pc += 3;
      } else {
        pc += 1;
      }
    }
    return false;
  };
  for (int s = 0; s < d.n_states; ++s)
    if (reads(d.states[s].prog_off, d.states[s].prog_len)) return -1;
  if (reads(d.shape_prog_off, d.shape_prog_len)) return -1;
  return c;
}

// After a push: keep the tag column's values of the rows the engine still carries (the only earlier rows a later
// match can name as e1): [push_end - lag, push_end) from the caller's columns and the previous history.
void keep_history(sg_node& nd, const sg_node_batch& b) {
  const int c = nd.tag_col;
  const int64_t end = (int64_t)(b.base_index + (uint64_t)b.n);
  HIPCHK(hipSetDevice(nd.dev[0]));
  const int64_t lag = sg_every_next_carry_max_lag(&nd.h[0]->h, c, (uint32_t)end);
  if (lag <= 0) {
    nd.hist_n = 0;
    return;
  }
  const int64_t lo = end - lag;
  std::vector<int64_t> h((size_t)lag);
  std::vector<uint8_t> hn;
  const bool nul = (b.nulls && b.nulls[c]) || !nd.hist_nul.empty();
  if (nul) hn.assign((size_t)lag, 0);
  const int wc = sg_col_width(nd.desc.col_type[c]);
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nd.threads, lag / 65536 + 1));
  bool miss = false;
  nd.pool->parallel_for(T, [&](int t) {
    const int64_t a = lo + lag * t / T, e = lo + lag * (t + 1) / T;
    for (int64_t g = a; g < e; ++g) {
      int64_t v = 0;
      uint8_t u = 0;
      if (g >= (int64_t)b.base_index) {
        const int64_t r = g - (int64_t)b.base_index;
        v = wc == 8 ? ((const int64_t*)b.cols[c])[r] : (int64_t)((const int32_t*)b.cols[c])[r];
        u = (b.nulls && b.nulls[c]) ? b.nulls[c][r] : 0;
      } else if (g >= nd.hist_lo && g < nd.hist_lo + nd.hist_n) {
        v = nd.hist[(size_t)(g - nd.hist_lo)];
        u = nd.hist_nul.empty() ? 0 : nd.hist_nul[(size_t)(g - nd.hist_lo)];
      } else {
        miss = true;
      }
      h[(size_t)(g - lo)] = v;
      if (nul) hn[(size_t)(g - lo)] = u;
    }
  });
  if (miss) throw SgError(SG_EINVAL, "internal: a carried row is older than the node's tag history");
  nd.hist.swap(h);
  nd.hist_nul.swap(hn);
  nd.hist_lo = lo;
  nd.hist_n = lag;
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
  nd->no_fill = getenv("SG_NODE_NO_FILL") != nullptr;
  nd->no_ts32 = getenv("SG_NODE_NO_TS32") != nullptr;
  nd->edesc = nd->desc;
  nd->tag_cand = (n_gpus == 1 && !nd->no_fill) ? tag_column(nd->desc) : -1;
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
  if (rc == SG_OK) nd->pool = new Pool(std::max(0, nd->threads - 1));
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
  nd->hist_n = 0;
  nd->hist.clear();
  nd->hist_nul.clear();
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
