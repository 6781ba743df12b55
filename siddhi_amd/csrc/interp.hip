// General NFA pass on MI355X (SG_SHAPE_GENERAL): one thread advances one partition key's runtime
// (interp.h KeyMachine, the flat restatement of the Pre/Post processor chain) over that key's rows.
//
// Per sg_push:
//   1. k_route      rows -> partition key (sentinel for rows no receiver reads / null keys);
//                   for playback queries with `not ... for T` also checks that timestamps never decrease
//   2. key partition stable radix sort of (key, row) (rocPRIM) + k_segments: each key's rows contiguous,
//                   in arrival order (PartitionStreamReceiver routing)
//   3. k_nfa        one thread per key that ever appeared: runs the key machine over its rows and the
//                   absence timers its schedulers fire on the global playback clock; every match is
//                   appended (atomic bump) with a sort key (trigger row, timer-before-event, key).
//      k_nfa_units  (shapes with a bounded horizon, interp.h sg_chunk_rule) one thread per (key, chunk of
//                   R rows): a unit rebuilds its key's state by replaying the rows inside the horizon before
//                   its chunk, so a key's rows run on many lanes instead of one
//   4. radix sort of the sort keys (stable: per-key emission order is kept) + k_gather into the
//                   pending match store in the reference's delivery order.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <string>

#include "sg_device.h"
#include "sg_engine.h"
#include "interp.h"
#include "pred.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct GeneralState {
  SgGeo geo;
  int32_t* arena = nullptr;
  int64_t keys_alloc = 0;     // arenas allocated
  SgGeo* dgeo = nullptr;
  int32_t* dfail = nullptr;
  PartialState* pp = nullptr; // partial-lane route (partial.hip) while the query and the stream allow it
  int pp_checked = 0;
  int64_t max_ts = INT64_MIN;  // largest timestamp pushed (INT64_MAX once a timestamp went back)
  int64_t clock = 0;           // playback clock after the last push (TimestampGeneratorImpl.lastEventTimestamp)
  int64_t grows = 0;           // capacity growths (pushes rerun with larger pools / lists / emission space)
};

static bool has_count_state(const sg_nfa_desc& d) {
  for (int s = 0; s < d.n_states; ++s)
    if (d.states[s].kind == SG_K_COUNT) return true;
  return false;
}

__global__ void k_route(int64_t n, const int32_t* __restrict__ stream, const int32_t* __restrict__ key,
                        const int64_t* __restrict__ ts, const DevDesc* __restrict__ dd, int partitioned,
                        uint32_t sentinel, int check_order, uint32_t* __restrict__ okey, uint32_t* __restrict__ orow,
                        int32_t* __restrict__ order_err) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int s = stream ? stream[i] : 0;
  bool own = s >= 0 && s < SG_MAX_STREAMS && dd->recv_of_stream[s] >= 0;
  uint32_t k = sentinel;
  if (own) {
    if (!partitioned) k = 0;
    else {
      int32_t kk = key ? key[i] : -1;
      if (kk >= 0) {
        // a key at or above the caller's key_bound would fall outside the sorted bits and the per-key tables
        if ((uint32_t)kk >= sentinel) atomicOr(order_err, 2);
        else k = (uint32_t)kk;
      }
    }
  }
  okey[i] = k;
  orow[i] = (uint32_t)i;
  if (check_order && i > 0 && ts[i - 1] > ts[i]) atomicOr(order_err, 1);
}

__global__ void k_segments(int64_t n, const uint32_t* __restrict__ skey, uint32_t sentinel, uint32_t* __restrict__ beg,
                           uint32_t* __restrict__ end) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint32_t k = skey[p];
  if (k == sentinel) return;
  if (p == 0 || skey[p - 1] != k) beg[k] = (uint32_t)p;
  if (p == n - 1 || skey[p + 1] != k) end[k] = (uint32_t)p + 1;
}

struct DevRows {
  const uint32_t* rows;   // sorted row indices of this key: rows[0..nown)
  int64_t nown;
  int64_t n;
  const int64_t* ts;
  const int32_t* stream;
  const SgCols* cols;
  const DevDesc* d;
  uint64_t base;
  const uint64_t* index;
  __device__ uint64_t index_of(int64_t r) { return index ? gptr<uint64_t>(index)[r] : base + (uint64_t)r; }
  __device__ int64_t first_after(int64_t pos) {
    if (!index) {
      int64_t p = pos - (int64_t)base + 1;
      return p < 0 ? 0 : (p > n ? n : p);
    }
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if ((int64_t)gptr<uint64_t>(index)[mid] <= pos) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
  __device__ int64_t n_own() { return nown; }
  __device__ int64_t own_local(int64_t i) { return (int64_t)gptr<uint32_t>(rows)[i]; }
  __device__ int stream_at(int64_t r) { return stream ? gptr<int32_t>(stream)[r] : 0; }
  __device__ int64_t n_rows() { return n; }
  __device__ int64_t ts_at(int64_t r) { return gptr<int64_t>(ts)[r]; }
  __device__ int64_t ts_(int64_t r) { return gptr<int64_t>(ts)[r]; }
  // playback clock (queries with absence): clk = running max of the batch's ts, clock0 = the clock before the push,
  // nfr[n - 1 - r] = first row >= r that notifies the schedulers (ts >= the clock before it), or n
  const int64_t* clk;
  const uint32_t* nfr;
  int64_t clock0;
  __device__ int64_t clock_at(int64_t r) {
    if (!clk) return gptr<int64_t>(ts)[r];
    const int64_t c = gptr<int64_t>(clk)[r];
    return c > clock0 ? c : clock0;
  }
  __device__ int64_t find_ge(int64_t from, int64_t v) {
    int64_t lo = from, hi = n;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if (clock_at(mid) < v) lo = mid + 1;
      else hi = mid;
    }
    if (!clk || lo >= n) return lo;
    return (int64_t)gptr<uint32_t>(nfr)[n - 1 - lo];
  }
  __device__ void fill(int64_t r, SgRow& row) {
    row.ts = gptr<int64_t>(ts)[r];
    row.index = index_of(r);
    row.stream = stream ? gptr<int32_t>(stream)[r] : 0;
    row.nullmask = 0;
    for (int k = 0; k < d->n_ret; ++k) {
      SgVal v = sg_read_col(*cols, d->ret_col[k], d->ret_type[k], r);
      if (v.null) row.nullmask |= 1 << k;
      row.vals[k] = sg_val_bits(v);
    }
  }
};
// sg_run_key calls rows.ts(r)
struct DevRowsTs : DevRows {
  __device__ int64_t ts(int64_t r) { return gptr<int64_t>(DevRows::ts)[r]; }
};

// The descriptor (programs, state tables: ~9.6 KB) and the arena geometry are read hundreds of times per event;
// each workgroup copies them into LDS once so those reads are LDS hits instead of L2 round trips.
struct NfaLds {
  DevDesc d;
  SgGeo g;
  const uint64_t* lbits[SG_MAX_STATES];
  int32_t any_bits;
};
__device__ __forceinline__ void nfa_stage_desc(NfaLds& L, const DevDesc* __restrict__ dd, const SgGeo* __restrict__ geo,
                                               const uint64_t* const* lbits) {
  if (threadIdx.x < SG_MAX_STATES) L.lbits[threadIdx.x] = lbits[threadIdx.x];
  if (threadIdx.x == 0) {
    int any = 0;
    for (int s = 0; s < SG_MAX_STATES; ++s) any |= lbits[s] != nullptr;
    L.any_bits = any;
  }
  const uint32_t* src = (const uint32_t*)dd;
  uint32_t* dst = (uint32_t*)&L.d;
  for (uint32_t i = threadIdx.x; i < sizeof(DevDesc) / 4; i += blockDim.x) dst[i] = src[i];
  const uint32_t* gs = (const uint32_t*)geo;
  uint32_t* gd = (uint32_t*)&L.g;
  for (uint32_t i = threadIdx.x; i < sizeof(SgGeo) / 4; i += blockDim.x) gd[i] = gs[i];
  __syncthreads();
}

struct NfaArgs {
  int64_t n;
  uint64_t base_index;
  int64_t nkeys;
  int32_t partitioned;
  int32_t clone;
  const uint32_t* rows;
  const uint32_t* beg;
  const uint32_t* end;
  const int64_t* ts;
  const int32_t* stream;
  const uint64_t* index;
  const uint64_t* lbits[SG_MAX_STATES];   // predicate-pass condition bits per state (null: none)
  const int64_t* clk;                     // playback clock per row and next notifying row (DevRows); null: none
  const uint32_t* nfr;
  int64_t clock0;
};

__global__ void __launch_bounds__(64) k_nfa(NfaArgs a, SgCols cols, const DevDesc* __restrict__ dd,
                                            const SgGeo* __restrict__ geo, int32_t* __restrict__ arena,
                                            SgEmitSink sink, int32_t* __restrict__ fail_code) {
  __shared__ NfaLds L;
  nfa_stage_desc(L, dd, geo, a.lbits);
  dd = &L.d;
  geo = &L.g;
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.nkeys) return;
  int32_t* ar = arena + k * geo->key_words;
  uint32_t b = a.beg[k], e = a.end[k];
  // keys that never received a row have no runtime yet (and no timers)
  if (ar[K_CREATED] == 0 && e <= b && a.partitioned) return;
  KeyMachine m;
  m.d = dd;
  m.g = geo;
  m.a = (SG_GLOBAL int32_t*)ar;
  m.key = (int32_t)k;
  m.clone = a.clone;
  m.sink = sink;
  m.base_index = a.base_index;
  m.trigger = a.base_index;
  m.phase = 1;
  m.group = 0;
  m.now = 0;
  m.silent = 0;
  m.lbits = L.any_bits ? L.lbits : nullptr;
  m.failed = ar[K_OVERFLOW];
  if (m.failed) { atomicCAS(fail_code, 0, m.failed); return; }
  DevRowsTs rows;
  rows.rows = a.rows + b;
  rows.nown = (e > b) ? (int64_t)(e - b) : 0;
  rows.n = a.n;
  rows.DevRows::ts = a.ts;
  rows.stream = a.stream;
  rows.cols = &cols;
  rows.d = dd;
  rows.base = a.base_index;
  rows.index = a.index;
  rows.clk = a.clk;
  rows.nfr = a.nfr;
  rows.clock0 = a.clock0;
  sg_run_key(m, rows, !a.partitioned);
  if (m.failed) atomicCAS(fail_code, 0, m.failed);
}

// ---- chunked units (interp.h sg_chunk_rule): unit u = (key, chunk c) over the key's own rows
// [c*R, min(nown, (c+1)*R)).  Unit 0 continues the key's carried runtime in place; unit c > 0 runs in a
// scratch arena from a fresh runtime (or from the key's state at the push start when its horizon reaches
// the key's first row of this push) and replays its horizon without emitting.  After the pass the last
// unit's arena becomes the key's runtime.
struct UnitArgs {
  uint32_t R;
  SgChunkRule rule;
  const uint32_t* umap;     // unit -> key
  const uint32_t* uoff;     // key -> first unit
  int64_t n_units;
  int32_t* scratch;         // per-unit arenas
  const int32_t* snap;      // arenas at the push start
};

__global__ void k_unit_count(int64_t nkeys, const uint32_t* __restrict__ beg, const uint32_t* __restrict__ end,
                             uint32_t R, uint32_t* __restrict__ nch) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > nkeys) return;
  uint32_t rows = (k < nkeys && end[k] > beg[k]) ? end[k] - beg[k] : 0u;
  nch[k] = (rows + R - 1) / R;
}

__global__ void k_unit_map(int64_t nkeys, const uint32_t* __restrict__ uoff, uint32_t* __restrict__ umap) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  for (uint32_t u = uoff[k]; u < uoff[k + 1]; ++u) umap[u] = (uint32_t)k;
}

__global__ void __launch_bounds__(64) k_nfa_units(NfaArgs a, UnitArgs ua, SgCols cols, const DevDesc* __restrict__ dd,
                                                  const SgGeo* __restrict__ geo, int32_t* __restrict__ arena,
                                                  SgEmitSink sink, int32_t* __restrict__ fail_code) {
  __shared__ NfaLds L;
  nfa_stage_desc(L, dd, geo, a.lbits);
  dd = &L.d;
  geo = &L.g;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= ua.n_units) return;
  const uint32_t k = ua.umap[u];
  const uint32_t c = (uint32_t)(u - ua.uoff[k]);
  const uint32_t b = a.beg[k], e = a.end[k];
  const int64_t nown = (int64_t)(e - b);
  const int64_t p0 = (int64_t)c * ua.R, p1 = p0 + ua.R < nown ? p0 + ua.R : nown;
  const size_t kw = (size_t)geo->key_words;
  int32_t* ar;
  int64_t q = 0;
  if (c == 0) {
    ar = arena + (size_t)k * kw;
  } else {
    ar = ua.scratch + (size_t)u * kw;
    const uint32_t* own = a.rows + b;
    const int64_t* ts = a.ts;
    q = sg_replay_start(ua.rule, p0, [&](int64_t i) { return ts[own[i]]; });
    if (q == 0) {
      const int32_t* src = ua.snap + (size_t)k * kw;
      for (size_t w = 0; w < kw; ++w) ar[w] = src[w];
    } else {
      ar[K_CREATED] = 0;
      ar[K_OVERFLOW] = 0;
    }
  }
  KeyMachine m;
  m.d = dd;
  m.g = geo;
  m.a = (SG_GLOBAL int32_t*)ar;
  m.key = (int32_t)k;
  m.clone = a.clone;
  m.sink = sink;
  m.base_index = a.base_index;
  m.trigger = a.base_index;
  m.phase = 1;
  m.group = 0;
  m.now = 0;
  m.silent = 0;
  m.lbits = L.any_bits ? L.lbits : nullptr;
  m.failed = ar[K_OVERFLOW];
  if (m.failed) { atomicCAS(fail_code, 0, m.failed); return; }
  DevRowsTs rows;
  rows.rows = a.rows + b + q;
  rows.nown = p1 - q;
  rows.n = a.n;
  rows.DevRows::ts = a.ts;
  rows.stream = a.stream;
  rows.cols = &cols;
  rows.d = dd;
  rows.base = a.base_index;
  rows.index = a.index;
  rows.clk = a.clk;
  rows.nfr = a.nfr;
  rows.clock0 = a.clock0;
  sg_run_key(m, rows, !a.partitioned, p0 - q);
  if (m.failed) atomicCAS(fail_code, 0, m.failed);
}

// the last unit's runtime becomes the key's runtime (one block per key)
__global__ void k_unit_keep(int64_t nkeys, const uint32_t* __restrict__ uoff, const int32_t* __restrict__ scratch,
                            const SgGeo* __restrict__ geo, int32_t* __restrict__ arena) {
  for (int64_t k = blockIdx.x; k < nkeys; k += gridDim.x) {
    const uint32_t u0 = uoff[k], u1 = uoff[k + 1];
    if (u1 - u0 < 2) continue;
    const size_t kw = (size_t)geo->key_words;
    const int32_t* src = scratch + (size_t)(u1 - 1) * kw;
    int32_t* dst = arena + (size_t)k * kw;
    for (size_t w = threadIdx.x; w < kw; w += blockDim.x) dst[w] = src[w];
  }
}

// A key's runtime moved into a larger arena geometry (capacity growth): lists, pools and timer FIFOs keep their
// entries at the same indices (pool entries are addressed by index, never by arena offset); the new pool entries
// are put on the free lists and each timer FIFO is unrolled to start at 0.  One block per key.
__global__ void k_regeo(int64_t nkeys, const int32_t* __restrict__ old_arena, SgGeo og, int32_t* __restrict__ new_arena,
                        SgGeo ng) {
  for (int64_t k = blockIdx.x; k < nkeys; k += gridDim.x) {
    const int32_t* o = old_arena + (size_t)k * og.key_words;
    int32_t* a = new_arena + (size_t)k * ng.key_words;
    const int hw = sg_hdr_words(og.S);
    for (int w = threadIdx.x; w < hw; w += blockDim.x) a[w] = o[w];
    for (int l = 0; l < 2 * og.S; ++l)
      for (int w = threadIdx.x; w <= og.L; w += blockDim.x) a[ng.off_lists + l * (ng.L + 1) + w] = o[og.off_lists + l * (og.L + 1) + w];
    for (int w = threadIdx.x; w < og.P * og.part_words; w += blockDim.x) a[ng.off_part + w] = o[og.off_part + w];
    for (int w = threadIdx.x; w < og.E * og.ev_words; w += blockDim.x) a[ng.off_ev + w] = o[og.off_ev + w];
    for (int w = threadIdx.x; w < og.C * 3; w += blockDim.x) a[ng.off_chain + w] = o[og.off_chain + w];
    // new pool entries: a chain ending in the old free list, pushed in front of it
    for (int p = og.P + threadIdx.x; p < ng.P; p += blockDim.x)
      a[ng.off_part + p * ng.part_words + 2] = p + 1 < ng.P ? p + 1 : o[K_FREE_P];
    for (int e = og.E + threadIdx.x; e < ng.E; e += blockDim.x)
      a[ng.off_ev + e * ng.ev_words + 5] = e + 1 < ng.E ? e + 1 : o[K_FREE_E];
    for (int c = og.C + threadIdx.x; c < ng.C; c += blockDim.x)
      a[ng.off_chain + c * 3 + 2] = c + 1 < ng.C ? c + 1 : o[K_FREE_C];
    for (int i = 0; i < og.A; ++i) {
      const int32_t* oq = o + og.off_timer + i * (2 + 2 * og.Q);
      int32_t* nq = a + ng.off_timer + i * (2 + 2 * ng.Q);
      const int32_t head = oq[0], cnt = oq[1];
      for (int j = threadIdx.x; j < cnt; j += blockDim.x) {
        const int src = (head + j) % og.Q;
        nq[2 + 2 * j] = oq[2 + 2 * src];
        nq[3 + 2 * j] = oq[3 + 2 * src];
      }
      if (threadIdx.x == 0) {
        nq[0] = 0;
        nq[1] = cnt;
      }
    }
    if (threadIdx.x == 0 && o[K_CREATED]) {
      if (ng.P > og.P) { a[K_FREE_P] = og.P; a[K_NFREE_P] = o[K_NFREE_P] + (ng.P - og.P); }
      if (ng.E > og.E) { a[K_FREE_E] = og.E; a[K_NFREE_E] = o[K_NFREE_E] + (ng.E - og.E); }
      if (ng.C > og.C) { a[K_FREE_C] = og.C; a[K_NFREE_C] = o[K_NFREE_C] + (ng.C - og.C); }
    }
  }
}

__global__ void k_sortkeys(int64_t n, const char* __restrict__ buf, int32_t stride, uint64_t* __restrict__ sk,
                           uint32_t* __restrict__ idx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sk[i] = *(const uint64_t*)(buf + (size_t)i * stride);
  idx[i] = (uint32_t)i;
}

__global__ void k_gather(int64_t n, const char* __restrict__ buf, int32_t stride, const uint32_t* __restrict__ idx,
                         char* __restrict__ out, int32_t ostride) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t* src = (const uint64_t*)(buf + (size_t)idx[i] * stride + 8);
  uint64_t* dst = (uint64_t*)(out + (size_t)i * ostride);
  for (int w = 0; w < ostride / 8; ++w) dst[w] = src[w];
}

// The playback clock over a push (TimestampGeneratorImpl.setCurrentTimestamp, C/util/timestamp/
// TimestampGeneratorImpl.java:106-125): clk = running max of ts (scanned), then per row whether it notifies the
// schedulers (ts >= the clock before it) written in reverse, so a min scan gives each row's next notifying row.
__global__ void k_fire_rev(int64_t n, const int64_t* __restrict__ ts, const int64_t* __restrict__ clk, int64_t clock0,
                           uint32_t* __restrict__ rev) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t before = i ? clk[i - 1] : clock0;
  before = before > clock0 ? before : clock0;
  rev[n - 1 - i] = ts[i] >= before ? (uint32_t)i : (uint32_t)n;
}

static GeneralState* gstate(SgHandle* h) {
  if (!h->state) {
    GeneralState* g = new GeneralState();
    int q = h->opt.list_cap;
    g->geo = sg_make_geo(h->desc, h->opt.pool_partials, h->opt.pool_events, h->opt.pool_chain, h->opt.list_cap, q);
    if (hipMalloc(&g->dgeo, sizeof(SgGeo)) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc geo");
    hipMemcpy(g->dgeo, &g->geo, sizeof(SgGeo), hipMemcpyHostToDevice);
    if (hipMalloc(&g->dfail, sizeof(int32_t)) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc fail");
    h->state = g;
    h->state_kind = 2;
  }
  return (GeneralState*)h->state;
}

static uint32_t general_key_bound(SgHandle* h, const BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  uint32_t kb = 1;
  if (d.partitioned) {
    kb = bv.key_bound > 0 ? (uint32_t)bv.key_bound : 0;
    if (kb == 0) {
      int32_t* dmax = (int32_t*)h->ws.get("kmax", sizeof(int32_t), st);
      size_t tb = 0;
      HIPCHK(rocprim::reduce(nullptr, tb, bv.key, dmax, (int32_t)-1, (size_t)n, rocprim::maximum<int32_t>(), st));
      void* tmp = h->ws.get("kmax_tmp", tb, st);
      HIPCHK(rocprim::reduce(tmp, tb, bv.key, dmax, (int32_t)-1, (size_t)n, rocprim::maximum<int32_t>(), st));
      int32_t hm = 0;
      HIPCHK(hipMemcpyAsync(&hm, dmax, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      kb = (uint32_t)(hm + 1);
    }
  }
  if (kb < h->key_bound_seen) kb = h->key_bound_seen;
  h->key_bound_seen = kb;
  return kb;
}

static void run_machine(SgHandle* h, const BatchView& bv, int64_t n);

// rows [lo, lo + cnt) of a device batch view
BatchView sg_slice_view(const sg_nfa_desc& d, const BatchView& bv, int64_t lo, int64_t cnt) {
  if (lo == 0 && cnt == bv.n) return bv;
  BatchView v = bv;
  v.n = cnt;
  v.base_index = bv.base_index + (uint64_t)lo;
  v.ts = bv.ts + lo;
  if (bv.stream) v.stream = bv.stream + lo;
  if (bv.key) v.key = bv.key + lo;
  if (bv.index) v.index = bv.index + lo;
  for (int c = 0; c < d.n_cols; ++c) {
    if (bv.cols.col[c]) v.cols.col[c] = (const char*)bv.cols.col[c] + (size_t)sg_col_width(d.col_type[c]) * lo;
    if (bv.cols.nul[c]) v.cols.nul[c] = bv.cols.nul[c] + lo;
  }
  return v;
}

void sg_run_general(SgHandle* h, const BatchView& bv, int64_t n) {
  GeneralState* gs = gstate(h);
  if (!gs->pp_checked) {
    gs->pp = sg_partial_new(h->desc);
    gs->pp_checked = 1;
  }
  if (gs->pp && sg_partial_active(gs->pp) && h->opt.partial_lanes >= 0) {
    const uint32_t kb = general_key_bound(h, bv, n);
    // a push larger than the route's row budget runs as consecutive sub-pushes (carried state makes them one push)
    int64_t lo = 0;
    while (lo < n) {
      const int64_t room = sg_partial_max_rows(h, gs->pp);
      if (room < 1) throw SgError(SG_ECAPACITY, "partial-lane route: carried rows alone exceed the row budget");
      const int64_t cnt = std::min(n - lo, room);
      if (!sg_partial_push(h, gs->pp, sg_slice_view(h->desc, bv, lo, cnt), cnt, kb)) break;
      lo += cnt;
    }
    if (lo == n) return;
    // the route declined a push before anything was carried (sg_partial_push, seq_lanes_push): the per-key machine
    // takes the stream from here, exactly
    if (sg_partial_carried(gs->pp)) throw SgError(SG_EUNSUPPORTED, "partial-lane route left with carried partials");
    sg_partial_deactivate(gs->pp);
    run_machine(h, sg_slice_view(h->desc, bv, lo, n - lo), n - lo);
    return;
  }
  run_machine(h, bv, n);
}

// Move every key's runtime into geometry ng (larger pools / lists / timer FIFOs).
static void regeo(SgHandle* h, GeneralState* gs, const SgGeo& ng) {
  hipStream_t st = h->stream;
  const SgGeo og = gs->geo;
  if (gs->arena && gs->keys_alloc > 0) {
    const size_t bytes = (size_t)gs->keys_alloc * (size_t)ng.key_words * 4;
    int32_t* na = nullptr;
    if (hipMalloc(&na, bytes) != hipSuccess)
      throw SgError(SG_ECAPACITY, "cannot allocate grown per-key NFA arenas (" + std::to_string(bytes >> 20) + " MiB)");
    HIPCHK(hipMemsetAsync(na, 0, bytes, st));
    hipLaunchKernelGGL(k_regeo, dim3((unsigned)std::min<int64_t>(gs->keys_alloc, 65535)), dim3(256), 0, st,
                       gs->keys_alloc, gs->arena, og, na, ng);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    hipFree(gs->arena);
    gs->arena = na;
  }
  gs->geo = ng;
  HIPCHK(hipMemcpy(gs->dgeo, &gs->geo, sizeof(SgGeo), hipMemcpyHostToDevice));
}

// the next geometry when a key's pools, lists or timer FIFOs ran out: 4x each (as far as int32 indices allow)
static bool grown_geo(const sg_nfa_desc& d, const SgGeo& g, SgGeo& ng) {
  const int64_t lim = (int64_t)1 << 22;
  if ((int64_t)g.P * 4 > lim && (int64_t)g.L * 4 > lim) return false;
  auto up = [&](int32_t x) { return (int32_t)std::min<int64_t>(lim, std::max<int64_t>(4, (int64_t)x * 4)); };
  ng = sg_make_geo(d, up(g.P), up(g.E), up(g.C), up(g.L), up(g.Q));
  return ng.key_words < ((int64_t)1 << 31);
}

static void run_machine(SgHandle* h, const BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  GeneralState* gs = gstate(h);
  bool has_absent = gs->geo.A > 0;
  const uint32_t kb = general_key_bound(h, bv, n);
  // ---- grow arenas (new ones zeroed: runtime not created yet)
  if ((int64_t)kb > gs->keys_alloc) {
    int64_t nk = std::max<int64_t>((int64_t)kb, gs->keys_alloc * 3 / 2);
    size_t bytes = (size_t)nk * (size_t)gs->geo.key_words * 4;
    int32_t* na = nullptr;
    if (hipMalloc(&na, bytes) != hipSuccess)
      throw SgError(SG_ECAPACITY, "cannot allocate per-key NFA arenas (" + std::to_string(bytes >> 20) + " MiB)");
    HIPCHK(hipMemsetAsync(na, 0, bytes, st));
    if (gs->arena) {
      HIPCHK(hipMemcpyAsync(na, gs->arena, (size_t)gs->keys_alloc * gs->geo.key_words * 4, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
      hipFree(gs->arena);
    }
    gs->arena = na;
    gs->keys_alloc = nk;
  }
  int kbits = 1;
  while ((1ull << kbits) <= (uint64_t)kb) ++kbits;
  uint32_t sentinel = kb;
  int end_bit = 1;
  while ((1ull << end_bit) <= (uint64_t)sentinel) ++end_bit;
  dim3 blk(256), grd((unsigned)((n + 255) / 256));
  // ---- route + partition
  uint32_t* keys = (uint32_t*)h->ws.get("g_keys", sizeof(uint32_t) * n, st);
  uint32_t* rows = (uint32_t*)h->ws.get("g_rows", sizeof(uint32_t) * n, st);
  uint32_t* skeys = (uint32_t*)h->ws.get("g_skeys", sizeof(uint32_t) * n, st);
  uint32_t* srows = (uint32_t*)h->ws.get("g_srows", sizeof(uint32_t) * n, st);
  int32_t* order_err = (int32_t*)h->ws.get("order_err", sizeof(int32_t), st);
  HIPCHK(hipMemsetAsync(order_err, 0, sizeof(int32_t), st));
  h->mark(0);
  h->kbeg("route");
  const SgChunkRule rule = sg_chunk_rule(d);
  hipLaunchKernelGGL(k_route, grd, blk, 0, st, n, bv.stream, bv.key, bv.ts, h->ddesc, d.partitioned, sentinel,
                     (has_absent || rule.kind == 1) ? 1 : 0, keys, rows, order_err);
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(1);
  h->kbeg("key_sort");
  {
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, keys, skeys, rows, srows, (size_t)n, 0, end_bit, st));
    void* tmp = h->ws.get("g_sort_tmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, keys, skeys, rows, srows, (size_t)n, 0, end_bit, st));
  }
  uint32_t* beg = (uint32_t*)h->ws.get("g_beg", sizeof(uint32_t) * kb, st);
  uint32_t* end = (uint32_t*)h->ws.get("g_end", sizeof(uint32_t) * kb, st);
  HIPCHK(hipMemsetAsync(beg, 0, sizeof(uint32_t) * kb, st));
  HIPCHK(hipMemsetAsync(end, 0, sizeof(uint32_t) * kb, st));
  hipLaunchKernelGGL(k_segments, grd, blk, 0, st, n, skeys, sentinel, beg, end);
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(2);
  // ---- per-key machines
  int32_t stride = sg_emit_stride(d.n_select);
  int64_t cap = n + 65536;
  char* ebuf = nullptr;
  unsigned long long* ecount = (unsigned long long*)h->ws.get("g_ecount", 16, st);
  int32_t* eover = (int32_t*)h->ws.get("g_eover", 4, st);
  int32_t oerr = 0;
  int64_t tfl[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(&oerr, order_err, 4, hipMemcpyDeviceToHost, st));
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(&tfl[0], bv.ts, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&tfl[1], bv.ts + (n - 1), 8, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  if (oerr & 2) throw SgError(SG_EINVAL, "a partition key id is >= the batch's key_bound");
  // time-horizon units rebuild a key's state from the rows inside `within` before them: only sound while timestamps
  // never decrease, within this push and after the earlier ones
  const bool ts_monotone = !(oerr & 1) && (n == 0 || tfl[0] >= gs->max_ts);
  if (n > 0) gs->max_ts = std::max(gs->max_ts, ts_monotone ? tfl[1] : std::max(tfl[0], tfl[1]));
  if (!ts_monotone) gs->max_ts = INT64_MAX;   // from now on the order of the stream is unknown
  int64_t next_clock = gs->clock;
  NfaArgs na;
  na.n = n;
  na.base_index = bv.base_index;
  na.nkeys = kb;
  na.partitioned = d.partitioned;
  na.clone = d.partitioned;
  na.rows = srows;
  na.beg = beg;
  na.end = end;
  na.ts = bv.ts;
  na.stream = bv.stream;
  na.index = bv.index;
  na.clk = nullptr;
  na.nfr = nullptr;
  na.clock0 = gs->clock;
  if (has_absent && n > 0) {
    // absence timers fire on the playback clock, which a row whose time goes back leaves where it is
    int64_t* clk = (int64_t*)h->ws.get("g_clk", sizeof(int64_t) * n, st);
    uint32_t* rev = (uint32_t*)h->ws.get("g_fire_rev", sizeof(uint32_t) * n, st);
    uint32_t* nfr = (uint32_t*)h->ws.get("g_fire_next", sizeof(uint32_t) * n, st);
    size_t tb = 0;
    HIPCHK(rocprim::inclusive_scan(nullptr, tb, bv.ts, clk, (size_t)n, rocprim::maximum<int64_t>(), st));
    void* tmp = h->ws.get("g_clk_tmp", tb, st);
    HIPCHK(rocprim::inclusive_scan(tmp, tb, bv.ts, clk, (size_t)n, rocprim::maximum<int64_t>(), st));
    hipLaunchKernelGGL(k_fire_rev, grd, blk, 0, st, n, bv.ts, clk, gs->clock, rev);
    HIPCHK(hipGetLastError());
    tb = 0;
    HIPCHK(rocprim::inclusive_scan(nullptr, tb, rev, nfr, (size_t)n, rocprim::minimum<uint32_t>(), st));
    tmp = h->ws.get("g_nfr_tmp", tb, st);
    HIPCHK(rocprim::inclusive_scan(tmp, tb, rev, nfr, (size_t)n, rocprim::minimum<uint32_t>(), st));
    int64_t last = 0;
    HIPCHK(hipMemcpyAsync(&last, clk + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    na.clk = clk;
    na.nfr = nfr;
    next_clock = std::max(gs->clock, last);
  }
  // ---- predicate-evaluation pass: condition bits of every state whose filter reads only the arriving event
  for (int s = 0; s < SG_MAX_STATES; ++s) na.lbits[s] = nullptr;
  {
    const int64_t ntiles = (n + 255) / 256;
    bool any = false;
    for (int s = 0; s < d.n_states; ++s) {
      const sg_state_desc& x = d.states[s];
      if (!x.local || x.prog_len <= 0) continue;
      if (!any) h->kbeg("pred");
      any = true;
      PredArgs pa;
      memset(&pa, 0, sizeof(pa));
      pa.n = n;
      pa.stream = bv.stream;
      pa.s_a = x.stream;
      pa.prog_a_off = x.prog_off;
      pa.prog_a_len = x.prog_len;
      pa.val_col_a = -1;
      pa.val_col_b = -1;
      pa.cons_all = 1;
      uint64_t* bits = (uint64_t*)h->ws.get("g_lbits" + std::to_string(s), sizeof(uint64_t) * 4 * (ntiles + 1), st);
      launch_pred(d, pa, bv.stream, bv.cols, h->ddesc, bits, nullptr, st);
      HIPCHK(hipGetLastError());
      na.lbits[s] = bits;
    }
    if (any) h->kend();
  }
  // The reference's lists are unbounded (StreamPreStateProcessor.java:58-59): a push that runs out of a key's pool,
  // list or timer capacity, or out of emission space, is rolled back and rerun with 4x the capacity.
  unsigned long long total = 0;
  for (int attempt = 0;; ++attempt) {
  const size_t pre_bytes = (size_t)kb * (size_t)gs->geo.key_words * 4;
  int32_t* pre = (int32_t*)h->ws.get("g_pre", std::max<size_t>(pre_bytes, 4), st);
  if (pre_bytes) HIPCHK(hipMemcpyAsync(pre, gs->arena, pre_bytes, hipMemcpyDeviceToDevice, st));
  ebuf = (char*)h->ws.get("g_emit", (size_t)cap * stride, st);
  HIPCHK(hipMemsetAsync(ecount, 0, 8, st));
  HIPCHK(hipMemsetAsync(eover, 0, 4, st));
  HIPCHK(hipMemsetAsync(gs->dfail, 0, 4, st));
  SgEmitSink sink;
  sink.buf = ebuf;
  sink.cap = cap;
  sink.count = ecount;
  sink.overflow = eover;
  sink.stride = stride;
  sink.key_bits = kbits;
  // ---- unit plan: one unit per key, or (chunkable shapes) per (key, chunk of R rows)
  uint32_t R = 0;
  // A time-horizon unit's runtime is rebuilt from the rows inside `within` before its chunk, so it lacks the partials
  // parked in a count state since before that horizon: they never expire (CountPreStateProcessor.processAndReturn,
  // C/query/input/stream/state/CountPreStateProcessor.java:53-93) and a later push whose time goes back can complete
  // them -- queries with a count state are cut only by the sequence's event horizon
  const bool count_q = has_count_state(d);
  if (rule.kind != 0 && (rule.kind == 2 || (ts_monotone && !count_q)) && h->opt.chunk_rows >= 0 && n > 0) {
    if (h->opt.chunk_rows > 0) {
      R = (uint32_t)h->opt.chunk_rows;
    } else {
      // horizon rows per unit (rows of an average key inside `within`, or the sequence's event horizon);
      // units at least 4x their horizon, enough of them to fill the chip, scratch arenas within budget
      const int64_t span = std::max<int64_t>(1, tfl[1] - tfl[0]);
      const double per_key = (double)n / (double)std::max<uint32_t>(kb, 1);
      const double hz = rule.kind == 2 ? (double)rule.events : per_key * (double)rule.within / (double)span;
      // (measured on C3b/C3c: 131k -> 524k units took 372 -> 245 ms and 3150 -> 2347 ms per 100M events;
      // 1M units gained nothing more)
      const int64_t target_units = 256 * 32 * 64;
      const int64_t mem_units = std::max<int64_t>(1, ((int64_t)24 << 30) / ((int64_t)gs->geo.key_words * 4));
      int64_t r = std::max<int64_t>({(int64_t)(4.0 * hz) + 1, 32, (n + target_units - 1) / target_units,
                                     (n + mem_units - 1) / mem_units});
      R = (uint32_t)std::min<int64_t>(r, 1 << 30);
      if ((double)R >= per_key * 2.0) R = 0;   // hardly any key would be cut
    }
  }
  if (R > 0) {
    uint32_t* nch = (uint32_t*)h->ws.get("g_nch", sizeof(uint32_t) * (kb + 1), st);
    uint32_t* uoff = (uint32_t*)h->ws.get("g_uoff", sizeof(uint32_t) * (kb + 1), st);
    hipLaunchKernelGGL(k_unit_count, dim3((unsigned)((kb + 1 + 255) / 256)), blk, 0, st, (int64_t)kb, beg, end, R, nch);
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, nch, uoff, (uint32_t)0, (size_t)kb + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("g_uscan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, nch, uoff, (uint32_t)0, (size_t)kb + 1, rocprim::plus<uint32_t>(), st));
    uint32_t U = 0;
    HIPCHK(hipMemcpyAsync(&U, uoff + kb, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const size_t kw = (size_t)gs->geo.key_words;
    UnitArgs ua;
    ua.R = R;
    ua.rule = rule;
    ua.n_units = U;
    ua.uoff = uoff;
    uint32_t* umap = (uint32_t*)h->ws.get("g_umap", sizeof(uint32_t) * std::max<uint32_t>(U, 1), st);
    ua.umap = umap;
    ua.scratch = (int32_t*)h->ws.get("g_uarena", sizeof(int32_t) * kw * std::max<uint32_t>(U, 1), st);
    int32_t* snap = (int32_t*)h->ws.get("g_snap", sizeof(int32_t) * kw * kb, st);
    HIPCHK(hipMemcpyAsync(snap, gs->arena, sizeof(int32_t) * kw * kb, hipMemcpyDeviceToDevice, st));
    ua.snap = snap;
    hipLaunchKernelGGL(k_unit_map, dim3((unsigned)((kb + 255) / 256)), blk, 0, st, (int64_t)kb, uoff, umap);
    h->kbeg("nfa_units");
    if (U)
      hipLaunchKernelGGL(k_nfa_units, dim3((unsigned)((U + 63) / 64)), dim3(64), 0, st, na, ua, bv.cols, h->ddesc,
                         gs->dgeo, gs->arena, sink, gs->dfail);
    h->kend();
    hipLaunchKernelGGL(k_unit_keep, dim3((unsigned)std::min<uint32_t>(std::max<uint32_t>(kb, 1), 65535)), blk, 0, st,
                       (int64_t)kb, uoff, ua.scratch, gs->dgeo, gs->arena);
  } else {
    h->kbeg("nfa_keys");
    hipLaunchKernelGGL(k_nfa, dim3((unsigned)((kb + 63) / 64)), dim3(64), 0, st, na, bv.cols, h->ddesc, gs->dgeo,
                       gs->arena, sink, gs->dfail);
    h->kend();
  }
  HIPCHK(hipGetLastError());
  h->mark(3);
  total = 0;
  int32_t over = 0, fcode = 0;
  HIPCHK(hipMemcpyAsync(&total, ecount, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&over, eover, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&fcode, gs->dfail, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  SgGeo ng;
  const bool grow_pools = fcode == SG_ECAPACITY && !h->opt.no_grow && grown_geo(d, gs->geo, ng);
  const bool grow_emit = over && !fcode && !h->opt.no_grow && cap < ((int64_t)1 << 31);
  if ((grow_pools || grow_emit) && attempt < 8) {
    if (pre_bytes) HIPCHK(hipMemcpyAsync(gs->arena, pre, pre_bytes, hipMemcpyDeviceToDevice, st));   // roll back
    if (grow_pools) regeo(h, gs, ng);
    if (grow_emit) cap = std::min<int64_t>((int64_t)1 << 31, cap * 4);
    ++gs->grows;
    continue;
  }
  if (fcode) throw SgError(fcode, fcode == SG_ECAPACITY
                                      ? "per-key pool/list capacity exceeded (raise sg_options pool_* / list_cap)"
                                      : "query shape hits a reference failure path (see DESIGN.md)");
  if (over) throw SgError(SG_ECAPACITY, "match buffer overflow: push smaller batches");
  break;
  }
  // ---- order matches by (trigger, timer-before-event, key) keeping per-key emission order
  if (total) {
    uint64_t* sk = (uint64_t*)h->ws.get("g_sk", 8 * total, st);
    uint64_t* sk2 = (uint64_t*)h->ws.get("g_sk2", 8 * total, st);
    uint32_t* ix = (uint32_t*)h->ws.get("g_ix", 4 * total, st);
    uint32_t* ix2 = (uint32_t*)h->ws.get("g_ix2", 4 * total, st);
    dim3 g2((unsigned)((total + 255) / 256));
    h->kbeg("match_order");
    hipLaunchKernelGGL(k_sortkeys, g2, blk, 0, st, (int64_t)total, ebuf, stride, sk, ix);
    HIPCHK(hipGetLastError());
    int sbits = 31 + 1 + kbits;
    if (sbits > 64) sbits = 64;
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, sk, sk2, ix, ix2, (size_t)total, 0, sbits, st));
    void* tmp = h->ws.get("g_sort2_tmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, sk, sk2, ix, ix2, (size_t)total, 0, sbits, st));
    char* out = h->out.reserve((int64_t)total, d.n_select, st);
    int32_t ostride = 32 + 8 * d.n_select;
    hipLaunchKernelGGL(k_gather, g2, blk, 0, st, (int64_t)total, ebuf, stride, ix2, out + (size_t)h->out.n * ostride,
                       ostride);
    HIPCHK(hipGetLastError());
    h->kend();
    h->out.n += (int64_t)total;
  }
  h->mark(4);
  gs->clock = next_clock;
  h->last_events = n;
  h->last_spilled = 0;
  h->last_matches = (int64_t)total;
}

void sg_general_reset(SgHandle* h) {
  if (!h->state || h->state_kind != 2) return;
  GeneralState* gs = (GeneralState*)h->state;
  if (gs->arena) hipMemset(gs->arena, 0, (size_t)gs->keys_alloc * gs->geo.key_words * 4);
  sg_partial_reset(gs->pp);
  gs->max_ts = INT64_MIN;
  gs->clock = 0;
  h->key_bound_seen = 0;
}

void sg_general_release(SgHandle* h) {
  if (!h->state || h->state_kind != 2) return;
  GeneralState* gs = (GeneralState*)h->state;
  if (gs->arena) hipFree(gs->arena);
  if (gs->dgeo) hipFree(gs->dgeo);
  if (gs->dfail) hipFree(gs->dfail);
  sg_partial_free(gs->pp);
  delete gs;
  h->state = nullptr;
  h->state_kind = 0;
}

// Snapshot of the general machine: the per-key runtimes (pending / newAndEvery lists, partial, event-copy
// and chain pools, timer FIFOs) of the keys seen so far, i.e. what StreamPreStateProcessor.currentState,
// CountPreStateProcessor, LogicalPreStateProcessor and Scheduler.currentState persist per partition clone
// (C/query/input/stream/state/StreamPreStateProcessor.java:352-359, C/util/Scheduler.java:147-160,
// C/partition/PartitionRuntime.java:342-356).  The arena geometry must match on restore.
void sg_general_snapshot(SgHandle* h, SnapW& w) {
  GeneralState* gs = (h->state && h->state_kind == 2) ? (GeneralState*)h->state : nullptr;
  const int32_t route = (gs && gs->pp && sg_partial_active(gs->pp) && h->opt.partial_lanes >= 0) ? 1 : 0;   // 1: partial lanes' carried rows
  w.pod(route);
  w.pod(gs ? gs->max_ts : (int64_t)INT64_MIN);
  if (route) {
    sg_partial_snapshot(h, gs->pp, w);
    return;
  }
  const int64_t keys = gs ? std::min<int64_t>(gs->keys_alloc, (int64_t)h->key_bound_seen) : 0;
  w.pod(keys);
  if (!keys) return;
  w.pod(gs->geo);
  w.dev(gs->arena, (size_t)keys * gs->geo.key_words * 4, h->stream);
}

void sg_general_restore(SgHandle* h, SnapR& r) {
  GeneralState* gs = gstate(h);
  hipStream_t st = h->stream;
  if (!gs->pp_checked) {
    gs->pp = sg_partial_new(h->desc);
    gs->pp_checked = 1;
  }
  const int32_t route = r.pod<int32_t>();
  const int64_t max_ts = r.pod<int64_t>();
  if (route != 0 && route != 1) throw SgError(SG_EINVAL, "snapshot: bad general-route marker");
  if (route == 1) {
    if (!gs->pp || h->opt.partial_lanes < 0) throw SgError(SG_EINVAL, "snapshot: taken on the partial-lane route");
    sg_partial_restore(h, gs->pp, r);
    gs->max_ts = max_ts;
      // the machine's per-key runtimes from before the restore (a fallback taken earlier) are stale: a later fallback
    // rebuilds them from the restored carried rows alone
    if (gs->arena) HIPCHK(hipMemsetAsync(gs->arena, 0, (size_t)gs->keys_alloc * gs->geo.key_words * 4, st));
    HIPCHK(hipStreamSynchronize(st));
    return;
  }
  if (gs->pp) sg_partial_deactivate(gs->pp);
  gs->max_ts = max_ts;
  const int64_t keys = r.pod<int64_t>();
  if (keys < 0 || keys > (1ll << 31)) throw SgError(SG_EINVAL, "snapshot: bad key count");
  if (gs->arena) HIPCHK(hipMemsetAsync(gs->arena, 0, (size_t)gs->keys_alloc * gs->geo.key_words * 4, st));
  if (!keys) {
    HIPCHK(hipStreamSynchronize(st));
    return;
  }
  SgGeo g = r.pod<SgGeo>();
  const SgGeo& m = gs->geo;
  if (g.S != m.S || g.R != m.R || g.A != m.A || g.nsel != m.nsel)
    throw SgError(SG_EINVAL, "snapshot: per-key arena geometry differs (another query)");
  const SgGeo want = sg_make_geo(h->desc, g.P, g.E, g.C, g.L, g.Q);
  if (want.key_words != g.key_words) throw SgError(SG_EINVAL, "snapshot: inconsistent arena geometry");
  if (g.key_words != m.key_words || g.P != m.P || g.E != m.E || g.C != m.C || g.L != m.L || g.Q != m.Q) {
    // the snapshot's runtimes had grown (or this handle's have): adopt the snapshot's geometry
    HIPCHK(hipStreamSynchronize(st));
    if (gs->arena) hipFree(gs->arena);
    gs->arena = nullptr;
    gs->keys_alloc = 0;
    gs->geo = g;
    HIPCHK(hipMemcpy(gs->dgeo, &gs->geo, sizeof(SgGeo), hipMemcpyHostToDevice));
  }
  if (keys > gs->keys_alloc) {
    size_t bytes = (size_t)keys * (size_t)gs->geo.key_words * 4;
    int32_t* na = nullptr;
    if (hipMalloc(&na, bytes) != hipSuccess)
      throw SgError(SG_ECAPACITY, "cannot allocate per-key NFA arenas (" + std::to_string(bytes >> 20) + " MiB)");
    if (gs->arena) {
      HIPCHK(hipStreamSynchronize(st));
      hipFree(gs->arena);
    }
    gs->arena = na;
    gs->keys_alloc = keys;
  }
  r.dev(gs->arena, (size_t)keys * gs->geo.key_words * 4, st);
}
