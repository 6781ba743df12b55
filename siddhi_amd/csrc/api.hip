// C-ABI entry points of libsiddhi_gpu.so (declared in include/siddhi_gpu.h).
#include <cstring>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "sg_engine.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct sg_handle {
  SgHandle h;
};

int sg_col_width(int type) { return (type == SG_T_LONG || type == SG_T_DOUBLE) ? 8 : 4; }
static int out_cols(const sg_nfa_desc& d) { return d.n_out > 0 ? d.n_out : d.n_select; }

// ---- select expressions (QuerySelector.processNoGroupBy over math executors,
// C/query/selector/QuerySelector.java:125-163; SelectorParser.java:199-233): the engines project the matched
// slots the expressions read (n_select base values per record); this pass evaluates each output column's
// postfix program over them, one record per lane, in delivery order.
struct SelReader {
  const int64_t* vals;
  uint32_t vnull;
  __device__ SgVal read(int, int, int slot, int type) { return sg_val_from_bits(vals[slot], type, (vnull >> slot) & 1); }
};

// keep (optional): 1 if the match survives `having`, for the compaction that follows.
__global__ void k_select(int64_t n, const char* __restrict__ src, int sstride, char* __restrict__ dst, int dstride,
                         const DevDesc* __restrict__ d, uint32_t* __restrict__ keep) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* r = src + (size_t)i * sstride;
  char* o = dst + (size_t)i * dstride;
  SelReader rd;
  rd.vals = (const int64_t*)(r + 32);
  rd.vnull = *(const uint32_t*)(r + 24);
  ((uint64_t*)o)[0] = ((const uint64_t*)r)[0];   // trigger
  ((uint64_t*)o)[1] = ((const uint64_t*)r)[1];   // ts
  ((uint64_t*)o)[2] = ((const uint64_t*)r)[2];   // key, group
  uint32_t vn = 0;
  const int nout = d->n_out;
  int64_t* ov = (int64_t*)(o + 32);
  for (int k = 0; k < nout; ++k) {
    SgVal top;
    if (!sg_run(d->code + d->out_off[k], d->out_len[k], rd, top)) top.null = 1;
    if (top.null) vn |= 1u << k;
    ov[k] = sg_val_bits(top);
  }
  ((uint32_t*)o)[6] = vn;
  ((uint32_t*)o)[7] = 0;
  if (keep) {
    SelReader hr;
    hr.vals = ov;
    hr.vnull = vn;
    keep[i] = sg_eval(d->code + d->having_off, d->having_len, hr) ? 1u : 0u;
  }
}

// Stable compaction of the surviving matches (delivery order kept).
__global__ void k_having_scatter(int64_t n, const char* __restrict__ src, const uint32_t* __restrict__ keep,
                                 const uint32_t* __restrict__ pos, int stride, char* __restrict__ dst) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !keep[i]) return;
  const uint64_t* s = (const uint64_t*)(src + (size_t)i * stride);
  uint64_t* t = (uint64_t*)(dst + (size_t)pos[i] * stride);
  for (int w = 0; w < stride / 8; ++w) t[w] = s[w];
}

// Engines append base records to h.stage (swapped in for the push); the select pass appends the output
// records (those passing `having`) to h.out.
static void run_select(SgHandle& h) {
  const sg_nfa_desc& d = h.desc;
  hipStream_t st = h.stream;
  const int64_t n = h.stage.n;
  const int ostride = 32 + 8 * d.n_out;
  const dim3 grd((unsigned)((n + 255) / 256)), blk(256);
  if (n > 0 && d.having_len <= 0) {
    char* out = h.out.reserve(n, d.n_out, st);
    hipLaunchKernelGGL(k_select, grd, blk, 0, st, n, (const char*)h.stage.rec, 32 + 8 * d.n_select,
                       out + (size_t)h.out.n * ostride, ostride, h.ddesc, (uint32_t*)nullptr);
    HIPCHK(hipGetLastError());
    h.out.n += n;
  } else if (n > 0) {
    char* tmp = (char*)h.ws.get("having_rec", (size_t)n * ostride, st);
    uint32_t* keep = (uint32_t*)h.ws.get("having_keep", 4 * (size_t)(n + 1), st);
    uint32_t* pos = (uint32_t*)h.ws.get("having_pos", 4 * (size_t)(n + 1), st);
    HIPCHK(hipMemsetAsync(keep + n, 0, 4, st));
    hipLaunchKernelGGL(k_select, grd, blk, 0, st, n, (const char*)h.stage.rec, 32 + 8 * d.n_select, tmp, ostride,
                       h.ddesc, keep);
    HIPCHK(hipGetLastError());
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, keep, pos, 0u, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    void* tsc = h.ws.get("having_scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tsc, tb, keep, pos, 0u, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    uint32_t kept = 0;
    HIPCHK(hipMemcpyAsync(&kept, pos + n, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (kept) {
      char* out = h.out.reserve(kept, d.n_out, st);
      hipLaunchKernelGGL(k_having_scatter, grd, blk, 0, st, n, (const char*)tmp, keep, pos, ostride,
                         out + (size_t)h.out.n * ostride);
      HIPCHK(hipGetLastError());
      h.out.n += kept;
    }
  }
  h.stage.n = 0;
}

template <class F>
static int guard(sg_handle* hh, F&& f) {
  try {
    f();
    return SG_OK;
  } catch (SgError& e) {
    if (hh) hh->h.err = e.msg;
    return e.code;
  } catch (std::exception& e) {
    if (hh) hh->h.err = e.what();
    return SG_EINVAL;
  }
}

static void validate(const sg_nfa_desc* d) {
  if (d->abi_version != SG_ABI_VERSION) throw SgError(SG_EINVAL, "sg_nfa_desc ABI version mismatch");
  if (d->n_states < 1 || d->n_states > SG_MAX_STATES) throw SgError(SG_EINVAL, "bad n_states");
  if (d->n_streams < 1 || d->n_streams > SG_MAX_STREAMS) throw SgError(SG_EINVAL, "bad n_streams");
  if (d->n_cols < 0 || d->n_cols > SG_MAX_COLS) throw SgError(SG_EINVAL, "bad n_cols");
  if (d->n_ret < 0 || d->n_ret > SG_MAX_RET) throw SgError(SG_EINVAL, "bad n_ret");
  if (d->n_select < 0 || d->n_select > SG_MAX_SELECT) throw SgError(SG_EINVAL, "bad n_select");
  if (d->code_len < 0 || d->code_len > SG_MAX_CODE) throw SgError(SG_EINVAL, "bad code_len");
  if (d->n_out < 0 || d->n_out > SG_MAX_SELECT) throw SgError(SG_EINVAL, "bad n_out");
  if (d->having_len > 0 && (d->n_out <= 0 || d->having_off < 0 || d->having_off + d->having_len > d->code_len))
    throw SgError(SG_EINVAL, "bad having program");
  for (int k = 0; k < d->n_out; ++k)
    if (d->out_off[k] < 0 || d->out_len[k] < 1 || d->out_off[k] + d->out_len[k] > d->code_len)
      throw SgError(SG_EINVAL, "bad select program range");
  for (int s = 0; s < d->n_states; ++s) {
    const sg_state_desc& st = d->states[s];
    if (st.stream < 0 || st.stream >= d->n_streams) throw SgError(SG_EINVAL, "state stream out of range");
    if (st.prog_off < 0 || st.prog_off + st.prog_len > d->code_len) throw SgError(SG_EINVAL, "bad program range");
  }
  for (int r = 0; r < d->n_ret; ++r)
    if (d->ret_col[r] < 0 || d->ret_col[r] >= d->n_cols) throw SgError(SG_EINVAL, "retained column out of range");
  int timed = 0;
  for (int s = 0; s < d->n_states; ++s) timed += (d->states[s].kind == SG_K_ABSENT || d->states[s].kind == SG_K_ALOGICAL);
  if (d->n_sched != timed) throw SgError(SG_EINVAL, "sched_state must list every absent state once");
  for (int k = 0; k < d->n_sched; ++k) {
    const int s = d->sched_state[k];
    if (s < 0 || s >= d->n_states || (d->states[s].kind != SG_K_ABSENT && d->states[s].kind != SG_K_ALOGICAL))
      throw SgError(SG_EINVAL, "bad sched_state entry");
    for (int j = 0; j < k; ++j) if (d->sched_state[j] == s) throw SgError(SG_EINVAL, "duplicate sched_state entry");
  }
}

// One push of rows already in HBM: the engine route, then the select pass.
void sg_push_view(SgHandle& h, BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h.desc;
  for (int r = 0; r < d.n_ret; ++r)
    if (!bv.cols.col[d.ret_col[r]]) throw SgError(SG_EINVAL, "batch is missing a column the query reads");
  int shape = h.opt.force_general ? SG_SHAPE_GENERAL : d.shape;
  const bool sel = d.n_out > 0;
  h.bump_gen();   // the state changes from here on (a failed push leaves no valid snapshot cache either)
  h.n_km = 0;
  if (sel) std::swap(h.out, h.stage);   // engines append base records to the stage
  try {
    switch (shape) {
      case SG_SHAPE_EVERY_NEXT_CMP:
        sg_run_every_next(&h, bv, n);
        break;
      case SG_SHAPE_EVERY_ABSENT_EQ:
        sg_run_every_absent(&h, bv, n);
        break;
      case SG_SHAPE_NEXT_CMP_ONCE:
        sg_run_once(&h, bv, n);
        break;
      default:
        sg_run_general(&h, bv, n);
    }
  } catch (...) {
    if (sel) { std::swap(h.out, h.stage); h.stage.n = 0; }
    throw;
  }
  if (sel) {
    std::swap(h.out, h.stage);
    try {
      run_select(h);
    } catch (...) {
      h.stage.n = 0;   // base records of a failed select pass must not be delivered by the next push
      throw;
    }
  }
  h.pushes++;
}

static std::string slot_name(const char* what, int c, int slot) {
  char nm[48];
  snprintf(nm, sizeof nm, "in_%s%d#%d", what, c, slot);
  return nm;
}

SlotPtrs sg_reserve_slot(SgHandle& h, const sg_batch* b, int64_t rows, int slot) {
  const sg_nfa_desc& d = h.desc;
  SlotPtrs p;
  p.ts = h.ws.get(slot_name("ts", 0, slot), 8 * rows, h.stream);
  if (b->stream) p.stream = h.ws.get(slot_name("stream", 0, slot), 4 * rows, h.stream);
  if (b->key) p.key = h.ws.get(slot_name("key", 0, slot), 4 * rows, h.stream);
  if (b->index) p.index = h.ws.get(slot_name("index", 0, slot), 8 * rows, h.stream);
  for (int c = 0; c < d.n_cols; ++c) {
    if (b->cols && b->cols[c])
      p.col[c] = h.ws.get(slot_name("col", c, slot), (size_t)sg_col_width(d.col_type[c]) * rows, h.stream);
    if (b->nulls && b->nulls[c]) p.nul[c] = h.ws.get(slot_name("nul", c, slot), rows, h.stream);
  }
  return p;
}

// Copy rows [lo, lo + cnt) of a host batch into a slot on stream `st`; returns the device view.  Touches no
// handle state besides the descriptor, so it may run on a helper thread.
BatchView sg_upload_to(const sg_nfa_desc& d, const SlotPtrs& p, const sg_batch* b, int64_t lo, int64_t cnt,
                           hipStream_t st) {
  BatchView bv;
  bv.n = cnt;
  bv.base_index = b->base_index + (uint64_t)lo;
  bv.key_bound = b->key_bound;
  memset(&bv.cols, 0, sizeof(bv.cols));
  auto up = [&](void* dst, const void* src, size_t width) -> void* {
    if (!src) return nullptr;
    HIPCHK(hipMemcpyAsync(dst, (const char*)src + width * lo, width * cnt, hipMemcpyHostToDevice, st));
    return dst;
  };
  bv.ts = (const int64_t*)up(p.ts, b->ts, 8);
  bv.stream = (const int32_t*)up(p.stream, b->stream, 4);
  bv.key = (const int32_t*)up(p.key, b->key, 4);
  bv.index = (const uint64_t*)up(p.index, b->index, 8);
  for (int c = 0; c < d.n_cols; ++c) {
    bv.cols.col[c] = b->cols ? up(p.col[c], b->cols[c], (size_t)sg_col_width(d.col_type[c])) : nullptr;
    bv.cols.nul[c] = (const uint8_t*)(b->nulls ? up(p.nul[c], b->nulls[c], 1) : nullptr);
  }
  return bv;
}

static BatchView upload(SgHandle& h, const sg_batch* b, int64_t lo, int64_t cnt, int slot, hipStream_t st) {
  return sg_upload_to(h.desc, sg_reserve_slot(h, b, cnt, slot), b, lo, cnt, st);
}

struct ChunkHook {
  virtual void chunk_done() = 0;
  virtual ~ChunkHook() {}
};

static void check_batch(const sg_batch* b) {
  if (b->n >= (1ll << 30) - 1) throw SgError(SG_EINVAL, "batch too large (max 2^30-2 rows)");
  if (!b->ts) throw SgError(SG_EINVAL, "batch without timestamps");
}

static BatchView device_view(const sg_nfa_desc& d, const sg_batch* b) {
  BatchView bv;
  bv.n = b->n;
  bv.base_index = b->base_index;
  bv.key_bound = b->key_bound;
  bv.ts = b->ts;
  bv.stream = b->stream;
  bv.key = b->key;
  bv.index = b->index;
  memset(&bv.cols, 0, sizeof(bv.cols));
  for (int c = 0; c < d.n_cols; ++c) {
    bv.cols.col[c] = b->cols ? b->cols[c] : nullptr;
    bv.cols.nul[c] = b->nulls ? b->nulls[c] : nullptr;
  }
  return bv;
}

// ---- SoA match delivery (QuerySelector -> QueryCallback.receiveStreamEvent, C/query/output/callback/
// QueryCallback.java:52-85, as typed columns).  The pending AoS records are transposed on the GPU into a staging
// buffer of columns; the columns are copied to the caller on a D2H stream, double-buffered so one chunk's copy
// overlaps the next chunk's kernels.
ColLayout sg_col_layout(const sg_nfa_desc& d, int64_t cap) {
  ColLayout L;
  L.ns = out_cols(d);
  size_t o = 0;
  auto take = [&](size_t w) { size_t r = o; o += ((w * (size_t)cap + 255) / 256) * 256; return r; };
  L.off_trig = take(8);
  L.off_ts = take(8);
  L.off_key = take(4);
  L.off_grp = take(4);
  for (int k = 0; k < L.ns; ++k) {
    const int t = d.n_out > 0 ? d.out_type[k] : d.sel_type[k];
    L.width[k] = sg_col_width(t);
    L.off_col[k] = take((size_t)L.width[k]);
  }
  for (int k = 0; k < L.ns; ++k) L.off_nul[k] = take(1);
  L.bytes = o;
  return L;
}

// one thread per record: 16-B loads of the record, one coalesced store per column
__global__ void __launch_bounds__(256) k_to_columns(int64_t n, const char* __restrict__ rec, int stride, ColLayout L,
                                                    char* __restrict__ stage) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  typedef uint32_t U4 __attribute__((ext_vector_type(4)));
  const U4* r = (const U4*)(rec + (size_t)i * stride);
  const U4 h0 = r[0], h1 = r[1];   // trigger, ts | key, group, vnull, pad
  ((uint64_t*)(stage + L.off_trig))[i] = ((uint64_t)h0.y << 32) | h0.x;
  ((uint64_t*)(stage + L.off_ts))[i] = ((uint64_t)h0.w << 32) | h0.z;
  ((uint32_t*)(stage + L.off_key))[i] = h1.x;
  ((uint32_t*)(stage + L.off_grp))[i] = h1.y;
  const uint32_t vn = h1.z;
  const uint64_t* v = (const uint64_t*)(rec + (size_t)i * stride + 32);
  for (int k = 0; k < L.ns; ++k) {
    const uint64_t bits = v[k];
    if (L.width[k] == 8) ((uint64_t*)(stage + L.off_col[k]))[i] = bits;
    else ((uint32_t*)(stage + L.off_col[k]))[i] = (uint32_t)bits;
    ((uint8_t*)(stage + L.off_nul[k]))[i] = (uint8_t)((vn >> k) & 1u);
  }
}

void sg_launch_to_columns(int64_t n, const char* rec, int stride, const ColLayout& L, char* stage, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_to_columns, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, rec, stride, L, stage);
  HIPCHK(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_to_matches(int64_t n, const char* __restrict__ rec, int stride, int ns,
                                                    uint64_t* __restrict__ trig, int64_t* __restrict__ ts,
                                                    int32_t* __restrict__ key, uint32_t* __restrict__ grp,
                                                    int64_t* __restrict__ vals, uint32_t* __restrict__ vn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* r = rec + (size_t)i * stride;
  trig[i] = *(const uint64_t*)r;
  ts[i] = *(const int64_t*)(r + 8);
  key[i] = *(const int32_t*)(r + 16);
  grp[i] = *(const uint32_t*)(r + 20);
  vn[i] = *(const uint32_t*)(r + 24);
  for (int k = 0; k < ns; ++k) vals[(size_t)i * ns + k] = ((const int64_t*)(r + 32))[k];
}

void sg_egress_init(SgHandle& h) {
  if (h.eg.d2h) return;
  HIPCHK(hipStreamCreateWithFlags(&h.eg.d2h, hipStreamNonBlocking));
  for (int k = 0; k < 2; ++k) {
    HIPCHK(hipEventCreateWithFlags(&h.eg.ready[k], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&h.eg.done[k], hipEventDisableTiming));
    HIPCHK(hipEventRecord(h.eg.done[k], h.eg.d2h));
  }
}

// Staging slot `slot` holds at least `bytes` (grown only after its last copy has read it: hipFree synchronises the
// device, so sg_push_deliver sizes both slots before its chunk pipeline starts).
void sg_stage_reserve(SgHandle& h, int slot, int64_t bytes) {
  if (h.eg.cap[slot] >= bytes) return;
  HIPCHK(hipEventSynchronize(h.eg.done[slot]));
  if (h.eg.stage[slot]) HIPCHK(hipFree(h.eg.stage[slot]));
  h.eg.stage[slot] = nullptr;
  const size_t want = (size_t)bytes + (size_t)bytes / 4;
  HIPCHK(hipMalloc(&h.eg.stage[slot], want));
  h.eg.cap[slot] = (int64_t)want;
}

// Deliver up to `cap` pending matches into out (rows [row0, row0 + k)) through staging slot `slot`; returns k.
// The copies are left in flight on the D2H stream (the caller synchronises it before returning to its caller).
static int64_t deliver_pending(SgHandle& h, const sg_match_columns* out, int64_t row0, int64_t cap, int slot) {
  OutStore& o = h.out;
  const int64_t k = std::min<int64_t>(cap, o.n);
  if (k <= 0) return 0;
  sg_egress_init(h);
  const sg_nfa_desc& d = h.desc;
  const ColLayout L = sg_col_layout(d, k);
  sg_stage_reserve(h, slot, (int64_t)L.bytes);
  char* st = h.eg.stage[slot];
  HIPCHK(hipStreamWaitEvent(h.stream, h.eg.done[slot], 0));   // slot free again
  hipLaunchKernelGGL(k_to_columns, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, h.stream, k, (const char*)o.rec,
                     o.stride, L, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(h.eg.ready[slot], h.stream));
  o.consume(k, h.stream);   // (stream-ordered after the transpose)
  HIPCHK(hipStreamWaitEvent(h.eg.d2h, h.eg.ready[slot], 0));
  auto cp = [&](void* dst, size_t off, size_t w) {
    if (dst) HIPCHK(hipMemcpyAsync((char*)dst + w * (size_t)row0, st + off, w * (size_t)k, hipMemcpyDeviceToHost, h.eg.d2h));
  };
  cp(out->trigger, L.off_trig, 8);
  cp(out->ts, L.off_ts, 8);
  cp(out->key, L.off_key, 4);
  cp(out->group, L.off_grp, 4);
  for (int c = 0; c < L.ns; ++c) {
    cp(out->cols[c], L.off_col[c], (size_t)L.width[c]);
    cp(out->nulls[c], L.off_nul[c], 1);
  }
  HIPCHK(hipEventRecord(h.eg.done[slot], h.eg.d2h));
  return k;
}

struct DeliverHook : ChunkHook {
  SgHandle& h;
  const sg_match_columns* out;
  int64_t cap, rows = 0;
  int slot = 0;
  DeliverHook(SgHandle& hh, const sg_match_columns* o, int64_t c) : h(hh), out(o), cap(c) {}
  void chunk_done() override {
    rows += deliver_pending(h, out, rows, cap - rows, slot);
    slot ^= 1;
  }
};

// Host batch ingress in chunks (replacing StreamJunction's per-row fan-out,
// C/stream/StreamJunction.java:255-316): chunk k+1 is copied on a second HIP stream into the other of two HBM
// slots while chunk k runs on the handle's stream; consecutive chunks are consecutive sub-pushes, which the
// carried state makes identical to one push (no_carry handles are therefore never split).  `after` (optional)
// runs after each chunk's engine pass (match delivery, sg_push_deliver).
static void ingest_host(SgHandle& h, const sg_batch* b, ChunkHook* after) {
  const sg_nfa_desc& d = h.desc;
  const int64_t n = b->n;
  // Default (measured): batches of >= 32M rows in 4 chunks (copy-bound: 59.0 -> 55.1 ms per
  // 100M C2 events); smaller chunks lose to per-sub-push kernel overheads, smaller batches are one copy.
  int64_t C = h.opt.ingress_rows > 0 ? h.opt.ingress_rows : (n >= ((int64_t)32 << 20) ? (n + 3) / 4 : n);
  if (h.opt.ingress_rows < 0) C = n;
  if (h.opt.no_carry || n <= C) C = n;
  const int64_t nch = (n + C - 1) / C;
  if (nch == 1) {
    BatchView bv = upload(h, b, 0, n, 0, h.stream);
    sg_push_view(h, bv, n);
    if (after) after->chunk_done();
    return;
  }
  if (!h.copy_stream) {
    HIPCHK(hipStreamCreateWithFlags(&h.copy_stream, hipStreamNonBlocking));
    for (int k = 0; k < 2; ++k) {
      HIPCHK(hipEventCreateWithFlags(&h.ev_copied[k], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&h.ev_consumed[k], hipEventDisableTiming));
    }
  }
  SlotPtrs slots[2];
  for (int s = 0; s < 2; ++s) slots[s] = sg_reserve_slot(h, b, C, s);   // no workspace growth inside the pipeline
  BatchView cur = sg_upload_to(d, slots[0], b, 0, C, h.copy_stream);
  HIPCHK(hipEventRecord(h.ev_copied[0], h.copy_stream));
  // The next chunk's copies are issued from a helper thread: a large hipMemcpyAsync can hold the calling
  // thread, which would otherwise delay this chunk's kernels (measured).
  for (int64_t k = 0; k < nch; ++k) {
    const int64_t lo = k * C, cnt = std::min(C, n - lo);
    BatchView next;
    std::thread copier;
    int copy_rc = hipSuccess;
    if (k + 1 < nch) {
      const int s = (int)((k + 1) & 1);
      if (k + 1 >= 2) HIPCHK(hipStreamWaitEvent(h.copy_stream, h.ev_consumed[s], 0));
      copier = std::thread([&, s, lo] {
        try {
          if (hipSetDevice(h.device) != hipSuccess) { copy_rc = hipErrorInvalidDevice; return; }
          next = sg_upload_to(d, slots[s], b, lo + C, std::min(C, n - lo - C), h.copy_stream);
          copy_rc = hipEventRecord(h.ev_copied[s], h.copy_stream);
        } catch (...) {
          copy_rc = hipErrorUnknown;
        }
      });
    }
    try {
      HIPCHK(hipStreamWaitEvent(h.stream, h.ev_copied[k & 1], 0));
      sg_push_view(h, cur, cnt);
      HIPCHK(hipEventRecord(h.ev_consumed[k & 1], h.stream));
      if (after) after->chunk_done();
    } catch (...) {
      if (copier.joinable()) copier.join();
      hipStreamSynchronize(h.copy_stream);
      throw;
    }
    if (copier.joinable()) copier.join();
    if (copy_rc != hipSuccess) throw SgError(SG_EHIP, "ingress copy failed");
    if (k + 1 < nch) cur = next;
  }
  HIPCHK(hipStreamSynchronize(h.copy_stream));
}

// Pinned host memory for batches (cudaHostAlloc-style): the ingress copies from it run asynchronously at
// full PCIe rate, overlapped with the previous chunk's kernels.
extern "C" int sg_host_alloc(size_t bytes, void** p) {
  if (!p) return SG_EINVAL;
  return hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? SG_OK : SG_EHIP;
}
extern "C" int sg_host_free(void* p) { return hipHostFree(p) == hipSuccess ? SG_OK : SG_EHIP; }

extern "C" {

const char* sg_version(void) { return "siddhi_gpu 0.1 (gfx950)"; }

int sg_open(int hip_device, const sg_nfa_desc* nfa, const sg_options* opt, sg_handle** out) {
  if (!nfa || !out) return SG_EINVAL;
  sg_handle* hh = new sg_handle();
  SgHandle& h = hh->h;
  int rc = guard(hh, [&] {
    validate(nfa);
    h.device = hip_device;
    HIPCHK(hipSetDevice(hip_device));
    h.desc = *nfa;
    if (opt) h.opt = *opt;
    else memset(&h.opt, 0, sizeof(h.opt));
    if (h.opt.pool_partials <= 0) h.opt.pool_partials = 256;
    if (h.opt.pool_events <= 0) h.opt.pool_events = 256;
    if (h.opt.pool_chain <= 0) h.opt.pool_chain = 256;
    if (h.opt.list_cap <= 0) h.opt.list_cap = 256;
    if (h.opt.ring_cap < 0 || h.opt.ring_cap == 1 || h.opt.ring_cap > 256 || (h.opt.ring_cap & (h.opt.ring_cap - 1)))
      throw SgError(SG_EINVAL, "ring_cap must be 0 or a power of two in [2, 256]");
    HIPCHK(hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking));
    h.own_stream = true;
    for (auto& e : h.ev) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipMalloc(&h.ddesc, sizeof(DevDesc)));
    HIPCHK(hipMemcpy(h.ddesc, &h.desc, sizeof(DevDesc), hipMemcpyHostToDevice));
  });
  if (rc != SG_OK) {
    // keep the handle so the caller can read sg_last_error, but mark it unusable
    *out = hh;
    return rc;
  }
  *out = hh;
  return SG_OK;
}

int sg_push(sg_handle* hh, const sg_batch* b) {
  if (!hh || !b) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipSetDevice(h.device));
    const sg_nfa_desc& d = h.desc;
    int64_t n = b->n;
    if (n <= 0) return;
    check_batch(b);
    if (b->on_device) {
      BatchView bv = device_view(d, b);
      sg_push_view(h, bv, n);
      return;
    }
    ingest_host(h, b, nullptr);
  });
}

// A heartbeat is one clock-only row (stream -1): timers whose time has come fire in front of it, exactly as
// for an event row (TimestampGeneratorImpl.setCurrentTimestamp runs before the row is dispatched); no
// state consumes it.  trigger_index is its global event index (the sequence number the host assigned).
int sg_advance_time(sg_handle* hh, int64_t now, uint64_t trigger_index) {
  if (!hh) return SG_EINVAL;
  const sg_nfa_desc& d = hh->h.desc;
  int64_t ts = now;
  int32_t stream = -1, key = -1;
  uint64_t index = trigger_index;
  int64_t zero[SG_MAX_COLS] = {};
  const void* cols[SG_MAX_COLS];
  for (int c = 0; c < SG_MAX_COLS; ++c) cols[c] = &zero[c];
  sg_batch b;
  memset(&b, 0, sizeof(b));
  b.n = 1;
  b.base_index = trigger_index;
  b.ts = &ts;
  b.stream = &stream;
  b.key = &key;
  b.index = &index;
  b.cols = cols;
  b.on_device = 0;
  b.key_bound = 0;
  (void)d;
  return sg_push(hh, &b);
}

int sg_pending(sg_handle* hh, int64_t* n) {
  if (!hh || !n) return SG_EINVAL;
  *n = hh->h.out.n;
  return SG_OK;
}

int sg_device_records(sg_handle* hh, sg_match_records* v) {
  if (!hh || !v) return SG_EINVAL;
  OutStore& o = hh->h.out;
  v->n = o.n;
  v->record_bytes = 32 + 8 * out_cols(hh->h.desc);
  v->n_select = out_cols(hh->h.desc);
  v->base = o.rec;
  return SG_OK;
}

int sg_poll(sg_handle* hh, sg_matches* out, int64_t cap, int64_t* n) {
  if (!hh || !out) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipSetDevice(h.device));
    OutStore& o = h.out;
    const int64_t k = std::min<int64_t>(cap, o.n);
    if (k > 0) {
      // the sg_matches layout is built on the GPU (header fields split into columns, values row-major as in the
      // records), then copied field by field: no host-side transpose
      sg_egress_init(h);
      const int ns = out_cols(h.desc);
      const size_t need = (size_t)k * (8 + 8 + 4 + 4 + 4) + (size_t)k * 8 * ns + 1024;
      if (h.eg.cap[0] < (int64_t)need) {
        HIPCHK(hipEventSynchronize(h.eg.done[0]));
        if (h.eg.stage[0]) HIPCHK(hipFree(h.eg.stage[0]));
        h.eg.stage[0] = nullptr;
        HIPCHK(hipMalloc(&h.eg.stage[0], need + need / 4));
        h.eg.cap[0] = (int64_t)(need + need / 4);
      }
      char* st = h.eg.stage[0];
      HIPCHK(hipStreamWaitEvent(h.stream, h.eg.done[0], 0));   // the slot's last column copy has read it
      uint64_t* trig = (uint64_t*)st;
      int64_t* ts = (int64_t*)(trig + k);
      int64_t* vals = ts + k;
      int32_t* key = (int32_t*)(vals + (size_t)k * ns);
      uint32_t* grp = (uint32_t*)(key + k);
      uint32_t* vn = grp + k;
      hipLaunchKernelGGL(k_to_matches, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, h.stream, k, (const char*)o.rec,
                         o.stride, ns, trig, ts, key, grp, vals, vn);
      HIPCHK(hipGetLastError());
      auto cp = [&](void* dst, const void* src, size_t bytes) {
        if (dst) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h.stream));
      };
      cp(out->trigger, trig, 8 * (size_t)k);
      cp(out->ts, ts, 8 * (size_t)k);
      cp(out->key, key, 4 * (size_t)k);
      cp(out->group, grp, 4 * (size_t)k);
      cp(out->vnull, vn, 4 * (size_t)k);
      if (ns) cp(out->vals, vals, 8 * (size_t)k * ns);
      HIPCHK(hipStreamSynchronize(h.stream));
      o.consume(k, h.stream);
    }
    out->n = k;
    if (n) *n = k;
  });
}

int sg_poll_columns(sg_handle* hh, const sg_match_columns* out, int64_t cap, int64_t* n) {
  if (!hh || !out) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipSetDevice(h.device));
    const int64_t k = deliver_pending(h, out, 0, cap, 0);
    if (h.eg.d2h) HIPCHK(hipStreamSynchronize(h.eg.d2h));
    if (n) *n = k;
  });
}

int sg_push_deliver(sg_handle* hh, const sg_batch* b, const sg_match_columns* out, int64_t cap, int64_t* n) {
  if (!hh || !b || !out) return SG_EINVAL;
  SgHandle& h = hh->h;
  int64_t rows = 0;
  int rc = guard(hh, [&] {
    HIPCHK(hipSetDevice(h.device));
    DeliverHook dh(h, out, cap);
    {
      // size both staging slots for the largest delivery this call expects (pending matches, or one match per row of
      // the batch), so the chunk pipeline below does not allocate
      sg_egress_init(h);
      const int64_t expect = std::min<int64_t>(cap, std::max<int64_t>(h.out.n, b->n));
      if (expect > 0) {
        const int64_t bytes = (int64_t)sg_col_layout(h.desc, expect).bytes;
        sg_stage_reserve(h, 0, bytes);
        sg_stage_reserve(h, 1, bytes);
      }
    }
    try {
      dh.chunk_done();   // matches pending before this batch come first
      if (b->n > 0) {
        check_batch(b);
        if (b->on_device) {
          BatchView bv = device_view(h.desc, b);
          sg_push_view(h, bv, b->n);
          dh.chunk_done();
        } else {
          ingest_host(h, b, &dh);
        }
      }
    } catch (...) {
      if (h.eg.d2h) hipStreamSynchronize(h.eg.d2h);
      rows = dh.rows;
      throw;
    }
    if (h.eg.d2h) HIPCHK(hipStreamSynchronize(h.eg.d2h));
    rows = dh.rows;
    if (h.out.n) throw SgError(SG_ECAPACITY, "more matches than the output capacity: the rest stay pending");
  });
  if (n) *n = rows;
  return rc;
}

int sg_discard(sg_handle* hh) {
  if (!hh) return SG_EINVAL;
  hh->h.out.n = 0;
  return SG_OK;
}

int sg_flush(sg_handle* hh) {
  if (!hh) return SG_EINVAL;
  return guard(hh, [&] { HIPCHK(hipStreamSynchronize(hh->h.stream)); });
}

int sg_reset(sg_handle* hh) {
  if (!hh) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipStreamSynchronize(h.stream));
    h.out.n = 0;
    h.pushes = 0;
    h.ts_max_seen = INT64_MIN;
    h.bump_gen();
    sg_every_next_reset(&h);
    sg_every_absent_reset(&h);
    sg_general_reset(&h);
    sg_once_reset(&h);
  });
}

int sg_set_stream(sg_handle* hh, void* s) {
  if (!hh) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipStreamSynchronize(h.stream));
    if (h.own_stream) HIPCHK(hipStreamDestroy(h.stream));
    h.own_stream = false;
    h.stream = (hipStream_t)s;
  });
}

int sg_get_timing(sg_handle* hh, sg_timing* t) {
  if (!hh || !t) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipEventSynchronize(h.ev[4]));
    float a = 0, b = 0, c = 0, d = 0;
    HIPCHK(hipEventElapsedTime(&a, h.ev[0], h.ev[1]));
    HIPCHK(hipEventElapsedTime(&b, h.ev[1], h.ev[2]));
    HIPCHK(hipEventElapsedTime(&c, h.ev[2], h.ev[3]));
    HIPCHK(hipEventElapsedTime(&d, h.split_out ? h.ev[5] : h.ev[3], h.ev[4]));
    if (h.extra_marks) {
      float x = 0;
      HIPCHK(hipEventElapsedTime(&x, h.ev[6], h.ev[7]));
      c += x;
    }
    t->pred_ms = a;
    t->partition_ms = b;
    t->match_ms = c;
    t->output_ms = d;
    t->total_ms = a + b + c + d;
    t->events = h.last_events;
    t->matches = h.last_matches;
    t->spilled_units = h.last_spilled;
    t->n_kernels = h.n_km;
    for (int k = 0; k < h.n_km; ++k) {
      float x = 0;
      HIPCHK(hipEventElapsedTime(&x, h.km[k][0], h.km[k][1]));
      t->kernel_ms[k] = x;
      snprintf(t->kernel_name[k], sizeof t->kernel_name[k], "%s", h.km_name[k] ? h.km_name[k] : "?");
    }
  });
}

int sg_close(sg_handle* hh) {
  if (!hh) return SG_EINVAL;
  SgHandle& h = hh->h;
  hipSetDevice(h.device);
  if (h.stream) hipStreamSynchronize(h.stream);
  sg_every_next_release(&h);
  sg_every_absent_release(&h);
  sg_general_release(&h);
  sg_once_release(&h);
  h.ws.release();
  h.out.release();
  h.stage.release();
  if (h.eg.d2h) {
    hipStreamSynchronize(h.eg.d2h);
    for (int k = 0; k < 2; ++k) {
      if (h.eg.stage[k]) hipFree(h.eg.stage[k]);
      hipEventDestroy(h.eg.ready[k]);
      hipEventDestroy(h.eg.done[k]);
    }
    hipStreamDestroy(h.eg.d2h);
  }
  if (h.copy_stream) {
    hipStreamSynchronize(h.copy_stream);
    hipStreamDestroy(h.copy_stream);
    for (int k = 0; k < 2; ++k) { hipEventDestroy(h.ev_copied[k]); hipEventDestroy(h.ev_consumed[k]); }
  }
  if (h.ddesc) hipFree(h.ddesc);
  for (auto& e : h.ev) if (e) hipEventDestroy(e);
  for (auto& pr : h.km) for (auto& e : pr) if (e) hipEventDestroy(e);
  if (h.own_stream && h.stream) hipStreamDestroy(h.stream);
  delete hh;
  return SG_OK;
}

// ---- snapshot / restore -------------------------------------------------------------------------
static const char SNAP_MAGIC[8] = {'S', 'G', 'S', 'N', 'A', 'P', '0', '3'};   // 03: sequence-lane state layout recorded

// Fingerprint of everything the persisted state's meaning depends on: the lowered query and the engine
// route (closed form or general machine).  Field-wise, so struct padding never enters it.
static uint64_t query_fingerprint(const SgHandle& h) {
  const sg_nfa_desc& d = h.desc;
  uint64_t x = 1469598103934665603ull;
  auto mix = [&](int64_t v) {
    for (int b = 0; b < 8; ++b) { x ^= (uint64_t)((v >> (8 * b)) & 0xff); x *= 1099511628211ull; }
  };
  mix(d.type); mix(d.within); mix(d.playback); mix(d.partitioned);
  mix(d.n_states); mix(d.n_streams); mix(d.n_cols); mix(d.n_ret); mix(d.n_select);
  mix(h.opt.force_general ? SG_SHAPE_GENERAL : d.shape);
  for (int k = 0; k < 8; ++k) mix(d.shape_args[k]);
  for (int s = 0; s < d.n_states; ++s) {
    const sg_state_desc& st = d.states[s];
    mix(st.kind); mix(st.stream); mix(st.is_start); mix(st.min_count); mix(st.max_count); mix(st.logical_type);
    mix(st.partner); mix(st.next_state); mix(st.next_every); mix(st.within_every); mix(st.waiting_time);
  }
  for (int c = 0; c < d.n_cols; ++c) { mix(d.col_type[c]); mix(d.col_stream[c]); }
  for (int k = 0; k < d.n_select; ++k) { mix(d.sel_state[k]); mix(d.sel_index[k]); mix(d.sel_ret[k]); }
  mix(d.n_out); mix(d.having_off); mix(d.having_len);
  for (int k = 0; k < d.n_out; ++k) { mix(d.out_type[k]); mix(d.out_off[k]); mix(d.out_len[k]); }
  mix(d.code_len);
  for (int k = 0; k < d.code_len; ++k) mix(d.code[k]);
  return x;
}

// Serialise the handle's state (persist between events: SiddhiAppRuntime.snapshot,
// C/SiddhiAppRuntime.java:613-623 -> SnapshotService.fullSnapshot, C/util/snapshot/SnapshotService.java:97-157).
// buf == NULL (or cap too small) only reports the size.  Matches not yet polled are not state -- the
// reference has delivered them inside send() -- so a handle with pending matches is refused.
int sg_snapshot(sg_handle* hh, void* buf, size_t cap, size_t* size) {
  if (!hh || !size) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipSetDevice(h.device));
    HIPCHK(hipStreamSynchronize(h.stream));
    if (h.out.n) throw SgError(SG_EINVAL, "snapshot with undelivered matches: poll or discard them first");
    // the usual two calls (size query, then copy) serialise the device state once
    if (buf && h.snap_gen == h.gen && !h.snap_cache.empty()) {
      *size = h.snap_cache.size();
      if (cap >= h.snap_cache.size()) {
        memcpy(buf, h.snap_cache.data(), h.snap_cache.size());
        h.snap_cache.clear();
        h.snap_cache.shrink_to_fit();
        h.snap_gen = ~0ull;
      }
      return;
    }
    SnapW w;
    w.put(SNAP_MAGIC, 8);
    w.pod((int32_t)SG_ABI_VERSION);
    w.pod((int32_t)h.state_kind);
    w.pod(query_fingerprint(h));
    w.pod((int64_t)h.pushes);
    w.pod((uint32_t)h.key_bound_seen);
    switch (h.state_kind) {
      case 1: sg_every_next_snapshot(&h, w); break;
      case 2: sg_general_snapshot(&h, w); break;
      case 3: sg_every_absent_snapshot(&h, w); break;
      case 4: sg_once_snapshot(&h, w); break;
      default: break;
    }
    *size = w.b.size();
    if (buf && cap >= w.b.size()) {
      memcpy(buf, w.b.data(), w.b.size());
    } else {
      h.snap_cache.swap(w.b);
      h.snap_gen = h.gen;
    }
  });
}

// Replace the handle's state by a snapshot of a handle opened with the same query and options
// (SiddhiAppRuntime.restore, C/SiddhiAppRuntime.java:625-635 -> SnapshotService.restore :271-345).
int sg_restore(sg_handle* hh, const void* buf, size_t size) {
  if (!hh || (!buf && size)) return SG_EINVAL;
  SgHandle& h = hh->h;
  return guard(hh, [&] {
    HIPCHK(hipSetDevice(h.device));
    HIPCHK(hipStreamSynchronize(h.stream));
    h.bump_gen();   // from here on the state changes (or is reset on error)
    SnapR r{(const char*)buf, (const char*)buf + size};
    if (memcmp(r.take(8), SNAP_MAGIC, 8) != 0) throw SgError(SG_EINVAL, "not a siddhi_gpu snapshot");
    if (r.pod<int32_t>() != SG_ABI_VERSION) throw SgError(SG_EINVAL, "snapshot ABI version mismatch");
    const int32_t kind = r.pod<int32_t>();
    if (r.pod<uint64_t>() != query_fingerprint(h)) throw SgError(SG_EINVAL, "snapshot was taken for another query");
    const int64_t pushes = r.pod<int64_t>();
    const uint32_t kb = r.pod<uint32_t>();
    if (kind < 0 || kind > 4 || (h.state_kind && kind && h.state_kind != kind))
      throw SgError(SG_EINVAL, "snapshot engine kind does not match the handle");
    h.out.n = 0;
    sg_every_next_reset(&h);
    sg_every_absent_reset(&h);
    sg_general_reset(&h);
    sg_once_reset(&h);
    switch (kind) {
      case 1: sg_every_next_restore(&h, r); break;
      case 2: sg_general_restore(&h, r); break;
      case 3: sg_every_absent_restore(&h, r); break;
      case 4: sg_once_restore(&h, r); break;
      default: break;
    }
    if (r.p != r.e) throw SgError(SG_EINVAL, "trailing bytes in snapshot");
    h.pushes = (int)pushes;
    h.key_bound_seen = kb;
    h.bump_gen();
  });
}

const char* sg_last_error(const sg_handle* hh) { return hh ? hh->h.err.c_str() : "null handle"; }

}  // extern "C"

void OutStore::consume(int64_t k, hipStream_t st) {
  if (k >= n) {
    n = 0;
    return;
  }
  int64_t rest = n - k;
  void* tmp = nullptr;
  if (hipMalloc(&tmp, (size_t)rest * stride) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc in consume");
  hipMemcpyAsync(tmp, rec + (size_t)k * stride, (size_t)rest * stride, hipMemcpyDeviceToDevice, st);
  hipMemcpyAsync(rec, tmp, (size_t)rest * stride, hipMemcpyDeviceToDevice, st);
  hipStreamSynchronize(st);
  hipFree(tmp);
  n = rest;
}
