// once.hip -- closed form for  A[l] -> B[l' and B.x OP A.x] (within T)  without `every` (SG_SHAPE_NEXT_CMP_ONCE):
// PatternPartitionTestCase's canonical shape `from e1=Stream1[price>20] -> e2=Stream2[price>e1.price]` under
// `partition with (volume of Stream1, volume of Stream2)` (T/query/partition/PatternPartitionTestCase.java:54-64).
//
// Semantics, restated from the reference processors (C/ = modules/siddhi-core/src/main/java/io/siddhi/core/):
//   * A is a start state without an `every` edge: init() puts ONE empty partial into A's newAndEvery list, and only
//     for a start state that was never initialised (StreamPreStateProcessor.init, C/query/input/stream/state/
//     StreamPreStateProcessor.java:157-166).  The first A-stream event passing l binds it; the partial is removed from
//     A (stateChanged, :314-315) and handed to B (StreamPostStateProcessor.process, .../StreamPostStateProcessor.java:
//     53-72); nothing ever re-arms A.  A-stream events that fail l leave the partial in place (:316-331).
//   * Each B-stream event of the key first checks expiry (isExpired, :102-113: |e1.ts - now| > within, B is not a
//     start state) and drops the partial if so; otherwise binds, and the partial completes iff l' and the cross
//     compare hold (a null operand compares false, CompareConditionExpressionExecutor.java:39-43).
//   * A partitioned query clones one such runtime per key on the key's first event (PartitionRuntime.clonePartition,
//     C/partition/PartitionRuntime.java:255-308), so per key:
//         e1 = the key's first A-stream row passing l;
//         e2 = the first later B-stream row that passes l' and the compare, provided no B-stream row between them
//              (itself included) expired the partial first.
//     For one event both states are visited in reverse registration order (MultiProcessStreamReceiver.java:98-309),
//     B before A, so an event never completes the partial it binds.  None of this depends on time order: the rule
//     holds for any timestamps (expiry uses the absolute difference), so this route has no ordering precondition.
//
// GPU form: no key sort.  Two passes over the rows in arrival order with per-key atomicMin (a racy read of the
// current minimum skips the atomic for every row that cannot improve it -- after the first rows of each key, almost
// all), one pass over the keys between them, a compaction of the completed keys and a radix sort of their (trigger,
// key) pairs by trigger.  Per key the state carried between pushes is the phase (no e1 / e1 bound / done) and e1's
// timestamp, compared value and projected attributes.  O(rows) work and ~20 bytes read per row; the per-key machine
// took one lane per key (csrc/interp.hip).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <string>

#include "pred.h"
#include "sg_device.h"
#include "sg_engine.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace {

const uint32_t NONE = 0xffffffffu;

struct OnceState {
  int64_t kcap = 0;
  uint8_t* phase = nullptr;     // per key: 0 waiting for e1, 1 e1 bound, 2 done (matched or expired)
  int64_t* e1ts = nullptr;
  int64_t* e1x = nullptr;       // e1's compared value (bits)
  uint8_t* e1xn = nullptr;      // ... null
  int64_t* e1sel = nullptr;     // [n_select][kcap]: e1's projected attribute bits (select entries of state A)
  uint32_t* e1seln = nullptr;   // per key: null bits of those entries
  void release() {
    for (void* p : {(void*)phase, (void*)e1ts, (void*)e1x, (void*)e1xn, (void*)e1sel, (void*)e1seln})
      if (p) hipFree(p);
    *this = OnceState();
  }
};

struct OnceArgs {
  int64_t n;
  int64_t within;               // -1: none
  int32_t s_a, s_b;             // streams of A and B
  int32_t col_a, col_b;         // compared columns
  int32_t type;                 // their Attribute.Type (the lowering requires one type)
  int32_t op, dom;              // B.x OP A.x (sg_cmp codes), compare domain
  int32_t partitioned;
  uint32_t K;
  const int64_t* ts;
  const int32_t* stream;        // null: every row is stream 0
  const int32_t* key;
  const uint64_t* cand_m;       // rows passing A's local filter (A's stream only)
  const uint64_t* cons_m;       // rows passing B's local conjuncts (B's stream only); null: every B-stream row
};

__device__ __forceinline__ int row_stream(const OnceArgs& a, int64_t r) { return a.stream ? a.stream[r] : 0; }
__device__ __forceinline__ int64_t row_key(const OnceArgs& a, int64_t r) {
  return a.partitioned ? (int64_t)a.key[r] : 0;   // (-1: a clock-only row or a null partition key: no runtime)
}

// pass 1: the first row of each still-waiting key that passes A's filter
__global__ void __launch_bounds__(256) k_once_first(OnceArgs a, const uint8_t* __restrict__ phase,
                                                    uint32_t* __restrict__ first, uint32_t* __restrict__ err) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = row_key(a, r);
    if (k >= (int64_t)a.K) { atomicOr(err, 1u); continue; }   // beyond the caller's key_bound (every row checked)
    if (!mask_bit(a.cand_m, (uint64_t)r)) continue;
    if (k < 0 || phase[k] != 0) continue;
    if ((uint32_t)r < __hip_atomic_load(&first[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMin(&first[k], (uint32_t)r);
  }
}

struct SelPlan {
  int32_t n_select;
  int32_t a_state, b_state;
  int32_t sel_state[SG_MAX_SELECT], sel_ok[SG_MAX_SELECT], sel_col[SG_MAX_SELECT], sel_type[SG_MAX_SELECT];
};

// keys: bind the e1 found in this push (its attributes are kept: a later push's match projects them); lo[k] = first
// row that may complete the key's partial (NONE: none in this push).  A push with a key beyond key_bound (*err, from
// k_once_first) changes no key's state: every key gets lo = NONE, so the later passes do nothing, and the host raises
// the error with the push's one end-of-push readback.
__global__ void k_once_bind(OnceArgs a, SgCols bc, SelPlan sp, OnceState s, const uint32_t* __restrict__ first,
                            uint32_t* __restrict__ lo, const uint32_t* __restrict__ err) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)a.K) return;
  if (*err) { lo[k] = NONE; return; }
  const uint8_t ph = s.phase[k];
  if (ph == 1) { lo[k] = 0; return; }
  if (ph != 0 || first[k] == NONE) { lo[k] = NONE; return; }
  const uint32_t r = first[k];
  s.e1ts[k] = a.ts[r];
  const SgVal x = sg_read_col(bc, a.col_a, a.type, r);
  s.e1x[k] = sg_val_bits(x);
  s.e1xn[k] = (uint8_t)x.null;
  uint32_t nm = 0;
  for (int q = 0; q < sp.n_select; ++q) {
    if (sp.sel_state[q] != sp.a_state) continue;
    int64_t bits = 0;
    if (sp.sel_ok[q]) {
      const SgVal v = sg_read_col(bc, sp.sel_col[q], sp.sel_type[q], r);
      if (v.null) nm |= 1u << q;
      bits = sg_val_bits(v);
    } else {
      nm |= 1u << q;   // a chain index beyond a single-event slot reads null (StateEvent.getStreamEvent)
    }
    s.e1sel[(size_t)q * s.kcap + k] = bits;
  }
  s.e1seln[k] = nm;
  s.phase[k] = 1;
  lo[k] = r + 1;   // (B is visited before A for the binding event itself)
}

// pass 2: per waiting key, the first B-stream row that expires its partial and the first that completes it
__global__ void __launch_bounds__(256) k_once_second(OnceArgs a, SgCols bc, OnceState s, const uint32_t* __restrict__ lo,
                                                     uint32_t* __restrict__ hit, uint32_t* __restrict__ expd) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += (int64_t)gridDim.x * blockDim.x) {
    if (row_stream(a, r) != a.s_b) continue;
    const int64_t k = row_key(a, r);
    if (k < 0 || k >= (int64_t)a.K) continue;
    const uint32_t l = lo[k];
    if ((uint32_t)r < l || l == NONE) continue;
    const uint32_t cur = min(__hip_atomic_load(&hit[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                             __hip_atomic_load(&expd[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if ((uint32_t)r >= cur) continue;   // an earlier row already decided this key
    if (a.within >= 0) {
      const int64_t d = a.ts[r] - s.e1ts[k];
      if (d > a.within || -d > a.within) { atomicMin(&expd[k], (uint32_t)r); continue; }
    }
    if (a.cons_m && !mask_bit(a.cons_m, (uint64_t)r)) continue;
    if (s.e1xn[k]) continue;
    const SgVal xb = sg_read_col(bc, a.col_b, a.type, r);
    const SgVal xa = sg_val_from_bits(s.e1x[k], a.type, 0);
    if (sg_cmp(a.op, a.dom, xb, xa)) atomicMin(&hit[k], (uint32_t)r);
  }
}

// keys: completed partials -> (trigger row, key) pairs; completed or expired keys are done
__global__ void k_once_finish(OnceArgs a, OnceState s, const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hit,
                              const uint32_t* __restrict__ expd, uint32_t* __restrict__ cnt, uint32_t* __restrict__ prow,
                              uint32_t* __restrict__ pkey) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)a.K || lo[k] == NONE) return;
  const uint32_t h = hit[k], e = expd[k];
  if (h < e) {
    const uint32_t q = atomicAdd(cnt, 1u);
    prow[q] = h;
    pkey[q] = (uint32_t)k;
    s.phase[k] = 2;
  } else if (e != NONE) {
    s.phase[k] = 2;
  }
}

// match records (QuerySelector.processNoGroupBy, C/query/selector/QuerySelector.java:125-163) in trigger order
__global__ void k_once_project(int64_t m, const uint32_t* __restrict__ srow, const uint32_t* __restrict__ skey,
                               OnceArgs a, SgCols bc, SelPlan sp, OnceState s, uint64_t base_index,
                               const uint64_t* __restrict__ index, uint32_t grp, int stride, char* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t r = srow[i], k = skey[i];
  int64_t* o = (int64_t*)(out + (size_t)i * stride);
  uint32_t nm = 0;
  const uint32_t e1n = s.e1seln[k];
  for (int q = 0; q < sp.n_select; ++q) {
    int64_t bits = 0;
    if (sp.sel_state[q] == sp.a_state) {
      bits = s.e1sel[(size_t)q * s.kcap + k];
      nm |= e1n & (1u << q);
    } else if (sp.sel_ok[q]) {
      const SgVal v = sg_read_col(bc, sp.sel_col[q], sp.sel_type[q], r);
      if (v.null) nm |= 1u << q;
      bits = sg_val_bits(v);
    } else {
      nm |= 1u << q;
    }
    o[4 + q] = bits;
  }
  o[0] = (int64_t)(index ? index[r] : base_index + r);
  o[1] = a.ts[r];
  o[2] = (int64_t)((uint64_t)(a.partitioned ? k : 0u) | ((uint64_t)grp << 32));
  o[3] = (int64_t)nm;
}

template <class T>
void grow(T*& p, int64_t old_n, int64_t new_n, hipStream_t st) {
  T* np = nullptr;
  if (hipMalloc(&np, sizeof(T) * (size_t)new_n) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc once-route state");
  HIPCHK(hipMemsetAsync(np, 0, sizeof(T) * (size_t)new_n, st));
  if (p && old_n) HIPCHK(hipMemcpyAsync(np, p, sizeof(T) * (size_t)old_n, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  if (p) hipFree(p);
  p = np;
}

void ensure_keys(OnceState& s, int64_t K, int n_select, hipStream_t st) {
  if (K <= s.kcap) return;
  const int64_t nk = std::max<int64_t>(K, s.kcap * 3 / 2);
  const int ns = std::max(n_select, 1);
  grow(s.phase, s.kcap, nk, st);
  grow(s.e1ts, s.kcap, nk, st);
  grow(s.e1x, s.kcap, nk, st);
  grow(s.e1xn, s.kcap, nk, st);
  grow(s.e1seln, s.kcap, nk, st);
  // e1sel is [n_select][kcap]: re-stride
  int64_t* np = nullptr;
  if (hipMalloc(&np, 8 * (size_t)ns * (size_t)nk) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc once-route state");
  HIPCHK(hipMemsetAsync(np, 0, 8 * (size_t)ns * (size_t)nk, st));
  if (s.e1sel && s.kcap)
    for (int q = 0; q < ns; ++q)
      HIPCHK(hipMemcpyAsync(np + (size_t)q * nk, s.e1sel + (size_t)q * s.kcap, 8 * (size_t)s.kcap, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  if (s.e1sel) hipFree(s.e1sel);
  s.e1sel = np;
  s.kcap = nk;
}

OnceState* ostate(SgHandle* h) {
  if (!h->state) {
    h->state = new OnceState();
    h->state_kind = 4;
  }
  return (OnceState*)h->state;
}

unsigned grid_rows(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 64)); }

}  // namespace

void sg_run_once(SgHandle* h, const BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int* sa = d.shape_args;
  const int a_state = sa[0], b_state = sa[1];
  OnceState& s = *ostate(h);
  // ---- key bound (monotone over the stream)
  uint32_t kb = 1;
  if (d.partitioned) {
    kb = bv.key_bound > 0 ? (uint32_t)bv.key_bound : 0;
    if (kb == 0 && n > 0) {
      int32_t* dmax = (int32_t*)h->ws.get("kmax", sizeof(int32_t), st);
      size_t tb = 0;
      HIPCHK(rocprim::reduce(nullptr, tb, bv.key, dmax, (int32_t)-1, (size_t)n, rocprim::maximum<int32_t>(), st));
      void* tmp = h->ws.get("kmax_tmp", tb, st);
      HIPCHK(rocprim::reduce(tmp, tb, bv.key, dmax, (int32_t)-1, (size_t)n, rocprim::maximum<int32_t>(), st));
      int32_t hm = 0;
      HIPCHK(hipMemcpyAsync(&hm, dmax, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      kb = (uint32_t)std::max(hm + 1, 1);
    }
    kb = std::max<uint32_t>(kb, 1);
    if (kb < h->key_bound_seen) kb = h->key_bound_seen;
    h->key_bound_seen = kb;
  }
  if (n >= (int64_t)NONE) throw SgError(SG_EINVAL, "batch too large for the once route");
  ensure_keys(s, kb, d.n_select, st);
  h->split_out = 0;
  h->extra_marks = 0;
  h->mark(0);
  OnceArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.within = d.within;
  a.s_a = d.states[a_state].stream;
  a.s_b = d.states[b_state].stream;
  a.col_b = d.ret_col[sa[3]];
  a.col_a = d.ret_col[sa[4]];
  a.type = d.col_type[a.col_a];
  a.op = sa[2];
  a.dom = (a.type == SG_T_FLOAT) ? 1 : (a.type == SG_T_DOUBLE ? 2 : 0);
  a.partitioned = d.partitioned;
  a.K = kb;
  a.ts = bv.ts;
  a.stream = bv.stream;
  a.key = bv.key;
  // ---- 1. predicate-evaluation pass: A's local filter (nulls of the compared value do not stop e1 from binding) and
  //         B's local conjuncts
  PredArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.n = n;
  pa.stream = bv.stream;
  pa.s_a = a.s_a;
  pa.s_b = a.s_b;
  pa.val_col_a = -1;
  pa.val_col_b = a.col_b;   // (a null B.x compares false: such rows need no consumer bit; expiry is checked apart)
  pa.prog_a_off = d.states[a_state].prog_off;
  pa.prog_a_len = d.states[a_state].prog_len;
  pa.prog_b_off = d.shape_prog_off;
  pa.prog_b_len = d.shape_prog_len;
  // one stream and no local conjunct in B: every row is a consumer (k_once_second checks nulls); several streams:
  // the consumer bits are B's stream's rows (the 16-B pass over the stream column when A's filter is `col CMP const`)
  pa.cons_all = (d.shape_prog_len == 0 && !bv.stream && !bv.cols.nul[a.col_b]) ? 1 : 0;
  const int64_t ntiles = (n + 255) / 256;
  uint64_t* cand_m = (uint64_t*)h->ws.get("once_cand", sizeof(uint64_t) * 4 * (ntiles + 1), st);
  uint64_t* cons_m = pa.cons_all ? nullptr : (uint64_t*)h->ws.get("once_cons", sizeof(uint64_t) * 4 * (ntiles + 1), st);
  if (n > 0) {
    h->kbeg("pred");
    launch_pred(d, pa, bv.stream, bv.cols, h->ddesc, cand_m, cons_m, st);
    HIPCHK(hipGetLastError());
    h->kend();
  }
  a.cand_m = cand_m;
  a.cons_m = cons_m;
  h->mark(1);
  SelPlan sp;
  memset(&sp, 0, sizeof(sp));
  sp.n_select = d.n_select;
  sp.a_state = a_state;
  sp.b_state = b_state;
  for (int q = 0; q < d.n_select; ++q) {
    const int idx = d.sel_index[q];
    sp.sel_state[q] = d.sel_state[q];
    sp.sel_ok[q] = (idx == 0 || idx == -1) ? 1 : 0;
    sp.sel_col[q] = d.ret_col[d.sel_ret[q]];
    sp.sel_type[q] = d.sel_type[q];
  }
  uint32_t* first = (uint32_t*)h->ws.get("once_first", 4 * (size_t)kb, st);
  uint32_t* lo = (uint32_t*)h->ws.get("once_lo", 4 * (size_t)kb, st);
  uint32_t* hit = (uint32_t*)h->ws.get("once_hit", 4 * (size_t)kb, st);
  uint32_t* expd = (uint32_t*)h->ws.get("once_exp", 4 * (size_t)kb, st);
  uint32_t* cnt = (uint32_t*)h->ws.get("once_cnt", 8, st);
  uint32_t* prow = (uint32_t*)h->ws.get("once_prow", 4 * (size_t)kb, st);
  uint32_t* pkey = (uint32_t*)h->ws.get("once_pkey", 4 * (size_t)kb, st);
  HIPCHK(hipMemsetAsync(first, 0xff, 4 * (size_t)kb, st));
  HIPCHK(hipMemsetAsync(hit, 0xff, 4 * (size_t)kb, st));
  HIPCHK(hipMemsetAsync(expd, 0xff, 4 * (size_t)kb, st));
  HIPCHK(hipMemsetAsync(cnt, 0, 8, st));
  const dim3 blk(256), gk((unsigned)((kb + 255) / 256));
  h->kbeg("once_match");
  if (n > 0) hipLaunchKernelGGL(k_once_first, dim3(grid_rows(n)), blk, 0, st, a, s.phase, first, cnt + 1);
  hipLaunchKernelGGL(k_once_bind, gk, blk, 0, st, a, bv.cols, sp, s, first, lo, cnt + 1);
  if (n > 0) hipLaunchKernelGGL(k_once_second, dim3(grid_rows(n)), blk, 0, st, a, bv.cols, s, lo, hit, expd);
  hipLaunchKernelGGL(k_once_finish, gk, blk, 0, st, a, s, lo, hit, expd, cnt, prow, pkey);
  HIPCHK(hipGetLastError());
  h->kend();
  uint32_t hc[2] = {0, 0};   // matches, key-range error
  HIPCHK(hipMemcpyAsync(hc, cnt, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (hc[1]) throw SgError(SG_EINVAL, "a partition key id is >= the batch's key_bound");
  const uint32_t m = hc[0];
  h->mark(2);
  h->mark(3);
  if (m) {
    uint32_t* srow = (uint32_t*)h->ws.get("once_srow", 4 * (size_t)m, st);
    uint32_t* skey = (uint32_t*)h->ws.get("once_skey", 4 * (size_t)m, st);
    int end_bit = 1;
    while (end_bit < 32 && (1ull << end_bit) <= (uint64_t)n) ++end_bit;
    h->kbeg("once_order");
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, prow, srow, pkey, skey, (size_t)m, 0, end_bit, st));
    void* tmp = h->ws.get("once_sort_tmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, prow, srow, pkey, skey, (size_t)m, 0, end_bit, st));
    // group: one match per trigger (rank 0); a Multi receiver reports the visit slot of B (eventSequence = reversed
    // init order), as the other routes do
    const int rb = d.recv_of_stream[d.states[b_state].stream];
    uint32_t grp = (1u << 24) | 0x800000u;
    if (d.receivers[rb].multi) {
      const sg_receiver_desc& r = d.receivers[rb];
      for (int q = 0; q < r.n; ++q)
        if (r.pres[r.n - 1 - q] == b_state) grp = (1u << 24) | (uint32_t)q;
    }
    const int stride = 32 + 8 * d.n_select;
    char* out = h->out.reserve(m, d.n_select, st);
    hipLaunchKernelGGL(k_once_project, dim3((m + 255) / 256), blk, 0, st, (int64_t)m, srow, skey, a, bv.cols, sp, s,
                       bv.base_index, bv.index, grp, stride, out + (size_t)h->out.n * stride);
    HIPCHK(hipGetLastError());
    h->kend();
    h->out.n += m;
  }
  h->mark(4);
  h->last_events = n;
  h->last_matches = m;
  h->last_spilled = 0;
}

void sg_once_reset(SgHandle* h) {
  if (!h->state || h->state_kind != 4) return;
  OnceState& s = *(OnceState*)h->state;
  if (s.kcap) HIPCHK(hipMemset(s.phase, 0, (size_t)s.kcap));
}

void sg_once_release(SgHandle* h) {
  if (!h->state || h->state_kind != 4) return;
  OnceState* s = (OnceState*)h->state;
  s->release();
  delete s;
  h->state = nullptr;
  h->state_kind = 0;
}

// Snapshot: per key the phase and e1's kept attributes -- the pending partial of B's StreamPreStateProcessor and
// whether A's start partial is still there (StreamPreStateProcessor.currentState/restoreState,
// C/query/input/stream/state/StreamPreStateProcessor.java:352-367).
void sg_once_snapshot(SgHandle* h, SnapW& w) {
  OnceState* s = (h->state && h->state_kind == 4) ? (OnceState*)h->state : nullptr;
  const int64_t k = s ? s->kcap : 0;
  const int ns = std::max(h->desc.n_select, 1);
  w.pod(k);
  if (!k) return;
  w.dev(s->phase, (size_t)k, h->stream);
  w.dev(s->e1ts, 8 * (size_t)k, h->stream);
  w.dev(s->e1x, 8 * (size_t)k, h->stream);
  w.dev(s->e1xn, (size_t)k, h->stream);
  w.dev(s->e1seln, 4 * (size_t)k, h->stream);
  w.dev(s->e1sel, 8 * (size_t)ns * (size_t)k, h->stream);
}

void sg_once_restore(SgHandle* h, SnapR& r) {
  const int64_t k = r.pod<int64_t>();
  if (k < 0 || k > ((int64_t)1 << 31)) throw SgError(SG_EINVAL, "snapshot: bad key count");
  OnceState& s = *ostate(h);
  s.release();   // (a fresh state of exactly the snapshot's key capacity: e1sel is strided by it)
  if (!k) return;
  ensure_keys(s, k, h->desc.n_select, h->stream);
  const int ns = std::max(h->desc.n_select, 1);
  r.dev(s.phase, (size_t)k, h->stream);
  r.dev(s.e1ts, 8 * (size_t)k, h->stream);
  r.dev(s.e1x, 8 * (size_t)k, h->stream);
  r.dev(s.e1xn, (size_t)k, h->stream);
  r.dev(s.e1seln, 4 * (size_t)k, h->stream);
  r.dev(s.e1sel, 8 * (size_t)ns * (size_t)k, h->stream);
}
