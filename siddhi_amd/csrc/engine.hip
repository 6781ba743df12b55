// MI355X closed-form pipeline for  every A[l] -> B[l' and B.x OP A.x] within T
// (SG_SHAPE_EVERY_NEXT_CMP: configs C1/C2/C5).  Semantics: SURVEY.md A.7 — partial e1=i is completed
// by the first later B-row j of its key with B.x_j OP A.x_i, and emitted iff ts_j - ts_i <= T.
// Restated from StreamPreStateProcessor.processAndReturn (C/query/input/stream/state/
// StreamPreStateProcessor.java:292-337: lazy `within` expiry, bind, filter, remove on state change) and
// the `every` re-arm in StreamPostStateProcessor.process (:53-72).
//
// Pipeline per sg_push (one HIP stream, inputs resident in HBM):
//   1. k_pack        coalesced predicate-evaluation pass: per row evaluates A's filter and B's local
//                    conjuncts (postfix VM, sg_device.h) and packs one record
//                    {ts, row, flags, nulls, cmp value, projected attributes} + partition key
//                    (rows no state reads get the sentinel key and sort to the end).
//   2. key partition (partitioned queries): stable LSD radix sort of records by dense key (rocPRIM
//                    onesweep): every key's rows contiguous, in arrival order — the GPU form of
//                    PartitionStreamReceiver routing rows to per-key cloned runtimes.  Rows carried from
//                    the previous push (still inside the `within` window) are prepended.
//   3. k_match<COUNT> per consumer row j a backward scan over its key's earlier records, bounded by T
//                    and cut off once the running max/min of intermediate consumers makes every older
//                    candidate unreachable, counts the e1 partials j completes; count stored by arrival row.
//   4. exclusive scan over arrival order -> output offsets (reference delivery order: trigger event,
//                    then e1 arrival order within the trigger).
//   5. k_match<WRITE> re-runs the scan and writes one AoS match record (32 + 8*n_select bytes) per match.
//   6. carry: records with ts >= last_ts - T survive into the next push (they may still be completed,
//                    or consume, later).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "sg_device.h"
#include "sg_engine.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static const int F_CAND = 1, F_CONS = 2, F_CARRY = 4;
#define MAXP 4

struct RowReader {
  const SgCols* c;
  const int32_t* ret_col;
  int64_t row;
  __device__ SgVal read(int, int, int slot, int type) { return sg_read_col(*c, ret_col[slot], type, row); }
};

template <class T, int NP>
struct alignas(8) Rec {
  int64_t ts;
  uint32_t row;
  uint16_t flags;
  uint16_t pnull;
  T val;
  int64_t p[NP > 0 ? NP : 1];
};

struct ProjPlan {
  int32_t np;                 // projected columns carried in records
  int32_t col[MAXP];          // batch column of each
  int32_t type[MAXP];
  int32_t stream[MAXP];
  // per select: src 0 = candidate (A) record, 1 = consumer (B) record;
  // kind 0 = proj[idx], 1 = record value, 2 = null (chain index beyond a single-event slot), 3 = column gather
  int32_t src[SG_MAX_SELECT], kind[SG_MAX_SELECT], idx[SG_MAX_SELECT];
};

struct PackArgs {
  const int64_t* ts;
  const int32_t* stream;
  const int32_t* key;
  int64_t n;
  int64_t prev_clock;
  int32_t has_prev;
  int32_t s_a, s_b;
  int32_t partitioned;
  uint32_t sentinel;
  int32_t val_col_a, val_col_b;
  int32_t prog_a_off, prog_a_len, prog_b_off, prog_b_len;
  int64_t rec_off;            // records of this batch start after the carried ones
};

template <class T>
__device__ __forceinline__ T load_val(const SgCols& c, int col, int64_t row) {
  return ((const T*)c.col[col])[row];
}

template <class T, int NP>
__global__ void __launch_bounds__(256) k_pack(PackArgs a, SgCols cols, ProjPlan pp,
                                              const DevDesc* __restrict__ dd, Rec<T, NP>* __restrict__ rec,
                                              uint32_t* __restrict__ keys, int32_t* __restrict__ order_err) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  int s = a.stream ? a.stream[i] : 0;
  int64_t t = a.ts[i];
  int64_t tp = (i > 0) ? a.ts[i - 1] : (a.has_prev ? a.prev_clock : t);
  if (tp > t) atomicOr(order_err, 1);   // closed form needs non-decreasing timestamps
  RowReader rd{&cols, dd->ret_col, i};
  int flags = 0;
  T v = T(0);
  if (s == a.s_a) {
    bool nul = cols.nul[a.val_col_a] && cols.nul[a.val_col_a][i];
    if (!nul && sg_eval(dd->code + a.prog_a_off, a.prog_a_len, rd)) {
      flags |= F_CAND;
      v = load_val<T>(cols, a.val_col_a, i);
    }
  }
  if (s == a.s_b) {
    bool nul = cols.nul[a.val_col_b] && cols.nul[a.val_col_b][i];
    if (!nul && sg_eval(dd->code + a.prog_b_off, a.prog_b_len, rd)) {
      flags |= F_CONS;
      v = load_val<T>(cols, a.val_col_b, i);   // same column whenever s_a == s_b
    }
  }
  Rec<T, NP> r;
  r.ts = t;
  r.row = (uint32_t)i;
  r.flags = (uint16_t)flags;
  r.val = v;
  uint32_t pn = 0;
#pragma unroll
  for (int k = 0; k < (NP > 0 ? NP : 1); ++k) {
    r.p[k] = 0;
    if (k < NP && pp.stream[k] == s) {
      SgVal x = sg_read_col(cols, pp.col[k], pp.type[k], i);
      if (x.null) pn |= 1u << k;
      r.p[k] = sg_val_bits(x);
    }
  }
  r.pnull = (uint16_t)pn;
  rec[a.rec_off + i] = r;
  if (a.partitioned) {
    int32_t k = a.key ? a.key[i] : -1;
    keys[a.rec_off + i] = (flags == 0 || k < 0) ? a.sentinel : (uint32_t)k;
  }
}

template <class T> __device__ __forceinline__ bool is_nan_val(T) { return false; }
template <> __device__ __forceinline__ bool is_nan_val<float>(float x) { return x != x; }
template <> __device__ __forceinline__ bool is_nan_val<double>(double x) { return x != x; }

template <class T, int OP>
__device__ __forceinline__ bool cmp_op(T b, T a) {
  if (OP == 2) return b > a;
  if (OP == 3) return b >= a;
  if (OP == 4) return b < a;
  return b <= a;
}
// i is still pending at j iff no intermediate consumer x satisfied (x OP a_i)
template <class T, int OP>
__device__ __forceinline__ bool not_consumed(T m, T a, bool have) {
  if (!have) return true;
  return !cmp_op<T, OP>(m, a);
}
template <class T, int OP>
__device__ __forceinline__ void fold(T& m, bool& have, T x) {
  if (is_nan_val<T>(x)) return;   // NaN compares false: it consumes nothing
  if (!have) { m = x; have = true; return; }
  if (OP <= 3) m = (x > m) ? x : m;
  else m = (x < m) ? x : m;
}
template <class T, int OP>
__device__ __forceinline__ bool stop_scan(T m, T b, bool have) {
  if (!have) return false;
  if (OP <= 3) return m >= b;   // every older candidate would need a_i >= m and a_i < b
  return m <= b;
}

struct MatchArgs {
  int64_t n;             // records (carry + batch)
  int64_t within;
  uint64_t base_index;
  int32_t partitioned;
  uint32_t sentinel;
  int32_t multi;
  int32_t b_slot;
  int32_t n_select;
  int32_t stride;        // output record bytes
  int64_t out_base;
  const uint64_t* index; // optional global index per batch row
};

template <class T>
__device__ __forceinline__ int64_t val_bits(T v);
template <> __device__ __forceinline__ int64_t val_bits<float>(float v) { return (int64_t)(uint32_t)__float_as_uint(v); }
template <> __device__ __forceinline__ int64_t val_bits<double>(double v) { return __double_as_longlong(v); }
template <> __device__ __forceinline__ int64_t val_bits<int32_t>(int32_t v) { return (int64_t)v; }
template <> __device__ __forceinline__ int64_t val_bits<int64_t>(int64_t v) { return v; }

template <class T, int NP, int OP, bool WRITE>
__global__ void __launch_bounds__(256) k_match(MatchArgs a, const Rec<T, NP>* __restrict__ rec,
                                               const uint32_t* __restrict__ keys, uint32_t* __restrict__ cnt,
                                               const uint32_t* __restrict__ off, ProjPlan pp, SgCols cols,
                                               const DevDesc* __restrict__ dd, char* __restrict__ out) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.n) return;
  const Rec<T, NP> q = rec[p];
  if (!(q.flags & F_CONS) || (q.flags & F_CARRY)) return;
  uint32_t k = a.partitioned ? keys[p] : 0u;
  if (a.partitioned && k == a.sentinel) return;
  if (is_nan_val<T>(q.val)) return;
  uint32_t total = 0;
  int64_t wbase = 0;
  if (WRITE) {
    total = cnt[q.row];
    if (total == 0) return;
    wbase = a.out_base + (int64_t)off[q.row];
  }
  T m = q.val;
  bool have = false;
  uint32_t c = 0;
  for (int64_t r = p - 1; r >= 0; --r) {
    if (a.partitioned && keys[r] != k) break;
    const Rec<T, NP> e = rec[r];
    if (q.ts - e.ts > a.within) break;   // expired at j, and so is every older row of the key
    if ((e.flags & F_CAND) && cmp_op<T, OP>(q.val, e.val) && not_consumed<T, OP>(m, e.val, have)) {
      if (WRITE) {
        uint32_t rank = total - 1 - c;   // the scan meets e1 rows newest first; delivery is oldest first
        char* o = out + (size_t)(wbase + rank) * (size_t)a.stride;
        uint32_t nm = 0;
        int64_t* vals = (int64_t*)(o + 32);
        for (int s = 0; s < a.n_select; ++s) {
          int kind = pp.kind[s];
          int src = pp.src[s];
          int64_t bits = 0;
          if (kind == 0) {
            int ix = pp.idx[s];
            bool nul = ((src ? q.pnull : e.pnull) >> ix) & 1u;
            bits = nul ? 0 : (src ? q.p[ix] : e.p[ix]);
            if (nul) nm |= 1u << s;
          } else if (kind == 1) {
            bits = val_bits<T>(src ? q.val : e.val);
          } else if (kind == 2) {
            nm |= 1u << s;
          } else {
            SgVal v = sg_read_col(cols, dd->ret_col[dd->sel_ret[s]], dd->sel_type[s], src ? q.row : e.row);
            if (v.null) nm |= 1u << s;
            bits = sg_val_bits(v);
          }
          vals[s] = bits;
        }
        uint64_t* h64 = (uint64_t*)o;
        h64[0] = a.index ? a.index[q.row] : a.base_index + q.row;
        h64[1] = (uint64_t)q.ts;
        uint32_t* h32 = (uint32_t*)(o + 16);
        h32[0] = k;
        h32[1] = (1u << 24) | (a.multi ? (uint32_t)a.b_slot : (0x800000u | rank));
        h32[2] = nm;
        h32[3] = 0;
      }
      ++c;
    }
    if (e.flags & F_CONS) fold<T, OP>(m, have, e.val);
    if (stop_scan<T, OP>(m, q.val, have)) break;
  }
  if (!WRITE && c) cnt[q.row] = c;
}

// carry selection: records that may still matter for a later push
template <class T, int NP>
__global__ void k_carry_flags(const Rec<T, NP>* __restrict__ rec, const uint32_t* __restrict__ keys, int64_t n,
                              int64_t min_ts, uint32_t sentinel, int partitioned, uint8_t* __restrict__ fl) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  Rec<T, NP> r = rec[p];
  bool keep = (r.flags & (F_CAND | F_CONS)) && r.ts >= min_ts;
  if (partitioned && keys[p] == sentinel) keep = false;
  fl[p] = keep ? 1 : 0;
}

template <class T, int NP>
__global__ void k_mark_carry(Rec<T, NP>* __restrict__ rec, int64_t n) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) rec[p].flags |= F_CARRY;
}

// ----------------------------------------------------------------------------------------------
struct EveryNextState {
  int64_t n_carry = 0;
  int64_t clock = 0;
  bool has_clock = false;
};

static ProjPlan make_plan(const sg_nfa_desc& d, int b_state, int val_col_a, int val_col_b, int np_cap) {
  ProjPlan pp;
  memset(&pp, 0, sizeof(pp));
  bool overflow = false;
  for (int s = 0; s < d.n_select; ++s) {
    int st = d.sel_state[s];
    pp.src[s] = (st == b_state) ? 1 : 0;
    int col = d.ret_col[d.sel_ret[s]];
    int idx = d.sel_index[s];
    if (idx != 0 && idx != -1) { pp.kind[s] = 2; continue; }
    int vcol = pp.src[s] ? val_col_b : val_col_a;
    if (col == vcol) { pp.kind[s] = 1; continue; }
    int found = -1;
    for (int k = 0; k < pp.np; ++k) if (pp.col[k] == col) found = k;
    if (found < 0) {
      if (pp.np < np_cap) {
        found = pp.np++;
        pp.col[found] = col;
        pp.type[found] = d.col_type[col];
        pp.stream[found] = d.col_stream[col];
      } else overflow = true;
    }
    if (found >= 0) { pp.kind[s] = 0; pp.idx[s] = found; }
    else pp.kind[s] = 3;
  }
  if (overflow) {
    for (int s = 0; s < d.n_select; ++s) if (pp.kind[s] == 0) pp.kind[s] = 3;
    pp.np = 0;
  }
  return pp;
}

template <class T, int NP, int OP>
static void launch_match(bool write, dim3 g, dim3 b, hipStream_t st, MatchArgs ma, const Rec<T, NP>* rec,
                         const uint32_t* keys, uint32_t* cnt, const uint32_t* off, ProjPlan pp, SgCols cols,
                         const DevDesc* dd, char* out) {
  if (write) hipLaunchKernelGGL((k_match<T, NP, OP, true>), g, b, 0, st, ma, rec, keys, cnt, off, pp, cols, dd, out);
  else hipLaunchKernelGGL((k_match<T, NP, OP, false>), g, b, 0, st, ma, rec, keys, cnt, off, pp, cols, dd, out);
}

template <class T, int NP>
static void run_every_next(SgHandle* h, const BatchView& bv, int64_t n, ProjPlan pp) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int* sa = d.shape_args;
  int a_state = sa[0], b_state = sa[1], op = sa[2];
  EveryNextState* es = (EveryNextState*)h->state;
  PackArgs pa;
  pa.ts = bv.ts;
  pa.stream = bv.stream;
  pa.key = bv.key;
  pa.n = n;
  pa.prev_clock = es->clock;
  pa.has_prev = es->has_clock;
  pa.s_a = d.states[a_state].stream;
  pa.s_b = d.states[b_state].stream;
  pa.partitioned = d.partitioned;
  pa.val_col_a = d.ret_col[sa[4]];
  pa.val_col_b = d.ret_col[sa[3]];
  pa.prog_a_off = d.states[a_state].prog_off;
  pa.prog_a_len = d.states[a_state].prog_len;
  pa.prog_b_off = d.shape_prog_off;
  pa.prog_b_len = d.shape_prog_len;
  uint32_t kb = bv.key_bound > 0 ? (uint32_t)bv.key_bound : 0;
  if (d.partitioned && kb == 0) {
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
  // the sentinel must exceed every key still carried from earlier pushes
  if (kb < h->key_bound_seen) kb = h->key_bound_seen;
  h->key_bound_seen = kb;
  pa.sentinel = kb;
  int end_bit = 1;
  while ((1ull << end_bit) <= (uint64_t)kb) ++end_bit;

  typedef Rec<T, NP> R;
  int64_t nc = es->n_carry;
  int64_t nt = nc + n;
  R* rec = (R*)h->ws.get("rec", sizeof(R) * nt, st);
  uint32_t* keys = d.partitioned ? (uint32_t*)h->ws.get("keys", sizeof(uint32_t) * nt, st) : nullptr;
  if (nc) {
    HIPCHK(hipMemcpyAsync(rec, h->ws.get("carry_rec", sizeof(R) * nc, st), sizeof(R) * nc, hipMemcpyDeviceToDevice, st));
    if (d.partitioned)
      HIPCHK(hipMemcpyAsync(keys, h->ws.get("carry_keys", sizeof(uint32_t) * nc, st), sizeof(uint32_t) * nc,
                            hipMemcpyDeviceToDevice, st));
  }
  pa.rec_off = nc;
  int32_t* order_err = (int32_t*)h->ws.get("order_err", sizeof(int32_t), st);
  HIPCHK(hipMemsetAsync(order_err, 0, sizeof(int32_t), st));
  dim3 blk(256), grd((unsigned)((n + 255) / 256)), grdt((unsigned)((nt + 255) / 256));
  h->mark(0);
  hipLaunchKernelGGL((k_pack<T, NP>), grd, blk, 0, st, pa, bv.cols, pp, h->ddesc, rec, keys, order_err);
  HIPCHK(hipGetLastError());
  h->mark(1);
  R* srec = rec;
  uint32_t* skeys = keys;
  if (d.partitioned) {
    R* rec2 = (R*)h->ws.get("rec2", sizeof(R) * nt, st);
    uint32_t* keys2 = (uint32_t*)h->ws.get("keys2", sizeof(uint32_t) * nt, st);
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, keys, keys2, rec, rec2, (size_t)nt, 0, end_bit, st));
    void* tmp = h->ws.get("sort_tmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, keys, keys2, rec, rec2, (size_t)nt, 0, end_bit, st));
    srec = rec2;
    skeys = keys2;
  }
  h->mark(2);
  uint32_t* cnt = (uint32_t*)h->ws.get("cnt", sizeof(uint32_t) * (n + 1), st);
  uint32_t* off = (uint32_t*)h->ws.get("off", sizeof(uint32_t) * (n + 1), st);
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (n + 1), st));
  MatchArgs ma;
  ma.n = nt;
  ma.within = d.within;
  ma.base_index = bv.base_index;
  ma.partitioned = d.partitioned;
  ma.sentinel = kb;
  int rb = d.recv_of_stream[d.states[b_state].stream];
  ma.multi = d.receivers[rb].multi;
  ma.b_slot = 0;
  if (ma.multi) {
    const sg_receiver_desc& r = d.receivers[rb];
    for (int k = 0; k < r.n; ++k)
      if (r.pres[r.n - 1 - k] == b_state) ma.b_slot = k;   // eventSequence = reversed init order
  }
  ma.n_select = d.n_select;
  ma.stride = 32 + 8 * d.n_select;
  ma.out_base = 0;
  ma.index = bv.index;
  auto launch = [&](bool write, char* out) {
    switch (op) {
      case 2: launch_match<T, NP, 2>(write, grdt, blk, st, ma, srec, skeys, cnt, off, pp, bv.cols, h->ddesc, out); break;
      case 3: launch_match<T, NP, 3>(write, grdt, blk, st, ma, srec, skeys, cnt, off, pp, bv.cols, h->ddesc, out); break;
      case 4: launch_match<T, NP, 4>(write, grdt, blk, st, ma, srec, skeys, cnt, off, pp, bv.cols, h->ddesc, out); break;
      default: launch_match<T, NP, 5>(write, grdt, blk, st, ma, srec, skeys, cnt, off, pp, bv.cols, h->ddesc, out); break;
    }
    HIPCHK(hipGetLastError());
  };
  launch(false, nullptr);
  {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
  }
  h->mark(3);
  uint32_t total = 0;
  int32_t oerr = 0;
  int64_t last_ts = 0;
  HIPCHK(hipMemcpyAsync(&total, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&oerr, order_err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&last_ts, bv.ts + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (oerr) throw SgError(SG_EORDER, "closed-form kernel requires non-decreasing timestamps");
  if (total) {
    char* out = h->out.reserve(total, d.n_select, st);
    ma.out_base = h->out.n;
    launch(true, out);
    h->out.n += total;
  }
  h->mark(4);
  // ---- carry rows still inside the window into the next push: the surviving old carry plus the
  // time-ordered tail of this batch (pre-sort records [nc + lo, nt) with ts >= last_ts - T)
  if (h->opt.no_carry == 0) {
    int64_t min_ts = last_ts - d.within;
    int64_t lo = 0;
    {
      // first batch row with ts >= min_ts (timestamps are non-decreasing; checked above)
      std::vector<int64_t> probe(1);
      int64_t a0 = 0, a1 = n;
      while (a0 < a1) {
        int64_t mid = (a0 + a1) / 2;
        HIPCHK(hipMemcpy(probe.data(), bv.ts + mid, 8, hipMemcpyDeviceToHost));
        if (probe[0] < min_ts) a0 = mid + 1; else a1 = mid;
      }
      lo = a0;
    }
    int64_t tail = n - lo;
    int64_t keep_old = 0;
    R* crec = (R*)h->ws.get("carry_rec_tmp", sizeof(R) * (nc + tail + 1), st);
    uint32_t* ck = (uint32_t*)h->ws.get("carry_keys_tmp", sizeof(uint32_t) * (nc + tail + 1), st);
    if (nc) {
      // old carry sits unsorted at rec[0, nc) (copied before k_pack)
      uint8_t* fl = (uint8_t*)h->ws.get("carry_fl", nc, st);
      hipLaunchKernelGGL((k_carry_flags<T, NP>), dim3((unsigned)((nc + 255) / 256)), blk, 0, st, rec, keys, nc, min_ts,
                         kb, d.partitioned, fl);
      HIPCHK(hipGetLastError());
      int64_t* cnt_sel = (int64_t*)h->ws.get("carry_cnt", sizeof(int64_t), st);
      size_t tb = 0;
      HIPCHK(rocprim::select(nullptr, tb, rec, fl, crec, cnt_sel, (size_t)nc, st));
      void* tmp = h->ws.get("carry_tmp", tb, st);
      HIPCHK(rocprim::select(tmp, tb, rec, fl, crec, cnt_sel, (size_t)nc, st));
      if (d.partitioned) {
        size_t tb2 = 0;
        HIPCHK(rocprim::select(nullptr, tb2, keys, fl, ck, cnt_sel, (size_t)nc, st));
        void* tmp2 = h->ws.get("carry_tmp2", tb2, st);
        HIPCHK(rocprim::select(tmp2, tb2, keys, fl, ck, cnt_sel, (size_t)nc, st));
      }
      HIPCHK(hipMemcpyAsync(&keep_old, cnt_sel, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    if (tail) {
      HIPCHK(hipMemcpyAsync(crec + keep_old, rec + nc + lo, sizeof(R) * tail, hipMemcpyDeviceToDevice, st));
      if (d.partitioned)
        HIPCHK(hipMemcpyAsync(ck + keep_old, keys + nc + lo, sizeof(uint32_t) * tail, hipMemcpyDeviceToDevice, st));
    }
    int64_t ncar = keep_old + tail;
    if (ncar && pp.np == 0) {
      for (int s = 0; s < d.n_select; ++s)
        if (pp.kind[s] == 3 && pp.src[s] == 0)
          throw SgError(SG_EUNSUPPORTED, "carry across pushes needs <= 4 projected attributes");
    }
    R* keep = (R*)h->ws.get("carry_rec", sizeof(R) * std::max<int64_t>(ncar, 1), st);
    if (ncar) {
      HIPCHK(hipMemcpyAsync(keep, crec, sizeof(R) * ncar, hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL((k_mark_carry<T, NP>), dim3((unsigned)((ncar + 255) / 256)), blk, 0, st, keep, ncar);
      HIPCHK(hipGetLastError());
      if (d.partitioned) {
        uint32_t* keepk = (uint32_t*)h->ws.get("carry_keys", sizeof(uint32_t) * ncar, st);
        HIPCHK(hipMemcpyAsync(keepk, ck, sizeof(uint32_t) * ncar, hipMemcpyDeviceToDevice, st));
      }
    }
    es->n_carry = ncar;
  } else {
    es->n_carry = 0;
  }
  es->clock = last_ts;
  es->has_clock = true;
  h->last_events = n;
  h->last_matches = total;
}

template <class T>
static void dispatch_np(SgHandle* h, const BatchView& bv, int64_t n, const ProjPlan& pp) {
  switch (pp.np) {
    case 0: run_every_next<T, 0>(h, bv, n, pp); break;
    case 1: run_every_next<T, 1>(h, bv, n, pp); break;
    case 2: run_every_next<T, 2>(h, bv, n, pp); break;
    case 3: run_every_next<T, 3>(h, bv, n, pp); break;
    default: run_every_next<T, 4>(h, bv, n, pp); break;
  }
}

void sg_run_every_next(SgHandle* h, const BatchView& bv, int64_t n) {
  if (!h->state) { h->state = new EveryNextState(); h->state_kind = 1; }
  const sg_nfa_desc& d = h->desc;
  const int* sa = d.shape_args;
  ProjPlan pp = make_plan(d, sa[1], d.ret_col[sa[4]], d.ret_col[sa[3]], MAXP);
  switch (sa[5]) {
    case SG_T_FLOAT: dispatch_np<float>(h, bv, n, pp); break;
    case SG_T_DOUBLE: dispatch_np<double>(h, bv, n, pp); break;
    case SG_T_LONG: dispatch_np<int64_t>(h, bv, n, pp); break;
    default: dispatch_np<int32_t>(h, bv, n, pp); break;
  }
}

void sg_every_next_reset(SgHandle* h) {
  if (h->state && h->state_kind == 1) *(EveryNextState*)h->state = EveryNextState();
  h->key_bound_seen = 0;
}

void sg_every_next_release(SgHandle* h) {
  if (h->state_kind != 1) return;
  delete (EveryNextState*)h->state;
  h->state = nullptr;
  h->state_kind = 0;
}
