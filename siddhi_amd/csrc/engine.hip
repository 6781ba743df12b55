// MI355X state engine: C-ABI (include/siddhi_gpu.h) + the closed-form pipeline for
//   every A[l] -> B[l' and B.x OP A.x] within T        (SG_SHAPE_EVERY_NEXT_CMP; configs C1/C2/C5)
// The general per-key NFA interpreter lives in interp.hip, the absence closed form in absent.hip.
//
// Pipeline per sg_push (all on the handle's HIP stream, inputs resident in HBM):
//   1. k_pack       coalesced predicate-evaluation pass: per row evaluates A's filter and B's local
//                   conjuncts (postfix VM, sg_device.h) and writes a 16/24-byte record
//                   {ts, row|flags, value} plus the partition key (sentinel for rows no state reads).
//   2. key partition (partitioned queries): stable LSD radix sort of the records by dense key
//                   (rocPRIM onesweep) -> every key's events contiguous, in arrival order.  This is the
//                   GPU form of PartitionStreamReceiver routing rows to per-key runtimes.
//   3. k_match<COUNT> per consumer row j, a backward scan over its key's earlier records bounded by T
//                   finds the e1 partials j completes (i is matched by the first later
//                   B-row j with B.x OP A.x_i; the scan keeps the running max/min of intermediate
//                   consumers), writes the per-trigger match count in arrival order.
//   4. exclusive scan of counts over arrival order -> output offsets (reference delivery order:
//                   by trigger event, then e1 arrival order).
//   5. k_match<WRITE> re-runs the scan and writes projected match tuples at their offsets.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "sg_device.h"
#include "sg_engine.h"

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static const int F_CAND = 1, F_CONS = 2;

// ----------------------------------------------------------------------------------------------
// Local-predicate reader: every VAR refers to the row's own event (lowering marks such filters local).
struct RowReader {
  const SgCols* c;
  const int32_t* ret_col;
  const int32_t* ret_type;
  int64_t row;
  __device__ SgVal read(int, int, int slot, int type) { return sg_read_col(*c, ret_col[slot], type, row); }
};

template <class T>
struct alignas(8) Rec {
  int64_t ts;
  uint32_t rowf;   // row index (bits 0..29) | flags << 30
  T val;
};

struct PackArgs {
  const int64_t* ts;
  const int32_t* stream;
  const int32_t* key;
  int64_t n;
  int32_t s_a, s_b;
  int32_t partitioned;
  uint32_t sentinel;
  int32_t val_col_a, val_col_b;   // batch columns of A.x and B.x
  int32_t prog_a_off, prog_a_len, prog_b_off, prog_b_len;
};

template <class T>
__device__ __forceinline__ T load_val(const SgCols& c, int col, int64_t row) {
  return ((const T*)c.col[col])[row];
}

// Pass 1: predicate evaluation + record pack. One thread per row, fully coalesced.
template <class T>
__global__ void __launch_bounds__(256) k_pack(PackArgs a, SgCols cols, const DevDesc* __restrict__ dd,
                                              Rec<T>* __restrict__ rec, uint32_t* __restrict__ keys,
                                              int32_t* __restrict__ order_err) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  int s = a.stream ? a.stream[i] : 0;
  int64_t t = a.ts[i];
  if (i > 0 && a.ts[i - 1] > t) atomicOr(order_err, 1);   // closed form needs non-decreasing ts
  RowReader rd{&cols, dd->ret_col, dd->ret_type, i};
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
    // a null B.x never compares true and never consumes (compare with null -> false)
    if (!nul && sg_eval(dd->code + a.prog_b_off, a.prog_b_len, rd)) {
      flags |= F_CONS;
      v = load_val<T>(cols, a.val_col_b, i);   // same column when s_a == s_b
    }
  }
  Rec<T> r;
  r.ts = t;
  r.rowf = (uint32_t)i | ((uint32_t)flags << 30);
  r.val = v;
  rec[i] = r;
  if (a.partitioned) {
    int32_t k = a.key ? a.key[i] : -1;
    keys[i] = (flags == 0 || k < 0) ? a.sentinel : (uint32_t)k;
  }
}

// ----------------------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ bool is_nan_val(T x) { return false; }
template <>
__device__ __forceinline__ bool is_nan_val<float>(float x) { return x != x; }
template <>
__device__ __forceinline__ bool is_nan_val<double>(double x) { return x != x; }

template <class T>
__device__ __forceinline__ T lowest_val();
template <> __device__ __forceinline__ float lowest_val<float>() { return -__builtin_huge_valf(); }
template <> __device__ __forceinline__ double lowest_val<double>() { return -__builtin_huge_val(); }
template <> __device__ __forceinline__ int32_t lowest_val<int32_t>() { return INT32_MIN; }
template <> __device__ __forceinline__ int64_t lowest_val<int64_t>() { return INT64_MIN; }

struct MatchArgs {
  int64_t n;            // records
  int64_t within;
  uint64_t base_index;
  int32_t op;           // 2 >, 3 >=, 4 <, 5 <=
  int32_t partitioned;
  uint32_t sentinel;
  int32_t multi;        // B visited through a Multi receiver (group = slot), else Single (per-match group)
  int32_t b_slot;       // visit slot of B in the receiver's eventSequence
  int32_t n_select;
  int32_t state_a, state_b;
  int64_t out_base;     // pending matches already in the output store
};

struct OutPtrs {
  uint64_t* trigger;
  int64_t* ts;
  int32_t* key;
  uint32_t* group;
  int64_t* vals;
  uint32_t* vnull;
};

// For OP in {>, >=} the scan tracks M = max of intermediate consumers; i matches j iff
//   b_j OP a_i and (M <= a_i for '>' | M < a_i for '>=');  stop once M >= b_j.
// For {<, <=} values are mirrored by negation-free min tracking.
template <class T, int OP>
__device__ __forceinline__ bool cmp_op(T b, T a) {
  if (OP == 2) return b > a;
  if (OP == 3) return b >= a;
  if (OP == 4) return b < a;
  return b <= a;
}
template <class T, int OP>
__device__ __forceinline__ bool not_consumed(T m, T a, bool have) {
  // no intermediate consumer x with (x OP a)
  if (!have) return true;
  if (OP == 2) return !(m > a);
  if (OP == 3) return !(m >= a);
  if (OP == 4) return !(m < a);
  return !(m <= a);
}
template <class T, int OP>
__device__ __forceinline__ void fold(T& m, bool& have, T x) {
  if (is_nan_val<T>(x)) return;   // NaN never compares true: it consumes nothing
  if (!have) { m = x; have = true; return; }
  if (OP <= 3) m = (x > m) ? x : m;
  else m = (x < m) ? x : m;
}
template <class T, int OP>
__device__ __forceinline__ bool stop_scan(T m, T b, bool have) {
  if (!have) return false;
  if (OP <= 3) return m >= b;  // no a_i can satisfy a_i >= m (or > m) and a_i < b (or <= b)
  return m <= b;
}

template <class T, int OP, bool WRITE>
__global__ void __launch_bounds__(256) k_match(MatchArgs a, const Rec<T>* __restrict__ rec,
                                               const uint32_t* __restrict__ keys, uint32_t* __restrict__ cnt,
                                               const uint32_t* __restrict__ off, SgCols cols,
                                               const DevDesc* __restrict__ dd, OutPtrs out) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.n) return;
  Rec<T> q = rec[p];
  int qf = q.rowf >> 30;
  if (!(qf & F_CONS)) return;
  uint32_t k = a.partitioned ? keys[p] : 0;
  if (a.partitioned && k == a.sentinel) return;
  if (is_nan_val<T>(q.val)) return;
  uint32_t row_j = q.rowf & 0x3FFFFFFFu;
  T m = lowest_val<T>();
  bool have = false;
  uint32_t c = 0;
  uint32_t total = 0;
  int64_t wbase = 0;
  if (WRITE) {
    total = cnt[row_j];
    if (total == 0) return;
    wbase = a.out_base + (int64_t)off[row_j];
  }
  for (int64_t r = p - 1; r >= 0; --r) {
    if (a.partitioned && keys[r] != k) break;
    Rec<T> e = rec[r];
    if (q.ts - e.ts > a.within) break;   // expired for j and for every earlier row (ts non-decreasing)
    int ef = e.rowf >> 30;
    if ((ef & F_CAND) && cmp_op<T, OP>(q.val, e.val) && not_consumed<T, OP>(m, e.val, have)) {
      if (WRITE) {
        // scan yields e1 rows in descending arrival order; reference order is ascending
        int64_t o = wbase + (int64_t)(total - 1 - c);
        uint32_t row_i = e.rowf & 0x3FFFFFFFu;
        out.trigger[o] = a.base_index + row_j;
        out.ts[o] = q.ts;
        out.key[o] = (int32_t)k;
        out.group[o] = (1u << 24) | (a.multi ? (uint32_t)a.b_slot : (0x800000u | (total - 1 - c)));
        uint32_t nm = 0;
        for (int s = 0; s < a.n_select; ++s) {
          int st = dd->sel_state[s];
          int idx = dd->sel_index[s];
          int slot = dd->sel_ret[s];
          int typ = dd->sel_type[s];
          // a non-count slot holds one event: chain index 0 / CURRENT resolve to it, others are null
          if (idx != 0 && idx != -1) { nm |= 1u << s; out.vals[o * a.n_select + s] = 0; continue; }
          int64_t row = (st == a.state_a) ? (int64_t)row_i : (int64_t)row_j;
          SgVal v = sg_read_col(cols, dd->ret_col[slot], typ, row);
          if (v.null) nm |= 1u << s;
          out.vals[o * a.n_select + s] = sg_val_bits(v);
        }
        out.vnull[o] = nm;
      }
      ++c;
    }
    if (ef & F_CONS) fold<T, OP>(m, have, e.val);
    if (stop_scan<T, OP>(m, q.val, have)) break;
  }
  if (!WRITE && c) cnt[row_j] = c;
}

// ----------------------------------------------------------------------------------------------
template <class T>
static void run_every_next(SgHandle* h, const BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int* sa = d.shape_args;
  int a_state = sa[0], b_state = sa[1], op = sa[2];
  int slot_b = sa[3], slot_a = sa[4];
  PackArgs pa;
  pa.ts = bv.ts;
  pa.stream = bv.stream;   // may be null: every row is stream 0
  pa.key = bv.key;
  pa.n = n;
  pa.s_a = d.states[a_state].stream;
  pa.s_b = d.states[b_state].stream;
  pa.partitioned = d.partitioned;
  pa.val_col_a = d.ret_col[slot_a];
  pa.val_col_b = d.ret_col[slot_b];
  pa.prog_a_off = d.states[a_state].prog_off;
  pa.prog_a_len = d.states[a_state].prog_len;
  pa.prog_b_off = d.shape_prog_off;
  pa.prog_b_len = d.shape_prog_len;
  uint32_t kb = bv.key_bound > 0 ? (uint32_t)bv.key_bound : 0;
  if (d.partitioned && kb == 0) {
    // unknown bound: reduce max key on device
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
  pa.sentinel = kb;
  int end_bit = 1;
  while ((1ull << end_bit) <= (uint64_t)kb) ++end_bit;

  Rec<T>* rec = (Rec<T>*)h->ws.get("rec", sizeof(Rec<T>) * n, st);
  uint32_t* keys = d.partitioned ? (uint32_t*)h->ws.get("keys", sizeof(uint32_t) * n, st) : nullptr;
  int32_t* order_err = (int32_t*)h->ws.get("order_err", sizeof(int32_t), st);
  HIPCHK(hipMemsetAsync(order_err, 0, sizeof(int32_t), st));
  dim3 blk(256), grd((unsigned)((n + 255) / 256));
  h->mark(0);
  hipLaunchKernelGGL(k_pack<T>, grd, blk, 0, st, pa, bv.cols, h->ddesc, rec, keys, order_err);
  HIPCHK(hipGetLastError());
  h->mark(1);
  const Rec<T>* srec = rec;
  const uint32_t* skeys = nullptr;
  if (d.partitioned) {
    Rec<T>* rec2 = (Rec<T>*)h->ws.get("rec2", sizeof(Rec<T>) * n, st);
    uint32_t* keys2 = (uint32_t*)h->ws.get("keys2", sizeof(uint32_t) * n, st);
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, keys, keys2, rec, rec2, (size_t)n, 0, end_bit, st));
    void* tmp = h->ws.get("sort_tmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, keys, keys2, rec, rec2, (size_t)n, 0, end_bit, st));
    srec = rec2;
    skeys = keys2;
  }
  h->mark(2);
  uint32_t* cnt = (uint32_t*)h->ws.get("cnt", sizeof(uint32_t) * (n + 1), st);
  uint32_t* off = (uint32_t*)h->ws.get("off", sizeof(uint32_t) * (n + 1), st);
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (n + 1), st));
  MatchArgs ma;
  ma.n = n;
  ma.within = d.within;
  ma.base_index = bv.base_index;
  ma.op = op;
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
  ma.state_a = a_state;
  ma.state_b = b_state;
  ma.out_base = 0;
  OutPtrs none{};
  switch (op) {
    case 2: hipLaunchKernelGGL((k_match<T, 2, false>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, none); break;
    case 3: hipLaunchKernelGGL((k_match<T, 3, false>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, none); break;
    case 4: hipLaunchKernelGGL((k_match<T, 4, false>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, none); break;
    default: hipLaunchKernelGGL((k_match<T, 5, false>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, none); break;
  }
  HIPCHK(hipGetLastError());
  {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
  }
  h->mark(3);
  uint32_t total = 0;
  int32_t oerr = 0;
  HIPCHK(hipMemcpyAsync(&total, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&oerr, order_err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (oerr) throw SgError(SG_EORDER, "closed-form kernel requires non-decreasing timestamps in a batch");
  if (total) {
    OutPtrs o = h->out.reserve<OutPtrs>((int64_t)total, d.n_select, st);
    ma.out_base = h->out.n;
    switch (op) {
      case 2: hipLaunchKernelGGL((k_match<T, 2, true>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, o); break;
      case 3: hipLaunchKernelGGL((k_match<T, 3, true>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, o); break;
      case 4: hipLaunchKernelGGL((k_match<T, 4, true>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, o); break;
      default: hipLaunchKernelGGL((k_match<T, 5, true>), grd, blk, 0, st, ma, srec, skeys, cnt, off, bv.cols, h->ddesc, o); break;
    }
    HIPCHK(hipGetLastError());
    h->out.n += total;
  }
  h->mark(4);
  h->last_events = n;
  h->last_matches = total;
}

void sg_run_every_next(SgHandle* h, const BatchView& bv, int64_t n) {
  int t = h->desc.shape_args[5];
  switch (t) {
    case SG_T_FLOAT: run_every_next<float>(h, bv, n); break;
    case SG_T_DOUBLE: run_every_next<double>(h, bv, n); break;
    case SG_T_LONG: run_every_next<int64_t>(h, bv, n); break;
    default: run_every_next<int32_t>(h, bv, n); break;
  }
}
