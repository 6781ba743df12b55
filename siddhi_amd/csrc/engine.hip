// MI355X closed-form pipeline for  every A[l] -> B[l' and B.x OP A.x] within T
// (SG_SHAPE_EVERY_NEXT_CMP: configs C1/C2/C5).
//
// Semantics, restated from StreamPreStateProcessor.processAndReturn
// (C/query/input/stream/state/StreamPreStateProcessor.java:292-337: lazy `within` expiry, bind,
// filter, remove on state change), the `every` re-arm in StreamPostStateProcessor.process (:53-72) and
// the reverse-registration visit order of MultiProcessStreamReceiver (C/query/input/
// MultiProcessStreamReceiver.java:98-309, B's state is visited before A's for the same event):
//   per key, e2's pending list holds the e1 partials in arrival order; an event j of the key first
//   drops the partials whose e1 is older than ts_j - T, then (if it is a B event passing B's local
//   filter) completes every pending partial i with x_j OP x_i -- delivered in pending order -- and
//   finally (if it passes A's filter) appends itself as a new partial.
//
// Pipeline per sg_push (one HIP stream, inputs resident in HBM):
//   1. k_pred       predicate-evaluation pass: A's filter and B's local conjuncts per row -> two
//                   condition bitmasks (wave ballots), 0.125 B/row/state.  The only pass over the value
//                   columns that is not key-ordered.
//   2. partition    (partitioned queries) stable radix sort of row ids by dense key (rocPRIM onesweep):
//                   per key the row list in arrival order -- the GPU form of PartitionStreamReceiver
//                   routing rows to per-key cloned runtimes (C/partition/PartitionStreamReceiver.java:80-281).
//                   k_bounds turns the sorted keys into per-key segments.
//   3. k_walk<COUNT> one lane per (time chunk, key) unit walks its key's rows in order and runs the
//                   reference's pending list exactly.  When B's filter is only the cross compare and both
//                   sides read one attribute, the pending list is a monotone stack (every surviving
//                   partial has x_i NOT-OP x_j of the last consumer), so completion pops a suffix and
//                   `within` expiry advances the bottom: O(1) amortised per event, kept in LDS.  Otherwise
//                   the list is scanned and compacted.  A unit first replays (without emitting) the rows
//                   of its key inside the `within` window before its chunk, which rebuilds the exact
//                   pending list at the chunk start.  Units of one time chunk run together on one XCD,
//                   so their row-ordered gathers share L2 lines.  Counts per trigger row.
//   4. exclusive scan over arrival order -> output offsets (reference delivery order: trigger event,
//                   then pending order within the trigger).
//   5. k_walk<WRITE> replays the units and writes one AoS match record (32 + 8*n_select bytes) per match.
//   Units whose pending list outgrows the LDS ring (or whose time span exceeds 2^31 ms) are redone by the
//   same walker with an unbounded HBM-resident list (k_walk<BIG>), so capacity never changes results.
//   6. carry (multi-push streams): per key the rows still inside the window of its last event survive into
//                   the next push, prepended as virtual rows [0, nc) that are replayed but never emit.
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

static const uint32_t F_CAND = 1, F_CONS = 2;
static const int WALK_BLOCK = 256;
static const int STACK_CAP = 16;   // LDS pending-list ring entries per lane (power of two)
static const int PF = 8;           // rows prefetched per lane per step

// ---------------------------------------------------------------------------------------------
// 1. predicate-evaluation pass.  Bitmask layout ("interleaved"): tile g = rows [256g, 256g+256),
//    word[4g+s] bit l <-> row 256g + 4l + s  (lane l evaluates rows 4l..4l+3 with one 16-B load).
__device__ __forceinline__ uint32_t mask_bit(const uint64_t* m, uint64_t r) {
  return (uint32_t)(m[(r >> 8) * 4 + (r & 3)] >> ((r >> 2) & 63)) & 1u;
}

struct PredArgs {
  int64_t n;
  const int32_t* stream;
  int32_t s_a, s_b;
  int32_t val_col_a, val_col_b;
  int32_t prog_a_off, prog_a_len, prog_b_off, prog_b_len;
  int32_t cons_all;           // B's consumers are every row: skip the second mask
  // fast path: A's program is `col CMP const` on a 4-byte column read with 16-B loads
  int32_t simple;             // 0 general VM, 1 simple
  int32_t s_col, s_type, s_op, s_dom, s_ctype;
  int64_t s_cbits;
};

struct RowReader {
  const SgCols* c;
  const int32_t* ret_col;
  int64_t row;
  __device__ SgVal read(int, int, int slot, int type) { return sg_read_col(*c, ret_col[slot], type, row); }
};

__device__ __forceinline__ bool eval_row(const PredArgs& a, const SgCols& cols, const DevDesc* dd, int64_t i,
                                         bool side_b) {
  int s = a.stream ? a.stream[i] : 0;
  int want = side_b ? a.s_b : a.s_a;
  if (s != want) return false;
  int vc = side_b ? a.val_col_b : a.val_col_a;
  if (cols.nul[vc] && cols.nul[vc][i]) return false;
  RowReader rd{&cols, dd->ret_col, i};
  return side_b ? sg_eval(dd->code + a.prog_b_off, a.prog_b_len, rd)
                : sg_eval(dd->code + a.prog_a_off, a.prog_a_len, rd);
}

// general: any program, scalar loads (rows 4l+s of the tile)
__global__ void __launch_bounds__(256) k_pred(PredArgs a, SgCols cols, const DevDesc* __restrict__ dd,
                                              uint64_t* __restrict__ cand_m, uint64_t* __restrict__ cons_m) {
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (a.n + 255) >> 8;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t g = wave; g < ntiles; g += nwaves) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      int64_t i = g * 256 + lane * 4 + s;
      bool ca = false, co = false;
      if (i < a.n) {
        ca = eval_row(a, cols, dd, i, false);
        if (!a.cons_all) co = eval_row(a, cols, dd, i, true);
      }
      uint64_t ma = __ballot(ca);
      uint64_t mb = __ballot(co);
      if (lane == s) {
        cand_m[g * 4 + s] = ma;
        if (!a.cons_all) cons_m[g * 4 + s] = mb;
      }
    }
  }
}

// simple: A = `col CMP const` on a 4-byte column, stream column absent, B consumers = all rows.
// One 16-B load per lane per tile, 4 tiles in flight per wave.
template <class V>
__global__ void __launch_bounds__(256) k_pred_simple(PredArgs a, const V* __restrict__ col,
                                                     const uint8_t* __restrict__ nul,
                                                     uint64_t* __restrict__ cand_m) {
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (a.n + 255) >> 8;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t full = a.n >> 8;   // tiles without a tail
  SgVal c = sg_val_from_bits(a.s_cbits, a.s_ctype, 0);
  for (int64_t g0 = wave; g0 < ntiles; g0 += 4 * nwaves) {
    V x[4][4];
    bool nn[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int64_t g = g0 + (int64_t)u * nwaves;
      int64_t i = g * 256 + lane * 4;
      if (g < full) {
        typedef V V4 __attribute__((ext_vector_type(4)));
        V4 q = *(const V4*)(col + i);
        x[u][0] = q.x; x[u][1] = q.y; x[u][2] = q.z; x[u][3] = q.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) x[u][s] = (g < ntiles && i + s < a.n) ? col[i + s] : V(0);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) nn[u][s] = nul ? (g < ntiles && i + s < a.n && nul[i + s]) : false;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int64_t g = g0 + (int64_t)u * nwaves;
      if (g >= ntiles) break;
      int64_t i = g * 256 + lane * 4;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        SgVal v;
        v.type = a.s_type;
        v.null = nn[u][s];
        v.i = 0;
        v.d = 0.0;
        if (a.s_type == SG_T_FLOAT) v.d = (double)(float)x[u][s];
        else v.i = (int64_t)x[u][s];
        bool ok = (i + s < a.n) && !v.null && sg_cmp(a.s_op, a.s_dom, v, c);
        uint64_t m = __ballot(ok);
        if (lane == s) cand_m[g * 4 + s] = m;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// virtual row domain: [0, nc) carried rows of earlier pushes, [nc, nc + n) this batch
struct Virt {
  int64_t nc, n;
  const int64_t* ts;
  const int32_t* key;
  const uint64_t* cand_m;
  const uint64_t* cons_m;     // null: every batch row is a B consumer
  const void* val_a;
  const void* val_b;
  const int64_t* c_ts;
  const int32_t* c_key;
  const uint8_t* c_flags;
  const void* c_val_a;
  const void* c_val_b;
};

struct KeyOf {   // sort key of virtual row r (the dense partition key; -1 sorts last)
  const int32_t* key;
  const int32_t* c_key;
  uint32_t nc;
  __host__ __device__ uint32_t operator()(uint32_t r) const {
    return (uint32_t)(r < nc ? c_key[r] : key[r - nc]);
  }
};

__device__ __forceinline__ uint32_t v_flags(const Virt& v, uint32_t r) {
  if (r < v.nc) return v.c_flags[r];
  uint64_t b = r - v.nc;
  uint32_t f = mask_bit(v.cand_m, b);
  f |= v.cons_m ? (mask_bit(v.cons_m, b) << 1) : F_CONS;
  return f;
}
__device__ __forceinline__ int64_t v_ts(const Virt& v, uint32_t r) { return r < v.nc ? v.c_ts[r] : v.ts[r - v.nc]; }
template <class T>
__device__ __forceinline__ T v_val(const Virt& v, uint32_t r, bool side_a) {
  if (r < v.nc) return ((const T*)(side_a ? v.c_val_a : v.c_val_b))[r];
  return ((const T*)(side_a ? v.val_a : v.val_b))[r - v.nc];
}

__global__ void k_bounds(const uint32_t* __restrict__ skey, int64_t n, uint32_t kb, uint32_t* __restrict__ seg_b,
                         uint32_t* __restrict__ seg_e) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t k = skey[t];
  if (k >= kb) return;
  if (t == 0 || skey[t - 1] != k) seg_b[k] = (uint32_t)t;
  if (t == n - 1 || skey[t + 1] != k) seg_e[k] = (uint32_t)(t + 1);
}

// ---------------------------------------------------------------------------------------------
struct ProjPlan {
  // per select column: src 0 = e1 row (pending partial), 1 = e2 row (trigger);
  // kind 1 = the compared value, 2 = null (chain index beyond a single-event slot), 3 = column gather
  int32_t src[SG_MAX_SELECT], kind[SG_MAX_SELECT], col[SG_MAX_SELECT], type[SG_MAX_SELECT];
};

struct UnitDesc {
  uint32_t p0, p1, w, ovf;     // chunk positions [p0, p1), replay from w; ovf = 1 + HBM-list slot
};

struct WalkStats {
  uint32_t order_err;
  uint32_t n_ovf;
  uint32_t ovf_need;
  uint32_t pad;
};

struct WalkArgs {
  int64_t nt;                 // virtual rows
  int64_t within;
  uint32_t K;                 // keys (1 if unpartitioned)
  uint32_t C;                 // time chunks
  uint32_t R;                 // virtual rows per chunk
  uint32_t n_units;
  int32_t partitioned;
  int32_t op;                 // 2 > 3 >= 4 < 5 <=
  int32_t stack_mode;         // 1: monotone stack, 0: scanned list
  int32_t carry_out;          // WRITE pass: record per-key carry suffixes
  uint64_t base_index;
  const uint64_t* index;
  int32_t multi, b_slot;
  int32_t n_select;
  int32_t stride;
  int64_t out_base;
  uint32_t big_cap;           // entries per HBM list (BIG)
};

template <class T> __device__ __forceinline__ bool is_nan_val(T) { return false; }
template <> __device__ __forceinline__ bool is_nan_val<float>(float x) { return x != x; }
template <> __device__ __forceinline__ bool is_nan_val<double>(double x) { return x != x; }

template <class T>
__device__ __forceinline__ bool cmp_op(int op, T b, T a) {   // B.x OP A.x
  switch (op) {
    case 2: return b > a;
    case 3: return b >= a;
    case 4: return b < a;
    default: return b <= a;
  }
}

template <class T> __device__ __forceinline__ int64_t val_bits(T v);
template <> __device__ __forceinline__ int64_t val_bits<float>(float v) { return (int64_t)(uint32_t)__float_as_uint(v); }
template <> __device__ __forceinline__ int64_t val_bits<double>(double v) { return __double_as_longlong(v); }
template <> __device__ __forceinline__ int64_t val_bits<int32_t>(int32_t v) { return (int64_t)v; }
template <> __device__ __forceinline__ int64_t val_bits<int64_t>(int64_t v) { return v; }

// Pending list storage.  LDS: ring of STACK_CAP entries per lane (SoA, lane-strided: conflict-free),
// timestamps relative to the unit's first replayed row.  HBM (BIG): one unbounded list per overflowed
// unit, indexed by push count (no wrap).
template <class T, bool BIG>
struct PendList {
  T* val;
  int32_t* dts;
  int64_t* ts;
  uint32_t* row;
  int64_t base;
  __device__ __forceinline__ uint32_t ix(uint32_t s) const { return BIG ? s : (s & (STACK_CAP - 1)) * WALK_BLOCK; }
  __device__ __forceinline__ T gv(uint32_t s) const { return val[ix(s)]; }
  __device__ __forceinline__ int64_t gts(uint32_t s) const { return BIG ? ts[ix(s)] : base + (int64_t)dts[ix(s)]; }
  __device__ __forceinline__ uint32_t grow(uint32_t s) const { return row[ix(s)]; }
  __device__ __forceinline__ void put(uint32_t s, T v, int64_t t, uint32_t r) {
    val[ix(s)] = v;
    if (BIG) ts[ix(s)] = t; else dts[ix(s)] = (int32_t)(t - base);
    row[ix(s)] = r;
  }
};

__device__ __forceinline__ uint32_t lb_rows(const uint32_t* rows, uint32_t lo, uint32_t hi, uint32_t target,
                                            bool part) {
  if (!part) return target < lo ? lo : (target > hi ? hi : target);
  while (lo < hi) {
    uint32_t mid = lo + ((hi - lo) >> 1);
    if (rows[mid] < target) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t lb_ts(const Virt& v, const uint32_t* rows, uint32_t lo, uint32_t hi,
                                          int64_t tmin, bool part) {
  while (lo < hi) {
    uint32_t mid = lo + ((hi - lo) >> 1);
    uint32_t r = part ? rows[mid] : mid;
    if (v_ts(v, r) < tmin) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  // blocks are dealt round-robin over the 8 XCDs: give XCD x a contiguous range of logical blocks
  uint32_t x = b & 7, i = b >> 3, per = nb >> 3, rem = nb & 7;
  return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

template <class T>
__device__ void emit_match(const WalkArgs& a, const Virt& v, const ProjPlan& pp, const SgCols& bc,
                           const SgCols& cc, char* out, int64_t slot, uint32_t ri, T vi, uint32_t rj, T vj,
                           int64_t tj, uint32_t key, uint32_t rank) {
  char* o = out + (size_t)slot * (size_t)a.stride;
  uint32_t nm = 0;
  int64_t* vals = (int64_t*)(o + 32);
  for (int s = 0; s < a.n_select; ++s) {
    int kind = pp.kind[s];
    uint32_t r = pp.src[s] ? rj : ri;
    int64_t bits = 0;
    if (kind == 1) {
      bits = val_bits<T>(pp.src[s] ? vj : vi);
    } else if (kind == 2) {
      nm |= 1u << s;
    } else {
      SgVal x = r < v.nc ? sg_read_col(cc, pp.col[s], pp.type[s], r) : sg_read_col(bc, pp.col[s], pp.type[s], r - v.nc);
      if (x.null) nm |= 1u << s;
      bits = sg_val_bits(x);
    }
    vals[s] = bits;
  }
  uint64_t b = rj - v.nc;
  uint64_t trig = a.index ? a.index[b] : a.base_index + b;
  uint64_t* h64 = (uint64_t*)o;
  h64[0] = trig;
  h64[1] = (uint64_t)tj;
  h64[2] = (uint64_t)key | ((uint64_t)((1u << 24) | (a.multi ? (uint32_t)a.b_slot : (0x800000u | rank))) << 32);
  h64[3] = (uint64_t)nm;
}

// One lane per unit (chunk c, key k).  WRITE=false: count pass (also fixes the unit's replay range);
// WRITE=true: record pass.  BIG: only units that overflowed the LDS ring, with an HBM list.
template <class T, bool WRITE, bool BIG>
__global__ void __launch_bounds__(WALK_BLOCK) k_walk(WalkArgs a, Virt v, const uint32_t* __restrict__ rows,
                                                     const uint32_t* __restrict__ seg_b,
                                                     const uint32_t* __restrict__ seg_e, UnitDesc* __restrict__ ud,
                                                     uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                                     char* __restrict__ out, ProjPlan pp, SgCols bc, SgCols cc,
                                                     WalkStats* __restrict__ st, char* __restrict__ big,
                                                     uint32_t* __restrict__ carry_q0, uint32_t* __restrict__ carry_n) {
  __shared__ char lds[BIG ? 16 : (STACK_CAP * WALK_BLOCK * (sizeof(T) + 8))];
  const uint32_t u = xcd_block(blockIdx.x, gridDim.x) * WALK_BLOCK + threadIdx.x;
  if (u >= a.n_units) return;
  const bool part = a.partitioned != 0;
  const uint32_t c = u / a.K, k = u % a.K;
  uint32_t sb, se;
  if (part) {
    sb = seg_b[k];
    se = seg_e[k];
  } else {
    sb = 0;
    se = (uint32_t)a.nt;
  }
  uint32_t p0, p1, w, ovf = 0;
  if (!WRITE && !BIG) {
    if (sb >= se) { ud[u] = UnitDesc{0, 0, 0, 0}; return; }
    uint64_t lo_row = (uint64_t)c * a.R, hi_row = lo_row + a.R;
    p0 = c == 0 ? sb : lb_rows(rows, sb, se, (uint32_t)std::min<uint64_t>(lo_row, a.nt), part);
    p1 = c + 1 >= a.C ? se : lb_rows(rows, p0, se, (uint32_t)std::min<uint64_t>(hi_row, a.nt), part);
    if (p0 >= p1) { ud[u] = UnitDesc{p0, p0, p0, 0}; return; }
    int64_t t0 = v_ts(v, part ? rows[p0] : p0);
    w = lb_ts(v, rows, sb, p0, t0 - a.within, part);
    ud[u] = UnitDesc{p0, p1, w, 0};
  } else {
    UnitDesc d = ud[u];
    p0 = d.p0; p1 = d.p1; w = d.w; ovf = d.ovf;
    if (p0 >= p1) return;
    if (BIG != (ovf != 0)) return;
  }
  PendList<T, BIG> L;
  if (BIG) {
    size_t cap = a.big_cap;
    char* base = big + (size_t)(ovf - 1) * cap * (sizeof(T) + 12);
    L.val = (T*)base;
    L.ts = (int64_t*)(base + cap * sizeof(T));
    L.row = (uint32_t*)(base + cap * (sizeof(T) + 8));
    L.dts = nullptr;
  } else {
    L.val = (T*)lds + threadIdx.x;
    L.dts = (int32_t*)(lds + STACK_CAP * WALK_BLOCK * sizeof(T)) + threadIdx.x;
    L.row = (uint32_t*)(lds + STACK_CAP * WALK_BLOCK * (sizeof(T) + 4)) + threadIdx.x;
    L.ts = nullptr;
  }
  const uint32_t rw = part ? rows[w] : w;
  const int64_t tw = v_ts(v, rw);
  L.base = tw;
  if (!BIG && !WRITE) {
    int64_t tl = v_ts(v, part ? rows[p1 - 1] : p1 - 1);
    if (tl - tw > 0x7fffffffll || tl < tw) {   // relative timestamps would not fit (or order broken)
      uint32_t slot = atomicAdd(&st->n_ovf, 1u);
      atomicMax(&st->ovf_need, p1 - w);
      ud[u].ovf = slot + 1;
      return;
    }
  }
  int64_t prev_t = (w > sb) ? v_ts(v, part ? rows[w - 1] : w - 1) : tw;
  const int64_t T_ = a.within;
  const int op = a.op;
  uint32_t head = 0, top = 0;
  bool bad = false;
  for (uint32_t p = w; p < p1; p += PF) {
    uint32_t rr[PF], ff[PF];
    int64_t tt[PF];
    T vv[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) rr[i] = (p + i < p1) ? (part ? rows[p + i] : p + i) : 0u;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      ff[i] = 0;
      if (p + i < p1) {
        ff[i] = v_flags(v, rr[i]);
        tt[i] = v_ts(v, rr[i]);
        vv[i] = v_val<T>(v, rr[i], true);
      }
    }
    if (v.val_a != v.val_b) {
#pragma unroll
      for (int i = 0; i < PF; ++i)
        if (p + i < p1 && !(ff[i] & F_CAND)) vv[i] = v_val<T>(v, rr[i], false);
    }
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      uint32_t f = ff[i];
      if (!f) continue;
      const int64_t t = tt[i];
      const T x = vv[i];
      bad |= t < prev_t;
      prev_t = t;
      // lazy `within` expiry of the oldest partials (StreamPreStateProcessor.isExpired :102-113)
      while (head != top && t - L.gts(head) > T_) ++head;
      const uint32_t r = rr[i];
      const bool emit = (p + i >= p0) && (r >= v.nc);
      if ((f & F_CONS) && !is_nan_val<T>(x)) {
        uint32_t m = 0;
        if (a.stack_mode) {
          while (top != head && cmp_op<T>(op, x, L.gv(top - 1))) { --top; ++m; }
          if (emit && m) {
            if (!WRITE) {
              cnt[r - v.nc] = m;
            } else {
              int64_t o = a.out_base + off[r - v.nc];
              for (uint32_t q = 0; q < m; ++q)
                emit_match<T>(a, v, pp, bc, cc, out, o + q, L.grow(top + q), L.gv(top + q), r, x, t, k, q);
            }
          }
        } else {
          int64_t o = (WRITE && emit) ? a.out_base + off[r - v.nc] : 0;
          uint32_t wr = head;
          for (uint32_t s = head; s != top; ++s) {
            T e = L.gv(s);
            if (cmp_op<T>(op, x, e)) {
              if (WRITE && emit) emit_match<T>(a, v, pp, bc, cc, out, o + m, L.grow(s), e, r, x, t, k, m);
              ++m;
            } else {
              if (wr != s) L.put(wr, e, L.gts(s), L.grow(s));
              ++wr;
            }
          }
          top = wr;
          if (!WRITE && emit && m) cnt[r - v.nc] = m;
        }
      }
      if ((f & F_CAND) && !is_nan_val<T>(x)) {
        if (!BIG && top - head == STACK_CAP) {
          if (!WRITE) {
            uint32_t slot = atomicAdd(&st->n_ovf, 1u);
            atomicMax(&st->ovf_need, p1 - w);
            ud[u].ovf = slot + 1;
          }
          return;   // the HBM-list walker redoes this unit
        }
        L.put(top, x, t, r);
        ++top;
      }
    }
  }
  if (bad) atomicOr(&st->order_err, 1u);
  if (WRITE && a.carry_out && p1 == se) {
    // rows of this key still inside the window of its last event survive into the next push
    int64_t tl = v_ts(v, part ? rows[se - 1] : se - 1);
    uint32_t q0 = lb_ts(v, rows, sb, se, tl - T_, part);
    carry_q0[k] = q0;
    carry_n[k] = se - q0;
  }
}

// carry copy: one lane per key copies its surviving suffix (virtual rows) into the new carry buffers
struct CarryBufs {
  int64_t* ts;
  int32_t* key;
  uint8_t* flags;
  void* col[SG_MAX_COLS];
  uint8_t* nul[SG_MAX_COLS];
};

__global__ void k_carry_copy(Virt v, const uint32_t* __restrict__ rows, int partitioned, uint32_t K,
                             const uint32_t* __restrict__ q0s, const uint32_t* __restrict__ ns,
                             const uint32_t* __restrict__ offs, int n_cols, const int32_t* __restrict__ widths,
                             SgCols bc, SgCols cc, CarryBufs dst) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  uint32_t n = ns[k];
  if (!n) return;
  uint32_t q0 = q0s[k], o = offs[k];
  for (uint32_t q = 0; q < n; ++q) {
    uint32_t r = partitioned ? rows[q0 + q] : q0 + q;
    uint32_t d = o + q;
    dst.ts[d] = v_ts(v, r);
    dst.key[d] = r < v.nc ? v.c_key[r] : (v.key ? v.key[r - v.nc] : 0);
    dst.flags[d] = (uint8_t)v_flags(v, r);
    for (int c = 0; c < n_cols; ++c) {
      const SgCols& s = r < v.nc ? cc : bc;
      uint32_t rr = r < v.nc ? r : (uint32_t)(r - v.nc);
      if (!s.col[c]) continue;
      if (widths[c] == 8) ((int64_t*)dst.col[c])[d] = ((const int64_t*)s.col[c])[rr];
      else ((int32_t*)dst.col[c])[d] = ((const int32_t*)s.col[c])[rr];
      dst.nul[c][d] = s.nul[c] ? s.nul[c][rr] : 0;
    }
  }
}

// ----------------------------------------------------------------------------------------------
struct CarrySet {
  int64_t n = 0, cap = 0;
  int64_t* ts = nullptr;
  int32_t* key = nullptr;
  uint8_t* flags = nullptr;
  void* col[SG_MAX_COLS] = {};
  uint8_t* nul[SG_MAX_COLS] = {};
  void release() {
    hipFree(ts); hipFree(key); hipFree(flags);
    for (int c = 0; c < SG_MAX_COLS; ++c) { hipFree(col[c]); hipFree(nul[c]); col[c] = nullptr; nul[c] = nullptr; }
    ts = nullptr; key = nullptr; flags = nullptr;
    n = cap = 0;
  }
  void ensure(int64_t need, int n_cols, const int32_t* col_type) {
    if (need <= cap) return;
    release();
    int64_t c = std::max<int64_t>(need + need / 4, 1024);
    auto al = [](void** p, size_t b) { if (hipMalloc(p, b) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc carry"); };
    al((void**)&ts, c * 8); al((void**)&key, c * 4); al((void**)&flags, c);
    for (int i = 0; i < n_cols; ++i) {
      al(&col[i], c * ((col_type[i] == SG_T_LONG || col_type[i] == SG_T_DOUBLE) ? 8 : 4));
      al((void**)&nul[i], c);
    }
    cap = c;
  }
};

struct EveryNextState {
  CarrySet carry[2];
  int cur = 0;
};

static int pick_chunks(uint32_t K, int64_t nt) {
  const int64_t target = 160 * 1024;   // ≈10 waves on each of 256 CUs
  int64_t C = (target + K - 1) / K;
  C = std::min<int64_t>(C, 64);
  C = std::min<int64_t>(C, std::max<int64_t>(1, nt / 512));
  return (int)std::max<int64_t>(C, 1);
}

// `col CMP const` on a 4-byte column?  (the predicate pass then streams it with 16-B loads)
static bool simple_prog(const sg_nfa_desc& d, int off, int len, PredArgs& pa) {
  if (len != 11) return false;   // VAR(5 words) CONST(3) CMP(3)
  const int64_t* c = d.code + off;
  if (c[0] != SG_OP_VAR || c[5] != SG_OP_CONST || c[8] != SG_OP_CMP) return false;
  int slot = (int)c[3], type = (int)c[4];
  if (type != SG_T_FLOAT && type != SG_T_INT) return false;
  pa.s_col = d.ret_col[slot];
  pa.s_type = type;
  pa.s_ctype = (int)c[6];
  pa.s_cbits = c[7];
  pa.s_op = (int)c[9];
  pa.s_dom = (int)c[10];
  return true;
}

template <class T>
static void run_every_next(SgHandle* h, const BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int* sa = d.shape_args;
  const int a_state = sa[0], b_state = sa[1], op = sa[2];
  EveryNextState* es = (EveryNextState*)h->state;
  CarrySet& cs = es->carry[es->cur];
  const int64_t nc = h->opt.no_carry ? 0 : cs.n;
  const int64_t nt = nc + n;
  if (nt >= (1ll << 31)) throw SgError(SG_EINVAL, "batch plus carried rows exceed 2^31");
  const int val_col_a = d.ret_col[sa[4]], val_col_b = d.ret_col[sa[3]];

  // ---- key bound
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
      kb = (uint32_t)std::max(hm + 1, 1);
    }
    if (kb < h->key_bound_seen) kb = h->key_bound_seen;
    h->key_bound_seen = kb;
  }

  // ---- 1. predicate-evaluation pass
  PredArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.n = n;
  pa.stream = bv.stream;
  pa.s_a = d.states[a_state].stream;
  pa.s_b = d.states[b_state].stream;
  pa.val_col_a = val_col_a;
  pa.val_col_b = val_col_b;
  pa.prog_a_off = d.states[a_state].prog_off;
  pa.prog_a_len = d.states[a_state].prog_len;
  pa.prog_b_off = d.shape_prog_off;
  pa.prog_b_len = d.shape_prog_len;
  pa.cons_all = (!bv.stream && pa.s_b == 0 && pa.prog_b_len == 0 && !bv.cols.nul[val_col_b]) ? 1 : 0;
  const int64_t ntiles = (n + 255) / 256;
  uint64_t* cand_m = (uint64_t*)h->ws.get("cand_m", sizeof(uint64_t) * 4 * (ntiles + 1), st);
  uint64_t* cons_m = pa.cons_all ? nullptr : (uint64_t*)h->ws.get("cons_m", sizeof(uint64_t) * 4 * (ntiles + 1), st);
  h->mark(0);
  {
    PredArgs sp = pa;
    bool simple = pa.cons_all && !bv.stream && pa.s_a == 0 && simple_prog(d, pa.prog_a_off, pa.prog_a_len, sp) &&
                  sp.s_col == val_col_a && (((uintptr_t)bv.cols.col[sp.s_col]) & 15) == 0;
    int64_t waves = std::min<int64_t>((ntiles + 3) / 4, 256 * 16);
    dim3 grd((unsigned)std::max<int64_t>(1, (waves + 3) / 4)), blk(256);
    if (simple && sp.s_type == SG_T_FLOAT)
      hipLaunchKernelGGL(k_pred_simple<float>, grd, blk, 0, st, sp, (const float*)bv.cols.col[sp.s_col],
                         bv.cols.nul[sp.s_col], cand_m);
    else if (simple)
      hipLaunchKernelGGL(k_pred_simple<int32_t>, grd, blk, 0, st, sp, (const int32_t*)bv.cols.col[sp.s_col],
                         bv.cols.nul[sp.s_col], cand_m);
    else {
      int64_t w2 = std::min<int64_t>(ntiles, 256 * 16);
      hipLaunchKernelGGL(k_pred, dim3((unsigned)std::max<int64_t>(1, (w2 + 3) / 4)), blk, 0, st, pa, bv.cols,
                         h->ddesc, cand_m, cons_m);
    }
    HIPCHK(hipGetLastError());
  }
  h->mark(1);

  // ---- 2. key partition: per-key row lists in arrival order
  Virt v;
  v.nc = nc;
  v.n = n;
  v.ts = bv.ts;
  v.key = bv.key;
  v.cand_m = cand_m;
  v.cons_m = cons_m;
  v.val_a = bv.cols.col[val_col_a];
  v.val_b = bv.cols.col[val_col_b];
  v.c_ts = cs.ts;
  v.c_key = cs.key;
  v.c_flags = cs.flags;
  v.c_val_a = cs.col[val_col_a];
  v.c_val_b = cs.col[val_col_b];
  SgCols cc;
  memset(&cc, 0, sizeof(cc));
  for (int c = 0; c < d.n_cols; ++c) { cc.col[c] = cs.col[c]; cc.nul[c] = cs.nul[c]; }

  const uint32_t K = d.partitioned ? kb : 1;
  uint32_t* rows = nullptr;
  uint32_t* seg_b = nullptr;
  uint32_t* seg_e = nullptr;
  if (d.partitioned) {
    int end_bit = 1;
    while ((1ull << end_bit) <= (uint64_t)kb) ++end_bit;
    uint32_t* skeys = (uint32_t*)h->ws.get("skeys", sizeof(uint32_t) * nt, st);
    rows = (uint32_t*)h->ws.get("rows", sizeof(uint32_t) * nt, st);
    KeyOf kf{bv.key, cs.key, (uint32_t)nc};
    auto kit = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0), kf);
    auto vit = rocprim::make_counting_iterator<uint32_t>(0);
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, kit, skeys, vit, rows, (size_t)nt, 0, end_bit, st));
    void* tmp = h->ws.get("sort_tmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, kit, skeys, vit, rows, (size_t)nt, 0, end_bit, st));
    seg_b = (uint32_t*)h->ws.get("seg_b", sizeof(uint32_t) * K, st);
    seg_e = (uint32_t*)h->ws.get("seg_e", sizeof(uint32_t) * K, st);
    HIPCHK(hipMemsetAsync(seg_b, 0, sizeof(uint32_t) * K, st));
    HIPCHK(hipMemsetAsync(seg_e, 0, sizeof(uint32_t) * K, st));
    hipLaunchKernelGGL(k_bounds, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, skeys, nt, kb, seg_b, seg_e);
    HIPCHK(hipGetLastError());
  }
  h->mark(2);

  // ---- 3. count pass + scan
  WalkArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.nt = nt;
  wa.within = d.within;
  wa.K = K;
  wa.C = (uint32_t)pick_chunks(K, nt);
  wa.R = (uint32_t)((nt + wa.C - 1) / wa.C);
  const uint64_t units = (uint64_t)K * wa.C;
  if (units >= (1ull << 32)) throw SgError(SG_EINVAL, "too many (key, chunk) units");
  wa.n_units = (uint32_t)units;
  wa.partitioned = d.partitioned;
  wa.op = op;
  const bool same_col = (val_col_a == val_col_b) && (pa.s_a == pa.s_b);
  wa.stack_mode = (same_col && pa.prog_b_len == 0) ? 1 : 0;
  wa.carry_out = h->opt.no_carry ? 0 : 1;
  wa.base_index = bv.base_index;
  wa.index = bv.index;
  int rb = d.recv_of_stream[d.states[b_state].stream];
  wa.multi = d.receivers[rb].multi;
  wa.b_slot = 0;
  if (wa.multi) {
    const sg_receiver_desc& r = d.receivers[rb];
    for (int q = 0; q < r.n; ++q)
      if (r.pres[r.n - 1 - q] == b_state) wa.b_slot = q;   // eventSequence = reversed init order
  }
  wa.n_select = d.n_select;
  wa.stride = 32 + 8 * d.n_select;
  ProjPlan pp;
  memset(&pp, 0, sizeof(pp));
  for (int s = 0; s < d.n_select; ++s) {
    int stt = d.sel_state[s];
    pp.src[s] = (stt == b_state) ? 1 : 0;
    int col = d.ret_col[d.sel_ret[s]];
    int idx = d.sel_index[s];
    pp.col[s] = col;
    pp.type[s] = d.sel_type[s];
    if (idx != 0 && idx != -1) pp.kind[s] = 2;
    else if (col == (pp.src[s] ? val_col_b : val_col_a)) pp.kind[s] = 1;
    else pp.kind[s] = 3;
  }

  UnitDesc* ud = (UnitDesc*)h->ws.get("units", sizeof(UnitDesc) * units, st);
  WalkStats* wst = (WalkStats*)h->ws.get("walkstats", sizeof(WalkStats), st);
  uint32_t* cnt = (uint32_t*)h->ws.get("cnt", sizeof(uint32_t) * (n + 1), st);
  uint32_t* off = (uint32_t*)h->ws.get("off", sizeof(uint32_t) * (n + 1), st);
  uint32_t* carry_q0 = (uint32_t*)h->ws.get("carry_q0", sizeof(uint32_t) * K, st);
  uint32_t* carry_n = (uint32_t*)h->ws.get("carry_n", sizeof(uint32_t) * (K + 1), st);
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (n + 1), st));
  HIPCHK(hipMemsetAsync(wst, 0, sizeof(WalkStats), st));
  if (wa.carry_out) HIPCHK(hipMemsetAsync(carry_n, 0, sizeof(uint32_t) * (K + 1), st));
  const dim3 wblk(WALK_BLOCK), wgrd((unsigned)((units + WALK_BLOCK - 1) / WALK_BLOCK));
  hipLaunchKernelGGL((k_walk<T, false, false>), wgrd, wblk, 0, st, wa, v, rows, seg_b, seg_e, ud, cnt, off,
                     (char*)nullptr, pp, bv.cols, cc, wst, (char*)nullptr, carry_q0, carry_n);
  HIPCHK(hipGetLastError());
  auto scan_counts = [&]() {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
  };
  scan_counts();
  h->mark(3);
  WalkStats hs;
  uint32_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&hs, wst, sizeof(WalkStats), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  char* big = nullptr;
  h->extra_marks = 0;
  if (hs.n_ovf) {
    // units whose pending list outgrew the LDS ring: redo them with unbounded HBM lists
    wa.big_cap = (std::max<uint32_t>(hs.ovf_need, 1) + 1) & ~1u;
    big = (char*)h->ws.get("big_lists", (size_t)hs.n_ovf * wa.big_cap * (sizeof(T) + 12), st);
    h->mark(6);
    hipLaunchKernelGGL((k_walk<T, false, true>), wgrd, wblk, 0, st, wa, v, rows, seg_b, seg_e, ud, cnt, off,
                       (char*)nullptr, pp, bv.cols, cc, wst, big, carry_q0, carry_n);
    HIPCHK(hipGetLastError());
    scan_counts();
    h->mark(7);
    h->extra_marks = 1;
    HIPCHK(hipMemcpyAsync(&total, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&hs, wst, sizeof(WalkStats), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  if (hs.order_err) throw SgError(SG_EORDER, "closed-form kernel requires non-decreasing timestamps per key");

  // ---- 5. record pass
  char* out = nullptr;
  h->split_out = 1;
  if (!(total || wa.carry_out)) h->mark(5);
  if (total || wa.carry_out) {
    out = h->out.reserve(total, d.n_select, st);
    wa.out_base = h->out.n;
    h->mark(5);
    hipLaunchKernelGGL((k_walk<T, true, false>), wgrd, wblk, 0, st, wa, v, rows, seg_b, seg_e, ud, cnt, off, out,
                       pp, bv.cols, cc, wst, (char*)nullptr, carry_q0, carry_n);
    HIPCHK(hipGetLastError());
    if (hs.n_ovf) {
      hipLaunchKernelGGL((k_walk<T, true, true>), wgrd, wblk, 0, st, wa, v, rows, seg_b, seg_e, ud, cnt, off, out,
                         pp, bv.cols, cc, wst, big, carry_q0, carry_n);
      HIPCHK(hipGetLastError());
    }
    h->out.n += total;
  }
  h->mark(4);

  // ---- 6. carry into the next push
  if (wa.carry_out) {
    uint32_t* coff = (uint32_t*)h->ws.get("carry_off", sizeof(uint32_t) * (K + 1), st);
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, carry_n, coff, (uint32_t)0, (size_t)K + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("carry_scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, carry_n, coff, (uint32_t)0, (size_t)K + 1, rocprim::plus<uint32_t>(), st));
    uint32_t ncar = 0;
    HIPCHK(hipMemcpyAsync(&ncar, coff + K, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    CarrySet& nx = es->carry[es->cur ^ 1];
    nx.ensure(std::max<int64_t>(ncar, 1), d.n_cols, d.col_type);
    int32_t* widths = (int32_t*)h->ws.get("col_widths", sizeof(int32_t) * SG_MAX_COLS, st);
    int32_t hw[SG_MAX_COLS];
    for (int c = 0; c < SG_MAX_COLS; ++c)
      hw[c] = (c < d.n_cols && (d.col_type[c] == SG_T_LONG || d.col_type[c] == SG_T_DOUBLE)) ? 8 : 4;
    HIPCHK(hipMemcpyAsync(widths, hw, sizeof(hw), hipMemcpyHostToDevice, st));
    CarryBufs cb;
    memset(&cb, 0, sizeof(cb));
    cb.ts = nx.ts;
    cb.key = nx.key;
    cb.flags = nx.flags;
    for (int c = 0; c < d.n_cols; ++c) { cb.col[c] = nx.col[c]; cb.nul[c] = nx.nul[c]; }
    if (ncar)
      hipLaunchKernelGGL(k_carry_copy, dim3((K + 255) / 256), dim3(256), 0, st, v, rows, d.partitioned, K, carry_q0,
                         carry_n, coff, d.n_cols, widths, bv.cols, cc, cb);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    nx.n = ncar;
    cs.n = 0;
    es->cur ^= 1;
  }
  h->last_events = n;
  h->last_matches = total;
}

void sg_run_every_next(SgHandle* h, const BatchView& bv, int64_t n) {
  if (!h->state) { h->state = new EveryNextState(); h->state_kind = 1; }
  const sg_nfa_desc& d = h->desc;
  switch (d.shape_args[5]) {
    case SG_T_FLOAT: run_every_next<float>(h, bv, n); break;
    case SG_T_DOUBLE: run_every_next<double>(h, bv, n); break;
    case SG_T_LONG: run_every_next<int64_t>(h, bv, n); break;
    default: run_every_next<int32_t>(h, bv, n); break;
  }
}

void sg_every_next_reset(SgHandle* h) {
  if (h->state && h->state_kind == 1) {
    EveryNextState* es = (EveryNextState*)h->state;
    es->carry[0].n = 0;
    es->carry[1].n = 0;
  }
  h->key_bound_seen = 0;
}

void sg_every_next_release(SgHandle* h) {
  if (h->state_kind != 1) return;
  EveryNextState* es = (EveryNextState*)h->state;
  es->carry[0].release();
  es->carry[1].release();
  delete es;
  h->state = nullptr;
  h->state_kind = 0;
}
