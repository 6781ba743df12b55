#pragma once
// engine_impl.h — MI355X closed-form pipeline for  every A[l] -> B[l' and B.x OP A.x] within T
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
//   6. carry (multi-push streams): per key its final pending list -- the reference's whole state for the key
//                   (the `every` start state holds nothing) -- survives into the next push as candidate-only virtual
//                   rows [0, nc), replayed (re-appended in pending order) but never emitting.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <limits>
#include <type_traits>
#include <cstdio>
#include <string>
#include <vector>

#include "sg_device.h"
#include "sg_engine.h"

// (instantiated per value type by engine_{f32,f64,i32,i64}.hip so the build parallelises)

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static const uint32_t F_CAND = 1, F_CONS = 2;
static const int WALK_BLOCK = 256;
static const int STACK_CAP = 16;   // default LDS pending-list ring entries per lane (runtime: 16/32/64)
static const int PF = 8;           // rows prefetched per lane per step

#include "pred.h"

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
  const void* pcol;           // e1 payload column (one projected attribute carried in the pending list)
  const void* c_pcol;
  int32_t pw, pfloat;         // width 4/8; FLOAT bits zero-extended, integral sign-extended
  const int32_t* stream;      // batch stream column (null: every row is stream 0)
  int32_t s_b;                // B's stream: its rows visit e2's pending list (expiry), whatever their filters say
};

struct KeyOf {   // sort key of virtual row r (the dense partition key; -1 sorts last)
  const int32_t* key;
  const int32_t* c_key;
  uint32_t nc;
  __host__ __device__ uint32_t operator()(uint32_t r) const {
    return (uint32_t)(r < nc ? c_key[r] : key[r - nc]);
  }
};

// carried rows keep F_CAND / F_CONS in bits 0-1 and F_VISIT (a row of B's stream) in bit 2
static const uint32_t F_VISIT = 4;
__device__ __forceinline__ uint32_t v_flags(const Virt& v, uint32_t r) {
  if (r < v.nc) return v.c_flags[r] & 3u;
  uint64_t b = r - v.nc;
  uint32_t f = mask_bit(v.cand_m, b);
  f |= v.cons_m ? (mask_bit(v.cons_m, b) << 1) : F_CONS;
  return f;
}
// Does virtual row r visit e2's pending list?  Every row of B's stream does (MultiProcessStreamReceiver.receive ->
// StreamPreStateProcessor.processAndReturn, C/query/input/stream/state/StreamPreStateProcessor.java:292-337): its
// `within` expiry applies whether or not the row passes a filter.
__device__ __forceinline__ bool v_visit(const Virt& v, uint32_t r) {
  if (r < v.nc) return (v.c_flags[r] & F_VISIT) != 0;
  return (v.stream ? v.stream[r - v.nc] : 0) == v.s_b;
}
__device__ __forceinline__ int64_t v_ts(const Virt& v, uint32_t r) { return r < v.nc ? v.c_ts[r] : v.ts[r - v.nc]; }
template <class T>
__device__ __forceinline__ T v_val(const Virt& v, uint32_t r, bool side_a) {
  if (r < v.nc) return ((const T*)(side_a ? v.c_val_a : v.c_val_b))[r];
  return ((const T*)(side_a ? v.val_a : v.val_b))[r - v.nc];
}

__device__ __forceinline__ int64_t v_payload(const Virt& v, uint32_t r) {
  const void* c = r < v.nc ? v.c_pcol : v.pcol;
  uint32_t rr = r < v.nc ? r : (uint32_t)(r - v.nc);
  if (v.pw == 8) return ((const int64_t*)c)[rr];
  int32_t x = ((const int32_t*)c)[rr];
  return v.pfloat ? (int64_t)(uint32_t)x : (int64_t)x;
}

// Walker record: one row of one key as the walkers read it (key-sorted for partitioned queries).
// rowf = virtual row | condition flags << 30.  Narrow format (default): time as a 32-bit offset from the
// push's first virtual row, plus (4-byte values) e1's payload attribute in 32 bits -- 16 bytes, rocPRIM's
// tuned 8-bit-digit onesweep path and 8 records per 128-B line.  Wide format (fallback when a push spans
// more than 2^31 ms): 64-bit time, no payload.
static const uint32_t ROW_MASK = 0x3fffffffu;
template <class T, bool N, int S = (int)sizeof(T)>
struct WRec {   // wide
  int64_t ts;
  uint32_t rowf;
  T val;
  static constexpr bool has_pay = false;
  static constexpr bool narrow = false;
  __host__ __device__ int64_t t() const { return ts; }
  __host__ __device__ int64_t p(int) const { return 0; }
};
template <class T>
struct WRec<T, true, 4> {   // narrow, 4-byte value: room for a 32-bit payload
  int32_t dts;
  uint32_t rowf;
  T val;
  int32_t pay;
  static constexpr bool has_pay = true;
  static constexpr bool narrow = true;
  __host__ __device__ int64_t t() const { return dts; }
  __host__ __device__ int64_t p(int pzero) const { return pzero ? (int64_t)(uint32_t)pay : (int64_t)pay; }
};
template <class T>
struct WRec<T, true, 8> {   // narrow, 8-byte value
  int32_t dts;
  uint32_t rowf;
  T val;
  static constexpr bool has_pay = false;
  static constexpr bool narrow = true;
  __host__ __device__ int64_t t() const { return dts; }
  __host__ __device__ int64_t p(int) const { return 0; }
};
struct alignas(16) Blob16 { uint32_t w[4]; };   // 16-byte records sort as one opaque type

static const uint32_t PK_TS_RANGE = 1, PK_PAY_RANGE = 2, PK_KEY_RANGE = 4, PK_INTERNAL = 8;   // k_pack flags

template <class T, bool N>
struct PackFn {   // builds the walker record of virtual row r (coalesced when r is sequential)
  Virt v;
  __host__ __device__ WRec<T, N> operator()(uint32_t r) const {
    WRec<T, N> o;
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t f = v_flags(v, r);
    if constexpr (N) {
      o.dts = (int32_t)(v_ts(v, r) - v_ts(v, 0));
      if constexpr (WRec<T, N>::has_pay) o.pay = v.pcol ? (int32_t)v_payload(v, r) : 0;
    } else {
      o.ts = v_ts(v, r);
    }
    o.rowf = r | (f << 30);
    o.val = v_val<T>(v, r, (f & F_CAND) || v.val_a == v.val_b);
#else
    (void)r;
    memset(&o, 0, sizeof(o));
#endif
    return o;
  }
  // batch row b (virtual row nc + b) without the carried-row branches, so a run of rows issues its loads
  // back to back; also flags a time / payload outside the narrow format's 32 bits
  __device__ __forceinline__ WRec<T, N> batch(uint32_t b, int64_t t0, uint32_t& bad) const {
    WRec<T, N> o;
    uint32_t f = mask_bit(v.cand_m, b);
    f |= v.cons_m ? (mask_bit(v.cons_m, b) << 1) : F_CONS;
    const int64_t ts = v.ts[b];
    if constexpr (N) {
      const int64_t dt = ts - t0;
      bad |= (dt != (int64_t)(int32_t)dt) ? PK_TS_RANGE : 0u;
      o.dts = (int32_t)dt;
      if constexpr (WRec<T, N>::has_pay) {
        int64_t pv = 0;
        if (v.pcol) {   // (uniform)
          if (v.pw == 8) {
            pv = ((const int64_t*)v.pcol)[b];
            bad |= (pv != (int64_t)(int32_t)pv) ? PK_PAY_RANGE : 0u;
          } else {
            pv = ((const int32_t*)v.pcol)[b];
          }
        }
        o.pay = (int32_t)pv;
      }
    } else {
      o.ts = ts;
    }
    o.rowf = (uint32_t)(v.nc + b) | (f << 30);
    const T* src = ((f & F_CAND) || v.val_a == v.val_b) ? (const T*)v.val_a : (const T*)v.val_b;
    o.val = src[b];
    return o;
  }
};

template <class T, bool N>
struct Src {   // position -> record: the key-sorted records, or (unpartitioned) the rows themselves
  const WRec<T, N>* srec;
  PackFn<T, N> pk;
  __device__ __forceinline__ WRec<T, N> at(uint32_t p) const { return srec ? srec[p] : pk(p); }
  __device__ __forceinline__ uint32_t row(uint32_t p) const { return srec ? (srec[p].rowf & ROW_MASK) : p; }
  __device__ __forceinline__ int64_t ts(uint32_t p) const { return srec ? srec[p].t() : pk(p).t(); }
};

// Records per group load: G records = a whole number of 128-B lines, loaded by one lane at once so a
// line is fetched into registers exactly once (thousands of per-lane streams would otherwise thrash L2).
template <class T, bool N>
struct Grp {
  static constexpr int G = sizeof(WRec<T, N>) == 16 ? 8 : 16;
  static constexpr int QW = G * (int)sizeof(WRec<T, N>) / 16;
  typedef uint32_t U4 __attribute__((ext_vector_type(4)));
  U4 q[QW];
  __device__ __forceinline__ void load(const WRec<T, N>* base) {
    const U4* p = (const U4*)base;
#pragma unroll
    for (int j = 0; j < QW; ++j) q[j] = __builtin_nontemporal_load(p + j);
  }
  __device__ __forceinline__ WRec<T, N> rec(int i) const {
    WRec<T, N> r;
    __builtin_memcpy(&r, (const char*)q + i * sizeof(WRec<T, N>), sizeof(WRec<T, N>));
    return r;
  }
};

// walker records + sort keys of every virtual row, in arrival order (coalesced).  Narrow records flag a
// time outside +-2^31 ms of the first virtual row, or a payload that does not fit 32 bits.
template <class T, bool N>
__global__ void __launch_bounds__(256) k_pack(PackFn<T, N> pk, KeyOf kf, uint32_t kbound, int64_t nt,
                                              WRec<T, N>* __restrict__ rec, uint32_t* __restrict__ keys,
                                              uint32_t* __restrict__ flags) {
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t bad = 0;
  const int64_t t0 = N ? v_ts(pk.v, 0) : 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nt; r += stride) {
    rec[r] = pk((uint32_t)r);
    if (keys) {
      const uint32_t kk = kf((uint32_t)r);
      if (kk >= kbound && kk != 0xffffffffu) bad |= PK_KEY_RANGE;   // beyond the caller's key_bound
      keys[r] = kk;
    }
    if (N) {
      const int64_t d = v_ts(pk.v, (uint32_t)r) - t0;
      if (d != (int64_t)(int32_t)d) bad |= PK_TS_RANGE;
      if (WRec<T, N>::has_pay && pk.v.pcol && pk.v.pw == 8) {
        const int64_t pv = v_payload(pk.v, (uint32_t)r);
        if (pv != (int64_t)(int32_t)pv) bad |= PK_PAY_RANGE;
      }
    }
  }
  if (bad) atomicOr(flags, bad);
}

static __global__ void __launch_bounds__(256) k_bounds(const uint32_t* __restrict__ skey, int64_t n, uint32_t kb,
                                                       uint32_t* __restrict__ seg_b, uint32_t* __restrict__ seg_e) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t t0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; t0 < n; t0 += stride) {
    uint32_t k[6];
    k[0] = t0 > 0 ? skey[t0 - 1] : 0xffffffffu;
#pragma unroll
    for (int j = 0; j < 5; ++j) k[j + 1] = (t0 + j < n) ? skey[t0 + j] : 0xfffffffeu;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t t = t0 + j;
      uint32_t x = k[j + 1];
      if (t >= n || x >= kb) continue;
      if (k[j] != x) seg_b[x] = (uint32_t)t;
      if (k[j + 2] != x) seg_e[x] = (uint32_t)(t + 1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 2'. Key partition without a general sort (K <= 65536).  A stable MSD counting sort in one pass (K <= 256:
// digit = key) or two (digit = key group = high bits, then key within its group = low bits).  Each pass
// cuts its input into segments; a histogram kernel counts digits per segment, one exclusive scan over the
// (digit, segment) table gives every segment's output position per digit, and the scatter kernel ranks each
// 2048-row sub-tile stably by digit in LDS (wave ballots over the digit bits) and writes every digit run out
// as whole lines.  Pass 1 reads the raw columns and builds the walker records on the way (no pack pass);
// pass 2 reads pass 1's records and 1-byte in-group keys.  The per-key segments are read off the last
// pass's offsets (no bounds pass).  Same result as the radix sort: per key its rows in arrival order.
// Rows per thread per LDS-staged sub-tile, per pass (measured on C2, 100M events / 10k keys: pass 1 -- raw columns in,
// 16-B records out, 79 key-group digits -- is fastest with 1024-row sub-tiles (more resident workgroups: part_group
// 1.26 -> 1.04 ms); pass 2 -- records in, 128 in-group digits -- with 4096-row ones (longer runs per digit: part_key
// 0.90 -> 0.78 ms))
#ifndef SG_PT1
#define SG_PT1 4
#endif
#ifndef SG_PT2
#define SG_PT2 16
#endif
static const int PT1 = SG_PT1, PT1_ROWS = 256 * SG_PT1;
static const int PT2 = SG_PT2, PT2_ROWS = 256 * SG_PT2;
static const int PT_D = 256;       // digit values per pass (8 bits)

struct PartPlan {
  uint32_t K, lb, ng, two;    // keys; pass-2 digit bits (key & (2^lb - 1)); pass-1 digit values (key >> lb); 2 passes?
  uint32_t nb1, nb2;          // bits that tell the digits apart (ballots per 64-row step)
  uint32_t seg1, ns1;         // rows per pass-1 segment (multiple of PT1_ROWS); pass-1 segments
  uint32_t ts2, nj;           // pass-1 segments per pass-2 segment; pass-2 segments per group
};

template <class R, int PT, class TG = uint16_t>
struct PartLds {
  R stage[256 * PT];          // the sub-tile's records, sorted by digit
  TG tag[256 * PT];           // key (pass 1) / in-group key (pass 2) of each staged record
  uint32_t cw[4][PT_D];       // per-wave digit counts, then per-wave slot cursors
  uint32_t ls[PT_D];          // sub-tile start of each digit
  uint32_t tot[PT_D];         // sub-tile count of each digit
  uint32_t run[PT_D];         // next output position of each digit
  uint32_t wsum[4];
};

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t x, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t add = 0;
  for (int i = 0; i < w; ++i) add += wsum[i];
  return add + inc - x;
}

// lanes of the wave holding the same digit: rank among them (arrival order) and their count
__device__ __forceinline__ void peer_rank(bool valid, uint32_t d, uint32_t nb, uint32_t& rank, uint32_t& cnt) {
  uint64_t m = __ballot(valid);
  for (uint32_t b = 0; b < nb; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bb = __ballot(bit);
    m &= bit ? bb : ~bb;
  }
  rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  cnt = (uint32_t)__popcll(m);
}

// digit counts -> per-wave slot cursors and sub-tile digit starts; returns the sub-tile's staged rows
template <class R, int PT, class TG>
__device__ __forceinline__ uint32_t part_cursors(PartLds<R, PT, TG>& L) {
  const uint32_t t = threadIdx.x;
  const uint32_t c0 = L.cw[0][t], c1 = L.cw[1][t], c2 = L.cw[2][t], c3 = L.cw[3][t];
  const uint32_t tot = c0 + c1 + c2 + c3;
  const uint32_t ex = block_excl_scan256(tot, L.wsum);
  L.ls[t] = ex;
  L.tot[t] = tot;
  L.cw[0][t] = ex;
  L.cw[1][t] = ex + c0;
  L.cw[2][t] = ex + c0 + c1;
  L.cw[3][t] = ex + c0 + c1 + c2;
  __syncthreads();
  return L.ls[PT_D - 1] + L.tot[PT_D - 1];
}

// pass-1 histogram: segment j = virtual rows [j*seg1, (j+1)*seg1); h1[group * ns1 + j].  Per-wave counters
// (fewer same-address LDS atomics), eight rows per thread in flight.
static __global__ void __launch_bounds__(256) k_part1_hist(KeyOf kf, PartPlan pp, int64_t nt, uint32_t* __restrict__ h1,
                                                           uint32_t* __restrict__ flags) {
  __shared__ uint32_t cnt[4][PT_D];
  const uint32_t j = blockIdx.x, t = threadIdx.x, w = t >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) cnt[q][t] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)j * pp.seg1, r1 = (nt < r0 + pp.seg1) ? nt : r0 + pp.seg1;
  uint32_t bad = 0;
  for (int64_t rb = r0; rb < r1; rb += 256 * 8) {
    uint32_t k[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int64_t r = rb + s * 256 + t;
      k[s] = r < r1 ? kf((uint32_t)r) : 0xffffffffu;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (k[s] < pp.K) atomicAdd(&cnt[w][k[s] >> pp.lb], 1u);
      else if (k[s] != 0xffffffffu) bad |= PK_KEY_RANGE;   // beyond the caller's key_bound
    }
  }
  __syncthreads();
  if (t < pp.ng) h1[(size_t)t * pp.ns1 + j] = cnt[0][t] + cnt[1][t] + cnt[2][t] + cnt[3][t];
  if (bad) atomicOr(flags, bad);
}

// pass-1 scatter: records of segment j, grouped (two passes) or final (one pass).  TG holds a staged record's key
// (32 bits beyond 65536 keys), LK its in-group key.
template <class T, bool N, class TG = uint16_t, class LK = uint8_t, int P = PT1>
__global__ void __launch_bounds__(256) k_part1(PackFn<T, N> pk, KeyOf kf, PartPlan pp, int64_t nt,
                                               const uint32_t* __restrict__ o1, WRec<T, N>* __restrict__ orec,
                                               LK* __restrict__ olk, uint32_t* __restrict__ flags) {
  typedef WRec<T, N> R;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  PartLds<R, P, TG>& L = *(PartLds<R, P, TG>*)lds_raw;
  constexpr uint32_t PROWS = 256 * P;
  const uint32_t j = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t lmask = (1u << pp.lb) - 1u;
  if (t < pp.ng) L.run[t] = o1[(size_t)t * pp.ns1 + j];
  const int64_t rb = (int64_t)j * pp.seg1, re = (nt < rb + pp.seg1) ? nt : rb + pp.seg1;
  const int64_t t0 = N ? v_ts(pk.v, 0) : 0;
  uint32_t bad = 0;
  // the sub-tile's loads, all issued before the first use (one memory latency per sub-tile)
  auto load = [&](int64_t base, uint32_t* tg, R* rc) {
    const uint32_t rows = (uint32_t)((re - base < PROWS) ? re - base : PROWS);
    if (base >= (int64_t)pk.v.nc) {
      // batch rows only: branch-free loads (rows past the end re-read the last row and are dropped)
      const uint32_t b0 = (uint32_t)(base - pk.v.nc), last = rows - 1;
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const uint32_t i = w * (P * 64) + s * 64 + lane;
        const uint32_t b = b0 + (i < rows ? i : last);
        const uint32_t k = (uint32_t)pk.v.key[b];
        uint32_t bd = 0;
        rc[s] = pk.batch(b, t0, bd);
        tg[s] = (i < rows && k < pp.K) ? k : 0xffffffffu;
        bad |= (i < rows && k != 0xffffffffu) ? bd : 0u;
      }
    } else {
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const uint32_t i = w * (P * 64) + s * 64 + lane;
        const uint32_t r = (uint32_t)(base + i);
        const uint32_t k = i < rows ? kf(r) : 0xffffffffu;
        tg[s] = k < pp.K ? k : 0xffffffffu;
        if (k < pp.K) {
          rc[s] = pk(r);
          if (N) {
            const int64_t dt = v_ts(pk.v, r) - t0;
            if (dt != (int64_t)(int32_t)dt) bad |= PK_TS_RANGE;
            if (R::has_pay && pk.v.pcol && pk.v.pw == 8) {
              const int64_t pv = v_payload(pk.v, r);
              if (pv != (int64_t)(int32_t)pv) bad |= PK_PAY_RANGE;
            }
          }
        }
      }
    }
  };
  uint32_t tg[P], tn[P];
  R rc[P], rn[P];
  if (rb < re) load(rb, tg, rc);
  for (int64_t base = rb; base < re; base += PROWS) {
#pragma unroll
    for (int q = 0; q < 4; ++q) L.cw[q][t] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (tg[s] != 0xffffffffu) atomicAdd(&L.cw[w][tg[s] >> pp.lb], 1u);
    __syncthreads();
    const uint32_t staged = part_cursors(L);
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const bool valid = tg[s] != 0xffffffffu;
      const uint32_t d = valid ? tg[s] >> pp.lb : 0u;
      uint32_t rank, cnt;
      peer_rank(valid, d, pp.nb1, rank, cnt);
      if (valid) {
        const uint32_t slot = L.cw[w][d] + rank;
        if (rank == 0) L.cw[w][d] = slot + cnt;
        L.stage[slot] = rc[s];
        L.tag[slot] = (TG)tg[s];
      }
    }
    if (base + PROWS < re) load(base + PROWS, tn, rn);   // next sub-tile in flight during the write-out
    __syncthreads();
    for (uint32_t q = t; q < staged; q += 256) {
      const uint32_t k = L.tag[q], d = k >> pp.lb;
      const uint32_t dst = L.run[d] + q - L.ls[d];
      if ((int64_t)dst >= nt) { bad |= PK_INTERNAL; continue; }
      orec[dst] = L.stage[q];
      if (olk) olk[dst] = (LK)(k & lmask);
    }
    __syncthreads();
    L.run[t] += L.tot[t];
#pragma unroll
    for (int s = 0; s < P; ++s) { tg[s] = tn[s]; rc[s] = rn[s]; }
  }
  if (bad) atomicOr(flags, bad);
}

// pass-2 segment (g, jj): group g's rows that came from pass-1 segments [jj*ts2, (jj+1)*ts2)
__device__ __forceinline__ void part2_range(const PartPlan& pp, const uint32_t* o1, uint32_t g, uint32_t jj,
                                            uint32_t& lo, uint32_t& hi) {
  lo = o1[(size_t)g * pp.ns1 + jj * pp.ts2];
  hi = o1[(size_t)g * pp.ns1 + min(pp.ns1, (jj + 1) * pp.ts2)];
}

static __global__ void __launch_bounds__(256) k_part2_hist(PartPlan pp, const uint32_t* __restrict__ o1,
                                                           const uint8_t* __restrict__ glk, uint32_t* __restrict__ h2) {
  __shared__ uint32_t cnt[4][PT_D];
  const uint32_t g = blockIdx.x / pp.nj, jj = blockIdx.x % pp.nj, t = threadIdx.x, w = t >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) cnt[q][t] = 0;
  __syncthreads();
  uint32_t lo, hi;
  part2_range(pp, o1, g, jj, lo, hi);
  for (uint32_t pb = lo; pb < hi; pb += 256 * 8) {
    uint32_t d[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t p = pb + s * 256 + t;
      d[s] = p < hi ? (uint32_t)glk[p] : 0xffffffffu;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (d[s] != 0xffffffffu) atomicAdd(&cnt[w][d[s]], 1u);
  }
  __syncthreads();
  if (t < (1u << pp.lb)) h2[(size_t)((g << pp.lb) + t) * pp.nj + jj] = cnt[0][t] + cnt[1][t] + cnt[2][t] + cnt[3][t];
}

template <class R>
__global__ void __launch_bounds__(256) k_part2(PartPlan pp, const uint32_t* __restrict__ o1, const uint32_t* __restrict__ o2,
                                               const R* __restrict__ grec, const uint8_t* __restrict__ glk,
                                               R* __restrict__ srec, uint32_t cap, uint32_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  PartLds<R, PT2>& L = *(PartLds<R, PT2>*)lds_raw;
  const uint32_t g = blockIdx.x / pp.nj, jj = blockIdx.x % pp.nj;
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  if (t < (1u << pp.lb)) L.run[t] = o2[(size_t)((g << pp.lb) + t) * pp.nj + jj];
  uint32_t lo, hi;
  part2_range(pp, o1, g, jj, lo, hi);
  auto load = [&](uint32_t base, uint32_t* tg, R* rc) {
    const uint32_t rows = (hi - base < (uint32_t)PT2_ROWS) ? hi - base : (uint32_t)PT2_ROWS;
#pragma unroll
    for (int s = 0; s < PT2; ++s) {
      const uint32_t i = w * (PT2 * 64) + s * 64 + lane;
      const uint32_t p = base + (i < rows ? i : rows - 1);   // (clamped: branch-free loads)
      const uint32_t lk = glk[p];
      rc[s] = grec[p];
      tg[s] = i < rows ? lk : 0xffffffffu;
    }
  };
  uint32_t tg[PT2], tn[PT2];
  R rc[PT2], rn[PT2];
  if (lo < hi) load(lo, tg, rc);
  for (uint32_t base = lo; base < hi; base += PT2_ROWS) {
#pragma unroll
    for (int q = 0; q < 4; ++q) L.cw[q][t] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PT2; ++s)
      if (tg[s] != 0xffffffffu) atomicAdd(&L.cw[w][tg[s]], 1u);
    __syncthreads();
    const uint32_t staged = part_cursors(L);
#pragma unroll
    for (int s = 0; s < PT2; ++s) {
      const bool valid = tg[s] != 0xffffffffu;
      const uint32_t d = valid ? tg[s] : 0u;
      uint32_t rank, cnt;
      peer_rank(valid, d, pp.nb2, rank, cnt);
      if (valid) {
        const uint32_t slot = L.cw[w][d] + rank;
        if (rank == 0) L.cw[w][d] = slot + cnt;
        L.stage[slot] = rc[s];
        L.tag[slot] = (uint16_t)d;
      }
    }
    if (hi - base > (uint32_t)PT2_ROWS) load(base + PT2_ROWS, tn, rn);   // next sub-tile in flight during the write-out
    __syncthreads();
    for (uint32_t q = t; q < staged; q += 256) {
      const uint32_t d = L.tag[q];
      const uint32_t dst = L.run[d] + q - L.ls[d];
      if (dst >= cap) { atomicOr(flags, PK_INTERNAL); continue; }
      srec[dst] = L.stage[q];
    }
    __syncthreads();
    L.run[t] += L.tot[t];
#pragma unroll
    for (int s = 0; s < PT2; ++s) { tg[s] = tn[s]; rc[s] = rn[s]; }
  }
}

// pass 2 moves records as opaque words (vector / scalar members keep the 16 per thread in registers)
typedef uint32_t PtU4 __attribute__((ext_vector_type(4)));
struct PtB24 { uint64_t a, b, c; };
template <class R>
using PtRaw = typename std::conditional<sizeof(R) == 16, PtU4, PtB24>::type;

// per-key segments [seg_b, seg_e) of the sorted records from the last pass's offsets (stride = its segments)
static __global__ void k_part_segs(uint32_t K, const uint32_t* __restrict__ o, uint32_t stride,
                                   uint32_t* __restrict__ seg_b, uint32_t* __restrict__ seg_e) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  seg_b[k] = o[(size_t)k * stride];
  seg_e[k] = o[(size_t)(k + 1) * stride];
}

static PartPlan part_plan(uint32_t K, int64_t nt) {
  PartPlan p;
  memset(&p, 0, sizeof(p));
  p.K = K;
  uint32_t bits = 0;
  while ((1ull << bits) < (uint64_t)K) ++bits;
  auto nbits = [](uint32_t nd) { uint32_t b = 0; while ((1u << b) < nd) ++b; return b; };
  if (K <= (uint32_t)PT_D) {
    p.two = 0; p.lb = 0; p.ng = K;
  } else {
    const uint32_t hb = (bits + 1) / 2;
    p.two = 1; p.lb = bits - hb; p.ng = (K + (1u << p.lb) - 1) >> p.lb;
  }
  p.nb1 = nbits(p.ng);
  p.nb2 = p.lb;
  // >= ~2048 pass-1 segments when the batch allows (8 workgroups per CU), at most 32 sub-tiles each
  const int64_t sub = std::max<int64_t>(1, std::min<int64_t>(32, nt / ((int64_t)PT1_ROWS * 2048)));
  p.seg1 = (uint32_t)(PT1_ROWS * sub);
  p.ns1 = (uint32_t)std::max<int64_t>(1, (nt + p.seg1 - 1) / p.seg1);
  // pass-2 segments of ~8192 rows of one group
  p.ts2 = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(p.ns1, (int64_t)8192 * p.ng / p.seg1));
  p.nj = (p.ns1 + p.ts2 - 1) / p.ts2;
  return p;
}

// ---------------------------------------------------------------------------------------------
struct ProjPlan {
  // per select column: src 0 = e1 row (pending partial), 1 = e2 row (trigger); kind 0 = e1 payload carried
  // in the pending list, 1 = the compared value, 2 = null (chain index beyond a single-event slot),
  // 3 = column gather by row
  int32_t src[SG_MAX_SELECT], kind[SG_MAX_SELECT], col[SG_MAX_SELECT], type[SG_MAX_SELECT];
};

// A delivered match as the record walk leaves it at its final slot: e1/e2 virtual rows, e1's compared value
// and e1's payload attribute (both taken from the pending list, so no gather reaches back into the window).
struct MRec {
  uint32_t r1, r2;
  int64_t v1;                 // e1 compared-value bits
  int64_t p1;                 // e1 payload bits
};

// Where the record walk leaves each delivered match (k_project builds the output record from it).  Narrow form
// (narrow walker records of a 4-byte value type, whose LDS ring already keeps 32-bit payloads): 16 B per match in
// one store; wide form: MRec.
struct MRec16 {
  uint32_t r1, r2, v1, p1;
};
struct MatchSink {
  void* rec;
  int32_t narrow;
  uint32_t cap;               // slots allocated (a slot beyond it trips the internal guard)
  uint32_t* err;
  __device__ __forceinline__ void put(uint32_t slot, uint32_t r1, uint32_t r2, int64_t v1, int64_t p1) const {
    if (slot >= cap) { atomicOr(err, 8u); return; }
    if (narrow) {
      PtU4 q;
      q.x = r1; q.y = r2; q.z = (uint32_t)v1; q.w = (uint32_t)p1;
      ((PtU4*)rec)[slot] = q;
    } else {
      MRec m;
      m.r1 = r1; m.r2 = r2; m.v1 = v1; m.p1 = p1;
      ((MRec*)rec)[slot] = m;
    }
  }
};

struct UnitDesc {
  uint32_t p0, p1, w, ovf;     // chunk positions [p0, p1), replay from w; ovf = 1 + first entry of its HBM list
};

struct WalkStats {
  uint32_t order_err;
  uint32_t n_ovf;             // units on the HBM-list walker
  uint32_t ovf_total;         // HBM-list entries they take (each unit: one entry per row it walks)
  uint32_t internal;          // internal consistency guards tripped (bit 1 unit range, 2 tile source, 4 count row,
                              // 8 match slot, 16 HBM-list space): reported as SG_EINVAL instead of touching memory
                              // out of range
};

// an HBM list for unit u walking rows [w, p1): its first entry (the lists of a push are packed back to back)
__device__ __forceinline__ uint32_t take_hbm_list(WalkStats* st, uint32_t w, uint32_t p1) {
  const uint32_t need = p1 - w + 1;
  const uint32_t o = atomicAdd(&st->ovf_total, need);
  atomicAdd(&st->n_ovf, 1u);
  if (o > 0xffffffffu - need) atomicOr(&st->internal, 16u);
  return o;
}

struct LdsPlan {   // per-push layout of the walkers' LDS rings (count walk: value + time only)
  int32_t pay;     // 1: narrow payload plane
  int32_t row;     // 1: e1 row plane
  int32_t cap;     // ring entries per lane (power of two; deeper for long `within` windows)
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
  uint32_t big_total;         // entries of all HBM lists of the push (BIG)
  LdsPlan lp;                 // record walk LDS planes
  int32_t pay_in_rec;         // e1 payload rides in the (narrow) walker records
  // Keys whose rows (carried ones included) go back in time take the exact walker (see Walker::step_exact): one
  // unit per key on the HBM-list path.  kexact: per-key flag (null: no key does).
  const uint8_t* kexact;
  // Carry: the record pass of each key's last unit leaves the key's final pending list -- as virtual rows (alive,
  // alive_n: HBM lists, and LDS rings that keep e1's row) or as the entries' own time / value / payload (cv: LDS rings
  // without a row plane; the select needs no other e1 attribute then)
  uint32_t* alive;
  uint32_t* alive_n;
  int64_t* cv_ts;
  int32_t* cv_key;
  int64_t* cv_val;
  int64_t* cv_pay;
  uint32_t* cv_n;
  uint32_t cv_cap;
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

// Pending list: value + timestamp per partial, plus (record walk only) e1's payload attribute and e1's row
// when a select gathers other e1 attributes.  LDS: ring of `cap` (power of two) entries per lane, SoA planes,
// lane-strided (conflict-free); timestamps relative to the unit's first replayed row; payload narrowed to
// 32 bits (a LONG that does not fit sends the unit to the HBM path).  The count walk keeps 8 B per entry, so
// it runs at twice the residency of the record walk.  HBM (BIG): one unbounded list per overflowed unit,
// indexed by push count (no wrap), 64-bit times and payloads.
template <class T, bool BIG>
struct PendList {
  T* val;
  int32_t* dts;
  int64_t* ts;
  uint32_t* row;              // null: not kept
  int32_t* pay32;             // LDS narrow payload (null: none)
  int64_t* pay64;             // HBM payload
  int32_t pzero;              // narrow payload is zero-extended (FLOAT bits) rather than sign-extended
  int64_t base;
  uint32_t cmask;             // LDS ring: capacity - 1
  __device__ __forceinline__ uint32_t ix(uint32_t s) const { return BIG ? s : (s & cmask) * WALK_BLOCK; }
  __device__ __forceinline__ T gv(uint32_t s) const { return val[ix(s)]; }
  __device__ __forceinline__ int64_t gts(uint32_t s) const { return BIG ? ts[ix(s)] : base + (int64_t)dts[ix(s)]; }
  __device__ __forceinline__ uint32_t grow(uint32_t s) const { return row ? row[ix(s)] : 0u; }
  __device__ __forceinline__ int64_t gpay(uint32_t s) const {
    if (BIG) return pay64 ? pay64[ix(s)] : 0;
    if (!pay32) return 0;
    int32_t x = pay32[ix(s)];
    return pzero ? (int64_t)(uint32_t)x : (int64_t)x;
  }
  __device__ __forceinline__ void put(uint32_t s, T v, int64_t t, uint32_t r, int64_t p) {
    uint32_t i = ix(s);
    val[i] = v;
    if (BIG) ts[i] = t; else dts[i] = (int32_t)(t - base);
    if (row) row[i] = r;
    if (BIG) { if (pay64) pay64[i] = p; } else if (pay32) pay32[i] = (int32_t)p;
  }
};
template <class T>
struct PendBytes {   // bytes per entry
  static int lds(bool write, const LdsPlan& lp) { return (int)sizeof(T) + 4 + (write ? 4 * (lp.pay + lp.row) : 0); }
  static constexpr int hbm = sizeof(T) + 20;   // val, ts, row, payload
};
// LDS planes of one block: [val][dts][pay32?][row?], each cap * WALK_BLOCK entries
template <class T, bool BIG>
__device__ __forceinline__ void lds_planes(PendList<T, BIG>& L, char* lds, bool write, const LdsPlan& lp) {
  const size_t E = (size_t)(lp.cap) * WALK_BLOCK;
  L.cmask = (uint32_t)lp.cap - 1;
  char* p = lds;
  L.val = (T*)p + threadIdx.x; p += E * sizeof(T);
  L.dts = (int32_t*)p + threadIdx.x; p += E * 4;
  L.pay32 = nullptr;
  L.row = nullptr;
  if (write && lp.pay) { L.pay32 = (int32_t*)p + threadIdx.x; p += E * 4; }
  if (write && lp.row) { L.row = (uint32_t*)p + threadIdx.x; p += E * 4; }
  L.ts = nullptr;
  L.pay64 = nullptr;
}
template <class T, bool BIG>
__device__ __forceinline__ void hbm_planes(PendList<T, BIG>& L, char* big, uint32_t first, size_t total) {
  L.ts = (int64_t*)big + first;
  L.pay64 = (int64_t*)(big + total * 8) + first;
  L.val = (T*)(big + total * 16) + first;
  L.row = (uint32_t*)(big + total * (16 + sizeof(T))) + first;
  L.dts = nullptr;
  L.pay32 = nullptr;
}

template <class T, bool N>
__device__ __forceinline__ uint32_t lb_row(const Src<T, N>& src, uint32_t lo, uint32_t hi, uint32_t target, bool part) {
  if (!part) return target < lo ? lo : (target > hi ? hi : target);
  while (lo < hi) {
    uint32_t mid = lo + ((hi - lo) >> 1);
    if (src.row(mid) < target) lo = mid + 1; else hi = mid;
  }
  return lo;
}
template <class T, bool N>
__device__ __forceinline__ uint32_t lb_ts(const Src<T, N>& src, uint32_t lo, uint32_t hi, int64_t tmin) {
  while (lo < hi) {
    uint32_t mid = lo + ((hi - lo) >> 1);
    if (src.ts(mid) < tmin) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  // blocks are dealt round-robin over the 8 XCDs: give XCD x a contiguous range of logical blocks
  uint32_t x = b & 7, i = b >> 3, per = nb >> 3, rem = nb & 7;
  return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

// Match projection (QuerySelector.processNoGroupBy, C/query/selector/QuerySelector.java:125-163, with
// SelectiveStateEventPopulator, C/event/state/populater/SelectiveStateEventPopulator.java:36-56): one
// thread per delivered match builds its AoS record from the (e1 row, e2 row) pair the walker placed at the
// match's final slot.  Slots are in delivery order, so the e2 gathers stream and the e1 gathers stay within
// one `within` window behind them.
template <class T>
__global__ void __launch_bounds__(256) k_project(WalkArgs a, Virt v, ProjPlan pp, SgCols bc, SgCols cc,
                                                 const MatchSink ms, const uint32_t* __restrict__ off,
                                                 int64_t total, char* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char stage[];   // 256 records, written out contiguously
  const int64_t per = (int64_t)blockDim.x;
  // one match per thread (every gather in flight at once); each XCD takes a contiguous slot range so the
  // trigger-ordered gathers of neighbouring slots share its L2 instead of being fetched by all eight
  const int64_t s0 = (int64_t)xcd_block(blockIdx.x, gridDim.x) * per;
  const int64_t sl = s0 + threadIdx.x;
  if (sl < total) {
    MRec mr;
    if (ms.narrow) {   // 32-bit value / payload bits widened as val_bits and the LDS ring (pzero) widen them
      const PtU4 q = ((const PtU4*)ms.rec)[sl];
      mr.r1 = q.x;
      mr.r2 = q.y;
      mr.v1 = std::is_same<T, float>::value ? (int64_t)q.z : (int64_t)(int32_t)q.z;
      mr.p1 = v.pfloat ? (int64_t)q.w : (int64_t)(int32_t)q.w;
    } else {
      mr = ((const MRec*)ms.rec)[sl];
    }
    const uint32_t r1 = mr.r1, r2 = mr.r2;
    const uint64_t b = r2 - v.nc;
    const uint32_t ob = off[b];
    const uint32_t key = a.partitioned ? (uint32_t)v.key[b] : 0u;
    const int64_t t2 = v.ts[b];
    const uint64_t trig = a.index ? a.index[b] : a.base_index + b;
    int64_t* o = (int64_t*)(stage + (size_t)threadIdx.x * a.stride);
    uint32_t nm = 0;
    for (int s = 0; s < a.n_select; ++s) {
      const bool s2 = pp.src[s] != 0;
      const int kind = pp.kind[s];
      int64_t bits = 0;
      if (kind == 0) {
        bits = mr.p1;
      } else if (kind == 1) {
        bits = s2 ? val_bits<T>(v_val<T>(v, r2, v.val_a == v.val_b)) : mr.v1;
      } else if (kind == 2) {
        nm |= 1u << s;
      } else {
        const uint32_t r = s2 ? r2 : r1;
        SgVal x = r < v.nc ? sg_read_col(cc, pp.col[s], pp.type[s], r) : sg_read_col(bc, pp.col[s], pp.type[s], r - v.nc);
        if (x.null) nm |= 1u << s;
        bits = sg_val_bits(x);
      }
      o[4 + s] = bits;
    }
    const uint32_t rank = (uint32_t)(sl - (int64_t)ob);
    o[0] = (int64_t)trig;
    o[1] = t2;
    o[2] = (int64_t)((uint64_t)key | ((uint64_t)((1u << 24) | (a.multi ? (uint32_t)a.b_slot : (0x800000u | rank))) << 32));
    o[3] = (int64_t)nm;
  }
  __syncthreads();
  const int64_t nrec = (total - s0 < per) ? (total - s0) : per;
  const size_t bytes = (size_t)nrec * a.stride;
  char* dst = out + (size_t)(a.out_base + s0) * a.stride;
  if ((((uintptr_t)dst) & 15) == 0) {
    typedef uint32_t U4 __attribute__((ext_vector_type(4)));
    for (size_t q = (size_t)threadIdx.x * 16; q < bytes; q += (size_t)per * 16)
      *(U4*)(dst + q) = *(const U4*)(stage + q);
  } else {
    for (size_t q = (size_t)threadIdx.x * 8; q < bytes; q += (size_t)per * 8)
      *(uint64_t*)(dst + q) = *(const uint64_t*)(stage + q);
  }
}

// The reference's pending list for one event of one key (see the file header).
template <int OP, class T>
__device__ __forceinline__ bool cmp_sel(int op, T b, T a) { return cmp_op<T>(OP ? OP : op, b, a); }

template <class T, bool WRITE, bool BIG, int OP = 0>
struct Walker {
  // LDS path: times relative to the unit's first replayed row (the unit's span was checked to fit 31 bits);
  // HBM-list path: absolute 64-bit times.
  typedef typename std::conditional<BIG, int64_t, int32_t>::type TT;
  PendList<T, BIG> L;
  uint32_t head = 0, top = 0;
  TT hts = 0;                 // register copies (valid while head != top): time of the oldest partial and
  T tv = T();                 // value of the newest one -- the common step touches no LDS for either
  int64_t prev_t;             // time of the previous row (the records' own time domain): the order check
  int32_t prev32;             // (narrow records: their 32-bit times, compared as such)
  TT within;
  bool bad = false;
  // exact mode (a key whose time goes back; HBM list only): min / max time over the list while head != top
  bool exact = false;
  int64_t lo_t = 0, hi_t = 0;
  bool oob = false;           // internal guard: a row outside the batch (never expected)
  bool overflow = false;
  uint32_t ew = 0xffffffffu, ebits = 0;   // count pass: emit bitmap word being built
  __device__ __forceinline__ void set_within(int64_t w) {
    within = BIG ? (TT)w : (TT)(w > 0x7fffffffll ? 0x7fffffffll : w);   // a wider window never expires in-unit
  }
  __device__ __forceinline__ TT rel(int64_t t) const { return BIG ? (TT)t : (TT)(t - L.base); }
  // order check against the row before the replay window
  __device__ __forceinline__ void init_prev(int64_t before) {
    prev_t = before;
    prev32 = (int32_t)(before < INT32_MIN ? INT32_MIN : (before > INT32_MAX ? INT32_MAX : before));
  }
  __device__ __forceinline__ TT at(uint32_t s) const {
    return BIG ? (TT)L.ts[L.ix(s)] : (TT)L.dts[L.ix(s)];
  }
  __device__ __forceinline__ void flush_bits(uint32_t* __restrict__ emap) {
    if (ebits) atomicOr(&emap[ew], ebits);
    ebits = 0;
  }
  __device__ __forceinline__ void mark_emit(uint32_t pos, uint32_t* __restrict__ emap) {
    const uint32_t wi = pos >> 5;
    if (wi != ew) { flush_bits(emap); ew = wi; }
    ebits |= 1u << (pos & 31);
  }
  __device__ __forceinline__ void push(T x, int64_t tabs, uint32_t r, int64_t pay) {
    L.put(top, x, tabs, r, pay);
    if (top == head) hts = rel(tabs);
    tv = x;
    ++top;
  }
  // returns true when this event (inside the unit's chunk) completed partials
  template <class R>
  __device__ __forceinline__ bool step(const WalkArgs& a, const Virt& v, const R& rc, bool in_chunk,
                                       uint32_t ofs, uint32_t* __restrict__ cnt, const MatchSink& em,
                                       bool payload, int64_t pay = 0, bool pay_ready = false) {
    const uint32_t f = rc.rowf >> 30;
    // every row of the key takes part in the order check (a row that fails both filters still expires partials in
    // the reference): a key whose time goes back is redone by the exact walker
    const int64_t tabs = rc.t();
    if constexpr (R::narrow) {   // (a narrow record's time is a 32-bit offset: one 32-bit compare)
      bad |= rc.dts < prev32;
      prev32 = rc.dts;
    } else {
      bad |= tabs < prev_t;
      prev_t = tabs;
    }
    if (!f) return false;
    const T x = rc.val;
    const TT t = rel(tabs);
    // lazy `within` expiry of the oldest partials (StreamPreStateProcessor.isExpired :102-113)
    if (head != top && t - hts > within) {
      ++head;
      while (head != top) {
        hts = at(head);
        if (t - hts <= within) break;
        ++head;
      }
    }
    const uint32_t r = rc.rowf & ROW_MASK;
    const bool live = !is_nan_val<T>(x);
    uint32_t m = 0;
    if ((f & F_CONS) && live) {
      if (a.stack_mode) {
        // monotone stack: the completed partials are exactly a suffix, delivered oldest first
        if (top != head && cmp_sel<OP, T>(a.op, x, tv)) {
          --top;
          ++m;
          while (top != head) {
            tv = L.gv(top - 1);
            if (!cmp_sel<OP, T>(a.op, x, tv)) break;
            --top;
            ++m;
          }
        }
        if (WRITE && in_chunk && r >= v.nc) {
          for (uint32_t q = 0; q < m; ++q)
            em.put(ofs + q, L.grow(top + q), r, val_bits<T>(L.gv(top + q)), L.gpay(top + q));
        }
      } else {
        const bool emit = in_chunk && (r >= v.nc);
        uint32_t wr = head;
        for (uint32_t s = head; s != top; ++s) {
          T e = L.gv(s);
          if (cmp_sel<OP, T>(a.op, x, e)) {
            if (WRITE && emit) em.put(ofs + m, L.grow(s), r, val_bits<T>(e), L.gpay(s));
            ++m;
          } else {
            if (wr != s) L.put(wr, e, BIG ? (int64_t)at(s) : L.base + (int64_t)at(s), L.grow(s), L.gpay(s));
            ++wr;
          }
        }
        top = wr;
        if (head != top) {   // (compaction moved entries: refresh the register copies)
          hts = at(head);
          tv = L.gv(top - 1);
        }
      }
    }
    const bool emitted = m && in_chunk && (r >= v.nc);
    if (!WRITE && emitted) {
      if (r - v.nc < (uint64_t)v.n) cnt[r - v.nc] = m;
      else oob = true;
    }
    if ((f & F_CAND) && live) {
      if (!BIG && top - head == L.cmask + 1) { overflow = true; return emitted; }
      int64_t pv = 0;
      if (WRITE && payload) {
        if (R::has_pay && a.pay_in_rec) pv = rc.p(v.pfloat);
        else pv = pay_ready ? pay : v_payload(v, r);
      }
      // the LDS ring keeps 32 payload bits: a wider LONG value sends the unit to the HBM path
      if (!BIG && WRITE && payload && L.pay32 && !L.pzero && pv != (int64_t)(int32_t)pv) { overflow = true; return emitted; }
      push(x, rc.t(), r, pv);
    }
    return emitted;
  }
  __device__ __forceinline__ void keep(uint32_t& wr, uint32_t s, T e, int64_t ti) {
    if (wr != s) L.put(wr, e, ti, L.grow(s), L.gpay(s));
    ++wr;
    if (wr == head + 1) { lo_t = ti; hi_t = ti; } else { lo_t = ti < lo_t ? ti : lo_t; hi_t = ti > hi_t ? ti : hi_t; }
  }
  // The reference's list for any arrival order (HBM list only): a row of B's stream first drops every pending
  // partial with |e1.ts - ts| > within -- on either side, not only the oldest (StreamPreStateProcessor.isExpired,
  // C/query/input/stream/state/StreamPreStateProcessor.java:102-113) -- then a B consumer completes, in pending
  // order, every partial its compare accepts (processAndReturn :292-337), then a candidate appends itself.
  template <class R>
  __device__ __forceinline__ bool step_exact(const WalkArgs& a, const Virt& v, const R& rc, bool in_chunk,
                                             uint32_t ofs, uint32_t* __restrict__ cnt, const MatchSink& em,
                                             bool payload) {
    const uint32_t f = rc.rowf >> 30;
    const uint32_t r = rc.rowf & ROW_MASK;
    const int64_t t = rc.t();
    const T x = rc.val;
    const bool live = !is_nan_val<T>(x);
    if (BIG && head != top && (t - lo_t > (int64_t)within || hi_t - t > (int64_t)within) && v_visit(v, r)) {
      uint32_t wr = head;
      for (uint32_t s = head; s != top; ++s) {
        const int64_t ti = (int64_t)at(s);
        if (t - ti > (int64_t)within || ti - t > (int64_t)within) continue;
        keep(wr, s, L.gv(s), ti);
      }
      top = wr;
    }
    uint32_t m = 0;
    if ((f & F_CONS) && live && head != top) {
      const bool emit = in_chunk && (r >= v.nc);
      uint32_t wr = head;
      for (uint32_t s = head; s != top; ++s) {
        const T e = L.gv(s);
        if (cmp_sel<OP, T>(a.op, x, e)) {
          if (WRITE && emit) em.put(ofs + m, L.grow(s), r, val_bits<T>(e), L.gpay(s));
          ++m;
        } else {
          keep(wr, s, e, (int64_t)at(s));
        }
      }
      top = wr;
    }
    const bool emitted = m && in_chunk && (r >= v.nc);
    if (!WRITE && emitted) {
      if (r - v.nc < (uint64_t)v.n) cnt[r - v.nc] = m;
      else oob = true;
    }
    if ((f & F_CAND) && live) {
      int64_t pv = 0;
      if (WRITE && payload) pv = (R::has_pay && a.pay_in_rec) ? rc.p(v.pfloat) : v_payload(v, r);
      if (head == top) { lo_t = t; hi_t = t; } else { lo_t = t < lo_t ? t : lo_t; hi_t = t > hi_t ? t : hi_t; }
      L.put(top, x, t, r, pv);
      ++top;
    }
    return emitted;
  }
};

// HBM-list walker: one lane per unit whose pending list outgrew the LDS ring, whose time span does not fit the ring's
// 31-bit times, or whose key's time goes back (exact mode: the key's whole segment in one unit).  WRITE=false: count
// pass; WRITE=true: record pass.
template <class T, bool N, bool WRITE, bool BIG>
__global__ void __launch_bounds__(WALK_BLOCK) k_walk(WalkArgs a, Src<T, N> src, const uint32_t* __restrict__ seg_b,
                                                     const uint32_t* __restrict__ seg_e, UnitDesc* __restrict__ ud,
                                                     uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                                     const MatchSink em, uint32_t* __restrict__ emap,
                                                     WalkStats* __restrict__ st, char* __restrict__ big) {
  static_assert(BIG, "the LDS-ring units run on the tiled walker (k_walk_t)");
  const uint32_t u = xcd_block(blockIdx.x, gridDim.x) * WALK_BLOCK + threadIdx.x;
  if (u >= a.n_units) return;
  const Virt& v = src.pk.v;
  const bool part = a.partitioned != 0;
  const uint32_t k = u % a.K;
  uint32_t sb, se;
  if (part) {
    sb = seg_b[k];
    se = seg_e[k];
  } else {
    sb = 0;
    se = (uint32_t)a.nt;
  }
  const UnitDesc d = ud[u];
  const uint32_t p0 = d.p0, p1 = d.p1, w = d.w, ovf = d.ovf;
  if (p0 >= p1 || ovf == 0) return;
  Walker<T, WRITE, BIG> W;
  hbm_planes<T, BIG>(W.L, big, ovf - 1, a.big_total);
  W.L.pzero = v.pfloat;
  W.exact = a.kexact && a.kexact[k];
  const bool payload = v.pcol != nullptr;
  const int64_t tw = src.ts(w);
  W.L.base = tw;
  W.set_within(a.within);
  W.init_prev((w > sb) ? src.ts(w - 1) : tw);
  // record walk: output offsets only for the positions the count pass marked as emitting
  auto off_of = [&](const WRec<T, N>& rc, uint32_t pos, uint32_t bits) -> uint32_t {
    uint32_t r = rc.rowf & ROW_MASK;
    return (bits && pos >= p0 && pos < p1 && r >= v.nc) ? off[r - v.nc] : 0u;
  };
  auto one = [&](const WRec<T, N>& rc, uint32_t p, uint32_t o) {
    const bool e = W.exact ? W.step_exact(a, v, rc, p >= p0, o, cnt, em, payload)
                           : W.step(a, v, rc, p >= p0, o, cnt, em, payload);
    if (e && !WRITE) W.mark_emit(p, emap);
  };
  if (src.srec) {
    // key-sorted records: whole-line group loads, next group in flight while this one is walked
    typedef Grp<T, N> GT;
    const uint32_t G = GT::G;
    GT cur, nxt;
    uint32_t g = w & ~(G - 1);
    cur.load(src.srec + g);
    uint32_t ofs[GT::G], nofs[GT::G];
    uint32_t eb = 0, neb = 0;
    if (WRITE) {
      eb = emap[g >> 5] >> (g & 31);
#pragma unroll
      for (int i = 0; i < GT::G; ++i) ofs[i] = off_of(cur.rec(i), g + i, (eb >> i) & 1u);
    }
    for (; g < p1; g += G) {
      const uint32_t gn = g + G;
      if (gn < p1) {
        nxt.load(src.srec + gn);
        if (WRITE) neb = emap[gn >> 5] >> (gn & 31);
      }
#pragma unroll
      for (int i = 0; i < GT::G; ++i) {
        const uint32_t p = g + i;
        if (p < w || p >= p1) continue;
        one(cur.rec(i), p, WRITE ? ofs[i] : 0u);
      }
      cur = nxt;
      if (WRITE) {
#pragma unroll
        for (int i = 0; i < GT::G; ++i) nofs[i] = (gn < p1) ? off_of(cur.rec(i), gn + i, (neb >> i) & 1u) : 0u;
#pragma unroll
        for (int i = 0; i < GT::G; ++i) ofs[i] = nofs[i];
      }
    }
  } else {
    // unpartitioned: the rows themselves, in order
    for (uint32_t p = w; p < p1; ++p) {
      WRec<T, N> rc = src.pk(p);
      one(rc, p, WRITE ? off_of(rc, p, (emap[p >> 5] >> (p & 31)) & 1u) : 0u);
    }
  }
  if (!WRITE) W.flush_bits(emap);
  if (W.oob) atomicOr(&st->internal, 4u);
  if (W.bad && !W.exact) atomicOr(&st->order_err, 1u);
  if (WRITE && a.carry_out && p1 == se) {
    // the key's pending list survives: its partials as rows, in pending order (replaying them as candidates rebuilds
    // the list -- a carried row neither expires nor completes anything)
    const uint32_t m = W.top - W.head;
    const uint32_t o = m ? atomicAdd(a.alive_n, m) : 0u;
    if ((uint64_t)o + m > (uint64_t)a.nt) atomicOr(&st->internal, 32u);
    else for (uint32_t s = 0; s < m; ++s) a.alive[o + s] = W.L.grow(W.head + s);
  }
}

// ---------------------------------------------------------------------------------------------
// Lane-interleaved ("transposed") walker tiles for partitioned queries.  Logical wave W owns units
// 64W..64W+63; row i of its tile holds record (w_u + i) of each of its units, so one wave-wide record load
// is one contiguous 1 KB access and the emit flags of a row are one ballot word.

// unit replay ranges (p0, p1, w) + per-wave tile length (rows, padded to TROWS)
static const int TROWS = 16;
template <class T, bool N>
__global__ void __launch_bounds__(256) k_units(WalkArgs a, Src<T, N> src, const uint32_t* __restrict__ seg_b,
                                               const uint32_t* __restrict__ seg_e, UnitDesc* __restrict__ ud,
                                               uint32_t* __restrict__ wlen, WalkStats* __restrict__ st) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t len = 0;
  if (u < a.n_units) {
    const uint32_t c = u / a.K, k = u % a.K;
    uint32_t sb = seg_b[k], se = seg_e[k];
    UnitDesc d{0, 0, 0, 0};
    if (se > a.nt || sb > se) { atomicOr(&st->internal, 1u); sb = se = 0; }
    if (sb < se && a.kexact && a.kexact[k]) {
      // a key whose time goes back: its whole segment in one exact unit (chunk 0) on the HBM-list walker
      if (c == 0) d = UnitDesc{sb, se, sb, take_hbm_list(st, sb, se) + 1};
    } else if (sb < se) {
      uint64_t lo_row = (uint64_t)c * a.R, hi_row = lo_row + a.R;
      uint32_t p0 = c == 0 ? sb : lb_row(src, sb, se, (uint32_t)(lo_row < (uint64_t)a.nt ? lo_row : a.nt), true);
      uint32_t p1 = c + 1 >= a.C ? se : lb_row(src, p0, se, (uint32_t)(hi_row < (uint64_t)a.nt ? hi_row : a.nt), true);
      d = UnitDesc{p0, p0, p0, 0};
      if (p0 < p1) {
        uint32_t w = lb_ts(src, sb, p0, src.ts(p0) - a.within);
        d = UnitDesc{p0, p1, w, 0};
        int64_t tw = src.ts(w), tl = src.ts(p1 - 1);
        if (tl - tw > 0x7fffffffll || tl < tw) {   // relative ts would not fit: HBM-list walker
          d.ovf = take_hbm_list(st, w, p1) + 1;
        } else {
          len = p1 - w;
        }
      }
    }
    ud[u] = d;
  }
  // wave max -> tile rows
  uint32_t m = len;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0 && (u >> 6) < (a.n_units + 63) / 64) wlen[u >> 6] = (m + TROWS - 1) / TROWS * TROWS;
}

// row-block -> wave map
static __global__ void k_rowmap(const uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wrow, uint32_t nw,
                         uint32_t* __restrict__ map) {
  uint32_t W = blockIdx.x * blockDim.x + threadIdx.x;
  if (W >= nw) return;
  for (uint32_t q = wrow[W] / TROWS, e = (wrow[W] + wlen[W]) / TROWS; q < e; ++q) map[q] = W;
}

// sorted records -> tiles, through an LDS transpose (coalesced reads per unit, 1 KB rows out)
template <class T, bool N>
__global__ void __launch_bounds__(256) k_transpose(const WRec<T, N>* __restrict__ srec, const UnitDesc* __restrict__ ud,
                                                   const uint32_t* __restrict__ wrow, const uint32_t* __restrict__ map,
                                                   uint32_t nq, WRec<T, N>* __restrict__ tile, uint32_t nsrc,
                                                   uint32_t n_units, WalkStats* __restrict__ st) {
  __shared__ WRec<T, N> t[TROWS][64];
  for (uint32_t q = blockIdx.x; q < nq; q += gridDim.x) {
    const uint32_t W = map[q];
    const uint32_t i0 = q * TROWS - wrow[W];
    for (uint32_t idx = threadIdx.x; idx < TROWS * 64; idx += blockDim.x) {
      const uint32_t l = idx / TROWS, ii = idx % TROWS;
      const uint32_t u = W * 64 + l;   // (the last wave's lanes past n_units have no descriptor)
      const UnitDesc d = u < n_units ? ud[u] : UnitDesc{0, 0, 0, 0};
      WRec<T, N> r;
      const uint32_t len = (d.p1 > d.p0 && !d.ovf) ? d.p1 - d.w : 0;
      const uint32_t p = d.w + i0 + ii;
      if (i0 + ii < len && p < nsrc) {
        r = srec[p];
      } else {
        if (i0 + ii < len) atomicOr(&st->internal, 2u);
        memset(&r, 0, sizeof(r));
      }
      t[ii][l ^ ii] = r;
    }
    __syncthreads();
    for (uint32_t idx = threadIdx.x; idx < TROWS * 64; idx += blockDim.x) {
      const uint32_t ii = idx / 64, l = idx % 64;
      tile[(size_t)(q * TROWS + ii) * 64 + l] = t[ii][l ^ ii];
    }
    __syncthreads();
  }
}

// walker over tiles (partitioned, LDS list).  All 64 lanes step through rows together.
// (launch bounds: the record walk's LDS ring (12 B per entry, 16 entries per lane) fits three blocks per CU -- three
// waves per SIMD -- which its registers must allow too: at 2 waves per SIMD C2's record walk took 3.2 ms, at 3 1.6 ms)
template <class T, bool N, int OP, bool WRITE>
__global__ void __launch_bounds__(WALK_BLOCK, WRITE ? 3 : 5) k_walk_t(WalkArgs a, Src<T, N> src, const uint32_t* __restrict__ seg_b,
                                                       const uint32_t* __restrict__ seg_e,
                                                       const UnitDesc* __restrict__ ud,
                                                       const uint32_t* __restrict__ wlen,
                                                       const uint32_t* __restrict__ wrow,
                                                       const WRec<T, N>* __restrict__ tile, uint32_t* __restrict__ cnt,
                                                       const uint32_t* __restrict__ off, const MatchSink em,
                                                       uint64_t* __restrict__ emask, WalkStats* __restrict__ st,
                                                       UnitDesc* __restrict__ ud_w) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const uint32_t u = xcd_block(blockIdx.x, gridDim.x) * WALK_BLOCK + threadIdx.x;
  const uint32_t W = __builtin_amdgcn_readfirstlane(u >> 6), lane = threadIdx.x & 63;
  if ((W << 6) >= a.n_units) return;   // whole wave out of range (n_units need not be a multiple of 64)
  const Virt& v = src.pk.v;
  const UnitDesc d = u < a.n_units ? ud[u] : UnitDesc{0, 0, 0, 0};
  bool active = d.p0 < d.p1 && !d.ovf;
  const uint32_t p0 = d.p0, p1 = d.p1, w = d.w;
  const uint32_t len = active ? p1 - w : 0;
  const uint32_t rows = __builtin_amdgcn_readfirstlane(wlen[W]), base = __builtin_amdgcn_readfirstlane(wrow[W]);
  Walker<T, WRITE, false, OP> Wk;
  lds_planes<T, false>(Wk.L, lds, WRITE, a.lp);
  Wk.L.pzero = v.pfloat;
  const uint32_t k = u % a.K;
  const uint32_t sb = active ? seg_b[k] : 0;
  const int64_t tw = active ? src.ts(w) : 0;
  Wk.L.base = tw;
  Wk.set_within(a.within);
  Wk.init_prev((active && w > sb) ? src.ts(w - 1) : tw);
  const bool payload = v.pcol != nullptr;
  const uint32_t chunk_i = active ? p0 - w : 0;   // rows before this index only rebuild the pending list
  const WRec<T, N>* tp = tile + (size_t)base * 64 + lane;
  WRec<T, N> ba[PF], bb[PF];
  uint32_t oa[PF], ob[PF];
  auto load_rows = [&](WRec<T, N>* buf, uint32_t i0) {
#pragma unroll
    for (int j = 0; j < PF; ++j) buf[j] = (i0 + j < rows) ? tp[(size_t)(i0 + j) * 64] : WRec<T, N>{};
  };
  auto gather_offs = [&](const WRec<T, N>* buf, uint32_t i0, uint32_t* ofs) {   // rows the count pass marked
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const uint64_t mj = (i0 + j < rows) ? emask[base + i0 + j] : 0ull;
      const uint32_t r = buf[j].rowf & ROW_MASK;
      ofs[j] = ((mj >> lane) & 1ull) ? off[r - v.nc] : 0u;
    }
  };
  auto process = [&](const WRec<T, N>* buf, uint32_t i0, const uint32_t* ofs) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      bool e = false;
      if (active && i0 + j < len && !Wk.overflow)
        e = Wk.step(a, v, buf[j], i0 + j >= chunk_i, WRITE ? ofs[j] : 0u, cnt, em, payload);
      if (!WRITE) {
        const uint64_t b = __ballot(e);
        if (lane == 0) emask[base + i0 + j] = b;
      }
    }
  };
  // Explicit drain at each batch boundary: the batch about to be walked (loaded one batch earlier) and the
  // stores of the last batch are complete, so the branchy walk of a batch never waits on memory -- without it
  // the compiler drains every outstanding access (including the prefetch) inside each step.
  load_rows(ba, 0);
  if (WRITE) gather_offs(ba, 0, oa);
  for (uint32_t i = 0; i < rows; i += 2 * PF) {   // rows is a multiple of TROWS = 2 * PF
    __builtin_amdgcn_s_waitcnt(0);
    load_rows(bb, i + PF);
    if (WRITE) gather_offs(bb, i + PF, ob);
    process(ba, i, oa);
    __builtin_amdgcn_s_waitcnt(0);
    load_rows(ba, i + 2 * PF);
    if (WRITE) gather_offs(ba, i + 2 * PF, oa);
    process(bb, i + PF, ob);
  }
  if (Wk.oob) atomicOr(&st->internal, 4u);
  if (active && Wk.overflow && !WRITE) ud_w[u].ovf = take_hbm_list(st, w, p1) + 1;
  if (active && !Wk.overflow && Wk.bad) atomicOr(&st->order_err, 1u);
  if (!WRITE || !a.carry_out) return;
  // the key's last unit: its final pending list is the carry -- slots reserved once per wave (every lane of the wave
  // is still here), not by one atomic per key on a single counter
  const uint32_t m = (active && !Wk.overflow && p1 == seg_e[k]) ? Wk.top - Wk.head : 0u;
  uint32_t incl = m;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
    if ((int)lane >= o) incl += y;
  }
  const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
  if (!tot) return;
  const bool by_row = Wk.L.row != nullptr;
  uint32_t cbase = 0;
  if (lane == 63) cbase = atomicAdd(by_row ? a.alive_n : a.cv_n, tot);
  cbase = (uint32_t)__shfl((int)cbase, 63);
  const uint32_t o = cbase + incl - m;
  if ((uint64_t)cbase + tot > (by_row ? (uint64_t)a.nt : (uint64_t)a.cv_cap)) {
    if (lane == 63) atomicOr(&st->internal, 32u);
    return;
  }
  if (by_row) {
    for (uint32_t s = 0; s < m; ++s) a.alive[o + s] = Wk.L.grow(Wk.head + s);
  } else {
    const int64_t t0 = N ? v_ts(v, 0) : 0;   // (narrow records keep times relative to the push's first row)
    for (uint32_t s = 0; s < m; ++s) {
      const uint32_t q = Wk.head + s;
      a.cv_ts[o + s] = t0 + Wk.L.gts(q);
      a.cv_key[o + s] = (int32_t)k;
      a.cv_val[o + s] = val_bits<T>(Wk.L.gv(q));
      a.cv_pay[o + s] = Wk.L.gpay(q);
    }
  }
}

#include "gwalk.h"

// carry copy: one lane per key copies its surviving suffix (virtual rows) into the new carry buffers
struct CarryBufs {
  int64_t* ts;
  int32_t* key;
  uint8_t* flags;
  void* col[SG_MAX_COLS];
  uint8_t* nul[SG_MAX_COLS];
};

// Carry of rows (HBM-list keys, and LDS rings that keep e1's row): the listed rows mark a bitmask, a count per
// 8192-row block and a scan place every survivor, and the survivors are copied in arrival order (per-key order stays
// arrival order = pending order, which is all the next push's stable key partition needs).
static const int CARRY_BLK = 8192;   // rows per block of the survivor count (256 bitmask words)

static __global__ void __launch_bounds__(256) k_carry_bcount(int64_t nt, const uint32_t* __restrict__ bits,
                                                             uint32_t* __restrict__ bcnt) {
  __shared__ uint32_t red[4];
  const int64_t wi = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t c = wi * 32 < nt ? (uint32_t)__popc(bits[wi]) : 0u;
  for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

static __global__ void __launch_bounds__(256) k_carry_gather(Virt v, int64_t nt, const uint32_t* __restrict__ bits,
                                                             const uint32_t* __restrict__ boff, int n_cols,
                                                             const int32_t* __restrict__ widths, SgCols bc, SgCols cc,
                                                             CarryBufs dst) {
  // 256 consecutive rows per step, one per thread: survivors of a step get consecutive slots (coalesced stores)
  __shared__ uint32_t wc[2][4];
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t base_d = boff[blockIdx.x];
  const int64_t r0 = (int64_t)blockIdx.x * CARRY_BLK;
  for (int step = 0; step < CARRY_BLK / 256; ++step) {
    const int64_t r64 = r0 + step * 256 + t;
    const bool live = r64 < nt && ((bits[r64 >> 5] >> (r64 & 31)) & 1u);
    const uint64_t m = __ballot(live);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (lane == 0) wc[step & 1][w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t q = 0; q < w; ++q) before += wc[step & 1][q];
    const uint32_t tot = wc[step & 1][0] + wc[step & 1][1] + wc[step & 1][2] + wc[step & 1][3];
    if (live) {
      const uint32_t d = base_d + before + below;
      const uint32_t r = (uint32_t)r64;
      dst.ts[d] = v_ts(v, r);
      dst.key[d] = r < v.nc ? v.c_key[r] : (v.key ? v.key[r - v.nc] : 0);
      dst.flags[d] = (uint8_t)(v_flags(v, r) | (v_visit(v, r) ? F_VISIT : 0u));
      const SgCols& s = r < v.nc ? cc : bc;
      const uint32_t rr = r < v.nc ? r : (uint32_t)(r - v.nc);
      for (int c = 0; c < n_cols; ++c) {
        if (!s.col[c]) continue;
        if (widths[c] == 8) ((int64_t*)dst.col[c])[d] = ((const int64_t*)s.col[c])[rr];
        else ((int32_t*)dst.col[c])[d] = ((const int32_t*)s.col[c])[rr];
        dst.nul[c][d] = s.nul[c] ? s.nul[c][rr] : 0;
      }
    }
    base_d += tot;
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
  bool nul_seen[SG_MAX_COLS] = {};   // a column that ever had nulls is gathered by row, never carried
};

// Time chunks per key.  More chunks = more resident walker lanes, but every unit also replays the `within`
// window before its chunk: keep units at >= 2 windows of rows (estimated from the batch's time span) and at
// most one round of resident lanes (LDS holds 160 KiB / (STACK_CAP * entry) lanes per CU).
static int64_t window_rows(uint32_t K, int64_t nt, int64_t within, int64_t span_ms) {   // rows per key per window
  int64_t per_key = std::max<int64_t>(1, nt / std::max<uint32_t>(K, 1));
  return span_ms > 0 ? (int64_t)((double)per_key * (double)within / (double)span_ms) : per_key;
}
static int pick_cap(int64_t win) {   // a monotone stack over w random rows holds ~ln(w) partials
  return win < 300 ? 16 : (win < 5000 ? 32 : 64);
}
static constexpr int64_t WALK_LDS_MAX = 160 * 1024;   // gfx950 LDS per CU = per workgroup ceiling
// Largest ring (power of two) whose write-walk planes fit one workgroup's LDS.
static int clamp_cap(int cap, int entry_bytes_write) {
  while (cap > 2 && (int64_t)cap * WALK_BLOCK * entry_bytes_write > WALK_LDS_MAX) cap >>= 1;
  return cap;
}
// Chunks per key.  Each (key, chunk) unit replays the `within` window before its chunk, so chunks shorter
// than ~2 windows waste walker steps -- unless even such chunks leave the chip short of one walker lane
// per SIMD slot (few keys, long windows: the C1 shape), where parallelism beats replay cost.
static int pick_chunks(uint32_t K, int64_t nt, int entry_bytes, int cap, int64_t win) {
  int64_t blocks_per_cu = WALK_LDS_MAX / ((int64_t)cap * WALK_BLOCK * entry_bytes);
  int64_t target = std::max<int64_t>(blocks_per_cu, 1) * WALK_BLOCK * 256;
  int64_t per_key = std::max<int64_t>(1, nt / std::max<uint32_t>(K, 1));
  int64_t C = std::max<int64_t>(1, target / K);
  const int64_t c_cheap = std::max<int64_t>(1, per_key / std::max<int64_t>(256, 2 * win));
  const int64_t c_short = std::max<int64_t>(1, per_key / 256);
  const bool starved = (int64_t)K * c_cheap < 64 * 256;
  C = std::min<int64_t>(C, starved ? c_short : c_cheap);
  return (int)std::min<int64_t>(C, 1 << 16);
}

struct PushPlan {
  ProjPlan pp;
  int pcol = -1;              // e1 payload column carried in the pending list
  bool e1_row = false;        // some select gathers another e1 attribute by row
};

template <class T, bool N, bool WRITE>
static void launch_walk_t(int op, dim3 g, dim3 b, size_t lds, hipStream_t st, const WalkArgs& wa, const Src<T, N>& src,
                          const uint32_t* seg_b, const uint32_t* seg_e, UnitDesc* ud, const uint32_t* wlen,
                          const uint32_t* wrow, const WRec<T, N>* tile, uint32_t* cnt, const uint32_t* off, const MatchSink& ms,
                          uint64_t* emask, WalkStats* wst) {
#define SG_WALK_T(OPV)                                                                                          \
  if (lds > 65536)                                                                                              \
    HIPCHK(hipFuncSetAttribute((const void*)k_walk_t<T, N, OPV, WRITE>,                                        \
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                          \
  hipLaunchKernelGGL((k_walk_t<T, N, OPV, WRITE>), g, b, lds, st, wa, src, seg_b, seg_e, ud, wlen, wrow, tile, cnt, off, \
                     ms, emask, wst, ud)
  switch (op) {
    case 2: SG_WALK_T(2); break;
    case 3: SG_WALK_T(3); break;
    case 4: SG_WALK_T(4); break;
    default: SG_WALK_T(5); break;
  }
#undef SG_WALK_T
  HIPCHK(hipGetLastError());
}

// One push through the closed-form pipeline with walker records of format N (narrow / wide).  Returns false
// (having changed no state) when narrow records cannot represent the push (time span beyond 2^31 ms).
// ---------------------------------------------------------------------------------------------
// Unpartitioned streams: per-candidate search instead of the walker.  One key means the walker's units are
// time chunks of a single row sequence, each replaying a whole `within` window before it: few, long,
// latency-bound lanes (C1: 1000-row windows).  Every partial of this shape is independent:
// partial i leaves e2's list at the first later row of B's stream that either expires it (|ts_j - ts_i| > T,
// StreamPreStateProcessor.isExpired, C/query/input/stream/state/StreamPreStateProcessor.java:102-113 -- for any
// arrival order, so time going back needs no special case) or, as a consumer with x_j OP x_i, completes it
// (processAndReturn :292-337).  So one lane per candidate scans forward (lanes of a wave read neighbouring rows:
// coalesced); matches go to their slots by per-trigger counts, and a candidate whose scan reaches the end of the
// push is still pending: exactly those rows are carried into the next push.  A search longer than NGE_MAX_SCAN
// rows sends the push to the walker (bounded work per lane).
static const uint32_t NGE_MAX_SCAN = 4096;
static const uint32_t NGE_NONE = 0xffffffffu;

// per 64-row block of virtual rows: the most completing consumer value (max for > >=, min for < <=), whether the
// block has a live consumer at all, and the time range of its rows of B's stream -- a search skips a block that
// can neither complete nor expire its partial
template <class T, int OP>
__global__ void k_nge_blocks(Virt v, int64_t nt, T* __restrict__ best, uint8_t* __restrict__ has,
                             int64_t* __restrict__ bmin, int64_t* __restrict__ bmax) {
  const int64_t nb = (nt + 63) >> 6;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (int64_t)gridDim.x * blockDim.x) {
    T m{};
    bool any = false;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t q = b << 6, e = (q + 64 < nt ? q + 64 : nt); q < e; ++q) {
      if (v_visit(v, (uint32_t)q)) {
        const int64_t t = v_ts(v, (uint32_t)q);
        lo = t < lo ? t : lo;
        hi = t > hi ? t : hi;
      }
      if (!(v_flags(v, (uint32_t)q) & F_CONS)) continue;
      const T x = v_val<T>(v, (uint32_t)q, false);
      if (is_nan_val<T>(x)) continue;
      if (!any || ((OP == 2 || OP == 3) ? x > m : x < m)) m = x;
      any = true;
    }
    best[b] = m;
    has[b] = any ? 1 : 0;
    bmin[b] = lo;
    bmax[b] = hi;
  }
}

template <class T, int OP>
__global__ void __launch_bounds__(256) k_nge(Virt v, int64_t nt, int64_t within, int op, uint32_t* __restrict__ mj,
                                             uint32_t* __restrict__ rank, uint32_t* __restrict__ cnt,
                                             uint32_t* __restrict__ st_flags, const T* __restrict__ best,
                                             const uint8_t* __restrict__ has, const int64_t* __restrict__ bmin,
                                             const int64_t* __restrict__ bmax, uint32_t* __restrict__ alive) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nt; p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = v_flags(v, (uint32_t)p);
    uint32_t j = NGE_NONE;
    if (f & F_CAND) {
      const T xp = v_val<T>(v, (uint32_t)p, true);
      const int64_t tp = v_ts(v, (uint32_t)p);
      if (!is_nan_val<T>(xp)) {
        uint32_t steps = 0;
        bool open = true;   // still pending when the scan reaches the end of the push
        bool done = false;
        int64_t q = p + 1;
        while (q < nt && !done) {
          if ((q & 63) == 0 && q + 64 <= nt && !(has[q >> 6] && cmp_sel<OP, T>(op, best[q >> 6], xp)) &&
              bmax[q >> 6] <= tp + within && bmin[q >> 6] >= tp - within) {
            if (++steps > NGE_MAX_SCAN) { atomicOr(&st_flags[1], 1u); open = false; break; }
            q += 64;                                                       // nothing in this block ends i
            continue;
          }
          // the rows up to the next multiple of 8: every load issued before the first test (one memory latency per
          // eight rows instead of one per row; most searches end within a few rows)
          const int64_t ge = ((q & ~(int64_t)7) + 8) < nt ? (q & ~(int64_t)7) + 8 : nt;
          int64_t tq[8];
          uint32_t fq[8];
          bool vq[8];
          T xq[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int64_t r = q + u < ge ? q + u : ge - 1;
            tq[u] = v_ts(v, (uint32_t)r);
            fq[u] = v_flags(v, (uint32_t)r);
            vq[u] = v_visit(v, (uint32_t)r);
            xq[u] = v_val<T>(v, (uint32_t)r, false);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (done || q + u >= ge) continue;
            if (++steps > NGE_MAX_SCAN) { atomicOr(&st_flags[1], 1u); open = false; done = true; continue; }
            if ((tq[u] - tp > within || tp - tq[u] > within) && vq[u]) { open = false; done = true; continue; }   // expired
            if ((fq[u] & F_CONS) && !is_nan_val<T>(xq[u]) && cmp_sel<OP, T>(op, xq[u], xp)) {
              if (q + u >= v.nc) j = (uint32_t)(q + u);                    // (carried triggers were emitted before)
              open = false;
              done = true;
            }
          }
          q = ge;
        }
        if (open && alive) atomicOr(&alive[p >> 5], 1u << (p & 31));
      }
    }
    mj[p] = j;
    if (j != NGE_NONE) rank[p] = atomicAdd(&cnt[j - v.nc], 1u);   // (rank among the trigger's matches: any order)
  }
}

// every match to its delivery slot: the trigger's offset + the rank the search drew; then each trigger's matches in
// pending (= arrival) order of their partials
template <class T>
__global__ void k_nge_place(Virt v, int64_t nt, const uint32_t* __restrict__ mj, const uint32_t* __restrict__ rank,
                            const uint32_t* __restrict__ off, MRec* __restrict__ mrec) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nt; p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t j = mj[p];
    if (j == NGE_NONE) continue;
    MRec m;
    m.r1 = (uint32_t)p;
    m.r2 = j;
    m.v1 = val_bits<T>(v_val<T>(v, (uint32_t)p, true));
    m.p1 = v.pcol ? v_payload(v, (uint32_t)p) : 0;
    mrec[off[j - v.nc] + rank[p]] = m;
  }
}

// Each trigger's matches into pending order (ascending e1 row).  Triggers with up to NGE_ORDER_SMALL matches are
// insertion-sorted by their own lane; larger ones (a long run of candidates completed by one row) are flagged and
// sorted by a segmented radix sort afterwards, so no lane does quadratic work.
static const uint32_t NGE_ORDER_SMALL = 32;
static __global__ void k_nge_order(int64_t n, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                   MRec* __restrict__ mrec, uint32_t* __restrict__ nbig) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = cnt[b];
    if (c < 2) continue;
    if (c > NGE_ORDER_SMALL) { atomicAdd(nbig, c); continue; }
    MRec* e = mrec + off[b];
    for (uint32_t i = 1; i < c; ++i) {
      const MRec x = e[i];
      uint32_t k = i;
      while (k > 0 && e[k - 1].r1 > x.r1) {
        e[k] = e[k - 1];
        --k;
      }
      e[k] = x;
    }
  }
}

// large triggers: (trigger slot, e1 row) keys of their matches, then one stable radix sort orders every match
static __global__ void k_nge_bigkeys(int64_t total, const MRec* __restrict__ mrec, const uint32_t* __restrict__ mj,
                                     const uint32_t* __restrict__ off, int64_t nc, uint64_t* __restrict__ key,
                                     uint32_t* __restrict__ idx) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += (int64_t)gridDim.x * blockDim.x) {
    const MRec m = mrec[s];
    key[s] = ((uint64_t)off[m.r2 - nc] << 32) | m.r1;
    idx[s] = (uint32_t)s;
  }
}
static __global__ void k_nge_permute(int64_t total, const MRec* __restrict__ src, const uint32_t* __restrict__ idx,
                                     MRec* __restrict__ dst) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += (int64_t)gridDim.x * blockDim.x)
    dst[s] = src[idx[s]];
}

template <class T>
static bool run_nge(SgHandle* h, const BatchView& bv, int64_t n, int64_t nc, const PushPlan& plan, const Virt& v,
                    const SgCols& cc, int op, EveryNextState* es) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int64_t nt = nc + n;
  const int b_state = d.shape_args[1];
  auto grid = [](int64_t m) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 256 * 16))); };
  uint32_t* mj = (uint32_t*)h->ws.get("nge_mj", 4 * nt, st);
  uint32_t* rank = (uint32_t*)h->ws.get("nge_rank", 4 * nt, st);
  uint32_t* cnt = (uint32_t*)h->ws.get("cnt", sizeof(uint32_t) * (n + 1), st);
  uint32_t* off = (uint32_t*)h->ws.get("off", sizeof(uint32_t) * (n + 1), st);
  uint32_t* stf = (uint32_t*)h->ws.get("nge_flags", 16, st);
  const bool carry = !h->opt.no_carry && nt > 0;
  const int64_t cnb = (nt + CARRY_BLK - 1) / CARRY_BLK;
  uint32_t* cbits = carry ? (uint32_t*)h->ws.get("carry_bits", sizeof(uint32_t) * (size_t)(cnb * 256), st) : nullptr;
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (n + 1), st));
  HIPCHK(hipMemsetAsync(stf, 0, 16, st));
  if (carry) HIPCHK(hipMemsetAsync(cbits, 0, sizeof(uint32_t) * (size_t)(cnb * 256), st));
  const int64_t nb = (nt + 63) >> 6;
  T* best = (T*)h->ws.get("nge_best", sizeof(T) * (nb + 1), st);
  uint8_t* has = (uint8_t*)h->ws.get("nge_has", nb + 1, st);
  int64_t* bmin = (int64_t*)h->ws.get("nge_bmin", sizeof(int64_t) * (nb + 1), st);
  int64_t* bmax = (int64_t*)h->ws.get("nge_bmax", sizeof(int64_t) * (nb + 1), st);
#define SG_NGE_LAUNCH(OPV)                                                                                       \
  hipLaunchKernelGGL((k_nge_blocks<T, OPV>), grid(nb), dim3(256), 0, st, v, nt, best, has, bmin, bmax);        \
  hipLaunchKernelGGL((k_nge<T, OPV>), grid(nt), dim3(256), 0, st, v, nt, d.within, op, mj, rank, cnt, stf, best, has, \
                     bmin, bmax, cbits)
  h->kbeg("nge_search");
  switch (op) {
    case 2: SG_NGE_LAUNCH(2); break;
    case 3: SG_NGE_LAUNCH(3); break;
    case 4: SG_NGE_LAUNCH(4); break;
    default: SG_NGE_LAUNCH(5); break;
  }
#undef SG_NGE_LAUNCH
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(2);
  size_t tb = 0;
  HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
  void* tmp = h->ws.get("scan_tmp", tb, st);
  HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
  uint32_t hflags[4] = {0, 0, 0, 0};
  uint32_t total = 0;
  HIPCHK(hipMemcpyAsync(hflags, stf, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&total, off + n, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (hflags[1]) return false;   // a search outgrew NGE_MAX_SCAN: the walker takes this push
  MRec* mrec = nullptr;
  if (total) {
    mrec = (MRec*)h->ws.get("mrec", sizeof(MRec) * total, st);
    hipLaunchKernelGGL((k_nge_place<T>), grid(nt), dim3(256), 0, st, v, nt, mj, rank, off, mrec);
    hipLaunchKernelGGL(k_nge_order, grid(n), dim3(256), 0, st, n, cnt, off, mrec, stf + 2);
    HIPCHK(hipGetLastError());
    uint32_t nbig = 0;
    HIPCHK(hipMemcpyAsync(&nbig, stf + 2, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (nbig) {
      // a trigger completed more than NGE_ORDER_SMALL partials: order every match by (trigger slot, e1 row)
      uint64_t* k1 = (uint64_t*)h->ws.get("nge_k1", 8 * (size_t)total, st);
      uint64_t* k2 = (uint64_t*)h->ws.get("nge_k2", 8 * (size_t)total, st);
      uint32_t* i1 = (uint32_t*)h->ws.get("nge_i1", 4 * (size_t)total, st);
      uint32_t* i2 = (uint32_t*)h->ws.get("nge_i2", 4 * (size_t)total, st);
      MRec* m2 = (MRec*)h->ws.get("mrec2", sizeof(MRec) * total, st);
      hipLaunchKernelGGL(k_nge_bigkeys, grid(total), dim3(256), 0, st, (int64_t)total, mrec, mj, off, nc, k1, i1);
      size_t sb = 0;
      HIPCHK(rocprim::radix_sort_pairs(nullptr, sb, k1, k2, i1, i2, (size_t)total, 0, 64, st));
      void* stmp = h->ws.get("nge_sort_tmp", sb, st);
      HIPCHK(rocprim::radix_sort_pairs(stmp, sb, k1, k2, i1, i2, (size_t)total, 0, 64, st));
      hipLaunchKernelGGL(k_nge_permute, grid(total), dim3(256), 0, st, (int64_t)total, mrec, i2, m2);
      HIPCHK(hipGetLastError());
      mrec = m2;
    }
  }
  h->mark(3);
  h->extra_marks = 0;
  h->split_out = 1;
  WalkArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.partitioned = 0;
  wa.base_index = bv.base_index;
  wa.index = bv.index;
  const int rb = d.recv_of_stream[d.states[b_state].stream];
  wa.multi = d.receivers[rb].multi;
  if (wa.multi) {
    const sg_receiver_desc& r = d.receivers[rb];
    for (int q = 0; q < r.n; ++q)
      if (r.pres[r.n - 1 - q] == b_state) wa.b_slot = q;   // eventSequence = reversed init order
  }
  wa.n_select = d.n_select;
  wa.stride = 32 + 8 * d.n_select;
  char* out = h->out.reserve(total, d.n_select, st);
  wa.out_base = h->out.n;
  h->mark(5);
  if (total) {
    h->kbeg("project");
    hipLaunchKernelGGL((k_project<T>), dim3((unsigned)(((int64_t)total + 255) / 256)), dim3(256), (size_t)256 * wa.stride, st,
                       wa, v, plan.pp, bv.cols, cc, MatchSink{mrec, 0, (uint32_t)total, nullptr}, off, (int64_t)total, out);
    h->kend();
    HIPCHK(hipGetLastError());
  }
  h->out.n += total;
  h->mark(4);
  // carry: the partials still pending at the end of the push
  if (carry) {
    CarrySet& cs = es->carry[es->cur];
    uint32_t* cboff = (uint32_t*)h->ws.get("carry_boff", sizeof(uint32_t) * (size_t)(cnb + 1), st);
    uint32_t* bcnt = (uint32_t*)h->ws.get("carry_bcnt", sizeof(uint32_t) * (size_t)(cnb + 1), st);
    hipLaunchKernelGGL(k_carry_bcount, dim3((unsigned)cnb), dim3(256), 0, st, nt, cbits, bcnt);
    HIPCHK(hipMemsetAsync(bcnt + cnb, 0, sizeof(uint32_t), st));
    size_t cb_tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, cb_tb, bcnt, cboff, (uint32_t)0, (size_t)cnb + 1, rocprim::plus<uint32_t>(), st));
    void* ctmp = h->ws.get("carry_scan_tmp", cb_tb, st);
    HIPCHK(rocprim::exclusive_scan(ctmp, cb_tb, bcnt, cboff, (uint32_t)0, (size_t)cnb + 1, rocprim::plus<uint32_t>(), st));
    uint32_t ncar = 0;
    HIPCHK(hipMemcpyAsync(&ncar, cboff + cnb, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    CarrySet& nx = es->carry[es->cur ^ 1];
    nx.ensure(std::max<int64_t>(ncar, 1), d.n_cols, d.col_type);
    int32_t* widths = (int32_t*)h->ws.get("col_widths", sizeof(int32_t) * SG_MAX_COLS, st);
    int32_t hw[SG_MAX_COLS];
    for (int c = 0; c < SG_MAX_COLS; ++c)
      hw[c] = (c < d.n_cols && (d.col_type[c] == SG_T_LONG || d.col_type[c] == SG_T_DOUBLE)) ? 8 : 4;
    HIPCHK(hipMemcpyAsync(widths, hw, sizeof(hw), hipMemcpyHostToDevice, st));
    CarryBufs cbuf;
    memset(&cbuf, 0, sizeof(cbuf));
    cbuf.ts = nx.ts;
    cbuf.key = nx.key;
    cbuf.flags = nx.flags;
    for (int c = 0; c < d.n_cols; ++c) { cbuf.col[c] = nx.col[c]; cbuf.nul[c] = nx.nul[c]; }
    if (ncar)
      hipLaunchKernelGGL(k_carry_gather, dim3((unsigned)cnb), dim3(256), 0, st, v, nt, cbits, cboff, d.n_cols, widths,
                         bv.cols, cc, cbuf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    nx.n = ncar;
    cs.n = 0;
    es->cur ^= 1;
  }
  h->last_events = n;
  h->last_matches = total;
  h->last_spilled = 0;
  return true;
}

#include "part_wide.h"

// Pass 1 of the key partition beyond 256 key groups (up to 4096 groups of 2^pp.lb keys, e.g. C5's 1M keys): rows ->
// narrow walker records grouped by key group, arrival order kept inside a group, in two LDS counting passes --
// supergroups of 2^lbs groups (<= 64 of them, k_part1 with 32-bit staged keys), then the groups inside each
// supergroup (k_part1b) straight into the group positions o1[g * ns1 + j] of the per-(group, segment) histogram.
// Output: grec, glk (in-group key), o1.
template <class T>
static void part1_wide(SgHandle* h, const PackFn<T, true>& pk, KeyOf kf, uint32_t kb, int64_t nt, const PartPlan& pp,
                       uint32_t* h1, uint32_t* o1, WRec<T, true>* grec, uint8_t* glk, uint32_t* pk_flags) {
  typedef WRec<T, true> R;
  hipStream_t st = h->stream;
  const uint32_t lb = pp.lb, ng = pp.ng;
  const size_t n1 = (size_t)pp.ng * pp.ns1 + 1;
  auto scan_u32 = [&](const uint32_t* in, uint32_t* outp, size_t cnt, const char* tmpname) {
    size_t b = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, b, in, outp, (uint32_t)0, cnt, rocprim::plus<uint32_t>(), st));
    void* tp = h->ws.get(tmpname, b, st);
    HIPCHK(rocprim::exclusive_scan(tp, b, in, outp, (uint32_t)0, cnt, rocprim::plus<uint32_t>(), st));
  };
  {
    // two passes: supergroups of 2^lbs groups (<= 64 of them), then groups inside each supergroup.  (C5, 4096 groups,
    // per 500M-row push: 256 supergroups part_group 7.7 + part_split 3.8 ms; 64 supergroups 6.0 + 4.2 ms -- pass 1's
    // runs per supergroup are 4x longer; 32 supergroups 5.8 + 4.7 ms; profiles/r06/ab_lbs.sh)
    uint32_t lbs = 0;
    while (((ng + (1u << lbs) - 1) >> lbs) > 64u && lbs < 8) ++lbs;
    PartPlan pa2 = pp;
    pa2.lb = lb + lbs;
    pa2.ng = (kb + (1u << pa2.lb) - 1) >> pa2.lb;
    uint32_t nbA = 0;
    while ((1u << nbA) < pa2.ng) ++nbA;
    pa2.nb1 = nbA;
    const size_t nA = (size_t)pa2.ng * pp.ns1 + 1;
    uint32_t* hA = (uint32_t*)h->ws.get("part_hA", sizeof(uint32_t) * nA, st);
    uint32_t* oA = (uint32_t*)h->ws.get("part_oA", sizeof(uint32_t) * nA, st);
    R* grecA = (R*)h->ws.get("grecA", sizeof(R) * nt, st);
    uint16_t* glkA = (uint16_t*)h->ws.get("glkA", 2 * nt, st);
    h->kbeg("part_hist");
    HIPCHK(hipMemsetAsync(hA + nA - 1, 0, sizeof(uint32_t), st));
    HIPCHK(hipMemsetAsync(h1 + n1 - 1, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_hist_wide, dim3(pp.ns1), dim3(256), 0, st, kf, kb, lb, ng, pp.seg1, pp.ns1, nt, h1, lbs, pa2.ng, hA,
                       pk_flags);
    HIPCHK(hipGetLastError());
    scan_u32(hA, oA, nA, "part_scan_tmpA");
    scan_u32(h1, o1, n1, "part_scan_tmp");
    h->kend();
    h->kbeg("part_group");
    // (rows per thread per LDS sub-tile of this 256-digit pass: SG_DEBUG_P1_PT test hook)
    const char* pe = getenv("SG_DEBUG_P1_PT");
    const int p1 = pe ? atoi(pe) : 8;   // (C5: 8.1 -> 7.3 ms per 500M-row push against 4, profiles/r06/ab_p1.sh)
    auto launch_a = [&](auto pt) {
      constexpr int P = decltype(pt)::value;
      const size_t ldsA = sizeof(PartLds<R, P, uint32_t>);
      HIPCHK(hipFuncSetAttribute((const void*)k_part1<T, true, uint32_t, uint16_t, P>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsA));
      hipLaunchKernelGGL((k_part1<T, true, uint32_t, uint16_t, P>), dim3(pp.ns1), dim3(256), ldsA, st, pk, kf, pa2, nt, oA,
                         grecA, glkA, pk_flags);
    };
    if (p1 == 8) launch_a(std::integral_constant<int, 8>());
    else if (p1 == 16) launch_a(std::integral_constant<int, 16>());
    else launch_a(std::integral_constant<int, PT1>());
    HIPCHK(hipGetLastError());
    h->kend();
    h->kbeg("part_split");
    Part1bArgs B;
    B.lb = lb;
    B.lbs = lbs;
    B.ns1 = pp.ns1;
    const int64_t per_sg = std::max<int64_t>(1, nt / pa2.ng);
    B.nsb = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(pp.ns1, per_sg / 32768));
    B.tsb = (pp.ns1 + B.nsb - 1) / B.nsb;
    B.nsb = (pp.ns1 + B.tsb - 1) / B.tsb;
    B.oa = oA;
    B.o1 = o1;
    const size_t ldsB = sizeof(Part1bLds<16>);
    HIPCHK(hipFuncSetAttribute((const void*)k_part1b<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsB));
    hipLaunchKernelGGL((k_part1b<16>), dim3(pa2.ng * B.nsb), dim3(256), ldsB, st, B, (const PtU4*)grecA, glkA,
                       (PtU4*)grec, glk, (uint32_t)nt, pk_flags);
    HIPCHK(hipGetLastError());
    h->kend();
  }
}

// keys whose rows (sorted positions of one key, carried rows first) go back in time
template <class T, bool N>
__global__ void k_order_keys(Src<T, N> src, KeyOf kf, const uint32_t* __restrict__ seg_b, uint32_t K, int64_t nt,
                             uint8_t* __restrict__ kx) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; p < nt; p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = kf(src.row((uint32_t)p));
    if (k < K && (uint32_t)p > seg_b[k] && src.ts((uint32_t)p) < src.ts((uint32_t)(p - 1))) kx[k] = 1;
  }
}

// rows listed in rows[0, *n) -> carry bitmask (the pending partials of every key the rows list)
static __global__ void k_carry_mark_list(const uint32_t* __restrict__ rows, const uint32_t* __restrict__ n,
                                         uint32_t* __restrict__ bits) {
  const uint32_t m = *n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
    atomicOr(&bits[rows[i] >> 5], 1u << (rows[i] & 31));
}

// pending entries kept as values (LDS rings without a row plane) -> carried candidate rows [base, base + n): time,
// key, the compared value and e1's payload attribute; every other column of such a row is never read (no select
// gathers an e1 attribute by row when the ring has no row plane, and a carried row is never a B row)
template <class T>
__global__ void k_carry_vals(uint32_t n, const int64_t* __restrict__ cts, const int32_t* __restrict__ ckey,
                             const int64_t* __restrict__ cval, const int64_t* __restrict__ cpay, int val_col, int pay_col,
                             int pay_w, int n_cols, uint32_t base, CarryBufs dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t d = base + i;
  dst.ts[d] = cts[i];
  dst.key[d] = ckey[i];
  dst.flags[d] = (uint8_t)F_CAND;
  const uint64_t vb = (uint64_t)cval[i];
  T x;
  if constexpr (sizeof(T) == 4) { const uint32_t w = (uint32_t)vb; __builtin_memcpy(&x, &w, 4); }
  else __builtin_memcpy(&x, &vb, 8);
  ((T*)dst.col[val_col])[d] = x;
  if (pay_col >= 0) {
    if (pay_w == 8) ((int64_t*)dst.col[pay_col])[d] = cpay[i];
    else ((int32_t*)dst.col[pay_col])[d] = (int32_t)cpay[i];
  }
  for (int c = 0; c < n_cols; ++c) dst.nul[c][d] = 0;
}

// The next push's carried rows: every key's final pending list -- listed rows (alive) copied in arrival order, then
// the entries kept as values (cv) appended.  Per key one of the two; per key pending order.
template <class T, bool N>
static void carry_out_rows(SgHandle* h, EveryNextState* es, int64_t nt, const Virt& v, const BatchView& bv,
                           const SgCols& cc, const WalkArgs& wa, int val_col, int pay_col, int pay_w) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  CarrySet& cs = es->carry[es->cur];
  uint32_t* ccount = (uint32_t*)h->ws.get("carry_count", sizeof(uint32_t) * 2, st);
  h->kbeg("carry");
  const int64_t nb = (nt + CARRY_BLK - 1) / CARRY_BLK;
  uint32_t* cbits = (uint32_t*)h->ws.get("carry_bits", sizeof(uint32_t) * (size_t)(nb * 256), st);
  uint32_t* cboff = (uint32_t*)h->ws.get("carry_boff", sizeof(uint32_t) * (size_t)(nb + 1), st);
  uint32_t* bcnt = (uint32_t*)h->ws.get("carry_bcnt", sizeof(uint32_t) * (size_t)(nb + 1), st);
  HIPCHK(hipMemsetAsync(cbits, 0, sizeof(uint32_t) * (size_t)(nb * 256), st));
  hipLaunchKernelGGL(k_carry_mark_list, dim3((unsigned)std::min<int64_t>((nt + 255) / 256, 4096)), dim3(256), 0, st,
                     wa.alive, wa.alive_n, cbits);
  hipLaunchKernelGGL(k_carry_bcount, dim3((unsigned)nb), dim3(256), 0, st, nt, cbits, bcnt);
  HIPCHK(hipMemsetAsync(bcnt + nb, 0, sizeof(uint32_t), st));
  HIPCHK(hipGetLastError());
  size_t tb = 0;
  HIPCHK(rocprim::exclusive_scan(nullptr, tb, bcnt, cboff, (uint32_t)0, (size_t)nb + 1, rocprim::plus<uint32_t>(), st));
  void* tmp = h->ws.get("carry_scan_tmp", tb, st);
  HIPCHK(rocprim::exclusive_scan(tmp, tb, bcnt, cboff, (uint32_t)0, (size_t)nb + 1, rocprim::plus<uint32_t>(), st));
  HIPCHK(hipMemcpyAsync(ccount, cboff + nb, sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync(ccount + 1, wa.cv_n, sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  h->kend();
  uint32_t hc[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(hc, ccount, sizeof(hc), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint32_t nrow = hc[0], nval = hc[1];
  CarrySet& nx = es->carry[es->cur ^ 1];
  nx.ensure(std::max<int64_t>((int64_t)nrow + nval, 1), d.n_cols, d.col_type);
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
  if (nrow)
    hipLaunchKernelGGL(k_carry_gather, dim3((unsigned)nb), dim3(256), 0, st, v, nt, cbits, cboff, d.n_cols, widths,
                       bv.cols, cc, cb);
  if (nval) {
    for (int c = 0; c < d.n_cols; ++c)   // (columns the value entries do not set: deterministic snapshots)
      if (c != val_col && c != pay_col)
        HIPCHK(hipMemsetAsync((char*)nx.col[c] + (size_t)hw[c] * nrow, 0, (size_t)hw[c] * nval, st));
    hipLaunchKernelGGL(k_carry_vals<T>, dim3((nval + 255) / 256), dim3(256), 0, st, nval, wa.cv_ts, wa.cv_key, wa.cv_val,
                       wa.cv_pay, val_col, pay_col, pay_w, d.n_cols, nrow, cb);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  nx.n = (int64_t)nrow + nval;
  cs.n = 0;
  es->cur ^= 1;
}

// The group walker (gwalk.h) for a push whose partition ran pass 1 in two (more than 65,536 keys): returns 1 when it
// delivered the push, 2 when the push needs wide records (the caller returns false), 0 when it declines -- nothing
// was delivered and no state changed, so the caller reruns the push on the tiled path.
struct GwPlan {
  bool ok = false;
  int cap = 0;
  GwSel sel;
};
template <class T>
static GwPlan gw_plan(SgHandle* h, const BatchView& bv, int64_t n, int64_t nc, uint32_t kb, const PushPlan& plan,
                      int val_col_a, int val_col_b, bool same_col, int prog_b_len) {
  const sg_nfa_desc& d = h->desc;
  GwPlan g;
  memset(&g.sel, 0, sizeof(g.sel));
  if (!d.partitioned || !same_col || plan.e1_row || d.n_select > SG_MAX_SELECT) return g;
  (void)val_col_b;
  (void)prog_b_len;
  for (int c = 0; c < d.n_cols; ++c)
    if (bv.cols.nul[c]) return g;
  for (int s = 0; s < d.n_select; ++s) {
    const int src = plan.pp.src[s], kind = plan.pp.kind[s];
    int code = -1;
    if (kind == 2) code = 4;
    else if (kind == 0 && src == 0) code = 0;
    else if (kind == 1) code = src ? 2 : 1;
    else if (kind == 3 && src == 1 && plan.pcol >= 0 && plan.pp.col[s] == plan.pcol) code = 3;
    if (code < 0) return g;
    g.sel.code[s] = code;
  }
  // ring capacity as the tiled walker picks it (rows per key per window from the push's time span)
  int64_t tfl[2] = {0, 0};
  hipStream_t st = h->stream;
  HIPCHK(hipMemcpyAsync(&tfl[0], bv.ts, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&tfl[1], bv.ts + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const int64_t win = window_rows(kb, nc + n, d.within, tfl[1] - tfl[0]);
  // the ring as the tiled walker sizes it (a key whose list outgrows it is walked again on an unbounded list by
  // k_gw_redo); the LDS chunk shrinks as the ring grows so two workgroups share a CU (launch_gwalk)
  const char* e = getenv("SG_DEBUG_GW_CAP");   // (test hook)
  int cap = h->opt.ring_cap > 0 ? h->opt.ring_cap : (e ? atoi(e) : pick_cap(win));
  if (cap > 32 || cap < 2 || (cap & (cap - 1))) return g;
  g.cap = cap;
  g.sel.n_select = d.n_select;
  g.sel.stride = 32 + 8 * d.n_select;
  g.sel.vfloat = std::is_same<T, float>::value ? 1 : 0;
  g.ok = true;
  return g;
}

template <class T, int OP, int PT, bool STACK>
static void launch_gwalk_pt(const GwArgs& ga, uint32_t ng, hipStream_t st) {
  const size_t lds = sizeof(GwLds<PT>) + (size_t)ga.cap * 256 * (sizeof(T) + 8);
  HIPCHK(hipFuncSetAttribute((const void*)k_gwalk<T, OP, PT, STACK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_gwalk<T, OP, PT, STACK>), dim3(ng), dim3(256), lds, st, ga);
  HIPCHK(hipGetLastError());
}
template <class T, int OP>
static void launch_gw_redo(const GwArgs& ga, uint32_t nk, uint32_t* rows, T* hv, int32_t* ht, int32_t* hp, hipStream_t st) {
  if (ga.stack_mode) hipLaunchKernelGGL((k_gw_redo<T, OP, true>), dim3(nk), dim3(256), 0, st, ga, rows, hv, ht, hp);
  else hipLaunchKernelGGL((k_gw_redo<T, OP, false>), dim3(nk), dim3(256), 0, st, ga, rows, hv, ht, hp);
  HIPCHK(hipGetLastError());
}
template <class T, int OP>
static void launch_gwalk(const GwArgs& ga, uint32_t ng, hipStream_t st) {
  // rows per thread per LDS chunk: the largest that leaves room for two workgroups per CU beside the ring (measured on
  // C5, profiles/r06/ab_gw.sh: 8 with an 8-entry ring, 6 with 16; with 32 one workgroup per CU whatever the chunk)
  const char* e = getenv("SG_DEBUG_GW_PT");   // (test hook)
  const int pt = e ? atoi(e) : (ga.cap <= 8 ? 8 : ga.cap <= 16 ? 6 : 4);
  if (ga.stack_mode) {
    if (pt == 4) launch_gwalk_pt<T, OP, 4, true>(ga, ng, st);
    else if (pt == 12) launch_gwalk_pt<T, OP, 12, true>(ga, ng, st);
    else if (pt == 10) launch_gwalk_pt<T, OP, 10, true>(ga, ng, st);
    else if (pt == 6) launch_gwalk_pt<T, OP, 6, true>(ga, ng, st);
    else launch_gwalk_pt<T, OP, 8, true>(ga, ng, st);
  } else {
    launch_gwalk_pt<T, OP, 8, false>(ga, ng, st);
  }
}

template <class T>
static int run_group_walk(SgHandle* h, const BatchView& bv, int64_t n, int64_t nc, uint32_t kb, const PartPlan& pp,
                          const uint32_t* o1, const WRec<T, true>* grec, const uint8_t* glk, uint32_t* pk_flags,
                          const GwPlan& gp, const PushPlan& plan, const Virt& v, const SgCols& cc, int op, int stack_mode,
                          int val_col_a, EveryNextState* es) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int64_t nt = nc + n;
  const uint32_t ng = (kb + 255) >> 8;
  // per-key rows -> each key's first row in the group domain (its match-area region starts at 3x that)
  uint32_t* kcnt = (uint32_t*)h->ws.get("gw_kcnt", sizeof(uint32_t) * ((size_t)kb + 1), st);
  uint32_t* kbase = (uint32_t*)h->ws.get("gw_kbase", sizeof(uint32_t) * ((size_t)kb + 1), st);
  h->kbeg("gw_count");
  HIPCHK(hipMemsetAsync(kcnt, 0, sizeof(uint32_t) * ((size_t)kb + 1), st));
  hipLaunchKernelGGL(k_gw_count, dim3(ng), dim3(256), 0, st, o1, pp.ns1, kb, glk, kcnt);
  HIPCHK(hipGetLastError());
  {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, kcnt, kbase, (uint32_t)0, (size_t)kb + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("gw_kscan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, kcnt, kbase, (uint32_t)0, (size_t)kb + 1, rocprim::plus<uint32_t>(), st));
  }
  h->kend();
  uint32_t pkf = 0;
  int64_t t0 = 0;   // narrow records' time origin: the push's first virtual row
  HIPCHK(hipMemcpyAsync(&pkf, pk_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&t0, nc ? v.c_ts : v.ts, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (pkf & PK_KEY_RANGE) throw SgError(SG_EINVAL, "a partition key id is >= the batch's key_bound");
  if (pkf & PK_INTERNAL) throw SgError(SG_EINVAL, "internal: key partition offsets out of range");
  if (pkf & PK_TS_RANGE) return 2;
  if (pkf & PK_PAY_RANGE) return 0;   // a payload wider than 32 bits: the tiled path gathers e1 by row
  h->mark(2);

  GwArgs ga;
  memset(&ga, 0, sizeof(ga));
  ga.n = n;
  ga.nc = nc;
  ga.within = d.within;
  ga.t0 = t0;
  ga.K = kb;
  ga.ns1 = pp.ns1;
  ga.stack_mode = stack_mode;
  ga.cap = gp.cap;
  ga.chunk = 4096;
  ga.carry_out = h->opt.no_carry ? 0 : 1;
  ga.pzero = v.pfloat;
  ga.o1 = o1;
  ga.grec = (const PtU4*)grec;
  ga.glk = glk;
  ga.kbase = kbase;
  ga.trig = (uint64_t*)h->ws.get("gw_trig", sizeof(uint64_t) * ((size_t)n + 1), st);
  ga.area = (uint64_t*)h->ws.get("gw_area", sizeof(uint64_t) * 3 * (size_t)std::max<int64_t>(nt, 1), st);
  uint32_t* gflags = (uint32_t*)h->ws.get("gw_flags", sizeof(uint32_t) * 4, st);
  ga.flags = gflags;
  ga.cv_n = gflags + 1;
  ga.ovf_n = gflags + 2;
  ga.ovf_cap = std::min<uint32_t>(kb, 1u << 16);
  ga.ovf_keys = (uint32_t*)h->ws.get("gw_ovf_keys", sizeof(uint32_t) * ga.ovf_cap, st);
  ga.match_n = gflags + 3;
  // carry: at most `cap` entries per key from the LDS rings, and a redone key's whole list -- room for 4M of those
  // (more sends the push to the tiled path)
  ga.cv_cap = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(nt, (int64_t)kb * gp.cap + (1 << 22)));
  ga.cv_ts = (int64_t*)h->ws.get("cv_ts", sizeof(int64_t) * (size_t)ga.cv_cap, st);
  ga.cv_val = (int64_t*)h->ws.get("cv_val", sizeof(int64_t) * (size_t)ga.cv_cap, st);
  ga.cv_pay = (int64_t*)h->ws.get("cv_pay", sizeof(int64_t) * (size_t)ga.cv_cap, st);
  ga.cv_key = (int32_t*)h->ws.get("cv_key", sizeof(int32_t) * (size_t)ga.cv_cap, st);
  HIPCHK(hipMemsetAsync(gflags, 0, sizeof(uint32_t) * 4, st));
  HIPCHK(hipMemsetAsync(ga.trig, 0, sizeof(uint64_t) * ((size_t)n + 1), st));
  h->kbeg("group_walk");
  switch (op) {
    case 2: launch_gwalk<T, 2>(ga, ng, st); break;
    case 3: launch_gwalk<T, 3>(ga, ng, st); break;
    case 4: launch_gwalk<T, 4>(ga, ng, st); break;
    default: launch_gwalk<T, 5>(ga, ng, st); break;
  }
  h->kend();
  uint32_t hf[4] = {0, 0, 0, 0}, total = 0;
  HIPCHK(hipMemcpyAsync(hf, gflags, sizeof(hf), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (hf[0] & GW_INTERNAL) throw SgError(SG_EINVAL, "internal: group walker guard tripped");
  if (hf[0]) return 0;   // a key whose time goes back (or more ring overflows than the list holds): the tiled path
  if (hf[2]) {
    // keys whose pending list outgrew the LDS ring: each walked again with an unbounded HBM list
    h->kbeg("gw_redo");
    uint32_t* rrows = (uint32_t*)h->ws.get("gw_redo_rows", sizeof(uint32_t) * (size_t)nt, st);
    char* rl = (char*)h->ws.get("gw_redo_list", (sizeof(T) + 8) * (size_t)nt, st);
    T* hv = (T*)rl;
    int32_t* ht = (int32_t*)(rl + sizeof(T) * (size_t)nt);
    int32_t* hp = ht + nt;
    switch (op) {
      case 2: launch_gw_redo<T, 2>(ga, hf[2], rrows, hv, ht, hp, st); break;
      case 3: launch_gw_redo<T, 3>(ga, hf[2], rrows, hv, ht, hp, st); break;
      case 4: launch_gw_redo<T, 4>(ga, hf[2], rrows, hv, ht, hp, st); break;
      default: launch_gw_redo<T, 5>(ga, hf[2], rrows, hv, ht, hp, st); break;
    }
    h->kend();
    HIPCHK(hipMemcpyAsync(hf, gflags, sizeof(hf), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (hf[0] & GW_INTERNAL) throw SgError(SG_EINVAL, "internal: group walker redo guard tripped");
    if (hf[0]) return 0;
  }
  h->last_spilled = hf[2];
  total = hf[3];   // matches, counted by the walkers
  h->mark(3);
  h->split_out = 1;
  h->mark(5);
  if (total) {
    char* out = h->out.reserve(total, d.n_select, st);
    GwSel sel = gp.sel;
    int rb = d.recv_of_stream[d.states[d.shape_args[1]].stream];
    sel.multi = d.receivers[rb].multi;
    sel.b_slot = 0;
    if (sel.multi) {
      const sg_receiver_desc& r = d.receivers[rb];
      for (int q = 0; q < r.n; ++q)
        if (r.pres[r.n - 1 - q] == d.shape_args[1]) sel.b_slot = q;
    }
    sel.pzero = v.pfloat;
    // per-tile match counts -> tile bases (scan) -> output records per tile (block scan inside the tile)
    const int64_t ntile = (n + GW_TILE - 1) / GW_TILE;
    uint32_t* tcount = (uint32_t*)h->ws.get("gw_tcount", sizeof(uint32_t) * ((size_t)ntile + 1), st);
    uint32_t* tbase = (uint32_t*)h->ws.get("gw_tbase", sizeof(uint32_t) * ((size_t)ntile + 1), st);
    h->kbeg("gw_tiles");
    HIPCHK(hipMemsetAsync(tcount + ntile, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_gtile_count, dim3((unsigned)((ntile + 7) / 8)), dim3(256), 0, st, n, (const uint64_t*)ga.trig, tcount,
                       ntile);
    HIPCHK(hipGetLastError());
    {
      size_t tb = 0;
      HIPCHK(rocprim::exclusive_scan(nullptr, tb, tcount, tbase, (uint32_t)0, (size_t)ntile + 1, rocprim::plus<uint32_t>(), st));
      void* tmp = h->ws.get("gw_tscan_tmp", tb, st);
      HIPCHK(rocprim::exclusive_scan(tmp, tb, tcount, tbase, (uint32_t)0, (size_t)ntile + 1, rocprim::plus<uint32_t>(), st));
    }
    h->kend();
    uint32_t tsum = 0;
    HIPCHK(hipMemcpyAsync(&tsum, tbase + ntile, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    h->kbeg("gw_project");
    const size_t plds = (size_t)GW_PROJ_S * sel.stride;
    if (plds > 65536)
      HIPCHK(hipFuncSetAttribute((const void*)k_gscan_project, hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds));
    hipLaunchKernelGGL(k_gscan_project, dim3((unsigned)ntile), dim3(256), plds, st, n, ga.t0, bv.base_index, bv.index,
                       (const uint64_t*)ga.trig, (const uint64_t*)ga.area, sel, (int64_t)h->out.n, out,
                       (const uint32_t*)tbase);
    HIPCHK(hipGetLastError());
    h->kend();
    HIPCHK(hipStreamSynchronize(st));
    if (tsum != total) throw SgError(SG_EINVAL, "internal: group walker match count mismatch");
    h->out.n += total;
  }
  h->mark(4);
  if (ga.carry_out) {
    WalkArgs wa;
    memset(&wa, 0, sizeof(wa));
    wa.alive = (uint32_t*)h->ws.get("alive_rows", sizeof(uint32_t), st);
    wa.alive_n = (uint32_t*)h->ws.get("gw_alive_n", sizeof(uint32_t), st);
    HIPCHK(hipMemsetAsync(wa.alive_n, 0, sizeof(uint32_t), st));
    wa.cv_n = ga.cv_n;
    wa.cv_ts = ga.cv_ts;
    wa.cv_key = ga.cv_key;
    wa.cv_val = ga.cv_val;
    wa.cv_pay = ga.cv_pay;
    carry_out_rows<T, true>(h, es, nt, v, bv, cc, wa, val_col_a, v.pcol ? plan.pcol : -1, v.pw);
  }
  h->last_events = n;
  h->last_matches = total;
  return 1;
}

template <class T, bool N>
static bool run_every_next(SgHandle* h, const BatchView& bv, int64_t n, PushPlan plan, bool allow_group = true) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int* sa = d.shape_args;
  const int a_state = sa[0], b_state = sa[1], op = sa[2];
  EveryNextState* es = (EveryNextState*)h->state;
  CarrySet& cs = es->carry[es->cur];
  const int64_t nc = h->opt.no_carry ? 0 : cs.n;
  const int64_t nt = nc + n;
  if (nt >= (1ll << 30)) throw SgError(SG_EINVAL, "batch plus carried rows exceed 2^30");
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
  h->kbeg("pred");
  launch_pred(d, pa, bv.stream, bv.cols, h->ddesc, cand_m, cons_m, st);
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(1);

  // ---- 2. key partition: per-key walker records in arrival order
  Virt v;
  memset(&v, 0, sizeof(v));
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
  v.stream = bv.stream;
  v.s_b = pa.s_b;
  v.c_val_a = cs.col[val_col_a];
  v.c_val_b = cs.col[val_col_b];
  if (plan.pcol >= 0) {
    const int c = plan.pcol;
    v.pcol = bv.cols.col[c];
    v.c_pcol = cs.col[c];
    v.pw = (d.col_type[c] == SG_T_LONG || d.col_type[c] == SG_T_DOUBLE) ? 8 : 4;
    v.pfloat = d.col_type[c] == SG_T_FLOAT;
  }
  SgCols cc;
  memset(&cc, 0, sizeof(cc));
  for (int c = 0; c < d.n_cols; ++c) { cc.col[c] = cs.col[c]; cc.nul[c] = cs.nul[c]; }
  if (!d.partitioned && !h->opt.walker_only && run_nge<T>(h, bv, n, nc, plan, v, cc, op, es)) return true;

  typedef WRec<T, N> R;
  Src<T, N> src;
  src.srec = nullptr;
  src.pk.v = v;
  const uint32_t K = d.partitioned ? kb : 1;
  uint32_t* pk_flags = nullptr;
  uint32_t* seg_b = nullptr;   // (unpartitioned: one segment [0, nt))
  uint32_t* seg_e = nullptr;
  pk_flags = (uint32_t*)h->ws.get("pack_flags", sizeof(uint32_t), st);
  HIPCHK(hipMemsetAsync(pk_flags, 0, sizeof(uint32_t), st));
  R* prec = (R*)h->ws.get("prec", sizeof(R) * nt, st);
  seg_b = (uint32_t*)h->ws.get("seg_b", sizeof(uint32_t) * K, st);
  seg_e = (uint32_t*)h->ws.get("seg_e", sizeof(uint32_t) * K, st);
  const dim3 pgrd((unsigned)std::min<int64_t>((nt + 255) / 256, 256 * 32));
  // beyond 65536 keys (C5: 1M per GPU) the LDS partition runs its first pass in two (part1_wide: narrow records only,
  // up to 4096 groups of 256 keys) -- three counting passes in place of pack + a 3-pass onesweep sort + bounds
  const bool wide_part = N && sizeof(R) == 16 && sizeof(T) == 4 && kb > 65536u && kb <= (4096u << 8);
  const bool lds_part = d.partitioned && (kb <= 65536u || wide_part) && h->opt.partition_sort == 0;
  if (lds_part) {
    PartPlan pp = part_plan(kb, nt);
    if (kb > 65536u) {   // groups of 256 keys: pass 2 sorts by the low 8 bits
      pp.two = 1;
      pp.lb = 8;
      pp.ng = (kb + 255u) >> 8;
      pp.nb1 = 0;
      while ((1u << pp.nb1) < pp.ng) ++pp.nb1;
      pp.nb2 = 8;
      pp.ts2 = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(pp.ns1, (int64_t)8192 * pp.ng / pp.seg1));
      pp.nj = (pp.ns1 + pp.ts2 - 1) / pp.ts2;
    }
    KeyOf kf{bv.key, cs.key, (uint32_t)nc};
    const size_t n1 = (size_t)pp.ng * pp.ns1 + 1;
    uint32_t* h1 = (uint32_t*)h->ws.get("part_h1", sizeof(uint32_t) * n1, st);
    uint32_t* o1 = (uint32_t*)h->ws.get("part_o1", sizeof(uint32_t) * n1, st);
    R* srec = (R*)h->ws.get("srec", sizeof(R) * nt, st);
    typedef PtRaw<R> RW;
    static_assert(sizeof(RW) == sizeof(R), "raw record layout");
    const size_t lds1 = sizeof(PartLds<R, PT1>), lds2 = sizeof(PartLds<RW, PT2>);
    HIPCHK(hipFuncSetAttribute((const void*)k_part1<T, N>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
    HIPCHK(hipFuncSetAttribute((const void*)k_part2<RW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
    size_t tb = 0;
    void* tmp = nullptr;
    if (kb <= 65536u) {
      h->kbeg("part_hist");
      HIPCHK(hipMemsetAsync(h1 + n1 - 1, 0, sizeof(uint32_t), st));
      hipLaunchKernelGGL(k_part1_hist, dim3(pp.ns1), dim3(256), 0, st, kf, pp, nt, h1, pk_flags);
      HIPCHK(hipGetLastError());
      HIPCHK(rocprim::exclusive_scan(nullptr, tb, h1, o1, (uint32_t)0, n1, rocprim::plus<uint32_t>(), st));
      tmp = h->ws.get("part_scan_tmp", tb, st);
      HIPCHK(rocprim::exclusive_scan(tmp, tb, h1, o1, (uint32_t)0, n1, rocprim::plus<uint32_t>(), st));
      h->kend();
    }
    if (!pp.two) {
      h->kbeg("part_scatter");
      hipLaunchKernelGGL((k_part1<T, N>), dim3(pp.ns1), dim3(256), lds1, st, src.pk, kf, pp, nt, o1, srec, (uint8_t*)nullptr,
                         pk_flags);
      HIPCHK(hipGetLastError());
      h->kend();
      hipLaunchKernelGGL(k_part_segs, dim3((kb + 255) / 256), dim3(256), 0, st, kb, o1, pp.ns1, seg_b, seg_e);
    } else {
      R* grec = (R*)h->ws.get("grec", sizeof(R) * nt, st);
      uint8_t* glk = (uint8_t*)h->ws.get("glk", nt, st);
      const size_t n2 = ((size_t)pp.ng << pp.lb) * pp.nj + 1;
      uint32_t* h2 = (uint32_t*)h->ws.get("part_h2", sizeof(uint32_t) * n2, st);
      uint32_t* o2 = (uint32_t*)h->ws.get("part_o2", sizeof(uint32_t) * n2, st);
      if (kb > 65536u) {
        if constexpr (N && sizeof(R) == 16 && sizeof(T) == 4) {
          // many keys: the group walker (gwalk.h) when the query and the push allow it, else the tiled path below
          GwPlan gp;
          const bool same = (val_col_a == val_col_b) && (pa.s_a == pa.s_b);
          if (allow_group) gp = gw_plan<T>(h, bv, n, nc, kb, plan, val_col_a, val_col_b, same, pa.prog_b_len);
          part1_wide<T>(h, src.pk, kf, kb, nt, pp, h1, o1, grec, glk, pk_flags);
          if (gp.ok) {
            const int rc = run_group_walk<T>(h, bv, n, nc, kb, pp, o1, grec, glk, pk_flags, gp, plan, v, cc, op,
                                             (same && pa.prog_b_len == 0) ? 1 : 0, val_col_a, es);
            if (rc == 1) return true;
            if (rc == 2) return false;
            return run_every_next<T, N>(h, bv, n, plan, false);
          }
        }
      } else {
        h->kbeg("part_group");
        hipLaunchKernelGGL((k_part1<T, N>), dim3(pp.ns1), dim3(256), lds1, st, src.pk, kf, pp, nt, o1, grec, glk, pk_flags);
        HIPCHK(hipGetLastError());
        h->kend();
      }
      h->kbeg("part_hist2");
      HIPCHK(hipMemsetAsync(h2 + n2 - 1, 0, sizeof(uint32_t), st));
      hipLaunchKernelGGL(k_part2_hist, dim3(pp.ng * pp.nj), dim3(256), 0, st, pp, o1, glk, h2);
      HIPCHK(hipGetLastError());
      tb = 0;
      HIPCHK(rocprim::exclusive_scan(nullptr, tb, h2, o2, (uint32_t)0, n2, rocprim::plus<uint32_t>(), st));
      tmp = h->ws.get("part_scan_tmp2", tb, st);
      HIPCHK(rocprim::exclusive_scan(tmp, tb, h2, o2, (uint32_t)0, n2, rocprim::plus<uint32_t>(), st));
      h->kend();
      h->kbeg("part_key");
      hipLaunchKernelGGL((k_part2<RW>), dim3(pp.ng * pp.nj), dim3(256), lds2, st, pp, o1, o2, (const RW*)grec, glk, (RW*)srec,
                         (uint32_t)nt, pk_flags);
      HIPCHK(hipGetLastError());
      h->kend();
      hipLaunchKernelGGL(k_part_segs, dim3((kb + 255) / 256), dim3(256), 0, st, kb, o2, pp.nj, seg_b, seg_e);
    }
    HIPCHK(hipGetLastError());
    src.srec = srec;
  } else if (d.partitioned) {
    int end_bit = 1;
    while ((1ull << end_bit) <= (uint64_t)kb) ++end_bit;
    uint32_t* skeys = (uint32_t*)h->ws.get("skeys", sizeof(uint32_t) * nt, st);
    R* srec = (R*)h->ws.get("srec", sizeof(R) * nt, st);
    uint32_t* pkeys = (uint32_t*)h->ws.get("pkeys", sizeof(uint32_t) * nt, st);
    KeyOf kf{bv.key, cs.key, (uint32_t)nc};
    h->kbeg("pack");
    hipLaunchKernelGGL((k_pack<T, N>), pgrd, dim3(256), 0, st, src.pk, kf, kb, nt, prec, pkeys, pk_flags);
    HIPCHK(hipGetLastError());
    h->kend();
    h->kbeg("key_sort");
    size_t tb = 0;
    if constexpr (sizeof(R) == 16) {   // one onesweep instantiation for every 16-byte record format
      Blob16* pb = (Blob16*)prec;
      Blob16* sbb = (Blob16*)srec;
      HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, pkeys, skeys, pb, sbb, (size_t)nt, 0, end_bit, st));
      void* tmp = h->ws.get("sort_tmp", tb, st);
      HIPCHK(rocprim::radix_sort_pairs(tmp, tb, pkeys, skeys, pb, sbb, (size_t)nt, 0, end_bit, st));
    } else {
      HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, pkeys, skeys, prec, srec, (size_t)nt, 0, end_bit, st));
      void* tmp = h->ws.get("sort_tmp", tb, st);
      HIPCHK(rocprim::radix_sort_pairs(tmp, tb, pkeys, skeys, prec, srec, (size_t)nt, 0, end_bit, st));
    }
    h->kend();
    src.srec = srec;
    HIPCHK(hipMemsetAsync(seg_b, 0, sizeof(uint32_t) * K, st));
    HIPCHK(hipMemsetAsync(seg_e, 0, sizeof(uint32_t) * K, st));
    h->kbeg("bounds");
    hipLaunchKernelGGL(k_bounds, dim3((unsigned)std::min<int64_t>((nt + 1023) / 1024, 256 * 16)), dim3(256), 0, st, skeys,
                       nt, kb, seg_b, seg_e);
    h->kend();
    HIPCHK(hipGetLastError());
  } else {
    // unpartitioned: one key whose rows are already in arrival order
    KeyOf kf{nullptr, nullptr, 0};
    hipLaunchKernelGGL((k_pack<T, N>), pgrd, dim3(256), 0, st, src.pk, kf, kb, nt, prec, (uint32_t*)nullptr, pk_flags);
    HIPCHK(hipGetLastError());
    src.srec = prec;
    const uint32_t seg[2] = {0u, (uint32_t)nt};
    HIPCHK(hipMemcpyAsync(seg_b, &seg[0], sizeof(uint32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(seg_e, &seg[1], sizeof(uint32_t), hipMemcpyHostToDevice, st));
  }
  h->mark(2);
  // ---- 3. count pass + scan
  WalkArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.nt = nt;
  wa.within = d.within;
  wa.K = K;
  wa.lp.pay = plan.pcol >= 0 ? 1 : 0;
  wa.lp.row = plan.e1_row ? 1 : 0;
  wa.pay_in_rec = (R::has_pay && plan.pcol >= 0) ? 1 : 0;
  // (ring capacity and chunking from the batch's time span: rows per key per `within` window)
  int64_t span_ms = 0;
  {
    int64_t tfl[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&tfl[0], bv.ts, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&tfl[1], bv.ts + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    span_ms = tfl[1] - tfl[0];
  }
  const int64_t win = window_rows(K, nt, d.within, span_ms);
  wa.lp.cap = clamp_cap(h->opt.ring_cap > 0 ? h->opt.ring_cap : pick_cap(win), PendBytes<T>::lds(true, wa.lp));
  const size_t lds_count = (size_t)wa.lp.cap * WALK_BLOCK * PendBytes<T>::lds(false, wa.lp);
  const size_t lds_write = (size_t)wa.lp.cap * WALK_BLOCK * PendBytes<T>::lds(true, wa.lp);
  wa.C = (uint32_t)pick_chunks(K, nt, PendBytes<T>::lds(true, wa.lp), wa.lp.cap, win);   // record walk's ring
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
  UnitDesc* ud = (UnitDesc*)h->ws.get("units", sizeof(UnitDesc) * units, st);
  WalkStats* wst = (WalkStats*)h->ws.get("walkstats", sizeof(WalkStats), st);
  uint32_t* cnt = (uint32_t*)h->ws.get("cnt", sizeof(uint32_t) * (n + 1), st);
  uint32_t* off = (uint32_t*)h->ws.get("off", sizeof(uint32_t) * (n + 1), st);
  uint32_t* emap = (uint32_t*)h->ws.get("emap", sizeof(uint32_t) * (nt / 32 + 2), st);
  const dim3 wblk(WALK_BLOCK), wgrd((unsigned)((units + WALK_BLOCK - 1) / WALK_BLOCK));
  const uint32_t nw = (uint32_t)((units + 63) / 64);
  MatchSink ms{nullptr, 0, 0, &wst->internal};   // (record pass: set once the match list is allocated)
  uint32_t* wlen = (uint32_t*)h->ws.get("wlen", sizeof(uint32_t) * (nw + 1), st);
  uint32_t* wrow = (uint32_t*)h->ws.get("wrow", sizeof(uint32_t) * (nw + 1), st);
  R* tile = nullptr;
  uint64_t* emask = nullptr;
  auto scan_counts = [&]() {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
  };
  WalkStats hs;
  uint32_t total = 0;
  char* big = nullptr;
  h->extra_marks = 0;
  // Pass 0 walks every key on the fast path, which needs each key's time not to go back.  When some key's does
  // (its rows, carried ones included, out of time order), pass 1 redoes the count with those keys on the exact walker.
  for (int pass = 0;; ++pass) {
    HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (n + 1), st));
    HIPCHK(hipMemsetAsync(emap, 0, sizeof(uint32_t) * (nt / 32 + 2), st));
    HIPCHK(hipMemsetAsync(wst, 0, sizeof(WalkStats), st));
    // lane-interleaved tiles: unit ranges -> per-wave rows -> LDS transpose of the sorted records
    HIPCHK(hipMemsetAsync(wlen, 0, sizeof(uint32_t) * (nw + 1), st));
    h->kbeg("units");
    hipLaunchKernelGGL((k_units<T, N>), dim3((unsigned)(nw * 64 + 255) / 256), dim3(256), 0, st, wa, src, seg_b, seg_e,
                       ud, wlen, wst);
    HIPCHK(hipGetLastError());
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, wlen, wrow, (uint32_t)0, (size_t)nw + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("wscan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, wlen, wrow, (uint32_t)0, (size_t)nw + 1, rocprim::plus<uint32_t>(), st));
    h->kend();
    uint32_t rows_total = 0, pkf = 0;
    HIPCHK(hipMemcpyAsync(&rows_total, wrow + nw, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&pkf, pk_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (pkf & PK_KEY_RANGE) throw SgError(SG_EINVAL, "a partition key id is >= the batch's key_bound");
    if (pkf & PK_INTERNAL) throw SgError(SG_EINVAL, "internal: key partition offsets out of range");
    if (pkf & PK_TS_RANGE) return false;   // the push spans more than 2^31 ms: wide records
    if (pkf & PK_PAY_RANGE) {
      // a payload value wider than 32 bits: gather e1's attributes by row instead
      for (int s = 0; s < d.n_select; ++s)
        if (plan.pp.kind[s] == 0) { plan.pp.kind[s] = 3; plan.e1_row = true; }
      plan.pcol = -1;
      wa.lp.pay = 0;
      wa.lp.row = 1;
      wa.pay_in_rec = 0;
      v.pcol = nullptr;
      src.pk.v.pcol = nullptr;
    }
    tile = (R*)h->ws.get("tile", sizeof(R) * 64 * (size_t)std::max<uint32_t>(rows_total, 1), st);
    emask = (uint64_t*)h->ws.get("emask", sizeof(uint64_t) * std::max<uint32_t>(rows_total, 1), st);
    const uint32_t nq = rows_total / TROWS;
    if (nq) {
      uint32_t* rmap = (uint32_t*)h->ws.get("rowmap", sizeof(uint32_t) * nq, st);
      hipLaunchKernelGGL(k_rowmap, dim3((nw + 255) / 256), dim3(256), 0, st, wlen, wrow, nw, rmap);
      HIPCHK(hipGetLastError());
      h->kbeg("tile_transpose");
      hipLaunchKernelGGL((k_transpose<T, N>), dim3(std::min<uint32_t>(nq, 256 * 32)), dim3(256), 0, st, src.srec, ud, wrow,
                         rmap, nq, tile, (uint32_t)nt, wa.n_units, wst);
      HIPCHK(hipGetLastError());
      h->kend();
    }
    h->kbeg("walk_count");
    launch_walk_t<T, N, false>(op, wgrd, wblk, lds_count, st, wa, src, seg_b, seg_e, ud, wlen, wrow, tile, cnt, off, ms,
                               emask, wst);
    h->kend();
    h->kbeg("count_scan");
    scan_counts();
    h->kend();
    h->mark(3);
    HIPCHK(hipMemcpyAsync(&total, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&hs, wst, sizeof(WalkStats), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (hs.n_ovf) {
      // units whose pending list outgrew the LDS ring (or that walk exact): redo them with unbounded HBM lists
      if (hs.internal & 16u) throw SgError(SG_ECAPACITY, "HBM pending lists exceed 2^32 entries: push smaller batches");
      wa.big_total = hs.ovf_total;
      big = (char*)h->ws.get("big_lists", (size_t)hs.ovf_total * PendBytes<T>::hbm, st);
      h->mark(6);
      hipLaunchKernelGGL((k_walk<T, N, false, true>), wgrd, wblk, 0, st, wa, src, seg_b, seg_e, ud, cnt, off,
                         ms, emap, wst, big);
      HIPCHK(hipGetLastError());
      scan_counts();
      h->mark(7);
      h->extra_marks = 1;
      HIPCHK(hipMemcpyAsync(&total, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&hs, wst, sizeof(WalkStats), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    if (hs.internal) throw SgError(SG_EINVAL, "internal: walker guard tripped (" + std::to_string(hs.internal) + ")");
    if (!hs.order_err) break;
    if (pass) throw SgError(SG_EINVAL, "internal: a key's time went back on the fast walker after the exact pass");
    // keys whose time goes back (StreamPreStateProcessor.isExpired compares |e1.ts - ts| with `within`, and a playback
    // clock that stays put still processes the row, TimestampGeneratorImpl.java:106-125): exact walker
    uint8_t* kx = (uint8_t*)h->ws.get("kexact", K, st);
    if (d.partitioned) {
      HIPCHK(hipMemsetAsync(kx, 0, K, st));
      KeyOf kf{bv.key, cs.key, (uint32_t)nc};
      hipLaunchKernelGGL((k_order_keys<T, N>), dim3((unsigned)std::min<int64_t>((nt + 255) / 256, 256 * 64)), dim3(256), 0,
                         st, src, kf, seg_b, K, nt, kx);
      HIPCHK(hipGetLastError());
    } else {
      HIPCHK(hipMemsetAsync(kx, 1, K, st));
    }
    wa.kexact = kx;
  }

  // ---- 5. record pass
  char* out = nullptr;
  h->split_out = 1;
  if (!(total || wa.carry_out)) h->mark(5);
  if (total || wa.carry_out) {
    out = h->out.reserve(total, d.n_select, st);
    wa.out_base = h->out.n;
    // narrow match records when the value type is 4 bytes and every payload fits 32 bits (narrow walker records)
    ms.narrow = (N && sizeof(T) == 4) ? 1 : 0;
    ms.cap = total;
    ms.rec = h->ws.get("mrec", (ms.narrow ? sizeof(MRec16) : sizeof(MRec)) * std::max<uint32_t>(total, 1), st);
    h->mark(5);
    if (wa.carry_out) {   // each key's final pending list (k_walk / k_walk_t, record pass)
      wa.alive = (uint32_t*)h->ws.get("alive_rows", sizeof(uint32_t) * (size_t)std::max<int64_t>(nt, 1), st);
      wa.alive_n = (uint32_t*)h->ws.get("alive_n", sizeof(uint32_t) * 2, st);
      wa.cv_n = wa.alive_n + 1;
      HIPCHK(hipMemsetAsync(wa.alive_n, 0, sizeof(uint32_t) * 2, st));
      wa.cv_cap = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(nt, (int64_t)K * wa.lp.cap));
      wa.cv_ts = (int64_t*)h->ws.get("cv_ts", sizeof(int64_t) * (size_t)wa.cv_cap, st);
      wa.cv_val = (int64_t*)h->ws.get("cv_val", sizeof(int64_t) * (size_t)wa.cv_cap, st);
      wa.cv_pay = (int64_t*)h->ws.get("cv_pay", sizeof(int64_t) * (size_t)wa.cv_cap, st);
      wa.cv_key = (int32_t*)h->ws.get("cv_key", sizeof(int32_t) * (size_t)wa.cv_cap, st);
    }
    h->kbeg("walk_record");
    launch_walk_t<T, N, true>(op, wgrd, wblk, lds_write, st, wa, src, seg_b, seg_e, ud, wlen, wrow, tile, cnt, off, ms,
                              emask, wst);
    h->kend();
    if (hs.n_ovf) {
      hipLaunchKernelGGL((k_walk<T, N, true, true>), wgrd, wblk, 0, st, wa, src, seg_b, seg_e, ud, cnt, off, ms,
                         emap, wst, big);
      HIPCHK(hipGetLastError());
    }
    if (total) {
      h->kbeg("project");
      hipLaunchKernelGGL((k_project<T>), dim3((unsigned)(((int64_t)total + 255) / 256)),
                         dim3(256), (size_t)256 * wa.stride, st, wa, v, plan.pp, bv.cols, cc, ms, off, (int64_t)total, out);
      HIPCHK(hipGetLastError());
      h->kend();
    }
    h->out.n += total;
  }
  h->mark(4);

  // ---- 6. carry into the next push
  if (wa.carry_out) {
    uint32_t guard = 0;
    HIPCHK(hipMemcpyAsync(&guard, &wst->internal, sizeof(uint32_t), hipMemcpyDeviceToHost, st));   // record-pass guards
    HIPCHK(hipStreamSynchronize(st));
    if (guard) throw SgError(SG_EINVAL, "internal: record-pass guard tripped (" + std::to_string(guard) + ")");
    carry_out_rows<T, N>(h, es, nt, v, bv, cc, wa, val_col_a, v.pcol ? plan.pcol : -1, v.pw);
  }
  h->last_events = n;
  h->last_matches = total;
  h->last_spilled = hs.n_ovf;
  return true;
}

// Projection plan: which select columns are the compared value and which are gathered by row at emission.
static PushPlan make_plan(SgHandle* h, const BatchView& bv) {
  const sg_nfa_desc& d = h->desc;
  EveryNextState* es = (EveryNextState*)h->state;
  for (int c = 0; c < d.n_cols; ++c) if (bv.cols.nul[c]) es->nul_seen[c] = true;
  const int b_state = d.shape_args[1];
  const int val_col_a = d.ret_col[d.shape_args[4]], val_col_b = d.ret_col[d.shape_args[3]];
  PushPlan pl;
  memset(&pl.pp, 0, sizeof(pl.pp));
  for (int s = 0; s < d.n_select; ++s) {
    ProjPlan& pp = pl.pp;
    pp.src[s] = (d.sel_state[s] == b_state) ? 1 : 0;
    int col = d.ret_col[d.sel_ret[s]];
    int idx = d.sel_index[s];
    pp.col[s] = col;
    pp.type[s] = d.sel_type[s];
    if (idx != 0 && idx != -1) pp.kind[s] = 2;
    else if (col == (pp.src[s] ? val_col_b : val_col_a)) pp.kind[s] = 1;
    else if (pp.src[s] == 0 && !es->nul_seen[col] && d.col_type[col] != SG_T_DOUBLE && (pl.pcol < 0 || pl.pcol == col)) {
      pp.kind[s] = 0;
      pl.pcol = col;
    } else {
      pp.kind[s] = 3;
      if (pp.src[s] == 0) pl.e1_row = true;
    }
  }
  return pl;
}

template <class T>
static void dispatch_np(SgHandle* h, const BatchView& bv, int64_t n) {
  if (!h->state) { h->state = new EveryNextState(); h->state_kind = 1; }
  PushPlan pl = make_plan(h, bv);   // (needs the state: null history)
  // narrow walker records whenever the push fits them (partitioned queries); wide otherwise
  if (!run_every_next<T, true>(h, bv, n, pl)) run_every_next<T, false>(h, bv, n, pl);
}
