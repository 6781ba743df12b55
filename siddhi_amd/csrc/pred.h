// pred.h -- the predicate-evaluation pass: one coalesced pass over the batch evaluates a
// state's event-local filter (the conjuncts that read only the arriving event) for every row and writes one
// condition bit per row, so the NFA passes read bits instead of re-evaluating (FilterProcessor.process,
// C/query/processor/filter/FilterProcessor.java:55-69, CompareConditionExpressionExecutor.execute,
// C/executor/condition/compare/CompareConditionExpressionExecutor.java:39-43).  Shared by the closed-form
// pipeline (engine_impl.h) and the general machine (interp.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "sg_device.h"
#include "sg_engine.h"

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

template <class Stack>
__device__ __forceinline__ bool eval_row(const PredArgs& a, const SgCols& cols, const DevDesc* dd, int64_t i,
                                         bool side_b) {
  int s = a.stream ? a.stream[i] : 0;
  int want = side_b ? a.s_b : a.s_a;
  if (s != want) return false;
  int vc = side_b ? a.val_col_b : a.val_col_a;   // (-1: no compared-value column, the program decides on nulls)
  if (vc >= 0 && cols.nul[vc] && cols.nul[vc][i]) return false;
  RowReader rd{&cols, dd->ret_col, i};
  return side_b ? sg_eval<RowReader, Stack>(dd->code + a.prog_b_off, a.prog_b_len, rd)
                : sg_eval<RowReader, Stack>(dd->code + a.prog_a_off, a.prog_a_len, rd);
}

// general: any program, scalar loads (rows 4l+s of the tile).  The VM's operand stack is D register slots, D the
// programs' depth rounded up (sg_prog_depth, checked on the host): no private segment, so no per-queue scratch the
// runtime keeps after the kernel.
template <int D>
__global__ void __launch_bounds__(256) k_pred(PredArgs a, SgCols cols, const DevDesc* __restrict__ dd,
                                              uint64_t* __restrict__ cand_m, uint64_t* __restrict__ cons_m) {
  typedef SgRegStack<D> Stack;
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
        ca = eval_row<Stack>(a, cols, dd, i, false);
        if (!a.cons_all) co = eval_row<Stack>(a, cols, dd, i, true);
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
// The constant is pre-converted to the compare domain (f32 / f64 / i64, ExpressionParser's promotion);
// the operator is a template parameter.  One-shot grid: each wave owns 4 consecutive 256-row tiles
// (4 contiguous 1 KB wave loads in flight), loaded non-temporally -- the column is read exactly once
// and must not displace the walker's working set from L2 / MALL (measured: 3.3 -> 6.2 TB/s,
// exp/predbench.hip).  The 4 tile words are stored by lanes 0..3 in one 32-B write.
template <int OP, class D>
__device__ __forceinline__ bool cmp_op(D a, D b) {
  if (OP == 0) return a == b;
  if (OP == 1) return a != b;
  if (OP == 2) return a > b;
  if (OP == 3) return a >= b;
  if (OP == 4) return a < b;
  return a <= b;
}
constexpr int PRED_TILES_PER_WAVE = 4;
template <class V, class D, int OP>
__global__ void __launch_bounds__(256) k_pred_simple(int64_t n, D c, const V* __restrict__ col,
                                                     const uint8_t* __restrict__ nul, uint64_t* __restrict__ cand_m) {
  constexpr int U = PRED_TILES_PER_WAVE;
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (n + 255) >> 8;
  const int64_t g0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * U;
  typedef V V4 __attribute__((ext_vector_type(4)));
  V4 x[U];
  if (g0 + U <= (n >> 8)) {
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load((const V4*)(col + (g0 + u) * 256 + lane * 4));
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = (g0 + u) * 256 + lane * 4;
      x[u].x = i + 0 < n ? col[i + 0] : V(0);
      x[u].y = i + 1 < n ? col[i + 1] : V(0);
      x[u].z = i + 2 < n ? col[i + 2] : V(0);
      x[u].w = i + 3 < n ? col[i + 3] : V(0);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t g = g0 + u;
    if (g >= ntiles) break;
    const int64_t i = g * 256 + lane * 4;
    const V xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
    uint64_t mine = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bool ok = (i + s < n) && cmp_op<OP, D>((D)xs[s], c);
      if (nul && ok) ok = !nul[i + s];
      const uint64_t m = __ballot(ok);
      if (lane == s) mine = m;
    }
    if (lane < 4) cand_m[g * 4 + lane] = mine;
  }
}
// simple with a stream column (several streams, e.g. `e1=Stream1[price>20] -> e2=Stream2[..]`): A's bit also needs
// the row's stream to be A's, and B's consumers are exactly the rows of B's stream (B has no local conjunct and its
// compared value no nulls) -- the stream column is streamed with 16-B loads as well
template <class V, class D, int OP>
__global__ void __launch_bounds__(256) k_pred_simple_s(int64_t n, D c, const V* __restrict__ col,
                                                       const uint8_t* __restrict__ nul, const int32_t* __restrict__ stream,
                                                       int32_t sa, int32_t sb, uint64_t* __restrict__ cand_m,
                                                       uint64_t* __restrict__ cons_m) {
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (n + 255) >> 8;
  const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (g >= ntiles) return;
  typedef V V4 __attribute__((ext_vector_type(4)));
  typedef int32_t I4 __attribute__((ext_vector_type(4)));
  const int64_t i = g * 256 + lane * 4;
  V4 x;
  I4 t;
  if (i + 4 <= n) {
    x = __builtin_nontemporal_load((const V4*)(col + i));
    t = __builtin_nontemporal_load((const I4*)(stream + i));
  } else {
    x.x = i + 0 < n ? col[i + 0] : V(0);
    x.y = i + 1 < n ? col[i + 1] : V(0);
    x.z = i + 2 < n ? col[i + 2] : V(0);
    x.w = i + 3 < n ? col[i + 3] : V(0);
    t.x = i + 0 < n ? stream[i + 0] : -1;
    t.y = i + 1 < n ? stream[i + 1] : -1;
    t.z = i + 2 < n ? stream[i + 2] : -1;
    t.w = i + 3 < n ? stream[i + 3] : -1;
  }
  const V xs[4] = {x.x, x.y, x.z, x.w};
  const int32_t ts[4] = {t.x, t.y, t.z, t.w};
  uint64_t ma = 0, mb = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bool ok = (i + s < n) && ts[s] == sa && cmp_op<OP, D>((D)xs[s], c);
    if (nul && ok) ok = !nul[i + s];
    const uint64_t a = __ballot(ok);
    const uint64_t b = __ballot((i + s < n) && ts[s] == sb);
    if (lane == s) { ma = a; mb = b; }
  }
  if (lane < 4) {
    cand_m[g * 4 + lane] = ma;
    cons_m[g * 4 + lane] = mb;
  }
}

template <class V, class D>
static void launch_pred_simple_s(int op, int64_t n, D c, const V* col, const uint8_t* nul, const int32_t* stream,
                                 int sa, int sb, uint64_t* cand_m, uint64_t* cons_m, hipStream_t st) {
  const int64_t ntiles = (n + 255) >> 8;
  const dim3 grd((unsigned)std::max<int64_t>(1, (ntiles + 3) / 4)), blk(256);
#define SG_PRED_S(OPV) hipLaunchKernelGGL((k_pred_simple_s<V, D, OPV>), grd, blk, 0, st, n, c, col, nul, stream, sa, sb, \
                                          cand_m, cons_m)
  switch (op) {
    case 0: SG_PRED_S(0); break;
    case 1: SG_PRED_S(1); break;
    case 2: SG_PRED_S(2); break;
    case 3: SG_PRED_S(3); break;
    case 4: SG_PRED_S(4); break;
    default: SG_PRED_S(5); break;
  }
#undef SG_PRED_S
}

template <class V, class D>
static void launch_pred_simple(int op, int64_t n, D c, const V* col, const uint8_t* nul, uint64_t* cand_m,
                               hipStream_t st) {
  const int64_t ntiles = (n + 255) >> 8;
  const int64_t waves = (ntiles + PRED_TILES_PER_WAVE - 1) / PRED_TILES_PER_WAVE;
  const dim3 grd((unsigned)std::max<int64_t>(1, (waves + 3) / 4)), blk(256);
  switch (op) {
    case 0: hipLaunchKernelGGL((k_pred_simple<V, D, 0>), grd, blk, 0, st, n, c, col, nul, cand_m); break;
    case 1: hipLaunchKernelGGL((k_pred_simple<V, D, 1>), grd, blk, 0, st, n, c, col, nul, cand_m); break;
    case 2: hipLaunchKernelGGL((k_pred_simple<V, D, 2>), grd, blk, 0, st, n, c, col, nul, cand_m); break;
    case 3: hipLaunchKernelGGL((k_pred_simple<V, D, 3>), grd, blk, 0, st, n, c, col, nul, cand_m); break;
    case 4: hipLaunchKernelGGL((k_pred_simple<V, D, 4>), grd, blk, 0, st, n, c, col, nul, cand_m); break;
    default: hipLaunchKernelGGL((k_pred_simple<V, D, 5>), grd, blk, 0, st, n, c, col, nul, cand_m); break;
  }
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

static SgVal sg_val_from_bits_host(int64_t bits, int type) {
  SgVal v;
  v.type = type;
  v.null = 0;
  v.i = 0;
  v.d = 0.0;
  if (type == SG_T_FLOAT) {
    uint32_t u = (uint32_t)bits;
    float f;
    memcpy(&f, &u, 4);
    v.d = f;
  } else if (type == SG_T_DOUBLE) {
    memcpy(&v.d, &bits, 8);
  } else {
    v.i = bits;
  }
  return v;
}

// Condition bits of program A (and B unless a.cons_all) over the batch: the 16-B streaming kernel for `col CMP const`
// on a 4-byte column of a single-stream batch, the VM kernel otherwise.
static void launch_pred(const sg_nfa_desc& d, const PredArgs& pa, const int32_t* stream, const SgCols& cols,
                        const DevDesc* ddesc, uint64_t* cand_m, uint64_t* cons_m, hipStream_t st) {
  const int64_t n = pa.n;
  const int64_t ntiles = (n + 255) / 256;
  PredArgs sp = pa;
  bool simple = pa.cons_all && !stream && pa.s_a == 0 && simple_prog(d, pa.prog_a_off, pa.prog_a_len, sp) &&
                (pa.val_col_a < 0 || sp.s_col == pa.val_col_a) && (((uintptr_t)cols.col[sp.s_col]) & 15) == 0;
  const dim3 blk(256);
  // several streams: the same pass with the stream column when B's consumers are just B's stream's rows
  if (!simple && stream && cons_m && pa.prog_b_len == 0 && pa.val_col_b >= 0 && !cols.nul[pa.val_col_b] &&
      simple_prog(d, pa.prog_a_off, pa.prog_a_len, sp) && (pa.val_col_a < 0 || sp.s_col == pa.val_col_a) &&
      (((uintptr_t)cols.col[sp.s_col]) & 15) == 0 && (((uintptr_t)stream) & 15) == 0 && sp.s_dom != 0 &&
      sp.s_type == SG_T_FLOAT) {
    SgVal cv = sg_val_from_bits_host(sp.s_cbits, sp.s_ctype);
    const float* colp = (const float*)cols.col[sp.s_col];
    const uint8_t* nul = cols.nul[sp.s_col];
    if (sp.s_dom == 1) {
      float c = (sp.s_ctype == SG_T_FLOAT || sp.s_ctype == SG_T_DOUBLE) ? (float)cv.d : (float)cv.i;
      launch_pred_simple_s<float, float>(sp.s_op, n, c, colp, nul, stream, pa.s_a, pa.s_b, cand_m, cons_m, st);
    } else {
      double c = (sp.s_ctype == SG_T_FLOAT || sp.s_ctype == SG_T_DOUBLE) ? cv.d : (double)cv.i;
      launch_pred_simple_s<float, double>(sp.s_op, n, c, colp, nul, stream, pa.s_a, pa.s_b, cand_m, cons_m, st);
    }
    return;
  }
  if (simple) {
    // constant in the compare domain (sg_cmp: 0 integral, 1 f32, 2 f64)
    SgVal cv = sg_val_from_bits_host(sp.s_cbits, sp.s_ctype);
    const void* colp = cols.col[sp.s_col];
    const uint8_t* nul = cols.nul[sp.s_col];
    if (sp.s_dom == 1) {
      float c = (sp.s_ctype == SG_T_FLOAT || sp.s_ctype == SG_T_DOUBLE) ? (float)cv.d : (float)cv.i;
      if (sp.s_type == SG_T_FLOAT)
        launch_pred_simple<float, float>(sp.s_op, n, c, (const float*)colp, nul, cand_m, st);
      else
        launch_pred_simple<int32_t, float>(sp.s_op, n, c, (const int32_t*)colp, nul, cand_m, st);
    } else if (sp.s_dom == 2) {
      double c = (sp.s_ctype == SG_T_FLOAT || sp.s_ctype == SG_T_DOUBLE) ? cv.d : (double)cv.i;
      if (sp.s_type == SG_T_FLOAT)
        launch_pred_simple<float, double>(sp.s_op, n, c, (const float*)colp, nul, cand_m, st);
      else
        launch_pred_simple<int32_t, double>(sp.s_op, n, c, (const int32_t*)colp, nul, cand_m, st);
    } else {
      int64_t c = (sp.s_ctype == SG_T_FLOAT || sp.s_ctype == SG_T_DOUBLE) ? (int64_t)cv.d : cv.i;
      if (sp.s_type == SG_T_FLOAT)
        simple = false;   // integral domain on a float column: leave it to the VM's conversions
      else
        launch_pred_simple<int32_t, int64_t>(sp.s_op, n, c, (const int32_t*)colp, nul, cand_m, st);
    }
  }
  if (!simple) {
    int64_t w2 = std::min<int64_t>(ntiles, 256 * 16);
    PredArgs ga = pa;
    ga.stream = stream;
    int depth = sg_prog_depth(d.code + pa.prog_a_off, pa.prog_a_len);
    if (!pa.cons_all) depth = std::max(depth, sg_prog_depth(d.code + pa.prog_b_off, pa.prog_b_len));
    const dim3 grd((unsigned)std::max<int64_t>(1, (w2 + 3) / 4));
    if (depth <= 2) hipLaunchKernelGGL(k_pred<2>, grd, blk, 0, st, ga, cols, ddesc, cand_m, cons_m);
    else if (depth <= 4) hipLaunchKernelGGL(k_pred<4>, grd, blk, 0, st, ga, cols, ddesc, cand_m, cons_m);
    else if (depth <= 8) hipLaunchKernelGGL(k_pred<8>, grd, blk, 0, st, ga, cols, ddesc, cand_m, cons_m);
    else if (depth <= SG_VM_STACK) hipLaunchKernelGGL(k_pred<SG_VM_STACK>, grd, blk, 0, st, ga, cols, ddesc, cand_m, cons_m);
    else throw SgError(SG_EUNSUPPORTED, "predicate program deeper than the VM stack");
  }
}
