// Partial lanes (chain.h): the general machine's route for patterns whose partial matches never interact
// (sg_pp_rule: `every e1=S[local] -> ... within T` over stream / count / logical states of one stream).
//
// Per sg_push, with the rows carried from earlier pushes listed first ("carried rows": the rows every partial still
// pending holds -- its e1, its bound slots, its count chains -- with the e1 rows marked as starts; replaying them
// rebuilds exactly those partials, whatever the order of time, chain.h PpLane::witnesses):
//   1. k_pp_route      combined rows (carried, then the batch) -> partition key (PartitionStreamReceiver routing)
//   2. key partition   stable radix sort of (key, combined row): each key's rows contiguous, in arrival order;
//                      k_pp_segments: per-key bounds and the route's precondition -- a key's timestamps never decrease
//                      (also across pushes), as for the closed forms
//   3. predicate pass  condition bits of every event-local filter over the batch (pred.h)
//   4. k_pp_lanes      one lane per row that starts a partial (a batch row passing the start state's filter, or a
//                      carried start): chain.h's PpLane runs that partial alone over the key's following rows until it
//                      dies (|ts - e1.ts| > within drops it everywhere but in a count state short of its minimum); a
//                      match is written with its sort key (trigger row, visit slot) and its insertion history (tie key);
//                      a partial still pending at the key's last row marks the rows it holds for the carry
//   5. match order     stable radix sorts: tie words, then (trigger, visit slot) -> the reference's delivery order;
//                      k_pp_gather writes the match records
//   6. carry           the marked rows, in arrival order, with their start flags
// Time going back needs no special case: expiry compares |e1.ts - ts| with `within` in every step, a partial parked in
// a count state (CountPreStateProcessor never expires one, CountPreStateProcessor.java:53-93) keeps walking the key's
// rows and is carried however old it is, and a key whose time goes back skips rows only while it waits in a count
// state.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <string>

#include "sg_device.h"
#include "sg_engine.h"
#include "interp.h"
#include "chain.h"
#include "seq.h"
#include "pred.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Carried rows: SoA in the batch's own column formats (so the general machine can replay them as a batch).
struct PpRows {
  int64_t n = 0, cap = 0;
  int64_t* ts = nullptr;
  int32_t* key = nullptr;
  uint8_t* start = nullptr;     // partial lanes: the row is the e1 of a pending partial (its lane restarts there)
  void* col[SG_MAX_COLS] = {};
  uint8_t* nul[SG_MAX_COLS] = {};
};

struct PartialState {
  int mode = 1;         // 1: partial lanes (patterns, chain.h), 2: sequence lanes (seq.h)
  SgPpRule rule;
  SgPpRule* drule = nullptr;
  SgSeqRule srule;
  SgSeqRule* dsrule = nullptr;
  void* kst = nullptr;          // sequence lanes: per-key machine state SeqStateT<G> (zero = no runtime yet)
  void* kst_out = nullptr;      // the push's end states (swapped into kst when the push succeeds: a push that runs
                                // out of match space is rerun from kst with more space, StreamPreStateProcessor's
                                // lists being unbounded, C/query/input/stream/state/StreamPreStateProcessor.java:57-58)
  int sq_small = 0;             // the query fits seq.h's small state geometry (SqSmall)
  int pp_small = 0;             // the query fits chain.h's small lane geometry (PpSmall)
  int lanes_fast = 0;           // every filter is fast compares or event-local bits (chain.h sg_terms_fast)
  int shape_c3 = 0;             // the state table is C3c's family (chain.h PpShapeC3): the specialised lane kernel
  int shape_c3b = 0;            // the state table is C3b's family (seq.h SqShapeC3b): the specialised sequence lanes
  size_t sq_bytes = sizeof(SeqState);
  int64_t kst_keys = 0;
  int64_t seq_pushes = 0;       // pushes that left state behind (after the first, the route cannot be left exactly)
  int64_t last_reruns = 0;      // sequence units rerun from their predecessor's end state in the last push
  int64_t sq_cap_hint = 0;      // match space the last push that outgrew its default needed
  int nulls_seen = 0;           // a push had null flags in a column the query reads (carried rows may hold nulls)
  int8_t hot[SG_MAX_RET];       // record sort: slot -> word of the 16-B record (-1: gathered), see rec_plan
  int rec_ok = 0;
  int used_col[SG_MAX_COLS] = {};
  int col_bytes[SG_MAX_COLS] = {};
  PpRows rows[2];       // carried rows (cur) and the next push's (double buffer)
  int cur = 0;
  int has_count = 0;
  int active = 1;
};

static void rows_free(PpRows& r) {
  if (r.ts) hipFree(r.ts);
  if (r.key) hipFree(r.key);
  if (r.start) hipFree(r.start);
  for (int c = 0; c < SG_MAX_COLS; ++c) {
    if (r.col[c]) hipFree(r.col[c]);
    if (r.nul[c]) hipFree(r.nul[c]);
  }
  r = PpRows();
}

static void rows_reserve(PartialState* ps, PpRows& r, int64_t need) {
  if (need <= r.cap) return;
  const int64_t cap = std::max<int64_t>(need + need / 4, 1024);
  PpRows nr;
  nr.cap = cap;
  if (hipMalloc(&nr.ts, 8 * cap) != hipSuccess || hipMalloc(&nr.key, 4 * cap) != hipSuccess ||
      hipMalloc(&nr.start, cap) != hipSuccess)
    throw SgError(SG_EHIP, "hipMalloc carried rows");
  for (int c = 0; c < SG_MAX_COLS; ++c) {
    if (!ps->used_col[c]) continue;
    if (hipMalloc(&nr.col[c], (size_t)ps->col_bytes[c] * cap) != hipSuccess || hipMalloc(&nr.nul[c], cap) != hipSuccess)
      throw SgError(SG_EHIP, "hipMalloc carried rows");
  }
  rows_free(r);
  r = nr;
}

// FAST lane kernels whenever the query's terms allow them (sg_terms_fast)
static bool lanes_fast(const PartialState* ps) { return ps->lanes_fast; }

PartialState* sg_partial_new(const sg_nfa_desc& d) {
  SgPpRule ru = sg_pp_rule(d);
  SgSeqRule sr = sg_seq_rule(d);
  if (!ru.ok && !sr.ok) return nullptr;
  PartialState* ps = new PartialState();
  ps->mode = ru.ok ? 1 : 2;
  ps->rule = ru;
  ps->srule = sr;
  ps->pp_small = sg_pp_small(ru, d) ? 1 : 0;
  if (ps->mode == 2) {
    ps->rule.local_mask = sr.local_mask;
    ps->rule.start = sr.start;
    ps->rule.recv = sr.recv;
    ps->sq_small = sg_seq_small(sr, d) ? 1 : 0;
    ps->sq_bytes = ps->sq_small ? sizeof(SeqStateT<SqSmall>) : sizeof(SeqState);
    if (hipMalloc(&ps->dsrule, sizeof(SgSeqRule)) != hipSuccess) { delete ps; throw SgError(SG_EHIP, "hipMalloc rule"); }
    hipMemcpy(ps->dsrule, &ps->srule, sizeof(SgSeqRule), hipMemcpyHostToDevice);
  }
  ps->lanes_fast = (ps->mode == 2 ? sg_terms_fast(sr, d.n_states) : sg_terms_fast(ru, d.n_states)) ? 1 : 0;
  ps->shape_c3 = (ps->mode == 1 && sg_pp_shape_is<PpShapeC3>(d, ru)) ? 1 : 0;
  ps->shape_c3b = (ps->mode == 2 && sg_sq_shape_is<SqShapeC3b>(d, sr)) ? 1 : 0;
  for (int s = 0; s < d.n_states; ++s) ps->has_count |= d.states[s].kind == SG_K_COUNT;
  for (int k = 0; k < d.n_ret; ++k) {
    const int c = d.ret_col[k];
    ps->used_col[c] = 1;
    ps->col_bytes[c] = (d.col_type[c] == SG_T_LONG || d.col_type[c] == SG_T_DOUBLE) ? 8 : 4;
  }
  // Record sort (see k_pp_rec): the retained slots the non-local filters read must fit two 32-bit words; partial
  // lanes carry the timestamp in the record instead of condition bits, so only the start state may be event-local.
  {
    for (int k = 0; k < SG_MAX_RET; ++k) ps->hot[k] = -1;
    int words = 0;
    bool fits = true;
    for (int k = 0; k < d.n_ret && fits; ++k) {
      bool used = false;
      for (int s2 = 0; s2 < d.n_states && !used; ++s2) {
        const sg_state_desc& x = d.states[s2];
        if (x.local) continue;
        for (int pc = 0; pc < x.prog_len;) {
          const int64_t op = d.code[x.prog_off + pc];
          if (op == SG_OP_VAR) { if (d.code[x.prog_off + pc + 3] == k) used = true; pc += 5; }
          else if (op == SG_OP_CONST || op == SG_OP_CMP || op == SG_OP_MATH) pc += 3;
          else pc += 1;
        }
      }
      if (!used) continue;
      const bool wide = d.ret_type[k] == SG_T_LONG || d.ret_type[k] == SG_T_DOUBLE;
      if (words + (wide ? 2 : 1) > 2) { fits = false; break; }
      ps->hot[k] = (int8_t)(wide ? 2 : words);
      words += wide ? 2 : 1;
    }
    uint32_t local_mask = 0;
    for (int s2 = 0; s2 < d.n_states; ++s2) if (d.states[s2].local) local_mask |= 1u << s2;
    const int start = ps->mode == 1 ? ru.start : sr.start;
    ps->rec_ok = fits && (ps->mode == 2 || (local_mask & ~(1u << start)) == 0);
  }
  if (hipMalloc(&ps->drule, sizeof(SgPpRule)) != hipSuccess) { delete ps; throw SgError(SG_EHIP, "hipMalloc rule"); }
  hipMemcpy(ps->drule, &ps->rule, sizeof(SgPpRule), hipMemcpyHostToDevice);
  return ps;
}

void sg_partial_free(PartialState* ps) {
  if (!ps) return;
  rows_free(ps->rows[0]);
  rows_free(ps->rows[1]);
  if (ps->drule) hipFree(ps->drule);
  if (ps->dsrule) hipFree(ps->dsrule);
  if (ps->kst) hipFree(ps->kst);
  if (ps->kst_out) hipFree(ps->kst_out);
  delete ps;
}

void sg_partial_reset(PartialState* ps) {
  if (!ps) return;
  ps->rows[0].n = ps->rows[1].n = 0;
  ps->active = 1;
  ps->seq_pushes = 0;
  if (ps->kst) hipMemset(ps->kst, 0, ps->sq_bytes * (size_t)ps->kst_keys);
}

int sg_partial_active(const PartialState* ps) { return ps && ps->active; }
void sg_partial_deactivate(PartialState* ps) {
  if (ps) ps->active = 0;
}

// ---- device side --------------------------------------------------------------------------------------------
struct PpArgs {
  int64_t nc;                 // carried rows (combined rows [0, nc)); batch row r is combined row nc + r
  int64_t n;
  uint64_t base_index;
  const uint64_t* index;
  const int64_t* bts;
  const int64_t* cts;
  const int32_t* stream;
  const int32_t* bkey;
  const int32_t* ckey;
  const uint64_t* lbits[SG_MAX_STATES];
  int32_t any_bits;
  const uint8_t* cstart;      // partial lanes: carried row starts a lane
  uint32_t* keep;             // partial lanes: per sorted position, 1 = carried into the next push
  uint8_t* kstart;            // partial lanes: per sorted position, 1 = the carried row starts a lane
  const uint8_t* kback;       // partial lanes: per key, its time goes back somewhere in this push (carried rows included)
  int64_t drop_before;        // partial lanes: a pending partial whose e1 is older than this is not carried
                              // (sg_options.bounded_lateness; INT64_MIN = carry every pending partial)
  int64_t dead_after;         // partial lanes: a partial at a row more than this after e1 is dead (within + lateness;
                              // INT64_MAX without bounded_lateness)
};

// Key-ordered packed rows (position q = the q-th row of the key partition): what a lane reads at every step, so the
// 64 lanes of a wave (consecutive start rows of one key) read neighbouring addresses.
struct PpPacked {
  int64_t* ts;                  // (nullptr: read through sid, lazy -- sequence lanes only need it for matches)
  void* val[SG_MAX_RET];        // retained slot k: 4- or 8-byte bit patterns (nullptr: lazy, read through sid)
  int32_t wide[SG_MAX_RET];
  uint32_t* nul;                // null mask over retained slots (nullptr: no nulls in this push)
  uint32_t* lb;                 // condition bits of the event-local filters (rule.local_mask)
  // lazy reads: the row's own column through the combined row id (carried rows first)
  const uint32_t* sid;
  int64_t nc;
  const int64_t* bts;
  const int64_t* cts;
  const void* bcol[SG_MAX_RET];
  const void* ccol[SG_MAX_RET];
  // wait skipping (chain.h PpLane::wait_on): per wait attribute, {min, max} encodings of every 8 key-ordered rows
  const uint2* wsum;            // nullptr: no skipping in this push (no wait term, or nulls in a column)
  int64_t wnb;                  // 8-row blocks
  int8_t wix[SG_MAX_RET];       // retained slot -> summary index
};
__device__ __forceinline__ int64_t pp_lazy_ts(const PpPacked* P, int64_t q) {
  const int64_t c = P->sid[q];
  return c < P->nc ? P->cts[c] : P->bts[c - P->nc];
}
__device__ __forceinline__ int64_t pp_lazy_bits(const PpPacked* P, int64_t q, int k) {
  const int64_t c = P->sid[q];
  const bool cr = c < P->nc;
  const void* col = cr ? P->ccol[k] : P->bcol[k];
  const int64_t r = cr ? c : c - P->nc;
  return P->wide[k] ? ((const int64_t*)col)[r] : (int64_t)((const int32_t*)col)[r];
}

struct PpSrc {
  const PpPacked* P;
  __device__ int64_t ts(int64_t q) const { return P->ts[q]; }
  __device__ SgVal read(int64_t q, int slotk, int type) const {
    const int null = P->nul ? (int)((P->nul[q] >> slotk) & 1u) : 0;
    const int64_t bits = P->wide[slotk] ? ((const int64_t*)P->val[slotk])[q] : (int64_t)((const int32_t*)P->val[slotk])[q];
    return sg_val_from_bits(bits, type, null);
  }
  __device__ int lbit(int s, int64_t q) const { return (int)((P->lb[q] >> s) & 1u); }
  __device__ void read_bits(int64_t q, int slotk, int type, int64_t& bits, int& null) const {
    null = P->nul ? (int)((P->nul[q] >> slotk) & 1u) : 0;
    bits = P->wide[slotk] ? ((const int64_t*)P->val[slotk])[q] : (int64_t)((const int32_t*)P->val[slotk])[q];
  }
};

__global__ void k_pp_route(PpArgs a, const DevDesc* __restrict__ dd, int partitioned, uint32_t sentinel,
                           uint32_t* __restrict__ okey, uint32_t* __restrict__ orow, int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.nc + a.n) return;
  uint32_t k = sentinel;
  if (i < a.nc) {
    k = partitioned ? (uint32_t)a.ckey[i] : 0u;
  } else {
    const int64_t r = i - a.nc;
    const int s = a.stream ? a.stream[r] : 0;
    if (s >= 0 && s < SG_MAX_STREAMS && dd->recv_of_stream[s] >= 0) {
      if (!partitioned) k = 0;
      else {
        const int32_t kk = a.bkey ? a.bkey[r] : -1;
        if (kk >= 0) {
          if ((uint32_t)kk >= sentinel) atomicOr(err, 2);
          else k = (uint32_t)kk;
        }
      }
    }
  }
  okey[i] = k;
  orow[i] = (uint32_t)i;
}

// ---- record sort: the rows' per-step fields travel through the key sort as one 16-byte record, so the key-ordered
// rows come out of the sort instead of a gather over the whole batch.  Record: {combined row (| start flag << 31 for
// partial lanes), timestamp - tbase (partial lanes) or event-local condition bits (sequence lanes), hot word 0,
// hot word 1}.
struct alignas(16) PpRec { uint32_t w[4]; };

struct RecArgs {
  int32_t mode, start, partitioned;
  uint32_t sentinel;
  int64_t tbase;
  int8_t hot[SG_MAX_RET];
};

__global__ void __launch_bounds__(256) k_pp_rec(PpArgs a, SgCols bc, SgCols cc, const DevDesc* dd, RecArgs ra,
                                                uint32_t* __restrict__ okey, PpRec* __restrict__ orec,
                                                int32_t* __restrict__ err) {
  __shared__ SgCols colsl[2];
  __shared__ DevDesc dl;
  {
    const uint32_t* s1 = (const uint32_t*)&bc;
    const uint32_t* s2 = (const uint32_t*)&cc;
    for (uint32_t i = threadIdx.x; i < sizeof(SgCols) / 4; i += blockDim.x) {
      ((uint32_t*)&colsl[0])[i] = s1[i];
      ((uint32_t*)&colsl[1])[i] = s2[i];
    }
    const uint32_t* src = (const uint32_t*)dd;
    for (uint32_t i = threadIdx.x; i < sizeof(DevDesc) / 4; i += blockDim.x) ((uint32_t*)&dl)[i] = src[i];
    __syncthreads();
  }
  dd = &dl;
  // grid-stride: a few thousand blocks each stage the descriptors once and walk many rows
  const int64_t m_ = a.nc + a.n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m_; i += (int64_t)gridDim.x * blockDim.x) {
    const bool carried = i < a.nc;
    const int64_t r = carried ? i : i - a.nc;
    uint32_t k = ra.sentinel;
    if (carried) {
      k = ra.partitioned ? (uint32_t)a.ckey[r] : 0u;
    } else {
      const int s = a.stream ? a.stream[r] : 0;
      if (s >= 0 && s < SG_MAX_STREAMS && dd->recv_of_stream[s] >= 0) {
        if (!ra.partitioned) k = 0;
        else {
          const int32_t kk = a.bkey ? a.bkey[r] : -1;
          if (kk >= 0) {
            if ((uint32_t)kk >= ra.sentinel) atomicOr(err, 2);
            else k = (uint32_t)kk;
          }
        }
      }
    }
    okey[i] = k;
    PpRec rec;
    rec.w[0] = (uint32_t)i;
    rec.w[1] = rec.w[2] = rec.w[3] = 0;
    if (k != ra.sentinel) {
      const SgCols& cols = colsl[carried ? 1 : 0];
      uint32_t lb = 0;
      for (int s = 0; s < dd->n_states; ++s) {
        const sg_state_desc& x = dd->states[s];
        if (!x.local || (ra.mode == 1 && s != ra.start)) continue;
        bool ok;
        if (x.prog_len <= 0) ok = true;
        else if (!carried && a.lbits[s]) ok = mask_bit(a.lbits[s], (uint64_t)r) != 0;
        else {
          RowReader rd{&cols, dd->ret_col, r};
          ok = sg_eval(dd->code + x.prog_off, x.prog_len, rd);
        }
        if (ok) lb |= 1u << s;
      }
      if (ra.mode == 1) {
        rec.w[0] |= ((lb >> ra.start) & (carried ? (uint32_t)a.cstart[r] : 1u) & 1u) << 31;
        const int64_t dt = (carried ? a.cts[r] : a.bts[r]) - ra.tbase;
        if (dt != (int64_t)(int32_t)dt) atomicOr(err, 4);
        rec.w[1] = (uint32_t)(int32_t)dt;
      } else {
        rec.w[1] = lb;
      }
      for (int q = 0; q < dd->n_ret; ++q) {
        const int hw = ra.hot[q];
        if (hw < 0) continue;
        const int64_t bits = sg_val_bits(sg_read_col(cols, dd->ret_col[q], dd->ret_type[q], r));
        if (hw == 2) { rec.w[2] = (uint32_t)bits; rec.w[3] = (uint32_t)((uint64_t)bits >> 32); }
        else rec.w[2 + hw] = (uint32_t)bits;
      }
    }
    orec[i] = rec;
  }
}

// sorted records -> the key-ordered SoA rows the lanes read (retained slots outside the record are gathered)
__global__ void __launch_bounds__(256) k_pp_unpack(PpArgs a, SgCols bc, SgCols cc, const DevDesc* dd, RecArgs ra,
                                                   const uint32_t* __restrict__ skey, const PpRec* __restrict__ srec,
                                                   PpPacked P, uint32_t* __restrict__ sid, uint32_t* __restrict__ flag) {
  __shared__ SgCols colsl[2];
  __shared__ DevDesc dl;
  {
    const uint32_t* s1 = (const uint32_t*)&bc;
    const uint32_t* s2 = (const uint32_t*)&cc;
    for (uint32_t i = threadIdx.x; i < sizeof(SgCols) / 4; i += blockDim.x) {
      ((uint32_t*)&colsl[0])[i] = s1[i];
      ((uint32_t*)&colsl[1])[i] = s2[i];
    }
    const uint32_t* src = (const uint32_t*)dd;
    for (uint32_t i = threadIdx.x; i < sizeof(DevDesc) / 4; i += blockDim.x) ((uint32_t*)&dl)[i] = src[i];
    __syncthreads();
  }
  dd = &dl;
  // grid-stride: a few thousand blocks each stage the descriptors once and walk many rows
  const int64_t m_ = a.nc + a.n;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m_; q += (int64_t)gridDim.x * blockDim.x) {
    const PpRec rec = srec[q];
    const uint32_t c = rec.w[0] & 0x7FFFFFFFu;
    sid[q] = c;
    if (skey[q] == ra.sentinel) { flag[q] = 0; continue; }
    const bool carried = (int64_t)c < a.nc;
    const int64_t r = carried ? (int64_t)c : (int64_t)c - a.nc;
    if (ra.mode == 1) {
      const uint32_t f = rec.w[0] >> 31;
      P.ts[q] = ra.tbase + (int64_t)(int32_t)rec.w[1];
      P.lb[q] = f << ra.start;
      flag[q] = f;
    } else {
      P.lb[q] = rec.w[1];
      flag[q] = (rec.w[1] >> ra.start) & 1u;
    }
    const SgCols& cols = colsl[carried ? 1 : 0];
    for (int k = 0; k < dd->n_ret; ++k) {
      const int hw = ra.hot[k];
      if (!P.val[k]) continue;   // lazy slot
      int64_t bits;
      if (hw == 2) bits = (int64_t)(((uint64_t)rec.w[3] << 32) | rec.w[2]);
      else if (hw >= 0) bits = (int64_t)(int32_t)rec.w[2 + hw];
      else bits = sg_val_bits(sg_read_col(cols, dd->ret_col[k], dd->ret_type[k], r));
      if (P.wide[k]) ((int64_t*)P.val[k])[q] = bits;
      else ((int32_t*)P.val[k])[q] = (int32_t)bits;
    }
  }
}

// per-key bounds; check_order: kback[k] = 1 when the key's timestamps go back somewhere (carried rows included)
__global__ void k_pp_segments(int64_t m, PpArgs a, const uint32_t* __restrict__ skey, const uint32_t* __restrict__ sid,
                              const int64_t* __restrict__ qts, int check_order, uint32_t sentinel,
                              uint32_t* __restrict__ beg, uint32_t* __restrict__ end, uint8_t* __restrict__ kback) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m) return;
  const uint32_t k = skey[p];
  if (k == sentinel) return;
  auto ts_at = [&](int64_t q) -> int64_t {
    if (qts) return qts[q];
    const int64_t c = sid[q];
    return c < a.nc ? a.cts[c] : a.bts[c - a.nc];
  };
  if (p == 0 || skey[p - 1] != k) beg[k] = (uint32_t)p;
  else if (check_order && ts_at(p - 1) > ts_at(p)) kback[k] = 1;
  if (p == m - 1 || skey[p + 1] != k) end[k] = (uint32_t)p + 1;
}

struct PpOut {
  char* rec;                  // match records (sg_match_records layout, 32 + 8 * n_select bytes)
  uint64_t* k1;               // (trigger row << 8) | visit slot
  uint64_t* th;               // tie words
  uint64_t* tl;
  unsigned long long* count;
  int32_t* fail;
  uint32_t* jp;               // sorted position of the trigger row
  uint32_t* maxoff;           // largest (trigger position - start position) of a match
  int32_t rstride;
  uint64_t k1_none;           // k1 of a start row without a match (above every (row << 8 | slot) of this push)
};

__device__ __forceinline__ uint64_t pp_index(const PpArgs& a, int64_t r) { return a.index ? a.index[r] : a.base_index + (uint64_t)r; }

// pack: key-ordered rows (ts, retained values, nulls, event-local condition bits) and the start-row flags
__global__ void __launch_bounds__(256) k_pp_pack(PpArgs a, SgCols bc, SgCols cc, const DevDesc* dd,
                                                 uint32_t local_mask, int start, const uint32_t* __restrict__ skey,
                                                 const uint32_t* __restrict__ sid, uint32_t sentinel, PpPacked P,
                                                 uint32_t* __restrict__ flag) {
  __shared__ SgCols colsl[2];
  __shared__ DevDesc dl;
  {
    const uint32_t* s1 = (const uint32_t*)&bc;
    const uint32_t* s2 = (const uint32_t*)&cc;
    for (uint32_t i = threadIdx.x; i < sizeof(SgCols) / 4; i += blockDim.x) {
      ((uint32_t*)&colsl[0])[i] = s1[i];
      ((uint32_t*)&colsl[1])[i] = s2[i];
    }
    const uint32_t* src = (const uint32_t*)dd;
    for (uint32_t i = threadIdx.x; i < sizeof(DevDesc) / 4; i += blockDim.x) ((uint32_t*)&dl)[i] = src[i];
    __syncthreads();
  }
  dd = &dl;
  // grid-stride: a few thousand blocks each stage the descriptors once and walk many rows
  const int64_t m_ = a.nc + a.n;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m_; q += (int64_t)gridDim.x * blockDim.x) {
    if (skey[q] == sentinel) { flag[q] = 0; continue; }
    const int64_t c = sid[q];
    const bool carried = c < a.nc;
    const int64_t r = carried ? c : c - a.nc;
    const SgCols& cols = colsl[carried ? 1 : 0];
    P.ts[q] = carried ? a.cts[r] : a.bts[r];
    uint32_t nm = 0;
    for (int k = 0; k < dd->n_ret; ++k) {
      const SgVal v = sg_read_col(cols, dd->ret_col[k], dd->ret_type[k], r);
      if (v.null) nm |= 1u << k;
      const int64_t bits = sg_val_bits(v);
      if (P.wide[k]) ((int64_t*)P.val[k])[q] = bits;
      else ((int32_t*)P.val[k])[q] = (int32_t)bits;
    }
    if (P.nul) P.nul[q] = nm;
    uint32_t lb = 0;
    for (int s = 0; s < dd->n_states; ++s) {
      if (!((local_mask >> s) & 1u)) continue;
      const sg_state_desc& x = dd->states[s];
      bool ok;
      if (x.prog_len <= 0) ok = true;
      else if (!carried && a.lbits[s]) ok = mask_bit(a.lbits[s], (uint64_t)r) != 0;
      else {
        RowReader rd{&cols, dd->ret_col, r};
        ok = sg_eval(dd->code + x.prog_off, x.prog_len, rd);
      }
      if (ok) lb |= 1u << s;
    }
    P.lb[q] = lb;
    flag[q] = (lb >> start) & (carried && a.cstart ? (uint32_t)a.cstart[r] : 1u) & 1u;
  }
}

__global__ void k_pp_compact(int64_t m, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                             uint32_t* __restrict__ cand) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < m && flag[q]) cand[pos[q]] = (uint32_t)q;
}

// Block summaries of the wait attributes (chain.h pp_wenc): one thread per 8 key-ordered rows and attribute.
__global__ void k_pp_wsum(int64_t m, PpPacked P, uint32_t slots, uint32_t fslots, uint2* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P.wnb) return;
  const int64_t q0 = b * 8;
  const int nr = (int)(m - q0 < 8 ? m - q0 : 8);
  for (int k = 0; k < SG_MAX_RET; ++k) {
    if (!((slots >> k) & 1u)) continue;
    const int fast = ((fslots >> k) & 1u) ? 2 : 1;
    const uint32_t* v = (const uint32_t*)P.val[k] + q0;
    uint32_t mn = 0xffffffffu, mx = 0;
    if (nr == 8) {
      const uint4 a = *(const uint4*)v, c = *(const uint4*)(v + 4);
      const uint32_t x[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (pp_wnan(x[i], fast)) continue;
        const uint32_t e = pp_wenc(x[i], fast);
        mn = e < mn ? e : mn;
        mx = e > mx ? e : mx;
      }
    } else {
      for (int i = 0; i < nr; ++i) {
        if (pp_wnan(v[i], fast)) continue;
        const uint32_t e = pp_wenc(v[i], fast);
        mn = e < mn ? e : mn;
        mx = e > mx ? e : mx;
      }
    }
    out[(int64_t)P.wix[k] * P.wnb + b] = make_uint2(mn, mx);
  }
}

constexpr int PP_BLOCK = 256;
constexpr int64_t PP_WAVE_CANDS = 512;    // start rows per wave (C3c sweep 128..8192: 512 and below 20.4-20.5 ms, 2048 21.5, 8192 26.0; profiles/r04/lanes_ab.log)
template <class G, bool FAST = false, class SH = PpShapeAny>
__global__ void __launch_bounds__(PP_BLOCK, G::S <= 4 ? 8 : 4) k_pp_lanes(PpArgs a, PpPacked P, const DevDesc* __restrict__ ddg,
                                                       const SgPpRule* __restrict__ rug, const uint32_t* __restrict__ cand,
                                                       int64_t ncand, const uint32_t* __restrict__ skey,
                                                       const uint32_t* __restrict__ sid, const uint32_t* __restrict__ end,
                                                       PpOut o, int64_t wave_cands) {
  // the descriptor (9.6 KB) stays in global memory (cache-resident: every lane reads the same few hundred bytes of
  // it), so LDS holds more lanes
  __shared__ SgPpRule rl;
  __shared__ PpPacked pl;
  __shared__ PpArraysT<G> lanes[PP_BLOCK];
  {
    const uint32_t* s3 = (const uint32_t*)&P;
    for (uint32_t i = threadIdx.x; i < sizeof(PpPacked) / 4; i += blockDim.x) ((uint32_t*)&pl)[i] = s3[i];
    const uint32_t* rs = (const uint32_t*)rug;
    uint32_t* rd = (uint32_t*)&rl;
    for (uint32_t i = threadIdx.x; i < sizeof(SgPpRule) / 4; i += blockDim.x) rd[i] = rs[i];
    __syncthreads();
  }
  const DevDesc* dd = ddg;
  // each wave owns PP_WAVE_CANDS consecutive start rows; a lane whose partial is finished takes the next one, so the
  // wave never waits on its longest partial (ballot + popcount hand-out, no atomics)
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t lo = wave * wave_cands;
  const int64_t hi = lo + wave_cands < ncand ? lo + wave_cands : ncand;
  if (lo >= ncand) return;
  PpSrc src{&pl};
  PpLane<PpSrc, G, FAST, SH> L;
  L.d = dd;
  L.ru = &rl;
  L.src = src;
  L.A = &lanes[threadIdx.x];
  const int64_t within = dd->within;
  int64_t nxt = lo + 64;   // wave-uniform
  int64_t i = lo + lane;
  bool active = i < hi;
  int64_t q = 0, e = 0, p0 = 0;
  uint32_t k = 0;
  bool back = false;   // the key's time goes back in this push: skip rows only while waiting in a count state
  if (active) {
    const int64_t p = cand[i];
    k = skey[p];
    L.start(p);
    q = p + 1;
    p0 = p;
    e = end[k];
    back = a.kback && a.kback[k];
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  bool emitted = false;
  uint32_t nemit = 0, maxoff = 0;
  while (__ballot(active)) {
    bool done = false;
    if (active) {
      // wait skipping: the 8-row blocks in which no row can pass the partial's wait term change nothing
      // (PpLane::wait_on); at most 16 blocks per step, the row landed on is checked for expiry below (a key whose time
      // goes back skips only while the partial waits in a count state, which nothing expires)
      int ws, wop, wf;
      int64_t wc;
      if (pl.wsum && q < e && L.wait_on(ws, wop, wf, wc) && (L.wait_count || !back)) {
        // blocks whose summary rules the term out are skipped whole; in a block that may pass, the lane reads its 8
        // values at once and lands on the first row that passes (or moves on to the next block)
        const uint2* S = pl.wsum + (int64_t)pl.wix[ws] * pl.wnb;
        const uint32_t* V = (const uint32_t*)pl.val[ws];
        const int64_t mrows = a.nc + a.n;
        int64_t qq = q;
        for (int lim = 0; lim < 16 && qq < e; ++lim) {
          const int64_t b = qq >> 3;
          const uint2 mm = S[b];
          if (pp_may_pass(mm.x, mm.y, wop, wf, wc)) {
            uint32_t x[8];
            if ((b << 3) + 8 <= mrows) {
              const uint4 x0 = *(const uint4*)(V + (b << 3)), x1 = *(const uint4*)(V + (b << 3) + 4);
              x[0] = x0.x; x[1] = x0.y; x[2] = x0.z; x[3] = x0.w; x[4] = x1.x; x[5] = x1.y; x[6] = x1.z; x[7] = x1.w;
            } else {
#pragma unroll
              for (int k = 0; k < 8; ++k) x[k] = (b << 3) + k < mrows ? V[(b << 3) + k] : 0u;
            }
            uint32_t pm = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const bool ok = wf == 1 ? pp_cmp_i(wop, (int64_t)(int32_t)x[k], wc) : pp_cmp_f(wop, pp_f32((int64_t)x[k]), pp_f32(wc));
              pm |= (ok ? 1u : 0u) << k;
            }
            pm &= ~((1u << (qq & 7)) - 1u);
            if (pm) {
              qq = (b << 3) + __builtin_ctz(pm);
              break;
            }
          }
          qq = (b + 1) << 3;
        }
        q = qq < e ? qq : e;
      }
      const int64_t sdt = q < e ? src.ts(q) - L.e1_ts : 0;
      const int64_t dt = sdt < 0 ? -sdt : sdt;
      if (q < e && sdt > a.dead_after) {
        // bounded lateness: the clock is at least this row's time, so no later row can lie inside `within` of e1 --
        // the partial never emits again, in this push or a later one (not carried)
        done = true;
      } else if (q >= e) {
        done = true;
        // still pending after the key's last row (and not finished: a partial completes at most once): the rows it
        // holds are carried, its e1 marked as the start of its lane in the next push
        if (a.keep && !emitted && !L.overflow && !L.dead() && (L.waiting_count() || L.live_other()) &&
            L.e1_ts >= a.drop_before)
          L.witnesses([&](int32_t pos, bool st) {
            atomicOr(&a.keep[pos], 1u);
            if (st) a.kstart[pos] = 1;
          });
      } else if (dt > within && (!(a.keep || back) || !L.waiting_count())) {
        // expired everywhere it can still emit (sg_pp_rule).  A partial waiting in a count state never expires
        // (CountPreStateProcessor.java:53-93) and walks on -- but only a later row back inside `within` of e1 could
        // complete it: with no push after this one (no carry) and a key whose time never goes back here, none can
        done = true;
      } else {
        const int em = L.step(q);
        if (L.overflow) atomicCAS(o.fail, 0, SG_EUNSUPPORTED);
        if (em >= 0) {
          const int64_t c = sid[q];
          if (c >= a.nc) {
            // a partial completes at most once (sg_pp_rule): its match record goes to its start row's slot
            const int64_t w = i;
            emitted = true;
            const int64_t r = c - a.nc;
            o.k1[w] = ((uint64_t)r << 8) | (uint32_t)em;
            L.tie(o.th[w], o.tl[w]);
            o.jp[w] = (uint32_t)q;
            const uint32_t off = (uint32_t)(q - p0);
            maxoff = off > maxoff ? off : maxoff;
            uint32_t* em32 = (uint32_t*)(o.rec + (size_t)w * (size_t)o.rstride);   // compact: positions (k_em_scatter)
            em32[0] = (uint32_t)q;
            em32[1] = (uint32_t)c;
            em32[2] = k;
            em32[3] = (1u << 24) | (uint32_t)em;
            em32[4] = (uint32_t)L.pts_pos;
            for (int s = 0; s < dd->n_select; ++s) em32[5 + s] = (uint32_t)L.get_event(dd->sel_state[s], dd->sel_index[s]);
          }
        }
        ++q;
        done = L.dead() || L.overflow;
      }
    }
    const uint64_t dm = __ballot(done);
    if (dm) {
      if (done) {
        if (emitted) ++nemit;
        else o.k1[i] = o.k1_none;   // no match: sorts behind every match
        emitted = false;
        i = nxt + __popcll(dm & lt);
        active = i < hi;
        if (active) {
          const int64_t p = cand[i];
          k = skey[p];
          L.start(p);
          q = p + 1;
          p0 = p;
          e = end[k];
          back = a.kback && a.kback[k];
        }
      }
      nxt += __popcll(dm);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    nemit += __shfl_down(nemit, off, 64);
    const uint32_t x = __shfl_down(maxoff, off, 64);
    maxoff = x > maxoff ? x : maxoff;
  }
  if (lane == 0 && nemit) {
    atomicAdd(o.count, (unsigned long long)nemit);
    atomicMax(o.maxoff, maxoff);
  }
}

// One 64-bit delivery key per match when it fits: (trigger row, visit slot), then the insertion history as offsets
// back from the trigger's position (a later insertion = a smaller offset), newest first.
__global__ void k_pp_key(int64_t n, const uint64_t* __restrict__ k1, const uint64_t* __restrict__ th,
                         const uint64_t* __restrict__ tl, const uint32_t* __restrict__ jp, uint64_t k1_none, int n_hist,
                         uint32_t maxoff, int ob, uint64_t none, uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  idx[i] = (uint32_t)i;
  const uint64_t a = k1[i];
  if (a == k1_none) { key[i] = none; return; }
  uint64_t x = ((a >> 8) << 4) | (a & 15u);
  const uint32_t J = jp[i];
  for (int j = 0; j < n_hist; ++j) {
    const uint64_t w = j < 2 ? th[i] : tl[i];
    const uint32_t c = (uint32_t)((j & 1) ? (w & 0x7FFFFFFFu) : ((w >> 31) & 0x7FFFFFFFu));
    const uint32_t off = J - (c >> 4);
    x = (x << (ob + 4)) | ((uint64_t)(maxoff - off) << 4) | (c & 15u);
  }
  key[i] = x;
}

// After the stable sort by k1, the matches of one (trigger row, visit slot) sit together in start-row order: order each
// such run by its insertion history (th, then tl) in place -- what the two LSD tie sorts over all T slots would give,
// for the cost of the runs alone.  A run longer than max_run sets *over and the caller takes the LSD sorts.
__global__ void k_pp_ties(int64_t m, const uint64_t* __restrict__ key, uint32_t* __restrict__ idx,
                          const uint64_t* __restrict__ th, const uint64_t* __restrict__ tl, uint64_t tl_mask, int max_run,
                          int32_t* __restrict__ over) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t k = key[i];
  if (i > 0 && key[i - 1] == k) return;   // not the head of its run
  int64_t e = i + 1;
  while (e < m && key[e] == k) {
    if (e - i >= max_run) { atomicOr(over, 1); return; }
    ++e;
  }
  for (int64_t a = i + 1; a < e; ++a) {   // stable insertion sort: equal histories keep start-row order
    const uint32_t v = idx[a];
    const uint64_t hv = th[v], lv = tl[v] & tl_mask;
    int64_t b = a;
    while (b > i) {
      const uint32_t u = idx[b - 1];
      const uint64_t hu = th[u], lu = tl[u] & tl_mask;
      if (hu < hv || (hu == hv && lu <= lv)) break;
      idx[b] = u;
      --b;
    }
    idx[b] = v;
  }
}

__global__ void k_pp_iota(int64_t n, uint32_t* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = (uint32_t)i;
}
__global__ void k_pp_take(int64_t n, const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, uint64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}
__global__ void k_pp_gather(int64_t n, const char* __restrict__ rec, const uint32_t* __restrict__ idx, int32_t stride,
                            char* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t* s = (const uint64_t*)(rec + (size_t)idx[i] * stride);
  uint64_t* t = (uint64_t*)(out + (size_t)i * stride);
  for (int w = 0; w < stride / 8; ++w) t[w] = s[w];
}

struct PpCopyCols {
  const void* bsrc[SG_MAX_COLS];
  const uint8_t* bnul[SG_MAX_COLS];
  const void* csrc[SG_MAX_COLS];
  const uint8_t* cnul[SG_MAX_COLS];
  void* dst[SG_MAX_COLS];
  uint8_t* dnul[SG_MAX_COLS];
  int32_t bytes[SG_MAX_COLS];
  int32_t ncols;
};

__global__ void k_pp_carry(int64_t m, PpArgs a, const uint32_t* __restrict__ skey, const uint32_t* __restrict__ sid,
                           const uint32_t* __restrict__ keep, const uint32_t* __restrict__ pos, PpCopyCols cc,
                           int64_t* __restrict__ nts, int32_t* __restrict__ nkey, uint8_t* __restrict__ nstart) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m || !keep[p]) return;
  const int64_t c = sid[p];
  const int64_t o = pos[p];
  const bool carried = c < a.nc;
  const int64_t r = carried ? c : c - a.nc;
  nts[o] = carried ? a.cts[r] : a.bts[r];
  nkey[o] = (int32_t)skey[p];
  nstart[o] = a.kstart ? a.kstart[p] : 0;
  for (int j = 0; j < cc.ncols; ++j) {
    if (!cc.dst[j]) continue;
    const void* s = carried ? cc.csrc[j] : cc.bsrc[j];
    const uint8_t* sn = carried ? cc.cnul[j] : cc.bnul[j];
    if (cc.bytes[j] == 8) ((int64_t*)cc.dst[j])[o] = ((const int64_t*)s)[r];
    else ((int32_t*)cc.dst[j])[o] = ((const int32_t*)s)[r];
    cc.dnul[j][o] = sn ? sn[r] : 0;
  }
}

// ---- host side ------------------------------------------------------------------------------------------------
static SgCols carried_cols(const PartialState* ps, const PpRows& r) {
  SgCols c;
  for (int j = 0; j < SG_MAX_COLS; ++j) { c.col[j] = ps->used_col[j] ? r.col[j] : nullptr; c.nul[j] = ps->used_col[j] ? r.nul[j] : nullptr; }
  return c;
}

int64_t sg_partial_carried(const PartialState* ps) { return ps->rows[ps->cur].n; }

static void sort_pairs64(SgHandle* h, const char* tag, uint64_t* k_in, uint64_t* k_out, uint32_t* v_in, uint32_t* v_out,
                         int64_t n, int end_bit) {
  hipStream_t st = h->stream;
  size_t tb = 0;
  HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, k_in, k_out, v_in, v_out, (size_t)n, 0, end_bit, st));
  void* tmp = h->ws.get(std::string("pp_sorttmp_") + tag, tb, st);
  HIPCHK(rocprim::radix_sort_pairs(tmp, tb, k_in, k_out, v_in, v_out, (size_t)n, 0, end_bit, st));
}

// ---- sequence lanes (seq.h): one lane per key resumes the key's compact machine over its rows ----------------------
struct SeqSrcD {
  const PpPacked* P;
  int64_t base;
  __device__ int64_t ts(int64_t pos) const { return P->ts ? P->ts[base + pos] : pp_lazy_ts(P, base + pos); }
  __device__ void read_bits(int64_t pos, int slotk, int type, int64_t& bits, int& null) const {
    const int64_t q = base + pos;
    null = P->nul ? (int)((P->nul[q] >> slotk) & 1u) : 0;
    if (!P->val[slotk]) { bits = pp_lazy_bits(P, q, slotk); return; }
    bits = P->wide[slotk] ? ((const int64_t*)P->val[slotk])[q] : (int64_t)((const int32_t*)P->val[slotk])[q];
  }
  __device__ SgVal read(int64_t pos, int slotk, int type) const {
    int64_t bits;
    int null;
    read_bits(pos, slotk, type, bits, null);
    return sg_val_from_bits(bits, type, null);
  }
  __device__ int lbit(int s, int64_t pos) const { return (int)((P->lb[base + pos] >> s) & 1u); }
};

struct SqOut {
  char* rec;
  uint64_t* k1;               // (trigger row << 16) | emission index within the row
  uint32_t* runit;            // unit that wrote the slot (| 0x80000000 when written by a rerun)
  uint32_t* rerun;            // per unit: 1 = its speculative matches are void
  unsigned long long* dropped;
  unsigned long long* reserved;
  unsigned long long* count;
  int32_t* fail;
  int64_t cap;
  int32_t rstride;
  uint64_t k1_none;
};

constexpr int SQ_BLOCK = 64;
constexpr int SQ_CHUNK = 16;   // match slots a lane reserves at a time

// Units (key, c): the key's new rows [s0, s1) = [beg + ncar + c R, ...).  Unit 0 starts from the key's carried state;
// unit c > 0 from a guess -- a zeroed state warmed up over the W rows before it -- verified afterwards.
struct SqPlan {
  const uint32_t* beg;
  const uint32_t* end;
  const uint32_t* ncar;       // carried rows at the start of each key's positions
  const uint32_t* uoff;       // key -> first unit
  const uint32_t* umap;       // unit -> key
  int64_t R, W;
  int64_t nunits;
  void* kst;                  // per key (carried), SeqStateT<G>: the states the push starts from (read only)
  void* kst_out;              // per key: the states the push ends in
  void* ust;                  // per unit: start state
  void* uen;                  // per unit: end state
  unsigned long long* reruns;
};

__global__ void k_sq_ucount(int64_t kb, const uint32_t* __restrict__ beg, const uint32_t* __restrict__ end,
                            const uint32_t* __restrict__ sid, int64_t nc, int64_t R, uint32_t* __restrict__ ncar,
                            uint32_t* __restrict__ nu) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > kb) return;
  if (k == kb) { nu[k] = 0; return; }
  const int64_t b0 = beg[k], e0 = end[k];
  int64_t c = 0;
  while (b0 + c < e0 && (int64_t)sid[b0 + c] < nc) ++c;
  ncar[k] = (uint32_t)c;
  const int64_t own = e0 > b0 ? e0 - b0 - c : 0;
  nu[k] = (uint32_t)((own + R - 1) / R);
}

__global__ void k_sq_umap(int64_t kb, const uint32_t* __restrict__ uoff, uint32_t* __restrict__ umap) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= kb) return;
  for (uint32_t u = uoff[k]; u < uoff[k + 1]; ++u) umap[u] = (uint32_t)k;
}

template <class T>
__device__ __forceinline__ void sq_copy(T* __restrict__ dst, const T* __restrict__ src) {
  static_assert(sizeof(T) % 4 == 0, "state words");
  const uint32_t* s = (const uint32_t*)src;
  uint32_t* d = (uint32_t*)dst;
  for (uint32_t i = 0; i < sizeof(T) / 4; ++i) d[i] = s[i];
}
template <class T>
__device__ __forceinline__ void sq_zero(T* dst) {
  uint32_t* d = (uint32_t*)dst;
  for (uint32_t i = 0; i < sizeof(T) / 4; ++i) d[i] = 0;
}

struct SqEmit {   // match writer of the emitting pass (off: the warm-up, same code so the machine is inlined once)
  bool on;
  const PpArgs* a;
  const DevDesc* dd;
  const uint32_t* sid;
  SqOut o;
  int64_t slot, slot_end;
  uint32_t key, seq, nemit, unit;
  template <class Mach>
  __device__ void operator()(Mach& mm, int p, int grp) {
    if (!on) return;
    if (slot == slot_end) {
      slot = (int64_t)atomicAdd(o.reserved, (unsigned long long)SQ_CHUNK);
      slot_end = slot + SQ_CHUNK;
      if (slot_end > o.cap) { mm.fail(5); slot = slot_end; return; }
    }
    const int64_t w = slot++;
    ++nemit;
    const int64_t q = mm.src.base + mm.cur;   // the trigger row's sorted position; its batch row through sid
    const int64_t r = (int64_t)sid[q] - a->nc;
    o.k1[w] = ((uint64_t)r << 16) | seq++;
    o.runit[w] = unit;
    // positions only: k_em_scatter turns them into the match record, in slot order, once the delivery order is known (one thread
    // per match instead of dependent reads in the lane's critical path)
    uint32_t* em32 = (uint32_t*)(o.rec + (size_t)w * (size_t)o.rstride);
    const int64_t pp = mm.dec(mm.M->P[p].pts);
    em32[0] = (uint32_t)q;
    em32[1] = (uint32_t)(r + a->nc);
    em32[2] = key;
    em32[3] = (1u << 24) | (uint32_t)grp;
    em32[4] = (uint32_t)(pp >= 0 ? mm.src.base + pp : -1);
    for (int s = 0; s < dd->n_select; ++s) {
      const int64_t ev = mm.get_event(p, dd->sel_state[s], dd->sel_index[s]);
      em32[5 + s] = (uint32_t)(ev < 0 ? -1 : mm.src.base + ev);
    }
  }
};

// rows [q0, q1) of a key whose positions start at b0; emit != null: the emitting pass
template <class E, class Mach>
__device__ __forceinline__ void sq_run(Mach& m, int64_t b0, int64_t q0, int64_t q1, E& emit, uint32_t* seq) {
  m.begin();
  for (int64_t q = q0; q < q1 && !m.failed; ++q) {
    if (seq) *seq = 0;
    m.receive(q - b0, emit);
  }
  m.finish();
}

// The descriptor stays in global memory (L1-resident: every lane reads the same few hundred bytes of it); LDS holds
// the lanes' machine states, so more waves fit per CU.
#define SQ_KERNEL_PROLOGUE                                                                                     \
  const DevDesc& dl = *ddg;                                                                                    \
  __shared__ SgSeqRule rl;                                                                                     \
  __shared__ PpPacked pl;                                                                                      \
  __shared__ SeqStateT<G> lanes[SQ_BLOCK];                                                                         \
  {                                                                                                            \
    const uint32_t* s3 = (const uint32_t*)&P;                                                                  \
    for (uint32_t i = threadIdx.x; i < sizeof(PpPacked) / 4; i += blockDim.x) ((uint32_t*)&pl)[i] = s3[i];    \
    const uint32_t* rs = (const uint32_t*)rug;                                                                 \
    for (uint32_t i = threadIdx.x; i < sizeof(SgSeqRule) / 4; i += blockDim.x) ((uint32_t*)&rl)[i] = rs[i];   \
    __syncthreads();                                                                                           \
  }

// pass A: every unit from its (guessed) start state, emitting; its start and end states are kept for the check
template <class G, bool FAST = false, class SH = SqShapeAny>
__global__ void __launch_bounds__(SQ_BLOCK) k_sq_spec(PpArgs a, PpPacked P, const DevDesc* __restrict__ ddg,
                                                      const SgSeqRule* __restrict__ rug, const uint32_t* __restrict__ sid,
                                                      SqPlan pl_, SqOut o) {
  SQ_KERNEL_PROLOGUE
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= pl_.nunits) return;
  const uint32_t k = pl_.umap[u];
  const int64_t c = u - pl_.uoff[k];
  const int64_t b0 = pl_.beg[k], e0 = pl_.end[k];
  const int64_t s0 = b0 + pl_.ncar[k] + c * pl_.R, s1 = s0 + pl_.R < e0 ? s0 + pl_.R : e0;
  SeqStateT<G>& M = lanes[threadIdx.x];
  SeqMachine<SeqSrcD, G, FAST, SH> m;
  m.d = &dl;
  m.ru = &rl;
  m.src = SeqSrcD{&pl, b0};
  m.M = &M;
  m.cur = 0;
  int64_t q0 = s0;
  if (c == 0) {
    sq_copy(&M, (const SeqStateT<G>*)pl_.kst + k);
  } else {
    sq_zero(&M);
    q0 = s0 - pl_.W > b0 ? s0 - pl_.W : b0;
  }
  SqEmit em;
  em.on = false;
  em.a = &a;
  em.dd = &dl;
  em.sid = sid;
  em.o = o;
  em.slot = em.slot_end = 0;
  em.key = k;
  em.nemit = 0;
  em.seq = 0;
  em.unit = (uint32_t)u;
  // one loop over the warm-up rows [q0, s0) (emitter off) and the unit's rows [s0, s1): one inlined machine
  bool started = false;
  m.begin();
  for (int64_t q = q0; q < s1 && !m.failed; ++q) {
    if (q == s0) {
      m.finish();
      sq_copy((SeqStateT<G>*)pl_.ust + u, &M);
      started = true;
      em.on = true;
    }
    em.seq = 0;
    m.receive(q - b0, em);
  }
  m.finish();
  if (!started) sq_copy((SeqStateT<G>*)pl_.ust + u, &M);   // (a warm-up that failed: the push is rerun elsewhere)
  for (int64_t q = em.slot; q < em.slot_end && q < o.cap; ++q) o.k1[q] = o.k1_none;
  if (em.nemit) atomicAdd(o.count, (unsigned long long)em.nemit);
  if (m.failed) atomicCAS(o.fail, 0, m.failed);
  sq_copy((SeqStateT<G>*)pl_.uen + u, &M);
}

// pass B: per key, in unit order, a unit whose guessed start differs from its predecessor's end is rerun from that end
// (emitting again; its speculative matches are voided); then the key's final state is kept for the next push
template <class G>
__global__ void __launch_bounds__(SQ_BLOCK) k_sq_fix(PpArgs a, PpPacked P, const DevDesc* __restrict__ ddg,
                                                     const SgSeqRule* __restrict__ rug, const uint32_t* __restrict__ sid,
                                                     SqPlan pl_, int64_t kb, SqOut o) {
  SQ_KERNEL_PROLOGUE
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= kb) return;
  const uint32_t u0 = pl_.uoff[k], u1 = pl_.uoff[k + 1];
  if (u1 == u0) {   // no rows this push: the key's state carries over unchanged
    sq_copy((SeqStateT<G>*)pl_.kst_out + k, (const SeqStateT<G>*)pl_.kst + k);
    return;
  }
  const int64_t b0 = pl_.beg[k], e0 = pl_.end[k];
  SeqStateT<G>& M = lanes[threadIdx.x];
  SeqMachine<SeqSrcD, G> m;
  m.d = &dl;
  m.ru = &rl;
  m.src = SeqSrcD{&pl, b0};
  m.M = &M;
  m.cur = 0;
  SqEmit em;
  em.a = &a;
  em.dd = &dl;
  em.sid = sid;
  em.o = o;
  em.slot = em.slot_end = 0;
  em.key = (uint32_t)k;
  em.nemit = 0;
  em.seq = 0;
  em.on = true;
  uint32_t reruns = 0;
  for (uint32_t u = u0 + 1; u < u1; ++u) {
    if (sg_seq_equiv(((const SeqStateT<G>*)pl_.ust)[u], ((const SeqStateT<G>*)pl_.uen)[u - 1], dl, rl)) continue;
    ++reruns;
    o.rerun[u] = 1;
    em.unit = u | 0x80000000u;
    const int64_t c = u - u0;
    const int64_t s0 = b0 + pl_.ncar[k] + c * pl_.R, s1 = s0 + pl_.R < e0 ? s0 + pl_.R : e0;
    sq_copy(&M, (const SeqStateT<G>*)pl_.uen + (u - 1));
    sq_run(m, b0, s0, s1, em, &em.seq);
    if (m.failed) { atomicCAS(o.fail, 0, m.failed); return; }
    sq_copy((SeqStateT<G>*)pl_.uen + u, &M);
  }
  for (int64_t q = em.slot; q < em.slot_end && q < o.cap; ++q) o.k1[q] = o.k1_none;
  if (em.nemit) atomicAdd(o.count, (unsigned long long)em.nemit);
  if (reruns) atomicAdd(pl_.reruns, (unsigned long long)reruns);
  sq_copy(&M, (const SeqStateT<G>*)pl_.uen + (u1 - 1));
  const int64_t nk = e0 - b0;
  m.rebase(nk - 1, nk > rl.horizon ? nk - rl.horizon : 0);
  sq_copy((SeqStateT<G>*)pl_.kst_out + k, &M);
}

// void the speculative matches of rerun units
__global__ void k_sq_drop(int64_t n, SqOut o) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n || o.k1[w] == o.k1_none) return;
  const uint32_t u = o.runit[w];
  if (!(u & 0x80000000u) && o.rerun[u]) {
    o.k1[w] = o.k1_none;
    atomicAdd(o.dropped, 1ull);
  }
}

// Compact emission records {trigger position, trigger combined row, key, group, timestamp row position, position per
// select slot} -> match records {trigger index, ts, key, group, null mask, values}.
// one match record from its compact emission record e
__device__ __forceinline__ void em_build(const uint32_t* __restrict__ e, char* rec, const PpPacked& P,
                                         const DevDesc* __restrict__ dd, const uint64_t* __restrict__ index,
                                         uint64_t base_index) {
  int64_t* h64 = (int64_t*)rec;
  // the trigger row's own columns are read straight from the batch where the slot is lazy; other rows go through
  // their key-sorted position, and a row selected twice in a row is read once
  const uint32_t tq = e[0];
  const int64_t r = (int64_t)e[1] - P.nc;
  h64[0] = (int64_t)(index ? index[r] : base_index + (uint64_t)r);
  const int32_t tp = (int32_t)e[4];
  h64[1] = tp < 0 ? -1 : P.ts ? P.ts[tp] : (uint32_t)tp == tq ? P.bts[r] : pp_lazy_ts(&P, tp);
  uint64_t* h2 = (uint64_t*)(rec + 16);   // {key, group} and {null mask, 0} as two 8-byte stores
  h2[0] = (uint64_t)e[2] | ((uint64_t)e[3] << 32);
  uint32_t nm = 0;
  int64_t* vals = (int64_t*)(rec + 32);
  const int ns = dd->n_select;
  int32_t pq = -1;
  int prs = -1;
  int64_t pv = 0;
  for (int s = 0; s < ns; ++s) {
    const int32_t q = (int32_t)e[5 + s];
    const int rs = dd->sel_ret[s];
    if (q < 0 || (P.nul && ((P.nul[q] >> rs) & 1u))) { nm |= 1u << s; vals[s] = 0; continue; }
    if (q == pq && rs == prs) { vals[s] = pv; continue; }   // e.g. e2[0] and e2[last] of a one-event count
    int64_t bits;
    if ((uint32_t)q == tq && !P.val[rs]) bits = P.wide[rs] ? ((const int64_t*)P.bcol[rs])[r] : (int64_t)((const int32_t*)P.bcol[rs])[r];
    else if (P.val[rs]) bits = P.wide[rs] ? ((const int64_t*)P.val[rs])[q] : (int64_t)((const int32_t*)P.val[rs])[q];
    else bits = pp_lazy_bits(&P, q, rs);
    pv = sg_val_bits(sg_val_from_bits(bits, dd->ret_type[rs], 0));
    pq = q;
    prs = rs;
    vals[s] = pv;
  }
  h2[1] = (uint64_t)nm;
}

// delivery position of every slot (slots without a match keep ~0)
__global__ void k_em_dest(int64_t n, const uint32_t* __restrict__ idx, uint32_t* __restrict__ dest) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dest[idx[i]] = (uint32_t)i;
}

// Partial lanes: slot order is start-row order, i.e. key-ordered, so walking the slots reads the compact records and
// the packed rows they point at nearly coalesced; each record is then written to its delivery position.  The block's
// records are assembled in LDS first and written out by consecutive threads taking consecutive 8-byte words of the
// same record, so one store instruction covers whole records instead of one word of 64 scattered ones.
__global__ void __launch_bounds__(256) k_em_scatter(int64_t T, const uint32_t* __restrict__ dest,
                                                    const char* __restrict__ em, int32_t estride, char* __restrict__ out,
                                                    int32_t ostride, PpPacked P, const DevDesc* __restrict__ dd,
                                                    const uint64_t* __restrict__ index, uint64_t base_index) {
  extern __shared__ __align__(16) char em_lds[];
  __shared__ uint32_t dl[256];
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = 0xFFFFFFFFu;
  if (w < T) {
    d = dest[w];
    if (d != 0xFFFFFFFFu)
      em_build((const uint32_t*)(em + (size_t)w * estride), em_lds + (size_t)threadIdx.x * ostride, P, dd, index,
               base_index);
  }
  dl[threadIdx.x] = d;
  __syncthreads();
  const int words = ostride / 8;
  const int all = (int)blockDim.x * words;
  for (int x = threadIdx.x; x < all; x += blockDim.x) {
    const int rec = x / words, wd = x - rec * words;
    const uint32_t to = dl[rec];
    if (to == 0xFFFFFFFFu) continue;
    ((uint64_t*)(out + (size_t)to * ostride))[wd] = ((const uint64_t*)(em_lds + (size_t)rec * ostride))[wd];
  }
}

// carry for sequence lanes: the last H rows of every key
__global__ void k_seq_keep(int64_t m, const uint32_t* __restrict__ skey, const uint32_t* __restrict__ end, uint32_t sentinel,
                           int64_t H, uint32_t* __restrict__ keep) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m) return;
  const uint32_t k = skey[p];
  keep[p] = (k != sentinel && p >= (int64_t)end[k] - H) ? 1u : 0u;
}

static void carry_rows(SgHandle* h, PartialState* ps, const BatchView& bv, const PpArgs& a, int64_t m,
                       const uint32_t* skeys, const uint32_t* sids, uint32_t* keep);

static int seq_lanes_push(SgHandle* h, PartialState* ps, const BatchView& bv, int64_t n, uint32_t kb, const PpArgs& a,
                          const PpPacked& P, const uint32_t* skeys, const uint32_t* sids, const uint32_t* beg,
                          const uint32_t* end, uint32_t sentinel) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int64_t m = a.nc + a.n;
  const dim3 blk(256), grd((unsigned)((m + 255) / 256));
  // per-key machine states (grown with the key bound; new keys start zeroed = no runtime yet)
  if ((int64_t)kb > ps->kst_keys || !ps->kst_out) {
    const int64_t nk = std::max<int64_t>((int64_t)kb, ps->kst_keys * 3 / 2);
    void* ns = nullptr;
    void* no = nullptr;
    if (hipMalloc(&ns, ps->sq_bytes * (size_t)nk) != hipSuccess || hipMalloc(&no, ps->sq_bytes * (size_t)nk) != hipSuccess) {
      if (ns) hipFree(ns);
      throw SgError(SG_ECAPACITY, "hipMalloc sequence states");
    }
    HIPCHK(hipMemsetAsync(ns, 0, ps->sq_bytes * (size_t)nk, st));
    HIPCHK(hipMemsetAsync(no, 0, ps->sq_bytes * (size_t)nk, st));
    if (ps->kst) {
      HIPCHK(hipMemcpyAsync(ns, ps->kst, ps->sq_bytes * (size_t)ps->kst_keys, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
      hipFree(ps->kst);
    }
    if (ps->kst_out) hipFree(ps->kst_out);
    ps->kst = ns;
    ps->kst_out = no;
    ps->kst_keys = nk;
  }
  const int nsel = d.n_select;
  const int32_t rstride = 32 + 8 * nsel;
  int64_t cap = 0;   // set with the unit plan
  SqOut o;
  o.reserved = (unsigned long long*)h->ws.get("sq_cnt", 64, st);
  o.count = o.reserved + 1;
  o.fail = (int32_t*)(o.reserved + 2);
  o.cap = cap;
  o.rstride = 20 + 4 * nsel;   // compact match records (k_em_scatter writes the rstride-byte ones)
  int rb = 1;
  while ((1ll << rb) < n + 1) ++rb;
  const int k1_bits = std::min(64, rb + 16);
  o.k1_none = k1_bits >= 64 ? ~0ull : (1ull << k1_bits) - 1;
  HIPCHK(hipMemsetAsync(o.reserved, 0, 64, st));
  // ---- unit plan
  SqPlan pl_;
  const int64_t H = ps->srule.horizon;
  // the speculative pass's kernel variant
  const void* spec_fn = ps->sq_small && lanes_fast(ps) && ps->shape_c3b ? (const void*)k_sq_spec<SqSmall, true, SqShapeC3b>
                        : ps->sq_small && lanes_fast(ps)                ? (const void*)k_sq_spec<SqSmall, true>
                        : ps->sq_small                                  ? (const void*)k_sq_spec<SqSmall>
                                                                        : (const void*)k_sq_spec<SqBig>;
  pl_.R = std::max<int64_t>(64, (n + 262143) / 262144);
  if (h->opt.chunk_rows > 0) pl_.R = h->opt.chunk_rows;
  pl_.W = std::max<int64_t>(4 * H, 16);
  uint32_t* ncar = (uint32_t*)h->ws.get("sq_ncar", 4 * ((size_t)kb + 1), st);
  uint32_t* nu = (uint32_t*)h->ws.get("sq_nu", 4 * ((size_t)kb + 1), st);
  uint32_t* uoff = (uint32_t*)h->ws.get("sq_uoff", 4 * ((size_t)kb + 1), st);
  const dim3 gk((unsigned)((kb + 1 + 255) / 256));
  h->kbeg("sequence_units");
  hipLaunchKernelGGL(k_sq_ucount, gk, blk, 0, st, (int64_t)kb, beg, end, sids, a.nc, pl_.R, ncar, nu);
  {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, nu, uoff, (uint32_t)0, (size_t)kb + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("sq_uscan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, nu, uoff, (uint32_t)0, (size_t)kb + 1, rocprim::plus<uint32_t>(), st));
  }
  uint32_t U = 0;
  HIPCHK(hipMemcpyAsync(&U, uoff + kb, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  uint32_t* umap = (uint32_t*)h->ws.get("sq_umap", 4 * ((size_t)U + 1), st);
  hipLaunchKernelGGL(k_sq_umap, dim3((unsigned)((kb + 255) / 256)), blk, 0, st, (int64_t)kb, uoff, umap);
  pl_.beg = beg;
  pl_.end = end;
  pl_.ncar = ncar;
  pl_.uoff = uoff;
  pl_.umap = umap;
  pl_.nunits = U;
  pl_.kst = ps->kst;
  pl_.kst_out = ps->kst_out;
  pl_.ust = h->ws.get("sq_ust", ps->sq_bytes * ((size_t)U + 1), st);
  pl_.uen = h->ws.get("sq_uen", ps->sq_bytes * ((size_t)U + 1), st);
  pl_.reruns = o.reserved + 3;
  h->kend();
  // match space: every lane reserves SQ_CHUNK slots at a time; a push whose matches outgrow it is rerun from the
  // unchanged start states (kst) with four times the space -- the reference's lists are unbounded
  cap = n + (int64_t)SQ_CHUNK * ((int64_t)U + (int64_t)kb) + 65536;
  if (ps->sq_cap_hint > cap) cap = ps->sq_cap_hint;
  if (const char* e = getenv("SG_DEBUG_SQ_MATCH_CAP")) {   // (debug: a tiny match space exercises the regrowth)
    const int64_t v = atoll(e);
    if (v > 0) cap = std::max<int64_t>(v, SQ_CHUNK);
  }
  const dim3 gu((unsigned)((U + SQ_BLOCK - 1) / SQ_BLOCK)), gq((unsigned)((kb + SQ_BLOCK - 1) / SQ_BLOCK));
  unsigned long long cnt[5] = {0, 0, 0, 0, 0};
  int32_t fail = 0;
  for (int attempt = 0;; ++attempt) {
  o.cap = cap;
  o.rec = (char*)h->ws.get("sq_rec", (size_t)cap * rstride, st);
  o.k1 = (uint64_t*)h->ws.get("sq_k1", 8 * cap, st);
  o.runit = (uint32_t*)h->ws.get("sq_runit", 4 * (size_t)cap, st);
  o.rerun = (uint32_t*)h->ws.get("sq_rerun", 4 * ((size_t)U + 1), st);
  o.dropped = o.reserved + 4;
  HIPCHK(hipMemsetAsync(o.rerun, 0, 4 * ((size_t)U + 1), st));
  if (attempt) HIPCHK(hipMemsetAsync(o.reserved, 0, 64, st));
  h->kbeg("sequence_lanes");
  if (U) {
    const DevDesc* dd_ = h->ddesc;
    const SgSeqRule* ru_ = ps->dsrule;
    PpArgs a_ = a;
    PpPacked P_ = P;
    void* args[] = {&a_, &P_, &dd_, &ru_, &sids, &pl_, &o};
    HIPCHK(hipLaunchKernel(spec_fn, gu, dim3(SQ_BLOCK), args, 0, st));
  }
  HIPCHK(hipGetLastError());
  h->kend();
  h->kbeg("sequence_fix");
  if (U && ps->sq_small) hipLaunchKernelGGL(k_sq_fix<SqSmall>, gq, dim3(SQ_BLOCK), 0, st, a, P, h->ddesc, ps->dsrule, sids, pl_, (int64_t)kb, o);
  else if (U) hipLaunchKernelGGL(k_sq_fix<SqBig>, gq, dim3(SQ_BLOCK), 0, st, a, P, h->ddesc, ps->dsrule, sids, pl_, (int64_t)kb, o);
  HIPCHK(hipGetLastError());
  h->kend();
  // keys past this push's key bound keep their states as well
  if (ps->kst_keys > (int64_t)kb)
    HIPCHK(hipMemcpyAsync((char*)ps->kst_out + ps->sq_bytes * (size_t)kb, (const char*)ps->kst + ps->sq_bytes * (size_t)kb,
                          ps->sq_bytes * (size_t)(ps->kst_keys - (int64_t)kb), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync(cnt, o.reserved, 40, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  fail = (int32_t)(cnt[2] & 0xffffffffu);
  if (fail != 5) break;
  const int64_t grown = std::max<int64_t>(4 * cap, (int64_t)std::min<unsigned long long>(cnt[0], (1ull << 40)) + cap);
  cap = grown;
  ps->sq_cap_hint = cap;
  }
  if (cnt[3]) {   // some units were rerun: void their speculative matches
    const int64_t Rz = std::min<int64_t>((int64_t)cnt[0], cap);
    hipLaunchKernelGGL(k_sq_drop, dim3((unsigned)((Rz + 255) / 256)), blk, 0, st, Rz, o);
    HIPCHK(hipMemcpyAsync(&cnt[4], o.dropped, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  h->mark(3);
  cnt[1] -= cnt[4];
  ps->last_reruns = (int64_t)cnt[3];
  if (fail) {
    if (ps->seq_pushes == 0 && a.nc == 0) {   // nothing carried yet: the per-key machine can take the stream exactly
      HIPCHK(hipMemsetAsync(ps->kst, 0, ps->sq_bytes * (size_t)ps->kst_keys, st));
      return 0;
    }
    throw SgError(SG_ECAPACITY, "sequence machine capacity exceeded (reason " + std::to_string(fail) +
                                    ": 1 partials, 2 list, 3 returned, 4 chain)");
  }
  std::swap(ps->kst, ps->kst_out);   // the push's end states become the carried states
  const int64_t R = std::min<int64_t>((int64_t)cnt[0], cap), total = (int64_t)cnt[1];
  if (total) {
    const dim3 g2((unsigned)((R + 255) / 256));
    uint32_t* ia = (uint32_t*)h->ws.get("sq_ia", 4 * R, st);
    uint32_t* ib = (uint32_t*)h->ws.get("sq_ib", 4 * R, st);
    uint64_t* kb2 = (uint64_t*)h->ws.get("sq_kb", 8 * R, st);
    h->kbeg("match_order");
    hipLaunchKernelGGL(k_pp_iota, g2, blk, 0, st, R, ia);
    size_t tb = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, o.k1, kb2, ia, ib, (size_t)R, 0, k1_bits, st));
    void* tmp = h->ws.get("sq_sorttmp", tb, st);
    HIPCHK(rocprim::radix_sort_pairs(tmp, tb, o.k1, kb2, ia, ib, (size_t)R, 0, k1_bits, st));
    char* out = h->out.reserve(total, nsel, st);
    // records built in slot order (a lane's slots hold one key's matches: the compact records and the packed rows they
    // name are read nearly in order) and scattered to their delivery positions (k_em_scatter), as the partial lanes do
    uint32_t* dest = (uint32_t*)h->ws.get("sq_dest", 4 * (size_t)(R + 1), st);
    HIPCHK(hipMemsetAsync(dest, 0xFF, 4 * (size_t)R, st));
    hipLaunchKernelGGL(k_em_dest, dim3((unsigned)((total + 255) / 256)), blk, 0, st, total, ib, dest);
    if ((size_t)256 * rstride > 65536)
      HIPCHK(hipFuncSetAttribute((const void*)k_em_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(256 * rstride)));
    hipLaunchKernelGGL(k_em_scatter, g2, blk, (size_t)256 * rstride, st, R, dest, o.rec, o.rstride,
                       out + (size_t)h->out.n * rstride, rstride, P, h->ddesc, bv.index, bv.base_index);
    HIPCHK(hipGetLastError());
    h->kend();
    h->out.n += total;
  }
  if (!h->opt.no_carry && m) {
    uint32_t* keep = (uint32_t*)h->ws.get("pp_keep", 4 * (m + 1), st);
    hipLaunchKernelGGL(k_seq_keep, grd, blk, 0, st, m, skeys, end, sentinel, (int64_t)ps->srule.horizon, keep);
    carry_rows(h, ps, bv, a, m, skeys, sids, keep);
  } else if (h->opt.no_carry) {
    HIPCHK(hipMemsetAsync(ps->kst, 0, ps->sq_bytes * (size_t)ps->kst_keys, st));
  }
  ps->seq_pushes++;
  h->mark(4);
  h->last_events = n;
  h->last_spilled = 0;
  h->last_matches = total;
  return 1;
}

static void carry_rows(SgHandle* h, PartialState* ps, const BatchView& bv, const PpArgs& a, int64_t m,
                       const uint32_t* skeys, const uint32_t* sids, uint32_t* keep) {
  {
    const sg_nfa_desc& d = h->desc;
    hipStream_t st = h->stream;
    const dim3 blk(256), grd((unsigned)((m + 255) / 256));
    const PpRows& cr = ps->rows[ps->cur];
    h->kbeg("carry");
    uint32_t* pos = (uint32_t*)h->ws.get("pp_pos", 4 * (m + 1), st);
    HIPCHK(hipMemsetAsync(keep + m, 0, 4, st));
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, keep, pos, (uint32_t)0, (size_t)m + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("pp_scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, keep, pos, (uint32_t)0, (size_t)m + 1, rocprim::plus<uint32_t>(), st));
    uint32_t nn = 0;
    HIPCHK(hipMemcpyAsync(&nn, pos + m, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    PpRows& nr = ps->rows[1 - ps->cur];
    rows_reserve(ps, nr, nn);
    PpCopyCols c2;
    memset(&c2, 0, sizeof(c2));
    c2.ncols = d.n_cols;
    for (int j = 0; j < d.n_cols; ++j) {
      if (!ps->used_col[j]) continue;
      c2.bsrc[j] = bv.cols.col[j];
      c2.bnul[j] = bv.cols.nul[j];
      c2.csrc[j] = cr.col[j];
      c2.cnul[j] = cr.nul[j];
      c2.dst[j] = nr.col[j];
      c2.dnul[j] = nr.nul[j];
      c2.bytes[j] = ps->col_bytes[j];
    }
    hipLaunchKernelGGL(k_pp_carry, grd, blk, 0, st, m, a, skeys, sids, keep, pos, c2, nr.ts, nr.key, nr.start);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    nr.n = nn;
    ps->rows[ps->cur].n = 0;
    ps->cur = 1 - ps->cur;
    h->kend();
  }
}

// Rows the next push may carry (carried rows included) before a tie component's 27-bit combined row overflows:
// larger pushes are cut into sub-pushes by the caller (a stream without carry runs on the machine instead).
int64_t sg_partial_max_rows(SgHandle* h, PartialState* ps) {
  if (ps->mode != 1 || h->opt.no_carry) return INT64_MAX;
  const char* e = getenv("SG_DEBUG_PP_ROW_BUDGET");   // (debug: a lower budget exercises sub-pushes)
  const int64_t v = e ? atoll(e) : 0;
  const int64_t lim = v > 0 && v < ((int64_t)1 << 27) ? v : ((int64_t)1 << 27);
  return lim - 1 - ps->rows[ps->cur].n;
}

// Returns 1 when the push ran on partial lanes, 0 when it breaks the route's precondition (nothing was changed).
int sg_partial_push(SgHandle* h, PartialState* ps, const BatchView& bv, int64_t n, uint32_t kb) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const PpRows& cr = ps->rows[ps->cur];
  const int64_t nc = h->opt.no_carry ? 0 : cr.n;
  const int64_t m = nc + n;
  if (ps->mode == 1 && m >= ((int64_t)1 << 27)) {   // tie components hold a combined row in 27 bits
    // (the caller cuts pushes into sub-pushes of sg_partial_max_rows; the carried partials cannot leave the route)
    if (nc > 0) throw SgError(SG_ECAPACITY, "partial-lane route: push at most 2^27 rows at a time (carried rows included)");
    return 0;
  }
  // keys whose time goes back (k_pp_segments): their lanes skip rows only while waiting in a count state
  const int order_check = ps->mode == 1 ? 1 : 0;
  PpArgs a;
  memset(&a, 0, sizeof(a));
  a.nc = nc;
  a.n = n;
  a.base_index = bv.base_index;
  a.index = bv.index;
  a.bts = bv.ts;
  a.cts = cr.ts;
  a.stream = bv.stream;
  a.bkey = bv.key;
  a.ckey = cr.key;
  a.cstart = ps->mode == 1 && nc > 0 ? cr.start : nullptr;
  a.drop_before = INT64_MIN;
  a.dead_after = INT64_MAX;
  // (only when every state a partial can emit from expires it by `within`: a count state never does, so a query whose
  // count state is a final one keeps every partial)
  bool lat_ok = h->opt.bounded_lateness && n > 0 && d.within >= 0;
  for (int s = 0; s < d.n_states; ++s)
    if (d.states[s].kind == SG_K_COUNT && d.states[s].has_selector) lat_ok = false;
  if (lat_ok) {
    // the largest timestamp so far; every later row is at most max_lateness_ms behind it, so a partial whose e1 is
    // more than `within` before (that - max_lateness_ms) never sees a row it could emit at again
    int64_t* dmax = (int64_t*)h->ws.get("pp_tsmax", sizeof(int64_t), st);
    size_t tb = 0;
    HIPCHK(rocprim::reduce(nullptr, tb, bv.ts, dmax, INT64_MIN, (size_t)n, rocprim::maximum<int64_t>(), st));
    void* tmp = h->ws.get("pp_tsmax_tmp", tb, st);
    HIPCHK(rocprim::reduce(tmp, tb, bv.ts, dmax, INT64_MIN, (size_t)n, rocprim::maximum<int64_t>(), st));
    int64_t hm = INT64_MIN;
    HIPCHK(hipMemcpyAsync(&hm, dmax, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    h->ts_max_seen = std::max(h->ts_max_seen, hm);
    const int64_t lat = std::max<int64_t>(0, h->opt.max_lateness_ms);
    const int64_t w = std::max<int64_t>(0, d.within);
    if (h->ts_max_seen > INT64_MIN / 2 && w < (int64_t)1 << 60 && lat < (int64_t)1 << 60) {
      a.drop_before = h->ts_max_seen - lat - w;
      a.dead_after = w + lat;
    }
  }
  const SgCols cc = carried_cols(ps, cr);
  int end_bit = 1;
  while ((1ull << end_bit) <= (uint64_t)kb) ++end_bit;
  const uint32_t sentinel = kb;
  const dim3 blk(256), grd((unsigned)((m + 255) / 256));
  const dim3 grs((unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 4096)));
  uint32_t* keys = (uint32_t*)h->ws.get("pp_keys", 4 * m, st);
  uint32_t* skeys = (uint32_t*)h->ws.get("pp_skeys", 4 * m, st);
  uint32_t* sids = (uint32_t*)h->ws.get("pp_sids", 4 * m, st);
  int32_t* err = (int32_t*)h->ws.get("pp_err", 8, st);
  HIPCHK(hipMemsetAsync(err, 0, 8, st));
  h->mark(0);
  // ---- predicate-evaluation pass over the batch rows
  for (int s = 0; s < SG_MAX_STATES; ++s) a.lbits[s] = nullptr;
  {
    const int64_t ntiles = (n + 255) / 256;
    bool any = false;
    for (int s = 0; s < d.n_states && n > 0; ++s) {
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
      uint64_t* bits = (uint64_t*)h->ws.get("pp_lbits" + std::to_string(s), sizeof(uint64_t) * 4 * (ntiles + 1), st);
      launch_pred(d, pa, bv.stream, bv.cols, h->ddesc, bits, nullptr, st);
      HIPCHK(hipGetLastError());
      a.lbits[s] = bits;
    }
    if (any) h->kend();
  }
  h->mark(1);
  // ---- the key-ordered rows the lanes read
  bool batch_nul = false;
  for (int k = 0; k < d.n_ret; ++k) batch_nul |= bv.cols.nul[d.ret_col[k]] != nullptr;
  if (batch_nul) ps->nulls_seen = 1;
  const bool any_nul = batch_nul || (nc > 0 && ps->nulls_seen);
  PpPacked P;
  memset(&P, 0, sizeof(P));
  P.ts = (int64_t*)h->ws.get("pp_qts", 8 * m, st);
  for (int k = 0; k < d.n_ret; ++k) {
    P.wide[k] = (d.ret_type[k] == SG_T_LONG || d.ret_type[k] == SG_T_DOUBLE) ? 1 : 0;
    P.val[k] = h->ws.get("pp_qv" + std::to_string(k), (P.wide[k] ? 8 : 4) * m, st);
  }
  P.nul = any_nul ? (uint32_t*)h->ws.get("pp_qnul", 4 * m, st) : nullptr;
  P.lb = (uint32_t*)h->ws.get("pp_qlb", 4 * m, st);
  P.sid = sids;
  P.nc = nc;
  P.bts = bv.ts;
  P.cts = cr.ts;
  for (int k = 0; k < d.n_ret; ++k) {
    P.bcol[k] = bv.cols.col[d.ret_col[k]];
    P.ccol[k] = cc.col[d.ret_col[k]];
  }
  uint32_t* flag = (uint32_t*)h->ws.get("pp_flag", 4 * (m + 1), st);
  uint32_t* fpos = (uint32_t*)h->ws.get("pp_fpos", 4 * (m + 1), st);
  uint32_t* cand = (uint32_t*)h->ws.get("pp_cand", 4 * (m + 1), st);
  uint32_t* beg = (uint32_t*)h->ws.get("pp_beg", 4 * (size_t)kb, st);
  uint32_t* end = (uint32_t*)h->ws.get("pp_end", 4 * (size_t)kb, st);
  uint8_t* kback = nullptr;
  if (order_check) {
    kback = (uint8_t*)h->ws.get("pp_kback", (size_t)kb, st);
    HIPCHK(hipMemsetAsync(kback, 0, (size_t)kb, st));
    a.kback = kback;
  }
  bool rec_mode = ps->rec_ok && !any_nul && m > 0;
  if (rec_mode) {
    // record sort: one 16-B record per row through the key sort, unpacked into the SoA rows (no batch-wide gather)
    RecArgs ra;
    memset(&ra, 0, sizeof(ra));
    ra.mode = ps->mode;
    ra.start = ps->rule.start;
    ra.partitioned = d.partitioned;
    ra.sentinel = sentinel;
    for (int k = 0; k < SG_MAX_RET; ++k) ra.hot[k] = ps->hot[k];
    int64_t t0 = 0;
    HIPCHK(hipMemcpyAsync(&t0, n ? bv.ts : cr.ts, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    ra.tbase = t0;
    PpRec* recs = (PpRec*)h->ws.get("pp_recs", sizeof(PpRec) * m, st);
    PpRec* srecs = (PpRec*)h->ws.get("pp_srecs", sizeof(PpRec) * m, st);
    h->kbeg("route");
    hipLaunchKernelGGL(k_pp_rec, grs, blk, 0, st, a, bv.cols, cc, h->ddesc, ra, keys, recs, err);
    HIPCHK(hipGetLastError());
    h->kend();
    h->kbeg("key_sort");
    {
      size_t tb = 0;
      HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, keys, skeys, recs, srecs, (size_t)m, 0, end_bit, st));
      void* tmp = h->ws.get("pp_rsort_tmp", tb, st);
      HIPCHK(rocprim::radix_sort_pairs(tmp, tb, keys, skeys, recs, srecs, (size_t)m, 0, end_bit, st));
    }
    h->kend();
    int32_t herr = 0;
    HIPCHK(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (herr & 2) throw SgError(SG_EINVAL, "a partition key id is >= the batch's key_bound");
    if (herr & 4) {   // a timestamp more than 2^31 ms from the push's first: the gather path carries full timestamps
      rec_mode = false;
      HIPCHK(hipMemsetAsync(err, 0, 8, st));
    } else {
      // the lanes read only the record's hot slots (every slot a non-local filter reads); the others are read for
      // matches only, lazily at record build.  Sequence lanes read timestamps only for matches as well.
      if (ps->mode == 2) P.ts = nullptr;
      for (int k = 0; k < d.n_ret; ++k) if (ps->hot[k] < 0) P.val[k] = nullptr;
      h->kbeg("pack");
      hipLaunchKernelGGL(k_pp_unpack, grs, blk, 0, st, a, bv.cols, cc, h->ddesc, ra, skeys, srecs, P, sids, flag);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemsetAsync(beg, 0, 4 * (size_t)kb, st));
      HIPCHK(hipMemsetAsync(end, 0, 4 * (size_t)kb, st));
      hipLaunchKernelGGL(k_pp_segments, grd, blk, 0, st, m, a, skeys, sids, P.ts, order_check, sentinel, beg,
                         end, kback);
      HIPCHK(hipGetLastError());
      h->kend();
    }
  }
  if (!rec_mode) {
    uint32_t* ids = (uint32_t*)h->ws.get("pp_ids", 4 * m, st);
    h->kbeg("route");
    hipLaunchKernelGGL(k_pp_route, grd, blk, 0, st, a, h->ddesc, d.partitioned, sentinel, keys, ids, err);
    HIPCHK(hipGetLastError());
    h->kend();
    h->kbeg("key_sort");
    {
      size_t tb = 0;
      HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, keys, skeys, ids, sids, (size_t)m, 0, end_bit, st));
      void* tmp = h->ws.get("pp_sort_tmp", tb, st);
      HIPCHK(rocprim::radix_sort_pairs(tmp, tb, keys, skeys, ids, sids, (size_t)m, 0, end_bit, st));
    }
    HIPCHK(hipMemsetAsync(beg, 0, 4 * (size_t)kb, st));
    HIPCHK(hipMemsetAsync(end, 0, 4 * (size_t)kb, st));
    if (m) hipLaunchKernelGGL(k_pp_segments, grd, blk, 0, st, m, a, skeys, sids, (const int64_t*)nullptr,
                              order_check, sentinel, beg, end, kback);
    HIPCHK(hipGetLastError());
    h->kend();
    h->kbeg("pack");
    if (m) hipLaunchKernelGGL(k_pp_pack, grs, blk, 0, st, a, bv.cols, cc, h->ddesc, ps->rule.local_mask, ps->rule.start,
                              skeys, sids, sentinel, P, flag);
    HIPCHK(hipGetLastError());
    h->kend();
  }
  {
    int32_t herr = 0;
    HIPCHK(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (herr & 2) throw SgError(SG_EINVAL, "a partition key id is >= the batch's key_bound");
  }
  h->mark(2);
  if (ps->mode == 2) return seq_lanes_push(h, ps, bv, n, kb, a, P, skeys, sids, beg, end, sentinel);
  h->kbeg("start_rows");
  HIPCHK(hipMemsetAsync(flag + m, 0, 4, st));
  {
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, flag, fpos, (uint32_t)0, (size_t)m + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("pp_fscan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, flag, fpos, (uint32_t)0, (size_t)m + 1, rocprim::plus<uint32_t>(), st));
  }
  if (m) hipLaunchKernelGGL(k_pp_compact, grd, blk, 0, st, m, flag, fpos, cand);
  HIPCHK(hipGetLastError());
  h->kend();
  uint32_t ncand = 0;
  HIPCHK(hipMemcpyAsync(&ncand, fpos + m, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // ---- partial lanes
  const int nsel = d.n_select;
  const int32_t rstride = 32 + 8 * nsel;
  const int64_t cap = std::max<int64_t>(ncand, 1);   // a partial completes at most once (sg_pp_rule)
  PpOut o;
  o.rec = (char*)h->ws.get("pp_rec", (size_t)cap * rstride, st);
  o.k1 = (uint64_t*)h->ws.get("pp_k1", 8 * cap, st);
  o.th = (uint64_t*)h->ws.get("pp_th", 8 * cap, st);
  o.tl = (uint64_t*)h->ws.get("pp_tl", 8 * cap, st);
  o.count = (unsigned long long*)h->ws.get("pp_count", 16, st);
  o.maxoff = (uint32_t*)(o.count + 1);
  o.jp = (uint32_t*)h->ws.get("pp_jp", 4 * cap, st);
  o.fail = err + 1;
  o.rstride = 20 + 4 * nsel;   // compact match records (k_em_scatter writes the rstride-byte ones)
  int rb = 1;
  while ((1ll << rb) < n + 1) ++rb;
  const int k1_bits = std::min(64, rb + 8);
  o.k1_none = k1_bits >= 64 ? ~0ull : (1ull << k1_bits) - 1;
  HIPCHK(hipMemsetAsync(o.count, 0, 16, st));
  // the carry: lanes still pending after their key's last row mark the rows they hold (PpLane::witnesses)
  uint32_t* keep = nullptr;
  if (!h->opt.no_carry && m) {
    keep = (uint32_t*)h->ws.get("pp_keep", 4 * (m + 1), st);
    uint8_t* kst = (uint8_t*)h->ws.get("pp_kstart", (size_t)m + 1, st);
    HIPCHK(hipMemsetAsync(keep, 0, 4 * (m + 1), st));
    HIPCHK(hipMemsetAsync(kst, 0, (size_t)m + 1, st));
    a.keep = keep;
    a.kstart = kst;
  }
  // wait-term block summaries (chain.h PpWait): only without nulls (a null row passes `!=`), 4-byte attributes
  P.wsum = nullptr;
  if (ps->rule.wait_slots && !P.nul && m > 0) {
    uint32_t slots = 0, fslots = 0;
    int nw = 0;
    for (int k = 0; k < SG_MAX_RET; ++k) P.wix[k] = -1;
    for (int s = 0; s < d.n_states; ++s) {
      const PpWait& w = ps->rule.wait[s];
      if (!w.ok || w.slot >= d.n_ret || P.wide[w.slot] || !P.val[w.slot] || ((slots >> w.slot) & 1u)) continue;
      slots |= 1u << w.slot;
      if (w.fast == 2) fslots |= 1u << w.slot;
      P.wix[w.slot] = (int8_t)nw++;
    }
    bool all = true;   // every wait term's attribute summarized (wait_on may return any of them)
    for (int s = 0; s < d.n_states; ++s)
      if (ps->rule.wait[s].ok && !((slots >> ps->rule.wait[s].slot) & 1u)) all = false;
    if (nw && all) {
      P.wnb = (m + 7) / 8;
      uint2* ws = (uint2*)h->ws.get("pp_wsum", sizeof(uint2) * (size_t)nw * (size_t)P.wnb, st);
      P.wsum = ws;
      h->kbeg("wait_sum");
      hipLaunchKernelGGL(k_pp_wsum, dim3((unsigned)((P.wnb + 255) / 256)), blk, 0, st, m, P, slots, fslots, ws);
      HIPCHK(hipGetLastError());
      h->kend();
    }
  }
  h->kbeg("partial_lanes");
  if (ncand) {
    const int64_t wcands = PP_WAVE_CANDS;
    const dim3 gl((unsigned)((ncand + wcands * (PP_BLOCK / 64) - 1) / (wcands * (PP_BLOCK / 64))));
    if (ps->pp_small && lanes_fast(ps) && ps->shape_c3)
      hipLaunchKernelGGL((k_pp_lanes<PpSmall, true, PpShapeC3>), gl, dim3(PP_BLOCK), 0, st, a, P, h->ddesc, ps->drule,
                         cand, (int64_t)ncand, skeys, sids, end, o, wcands);
    else if (ps->pp_small && lanes_fast(ps))
      hipLaunchKernelGGL((k_pp_lanes<PpSmall, true>), gl, dim3(PP_BLOCK), 0, st, a, P, h->ddesc, ps->drule, cand,
                         (int64_t)ncand, skeys, sids, end, o, wcands);
    else if (ps->pp_small)
      hipLaunchKernelGGL(k_pp_lanes<PpSmall>, gl, dim3(PP_BLOCK), 0, st, a, P, h->ddesc, ps->drule, cand, (int64_t)ncand,
                         skeys, sids, end, o, wcands);
    else
      hipLaunchKernelGGL(k_pp_lanes<PpBig>, gl, dim3(PP_BLOCK), 0, st, a, P, h->ddesc, ps->drule, cand, (int64_t)ncand,
                         skeys, sids, end, o, wcands);
  }
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(3);
  unsigned long long total = 0;
  uint32_t hmaxoff = 0;
  int32_t fail = 0;
  HIPCHK(hipMemcpyAsync(&total, o.count, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&hmaxoff, o.maxoff, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&fail, o.fail, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (fail) throw SgError(fail, "partial lane capacity exceeded (query outside the route's shape)");
  // ---- delivery order: LSD stable sorts (tie low word, tie high word, then trigger row and visit slot)
  if (total) {
    const int64_t T = (int64_t)ncand;   // one slot per start row; rows without a match sort behind (k1 = ~0)
    const dim3 g2((unsigned)((T + 255) / 256));
    uint32_t* ia = (uint32_t*)h->ws.get("pp_ia", 4 * T, st);
    uint32_t* ib = (uint32_t*)h->ws.get("pp_ib", 4 * T, st);
    uint64_t* ka = (uint64_t*)h->ws.get("pp_ka", 8 * T, st);
    uint64_t* kb2 = (uint64_t*)h->ws.get("pp_kb", 8 * T, st);
    h->kbeg("match_order");
    int ob = 1;
    while ((1ull << ob) <= (uint64_t)hmaxoff) ++ob;
    const int need = rb + 4 + ps->rule.n_hist * (ob + 4);
    const int order_path = h->opt.partial_lanes;   // 1 / 2: tie runs / LSD sorts even where one key fits (testing)
    if (need <= 63 && order_path == 0) {   // one radix sort over a single composed key
      const uint64_t none = (1ull << need) - 1;
      hipLaunchKernelGGL(k_pp_key, g2, blk, 0, st, T, o.k1, o.th, o.tl, o.jp, o.k1_none, ps->rule.n_hist, hmaxoff, ob,
                         none, ka, ia);
      sort_pairs64(h, "one", ka, kb2, ia, ib, T, need);
      std::swap(ia, ib);
    } else {
    int tb = 1;
    while ((1ll << tb) < m) ++tb;
    const int comp_bits = tb + 4;   // one history component: combined row << 4 | visit slot
    const int eb = std::min(64, 31 + comp_bits);
    // k1 first, then the tie runs in place (k_pp_ties); the three LSD sorts only when a run is too long
    int32_t hover = 1;
    if (order_path != 2) {
      int32_t* over = (int32_t*)h->ws.get("pp_over", 4, st);
      HIPCHK(hipMemsetAsync(over, 0, 4, st));
      hipLaunchKernelGGL(k_pp_iota, g2, blk, 0, st, T, ia);
      sort_pairs64(h, "k1", o.k1, kb2, ia, ib, T, k1_bits);
      const uint64_t tl_mask = ps->rule.n_hist <= 2 ? 0ull : (eb >= 64 ? ~0ull : (1ull << eb) - 1);
      hipLaunchKernelGGL(k_pp_ties, dim3((unsigned)((total + 255) / 256)), blk, 0, st, (int64_t)total, kb2, ib, o.th,
                         o.tl, tl_mask, 256, over);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(&hover, over, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    if (!hover) {
      std::swap(ia, ib);
    } else {
    hipLaunchKernelGGL(k_pp_iota, g2, blk, 0, st, T, ia);
    if (ps->rule.n_hist > 2) {
      hipLaunchKernelGGL(k_pp_take, g2, blk, 0, st, T, o.tl, ia, ka);
      sort_pairs64(h, "lo", ka, kb2, ia, ib, T, eb);
      std::swap(ia, ib);
    }
    hipLaunchKernelGGL(k_pp_take, g2, blk, 0, st, T, o.th, ia, ka);
    sort_pairs64(h, "hi", ka, kb2, ia, ib, T, 64);
    std::swap(ia, ib);
    hipLaunchKernelGGL(k_pp_take, g2, blk, 0, st, T, o.k1, ia, ka);
    sort_pairs64(h, "k1", ka, kb2, ia, ib, T, k1_bits);
    std::swap(ia, ib);
    }
    }
    const int64_t M = (int64_t)total;
    char* out = h->out.reserve(M, nsel, st);
    uint32_t* dest = (uint32_t*)h->ws.get("pp_dest", 4 * (size_t)(T + 1), st);
    HIPCHK(hipMemsetAsync(dest, 0xFF, 4 * (size_t)T, st));
    hipLaunchKernelGGL(k_em_dest, dim3((unsigned)((M + 255) / 256)), blk, 0, st, M, ia, dest);
    if ((size_t)256 * rstride > 65536)   // (up to SG_MAX_SELECT selected attributes: 256 * 288 B of LDS)
      HIPCHK(hipFuncSetAttribute((const void*)k_em_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(256 * rstride)));
    hipLaunchKernelGGL(k_em_scatter, g2, blk, (size_t)256 * rstride, st, T, dest, o.rec, o.rstride,
                       out + (size_t)h->out.n * rstride, rstride, P, h->ddesc, bv.index, bv.base_index);
    HIPCHK(hipGetLastError());
    h->kend();
    h->out.n += M;
  }
  // ---- carry
  if (keep) carry_rows(h, ps, bv, a, m, skeys, sids, keep);
  h->mark(4);
  h->last_events = n;
  h->last_spilled = 0;
  h->last_matches = (int64_t)total;
  return 1;
}

// Snapshot of the route's state: the carried rows (the rows pending partials hold, each flagged when a partial starts at
// it -- replaying them rebuilds every partial the reference still holds in StreamPreStateProcessor.pendingStateEventList /
// newAndEveryStateEventList, C/query/input/stream/state/StreamPreStateProcessor.java:352-367) and the latest timestamp.
void sg_partial_snapshot(SgHandle* h, PartialState* ps, SnapW& w) {
  const PpRows& r = ps->rows[ps->cur];
  w.pod((int32_t)ps->mode);
  if (ps->mode == 2) {   // sequence lanes: the per-key machine states as well (seq.h SeqState, positions over the rows)
    w.pod((int64_t)ps->sq_bytes);   // (the state layout: a snapshot restores only into the same geometry)
    w.pod(ps->kst_keys);
    w.pod(ps->seq_pushes);
    if (ps->kst_keys) w.dev(ps->kst, ps->sq_bytes * (size_t)ps->kst_keys, h->stream);
  }
  w.pod(r.n);
  if (!r.n) return;
  w.dev(r.ts, 8 * r.n, h->stream);
  w.dev(r.key, 4 * r.n, h->stream);
  w.dev(r.start, r.n, h->stream);
  for (int j = 0; j < SG_MAX_COLS; ++j) {
    if (!ps->used_col[j]) continue;
    w.dev(r.col[j], (size_t)ps->col_bytes[j] * r.n, h->stream);
    w.dev(r.nul[j], r.n, h->stream);
  }
}

void sg_partial_restore(SgHandle* h, PartialState* ps, SnapR& rd) {
  sg_partial_reset(ps);
  ps->nulls_seen = 1;   // the restored rows may hold nulls
  if (rd.pod<int32_t>() != ps->mode) throw SgError(SG_EINVAL, "snapshot: lane route differs");
  if (ps->mode == 2) {
    if (rd.pod<int64_t>() != (int64_t)ps->sq_bytes) throw SgError(SG_EINVAL, "snapshot: sequence state layout differs");
    const int64_t keys = rd.pod<int64_t>();
    const int64_t pushes = rd.pod<int64_t>();
    if (keys < 0 || keys > ((int64_t)1 << 31)) throw SgError(SG_EINVAL, "snapshot: bad sequence state count");
    if (keys > ps->kst_keys) {
      if (ps->kst) hipFree(ps->kst);
      if (ps->kst_out) hipFree(ps->kst_out);
      ps->kst = ps->kst_out = nullptr;
      if (hipMalloc(&ps->kst, ps->sq_bytes * (size_t)keys) != hipSuccess ||
          hipMalloc(&ps->kst_out, ps->sq_bytes * (size_t)keys) != hipSuccess)
        throw SgError(SG_ECAPACITY, "hipMalloc sequence states");
      ps->kst_keys = keys;
    }
    if (ps->kst_keys) HIPCHK(hipMemset(ps->kst, 0, ps->sq_bytes * (size_t)ps->kst_keys));
    if (keys) rd.dev(ps->kst, ps->sq_bytes * (size_t)keys, h->stream);
    ps->seq_pushes = pushes;
  }
  const int64_t n = rd.pod<int64_t>();
  if (n < 0 || n >= ((int64_t)1 << 31)) throw SgError(SG_EINVAL, "snapshot: bad carried row count");
  PpRows& r = ps->rows[ps->cur];
  rows_reserve(ps, r, n);
  if (n) {
    rd.dev(r.ts, 8 * n, h->stream);
    rd.dev(r.key, 4 * n, h->stream);
    rd.dev(r.start, n, h->stream);
    for (int j = 0; j < SG_MAX_COLS; ++j) {
      if (!ps->used_col[j]) continue;
      rd.dev(r.col[j], (size_t)ps->col_bytes[j] * n, h->stream);
      rd.dev(r.nul[j], n, h->stream);
    }
  }
  r.n = n;
}
