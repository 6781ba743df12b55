// chain.h -- per-partial pattern machine (SG route "partial lanes") for MI355X.
//
// For a PATTERN whose only `every` re-arms its single start state (`every e1=S[local] -> ... within T`, every state on
// one stream, no absence), the partial matches started by different e1 rows never interact: each one is created by
// the start state's `every` clone (StreamPostStateProcessor.process -> addEveryState, C/query/input/stream/state/
// StreamPostStateProcessor.java:53-72, StreamPreStateProcessor.addEveryState :219-227), is handed from state to state
// by the object itself (addState :203-216), and every decision the Pre/Post processors take on it reads only its own
// slots (StreamPreStateProcessor.processAndReturn :292-337, isExpired :102-113, CountPreStateProcessor.processAndReturn
// :53-93, LogicalPreStateProcessor.processAndReturn :132-176).  So one GPU lane can run one partial from its e1 row
// forward, alone, over the rows of its key, instead of one lane walking every pending partial of the key per event.
//
// What other partials contribute is only ORDER: matches of one event are delivered state by state in the receiver's
// visit order (MultiProcessStreamReceiver.receive :271-309) and, within a state, in pending-list order.  A pending list
// is the survivors of earlier rows followed by the newAndEvery list moved in by updateState (:281-289), and
// newAndEvery is filled in the order addState is called -- which is the order the predecessor state walked ITS list
// at that row.  Hence a partial's position in any list is the lexicographic order of its insertion history read
// backwards: (row and visit slot of the latest addState, then of the one before, ... down to its e1 row).  Each lane
// records that history (`hist`) and the match records carry it as a tie-break key; a stable radix sort by
// (trigger row, visit slot, history) restores the reference's delivery order exactly.
//
// State kept per lane (LDS on the GPU): each state's slot (row) or count chain, list membership bits for the
// pending (l0) and newAndEvery (l1) lists, the partial's timestamp, the per-state processor flags and the history.
// Every method restates the KeyMachine method of interp.h with the same name (which cites its reference method).
#pragma once
#include <stdint.h>
#include <string.h>

#include "../../include/siddhi_gpu.h"

#ifndef SG_HD
#define SG_HD __host__ __device__
#endif

#define PP_MAX_S 8         // states of the query
#define PP_MAX_CHAIN 16   // count-chain entries over all count states of the query
#define PP_MAX_HIST 4     // insertions recorded (elements after the start state)
#define PP_MAX_TERMS 4    // conjunctive compare terms of a filter evaluated without the VM

// A filter that is a conjunction of `operand CMP operand` terms (operands: attribute or constant) is evaluated directly;
// anything else runs on the postfix VM (sg_device.h).  Same semantics: sg_cmp per term, AND of the results.
struct PpOperand {
  int32_t kind;      // SG_OP_VAR or SG_OP_CONST
  int32_t state, idx, slot, type;
  int64_t bits;
};
struct PpTerm {
  PpOperand l, r;
  int32_t op, dom;
  int32_t fast;      // 1: both operands INT/LONG in the integral domain, 2: both FLOAT in the float domain, 0: SgVal path
};

SG_HD inline bool pp_cmp_i(int op, int64_t a, int64_t b) {
  switch (op) {
    case 0: return a == b;
    case 1: return a != b;
    case 2: return a > b;
    case 3: return a >= b;
    case 4: return a < b;
    default: return a <= b;
  }
}
SG_HD inline bool pp_cmp_f(int op, float a, float b) {
  switch (op) {
    case 0: return a == b;
    case 1: return a != b;
    case 2: return a > b;
    case 3: return a >= b;
    case 4: return a < b;
    default: return a <= b;
  }
}
SG_HD inline float pp_f32(int64_t bits) {
  const uint32_t u = (uint32_t)bits;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// Wait skipping: a state whose filter is one fast compare of the arriving row's 4-byte attribute with an operand that
// stays fixed while the partial waits there (a constant or another state's event).  See PpLane::wait_on.
struct PpWait {
  int32_t ok;
  int32_t slot;      // retained slot of the arriving row's attribute (INT or FLOAT)
  int32_t op;        // normalized: row OP fixed
  int32_t fast;      // 1: integral domain, 2: float domain
  int32_t other;     // the fixed operand: 0 term.r, 1 term.l
};

struct SgPpRule {
  int32_t ok;
  int32_t start;                      // the start state
  int32_t recv;                       // the single (multi) receiver
  int32_t n_hist;                     // tie components of an emission (= elements after the start)
  uint32_t local_mask;                // states whose filter reads only the arriving event (precomputed bits)
  int32_t coff[PP_MAX_S];             // count state -> offset of its chain in PpLane.chain
  int32_t visit_rank[PP_MAX_S];       // state -> its slot in the receiver's visit order
  int32_t nterm[PP_MAX_S];            // -1: the VM evaluates the state's filter
  PpTerm term[PP_MAX_S][PP_MAX_TERMS];
  PpWait wait[PP_MAX_S];
  uint32_t wait_slots;                // retained slots some wait term reads (block summaries, partial.hip)
};

// Parse a postfix filter into conjunctive compare terms (t1 t2 AND t3 AND ...); false if it has another form.
SG_HD inline bool pp_operand(const int64_t* c, int len, int& pc, PpOperand& o) {
  if (pc < len && c[pc] == SG_OP_VAR && pc + 5 <= len) {
    o.kind = SG_OP_VAR;
    o.state = (int32_t)c[pc + 1];
    o.idx = (int32_t)c[pc + 2];
    o.slot = (int32_t)c[pc + 3];
    o.type = (int32_t)c[pc + 4];
    o.bits = 0;
    pc += 5;
    return true;
  }
  if (pc < len && c[pc] == SG_OP_CONST && pc + 3 <= len) {
    o.kind = SG_OP_CONST;
    o.state = o.idx = o.slot = 0;
    o.type = (int32_t)c[pc + 1];
    o.bits = c[pc + 2];
    pc += 3;
    return true;
  }
  return false;
}
SG_HD inline int pp_terms(const int64_t* c, int len, PpTerm* t) {
  int pc = 0, n = 0;
  while (pc < len) {
    if (n >= PP_MAX_TERMS) return -1;
    if (!pp_operand(c, len, pc, t[n].l) || !pp_operand(c, len, pc, t[n].r)) return -1;
    if (pc + 3 > len || c[pc] != SG_OP_CMP) return -1;
    t[n].op = (int32_t)c[pc + 1];
    t[n].dom = (int32_t)c[pc + 2];
    {
      const int lt = t[n].l.type, rt = t[n].r.type;
      const bool li = lt == SG_T_INT || lt == SG_T_LONG, ri = rt == SG_T_INT || rt == SG_T_LONG;
      t[n].fast = (t[n].dom == 0 && li && ri) ? 1 : (t[n].dom == 1 && lt == SG_T_FLOAT && rt == SG_T_FLOAT) ? 2 : 0;
    }
    pc += 3;
    ++n;
    if (n > 1) {
      if (pc >= len || c[pc] != SG_OP_AND) return -1;
      pc += 1;
    }
  }
  return n;
}

// The wait terms of a rule (PpWait): state s (not the start) whose filter is exactly one fast term with one side the
// arriving row's INT / FLOAT attribute (state s, index CURRENT = -1) and the other a constant or an event of another
// state.
SG_HD inline void pp_wait_rule(const sg_nfa_desc& d, SgPpRule& r) {
  static const int32_t flip[6] = {0, 1, 4, 5, 2, 3};   // a OP b  <=>  b flip(OP) a
  r.wait_slots = 0;
  for (int s = 0; s < PP_MAX_S; ++s) r.wait[s].ok = 0;
  for (int s = 0; s < d.n_states; ++s) {
    if (s == r.start || r.nterm[s] != 1 || ((r.local_mask >> s) & 1u)) continue;
    const PpTerm& t = r.term[s][0];
    if (!t.fast || t.op < 0 || t.op > 5) continue;
    const int want = t.fast == 1 ? SG_T_INT : SG_T_FLOAT;
    auto is_row = [&](const PpOperand& o) { return o.kind == SG_OP_VAR && o.state == s && o.idx == -1 && o.type == want; };
    auto fixed = [&](const PpOperand& o) { return o.kind == SG_OP_CONST || (o.kind == SG_OP_VAR && o.state != s); };
    PpWait w;
    w.ok = 0;
    if (is_row(t.l) && fixed(t.r)) {
      w.slot = t.l.slot;
      w.op = t.op;
      w.other = 0;
    } else if (is_row(t.r) && fixed(t.l)) {
      w.slot = t.r.slot;
      w.op = flip[t.op];
      w.other = 1;
    } else {
      continue;
    }
    if (w.slot < 0 || w.slot >= 32 || (t.fast == 2 && w.op == 1)) continue;   // (float `!=`: NaN rows pass it)
    w.fast = t.fast;
    w.ok = 1;
    r.wait[s] = w;
    r.wait_slots |= 1u << w.slot;
  }
}

// Block summaries of a wait attribute: min and max of an orderable 32-bit encoding over 8 key-ordered rows.  FLOAT:
// -0.0 is encoded as +0.0 (they compare equal) and NaN rows are left out (no compare but `!=` is true for them, and
// float `!=` never waits).  An empty summary (min > max) holds no row that can pass.
SG_HD inline uint32_t pp_wenc(uint32_t bits, int fast) {
  if (fast == 1) return bits ^ 0x80000000u;
  if (bits == 0x80000000u) bits = 0;
  return (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
}
SG_HD inline bool pp_wnan(uint32_t bits, int fast) { return fast == 2 && (bits & 0x7fffffffu) > 0x7f800000u; }
SG_HD inline int64_t pp_wdec_i(uint32_t e) { return (int64_t)(int32_t)(e ^ 0x80000000u); }
SG_HD inline float pp_wdec_f(uint32_t e) {
  const uint32_t u = (e & 0x80000000u) ? (e & 0x7fffffffu) : ~e;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
// can a row of the block pass `row OP c`?  (conservative: true unless no value in [min, max] passes)
SG_HD inline bool pp_may_pass(uint32_t mn, uint32_t mx, int op, int fast, int64_t cbits) {
  if (mn > mx) return false;
  if (fast == 1) {
    const int64_t lo = pp_wdec_i(mn), hi = pp_wdec_i(mx), c = cbits;
    switch (op) {
      case 0: return lo <= c && c <= hi;
      case 1: return !(lo == hi && lo == c);
      case 2: return hi > c;
      case 3: return hi >= c;
      case 4: return lo < c;
      default: return lo <= c;
    }
  }
  const float lo = pp_wdec_f(mn), hi = pp_wdec_f(mx), c = pp_f32(cbits);   // (c NaN: every compare is false)
  switch (op) {
    case 0: return lo <= c && c <= hi;
    case 2: return hi > c;
    case 3: return hi >= c;
    case 4: return lo < c;
    case 5: return lo <= c;
    default: return true;
  }
}

// Which queries may run as partial lanes (checked at lowering-independent level, on the flat descriptor).
SG_HD inline SgPpRule sg_pp_rule(const sg_nfa_desc& d) {
  SgPpRule r;
  r.ok = 0;
  r.start = -1;
  r.recv = -1;
  r.n_hist = 0;
  r.local_mask = 0;
  for (int s = 0; s < PP_MAX_S; ++s) { r.coff[s] = -1; r.visit_rank[s] = -1; r.nterm[s] = -1; }
  if (d.type != 0 || d.within < 0 || d.n_states < 2 || d.n_states > PP_MAX_S || d.n_sched != 0) return r;
  int nrecv = 0;
  for (int s = 0; s < SG_MAX_STREAMS; ++s)
    if (d.recv_of_stream[s] >= 0) { ++nrecv; r.recv = d.recv_of_stream[s]; }
  if (nrecv != 1) return r;
  const sg_receiver_desc& rv = d.receivers[r.recv];
  if (!rv.multi || rv.n != d.n_states || !rv.selector) return r;
  for (int k = 0; k < rv.n; ++k) r.visit_rank[rv.pres[rv.n - 1 - k]] = k;
  int starts = 0, chain = 0, elems = 0;
  for (int s = 0; s < d.n_states; ++s) {
    const sg_state_desc& x = d.states[s];
    if (r.visit_rank[s] < 0) return r;
    if (x.local) r.local_mask |= 1u << s;
    else r.nterm[s] = pp_terms(d.code + x.prog_off, x.prog_len, r.term[s]);
    if (x.kind != SG_K_STREAM && x.kind != SG_K_COUNT && x.kind != SG_K_LOGICAL) return r;
    if (x.callback >= 0) return r;
    if (x.is_start) {
      ++starts;
      r.start = s;
      if (x.kind != SG_K_STREAM || x.next_every != s || !x.local || x.has_selector || x.next_state < 0) return r;
      continue;
    }
    if (x.next_every >= 0 || x.within_every >= 0 || x.this_last != s) return r;
    if (x.kind == SG_K_COUNT) {
      if (x.min_count < 1 || x.max_count < x.min_count || x.max_count > 8 || x.has_selector) return r;
      if (x.next_state >= 0 && d.states[x.next_state].kind == SG_K_COUNT) return r;
      r.coff[s] = chain;
      chain += x.max_count;
    }
    if (x.kind == SG_K_LOGICAL && (x.partner < 0 || d.states[x.partner].kind != SG_K_LOGICAL)) return r;
    if (x.kind != SG_K_LOGICAL || s < x.partner) ++elems;
  }
  if (starts != 1 || d.n_start != 1 || chain > PP_MAX_CHAIN || elems > PP_MAX_HIST) return r;
  r.n_hist = elems;
  r.ok = 1;
  pp_wait_rule(d, r);
  return r;
}

// Carry of the partial-lane route: a lane still pending after its key's last row marks the rows it holds
// (PpLane::witnesses) and they survive into the next push, its e1 flagged as a start; nothing else is carried.  Count
// states never expire partials (CountPreStateProcessor.processAndReturn, C/query/input/stream/state/
// CountPreStateProcessor.java:53-93), so a partial waiting in one stays carried however old its e1 -- a later row whose
// time goes back can still complete it; every other state drops the partial at the first row more than `within` from
// e1 on either side (StreamPreStateProcessor.isExpired, :102-113).

// Tie key of an emission: the insertion history newest first, 31 bits per component (row << 4 | visit slot), two
// components per word (bit 63 is always set).  Rows only need to be in arrival order within one key.
SG_HD inline uint32_t pp_tkey(int64_t row, int rank) { return (uint32_t)(((uint64_t)row << 4) | (uint32_t)(rank & 15)); }

// Src interface: int64_t ts(int64_t row); SgVal read(int64_t row, int ret_slot, int type);
//                void read_bits(int64_t row, int ret_slot, int type, int64_t& bits, int& null) (INT sign-extended,
//                FLOAT as its 32-bit pattern -- the bit layout of sg_val_bits);
//                int lbit(int state, int64_t row) -> 0/1, or -1 when the state's filter must be evaluated.
// The dynamically indexed part of a lane's state (LDS on the GPU); the rest stays in registers.  Its geometry (S states,
// CH chain entries) sets how many lanes a CU holds: queries of C3's family (<= 4 states, <= 6 chain entries,
// sg_pp_small) run with 60-byte arrays instead of 120.
template <int S_, int CH_>
struct PpGeo {
  static constexpr int S = S_;
  static constexpr int CH = CH_;
};
using PpBig = PpGeo<PP_MAX_S, PP_MAX_CHAIN>;
using PpSmall = PpGeo<4, 6>;

template <class G>
struct PpArraysT {
  int32_t slot[G::S];
  int32_t chain[G::CH];
  uint32_t hist[PP_MAX_HIST];
  int8_t clen[G::S];
};
using PpArrays = PpArraysT<PpBig>;

SG_HD inline bool sg_pp_small(const SgPpRule& r, const sg_nfa_desc& d) {
  if (!r.ok || d.n_states > PpSmall::S) return false;
  int chain = 0;
  for (int s = 0; s < d.n_states; ++s)
    if (d.states[s].kind == SG_K_COUNT) chain += d.states[s].max_count;
  return chain <= PpSmall::CH;
}

// Every filter the lane evaluates is a list of fast compares or an event-local bit (sg_terms_fast): FAST lanes are
// compiled without the postfix VM and the SgVal compare, which shrinks the lane kernel's code to its hot loop.
template <class R>
SG_HD inline bool sg_terms_fast(const R& r, int n_states) {
  for (int s = 0; s < n_states; ++s) {
    if ((r.local_mask >> s) & 1u) continue;   // the GPU reads these from the packed condition bits, never the VM
    if (r.nterm[s] < 0) return false;
    for (int i = 0; i < r.nterm[s]; ++i)
      if (!r.term[s][i].fast) return false;
  }
  return true;
}

// State table of one query family known at compile time (kinds, successors, logical pairs, visit order): the lane's
// loops over the states unroll and their kind branches fold -- the interpreter's scalar control flow is what bounds
// the lane kernel.  Counts, windows and filters stay run-time values.  PpShapeAny reads the descriptor.
struct PpShapeAny {
  static constexpr bool known = false;
  static constexpr int n = 0;
  static constexpr int8_t kind[1] = {0}, next[1] = {0}, partner[1] = {0}, ltype[1] = {0}, sel[1] = {0}, pres[1] = {0};
};
// `every e1=S[..] -> e2=S[..]<m:n> -> e3=S[..] and e4=S[..]` (C3c's family: one stream, a count state feeding an
// `and` pair whose members both select)
struct PpShapeC3 {
  static constexpr bool known = true;
  static constexpr int n = 4;
  static constexpr int8_t kind[4] = {SG_K_STREAM, SG_K_COUNT, SG_K_LOGICAL, SG_K_LOGICAL};
  static constexpr int8_t next[4] = {1, 3, -1, -1};
  static constexpr int8_t partner[4] = {-1, -1, 3, 2};
  static constexpr int8_t ltype[4] = {0, 0, 0, 0};
  static constexpr int8_t sel[4] = {0, 0, 1, 1};
  static constexpr int8_t pres[4] = {0, 1, 2, 3};   // the receiver's processors (visited in reverse)
};
template <class SH>
SG_HD inline bool sg_pp_shape_is(const sg_nfa_desc& d, const SgPpRule& r) {
  if (!SH::known || !r.ok || d.n_states != SH::n || r.start != 0) return false;
  const sg_receiver_desc& rv = d.receivers[r.recv];
  if (rv.n != SH::n) return false;
  for (int s = 0; s < SH::n; ++s) {
    const sg_state_desc& x = d.states[s];
    if (x.kind != SH::kind[s] || x.next_state != SH::next[s] || x.partner != SH::partner[s] ||
        (x.kind == SG_K_LOGICAL && x.logical_type != SH::ltype[s]) || (x.has_selector != 0) != (SH::sel[s] != 0) ||
        rv.pres[s] != SH::pres[s])
      return false;
  }
  return true;
}

template <class Src, class G = PpBig, bool FAST = false, class SH = PpShapeAny>
struct PpLane {
  const sg_nfa_desc* d;
  const SgPpRule* ru;
  Src src;
  PpArraysT<G>* A;
  uint32_t l0, l1;
  uint32_t f_changed, f_returned, f_success;
  int64_t pts;
  int32_t pts_pos;   // the row whose timestamp pts is
  int64_t e1_ts;
  int32_t nh;
  int32_t overflow;
  bool wait_count;   // (set by wait_on) the partial waits in a count state: a skipped row cannot expire it
  // current row
  int32_t cur_row;
  int cur_rank;

  SG_HD const sg_state_desc& st(int s) const { return d->states[s]; }
  SG_HD static uint32_t bit(int s) { return 1u << s; }
  // the state table, from the compile-time shape when there is one
  static constexpr int NS = SH::known ? SH::n : G::S;   // states the loops cover
  SG_HD int nstates() const { if constexpr (SH::known) return SH::n; else return d->n_states; }
  SG_HD int kind_of(int s) const { if constexpr (SH::known) return SH::kind[s]; else return st(s).kind; }
  SG_HD int next_of(int s) const { if constexpr (SH::known) return SH::next[s]; else return st(s).next_state; }
  SG_HD int partner_of(int s) const { if constexpr (SH::known) return SH::partner[s]; else return st(s).partner; }
  SG_HD int ltype_of(int s) const { if constexpr (SH::known) return SH::ltype[s]; else return st(s).logical_type; }
  SG_HD bool sel_of(int s) const { if constexpr (SH::known) return SH::sel[s] != 0; else return st(s).has_selector != 0; }
  SG_HD int start_of() const { if constexpr (SH::known) return 0; else return ru->start; }

  // does the start state's armed partial accept this row (its filter, evaluated with e1 bound to the row)?
  SG_HD bool start_ok(int32_t row) {
#pragma unroll
    for (int s = 0; s < NS; ++s) { A->slot[s] = -1; A->clen[s] = 0; }
    A->slot[start_of()] = (int32_t)row;
    cur_row = row;
    return filter(start_of());
  }
  SG_HD void start(int32_t row) {   // the armed start partial takes e1 = row (process_and_return of the start state)
#pragma unroll
    for (int s = 0; s < NS; ++s) { A->slot[s] = -1; A->clen[s] = 0; }
    l0 = l1 = 0;
    f_changed = f_returned = f_success = 0;
    nh = 0;
    overflow = 0;
    cur_row = row;
    cur_rank = ru->visit_rank[start_of()];
    A->slot[start_of()] = (int32_t)row;
    e1_ts = src.ts(row);
    stream_post(start_of());   // the `every` clone it also makes stays behind in the start state's lists
  }

  // ---- event access (KeyMachine::get_event): row of (state, index in chain) or -1
  SG_HD int32_t get_event(int s, int idx) {
    if (kind_of(s) != SG_K_COUNT) {
      if (A->slot[s] < 0) return -1;
      return (idx == 0 || idx == -1) ? A->slot[s] : -1;
    }
    const int n = A->clen[s];
    if (n == 0) return -1;
    const int32_t* c = A->chain + ru->coff[s];
    int k;
    if (idx >= 0) k = idx;
    else if (idx == -1) k = n - 1;
    else if (idx == -2) k = n - 2;
    else k = n + idx;
    if (k < 0 || k >= n) return -1;
    return c[k];
  }
  SG_HD int64_t slot_ts(int s) {
    int32_t r = kind_of(s) == SG_K_COUNT ? (A->clen[s] ? A->chain[ru->coff[s]] : -1) : A->slot[s];
    return src.ts(r);
  }
  struct Reader {
    PpLane* m;
    SG_HD SgVal read(int s, int idx, int slotk, int type) {
      const int32_t r = m->get_event(s, idx);
      if (r < 0) {
        SgVal v;
        v.type = type;
        v.i = 0;
        v.d = 0;
        v.null = 1;
        return v;
      }
      return m->src.read(r, slotk, type);
    }
  };
  SG_HD void operand_bits(const PpOperand& o, int64_t& bits, int& null) {
    if (o.kind == SG_OP_CONST) {
      bits = o.bits;
      null = 0;
      return;
    }
    const int32_t r = get_event(o.state, o.idx);
    if (r < 0) { bits = 0; null = 1; return; }
    src.read_bits(r, o.slot, o.type, bits, null);
  }
  SG_HD SgVal operand(const PpOperand& o) {
    if (o.kind == SG_OP_CONST) return sg_val_from_bits(o.bits, o.type, 0);
    Reader rd{this};
    return rd.read(o.state, o.idx, o.slot, o.type);
  }
  SG_HD bool filter(int s) {
    if ((ru->local_mask >> s) & 1u) {
      const int b = src.lbit(s, cur_row);
      if (b >= 0) return b != 0;
    }
    const int nt = ru->nterm[s];
    if (FAST) {   // sg_terms_fast: every term is a fast compare
      for (int i = 0; i < nt; ++i) {
        const PpTerm& t = ru->term[s][i];
        int64_t a, b;
        int na, nb;
        operand_bits(t.l, a, na);
        operand_bits(t.r, b, nb);
        if (na || nb) {
          if (t.op != 1) return false;
          continue;
        }
        if (!(t.fast == 1 ? pp_cmp_i(t.op, a, b) : pp_cmp_f(t.op, pp_f32(a), pp_f32(b)))) return false;
      }
      return true;
    }
    if (nt >= 0) {
      for (int i = 0; i < nt; ++i) {
        const PpTerm& t = ru->term[s][i];
        if (t.fast) {   // same result as sg_cmp on the two values, without building SgVals
          int64_t a, b;
          int na, nb;
          operand_bits(t.l, a, na);
          operand_bits(t.r, b, nb);
          if (na || nb) {
            if (t.op != 1) return false;
            continue;
          }
          bool ok;
          if (t.fast == 1) ok = pp_cmp_i(t.op, a, b);
          else ok = pp_cmp_f(t.op, pp_f32(a), pp_f32(b));
          if (!ok) return false;
          continue;
        }
        if (!sg_cmp(t.op, t.dom, operand(t.l), operand(t.r))) return false;
      }
      return true;
    }
    Reader rd{this};
    return sg_eval(d->code + st(s).prog_off, st(s).prog_len, rd);
  }

  // ---- posts
  SG_HD void stream_post(int s) {
    f_changed |= bit(s);
    pts_pos = kind_of(s) == SG_K_COUNT ? (A->clen[s] ? A->chain[ru->coff[s]] : -1) : A->slot[s];
    pts = slot_ts(s);
    if (sel_of(s)) f_returned |= bit(s);
    if (next_of(s) >= 0) add_state(next_of(s));
  }
  SG_HD void count_post(int s) {
    const sg_state_desc& x = st(s);
    const int n = A->clen[s];
    f_success |= bit(s);
    pts_pos = A->chain[ru->coff[s] + n - 1];
    pts = src.ts(pts_pos);
    if (n >= x.min_count) {
      if (n == x.min_count && next_of(s) >= 0) add_state(next_of(s));   // count_min_reached (no selector)
      if (n == x.max_count) f_changed |= bit(s);
    }
  }
  SG_HD void logical_post(int s) {
    if (ltype_of(s) == 0) {
      if (A->slot[partner_of(s)] >= 0) stream_post(s);
      else f_changed |= bit(s);
    } else {
      stream_post(s);
    }
  }
  SG_HD void add_state(int s) {
    if (nh < PP_MAX_HIST) A->hist[nh++] = pp_tkey(cur_row, cur_rank);
    else overflow = 1;
    l1 |= bit(s);
    if (kind_of(s) == SG_K_LOGICAL) l1 |= bit(partner_of(s));
  }
  SG_HD bool is_expired(int64_t t) {
    int64_t dt = e1_ts - t;
    if (dt < 0) dt = -dt;
    return dt > d->within;
  }

  // ---- one row: updateState of every state, then the states in visit order (KeyMachine::receive)
  // Returns the visit slot that emitted (one emission per row at most: the partial leaves the emitting state), or -1.
  // visit k of the row: state s (returns false when the partial overflowed its arrays)
  SG_HD bool visit(int k, int s, int64_t t, int& emitted) {
    if (!(l0 & bit(s)) || s == start_of()) return true;
    cur_rank = k;
    bool remove = false;
    if (kind_of(s) == SG_K_COUNT) {
      if ((s + 1 < nstates() && get_any(s + 1)) || (s + 2 < nstates() && get_any(s + 2))) {
        l0 &= ~bit(s);
        return true;
      }
      if (A->clen[s] >= st(s).max_count) { overflow = 1; return false; }
      A->chain[ru->coff[s] + A->clen[s]++] = (int32_t)cur_row;
      f_success &= ~bit(s);
      f_changed &= ~bit(s);
      if (filter(s)) count_post(s);
      if (f_changed & bit(s)) remove = true;
      if (!(f_success & bit(s))) --A->clen[s];
    } else {
      if (is_expired(t)) { l0 &= ~bit(s); return true; }
      if (kind_of(s) == SG_K_LOGICAL && ltype_of(s) == 1 && A->slot[partner_of(s)] >= 0) { l0 &= ~bit(s); return true; }
      A->slot[s] = cur_row;
      f_changed &= ~bit(s);
      if (filter(s)) {
        if (kind_of(s) == SG_K_LOGICAL) logical_post(s);
        else stream_post(s);
      }
      if (f_returned & bit(s)) {
        f_returned &= ~bit(s);
        if (emitted < 0) emitted = k;
        else overflow = 1;
      }
      if (f_changed & bit(s)) remove = true;
      else A->slot[s] = -1;
    }
    if (remove) l0 &= ~bit(s);
    return true;
  }
  SG_HD int step(int32_t row) {
    cur_row = row;
    const uint32_t moved = l1;
    l0 |= moved;
    l1 = 0;
    const int64_t t = src.ts(row);
    int emitted = -1;
    if constexpr (SH::known) {
#pragma unroll
      for (int k = 0; k < SH::n; ++k)
        if (!visit(k, SH::pres[SH::n - 1 - k], t, emitted)) return -1;
    } else {
      const sg_receiver_desc& rv = d->receivers[ru->recv];
      for (int k = 0; k < rv.n; ++k)
        if (!visit(k, rv.pres[rv.n - 1 - k], t, emitted)) return -1;
    }
    return emitted;
  }
  SG_HD bool get_any(int s) { return kind_of(s) == SG_K_COUNT ? A->clen[s] > 0 : A->slot[s] >= 0; }
  SG_HD bool dead() const { return (l0 | l1) == 0; }
  // A count state still short of its minimum holds the partial: counts never expire by `within`
  // (CountPreStateProcessor.processAndReturn, C/query/input/stream/state/CountPreStateProcessor.java:53-93), so a later
  // row -- with time going back, one inside `within` of e1 -- can still complete it.  Every other live state is dropped
  // by the first row of the stream more than `within` from e1 (isExpired compares |e1.ts - ts|, :102-113), and a count
  // state past its minimum can no longer forward the partial.
  SG_HD bool waiting_count() const {
    const uint32_t live = l0 | l1;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (s < nstates() && ((live >> s) & 1u) && kind_of(s) == SG_K_COUNT && A->clen[s] < st(s).min_count) return true;
    return false;
  }
  SG_HD bool live_other() const {   // a live state that is not a count state
    const uint32_t live = l0 | l1;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (s < nstates() && ((live >> s) & 1u) && kind_of(s) != SG_K_COUNT) return true;
    return false;
  }
  // rows the partial holds (e1, every bound slot, every chain event): replaying a superset of them in arrival order,
  // within the rows that followed e1, rebuilds it exactly -- a row that changed it is among them, and any other row
  // changed nothing the first time (the same state meets the same row again)
  template <class F>
  SG_HD void witnesses(F mark) const {
    for (int s = 0; s < NS && s < nstates(); ++s) {
      if (kind_of(s) == SG_K_COUNT) {
        const int32_t* c = A->chain + ru->coff[s];
        for (int i = 0; i < A->clen[s]; ++i) mark(c[i], false);
      } else if (A->slot[s] >= 0) {
        mark(A->slot[s], s == start_of());
      }
    }
  }

  // Wait skipping.  While the partial's only live state s is a stream, count or logical state with a wait term
  // (PpWait), an arriving row that fails the term changes nothing: step() binds the row (slot or chain append), the
  // filter fails, and the binding is undone -- no post, no add_state, no emission; the flags it clears are rewritten
  // before they are next read.  The one other effect, expiry, the caller checks on the row it lands on when the key's
  // timestamps never decrease (a skipped row that had expired the partial means the landing row has too); in a count
  // state (wait_count) there is no expiry, and a key whose time goes back skips only there.  Not while the count state's successors hold the partial (step() would drop it from s) or a full chain, nor
  // for an `or` state whose partner has matched, nor while the fixed operand is null.  Returns whether the partial
  // waits, with the term `row.slot OP c`.
  SG_HD bool wait_on(int& slot, int& op, int& fast, int64_t& cbits) {
    if (l1 != 0 || l0 == 0 || (l0 & (l0 - 1u)) != 0) return false;
    int s = 0;
    while (!((l0 >> s) & 1u)) ++s;
    if (s == start_of() || !ru->wait[s].ok) return false;
    const int kd = kind_of(s);
    if (kd == SG_K_COUNT) {
      if ((s + 1 < nstates() && get_any(s + 1)) || (s + 2 < nstates() && get_any(s + 2))) return false;
      if (A->clen[s] >= st(s).max_count) return false;
    } else if (kd == SG_K_LOGICAL && ltype_of(s) == 1 && A->slot[partner_of(s)] >= 0) {
      return false;
    }
    const PpWait& w = ru->wait[s];
    const PpTerm& t = ru->term[s][0];
    int null = 0;
    operand_bits(w.other ? t.l : t.r, cbits, null);
    if (null) return false;
    wait_count = kd == SG_K_COUNT;
    slot = w.slot;
    op = w.op;
    fast = w.fast;
    return true;
  }

  // tie words of an emission (bit 63: partial lane)
  SG_HD void tie(uint64_t& hi, uint64_t& lo) const {
    uint32_t c[PP_MAX_HIST] = {0, 0, 0, 0};
    for (int i = 0; i < nh; ++i) c[i] = A->hist[nh - 1 - i] & 0x7FFFFFFFu;
    hi = (1ull << 63) | ((uint64_t)c[0] << 31) | c[1];
    lo = ((uint64_t)c[2] << 31) | c[3];
  }
};
