// seq.h -- compact per-key sequence machine (SG route "sequence lanes") for MI355X.
//
// A SEQUENCE keeps almost nothing alive: every event first resets the pending lists and moves the newAndEvery lists
// in (StateStreamRuntime.resetAndUpdate, C/query/input/stream/state/StateStreamRuntime.java:96-99), and addState admits
// one partial per newAndEvery list (StreamPreStateProcessor.addState :203-216, CountPreStateProcessor.addState :109-132,
// LogicalPreStateProcessor.addState :62-83).  So a key's runtime is a handful of partials, and for sequences whose
// start state re-arms with `every` it stays small: each live partial references only events among the key's last H
// rows (H = sum of the states' max counts) -- which partials are live, though, depends on the whole history (below).  This machine is interp.h's KeyMachine restricted to such sequences (stream, count and
// logical states of one stream, `every` only on the start state) with everything sized to that: partials in a pool of
// at most PQ_MAX_P entries with their count chains inline, lists of at most PQ_MAX_L entries, events as row positions
// (the rows stay in HBM, key-ordered) -- a few hundred bytes of LDS per lane instead of a 30 KB HBM arena.
//
// The runtime is NOT a function of a bounded suffix of the key's events: addState admitting one partial per list lets a
// partial's presence decide whether a later one is admitted, and so on without bound (tests/test_partial_lanes.py
// shows it), so a key is run by one lane from its carried state, and the state itself (with the rows its partials
// reference: the key's last H rows) is what is carried between pushes.
//
// Every method restates the KeyMachine method with the same name (interp.h), which cites its reference method; the
// type-1 (SEQUENCE) branches are the ones kept.
#pragma once
#include <stdint.h>

#include "../../include/siddhi_gpu.h"
#include "chain.h"   // PpTerm: conjunctive compare terms evaluated without the VM

#ifndef SG_HD
#define SG_HD __host__ __device__
#endif

#define PQ_MAX_S 6
#define PQ_MAX_P 6        // partials alive at once (pool)
#define PQ_MAX_L 4        // entries per pending / newAndEvery list
#define PQ_MAX_CHAIN 12   // count-chain entries per partial over all count states
#define PQ_MAX_RET 8      // partials one state returns for one event
// Positions are stored as their low 7 bits (-1: none) and decoded against the current row: a live partial's events
// are at most H rows back (a sequence partial advances on every event or dies; an `and` partial waits one event more),
// and H <= PQ_MAX_CHAIN + PQ_MAX_S = 18 < 128.

struct SgSeqRule {
  int32_t ok;
  int32_t start;
  int32_t recv;
  int32_t horizon;                  // H: a partial is at most H events old
  int32_t coff[PQ_MAX_S];           // count state -> offset of its chain inside a partial's chain
  int32_t chain;                    // chain entries per partial
  int32_t pool;                     // partials alive at once (<= PQ_MAX_P)
  uint32_t local_mask;              // states whose filter reads only the arriving event (precomputed bits)
  int32_t nterm[PQ_MAX_S];          // -1: the VM evaluates the state's filter
  PpTerm term[PQ_MAX_S][PP_MAX_TERMS];
};

SG_HD inline SgSeqRule sg_seq_rule(const sg_nfa_desc& d) {
  SgSeqRule r;
  r.ok = 0;
  r.start = -1;
  r.recv = -1;
  r.horizon = 0;
  r.chain = 0;
  r.pool = 0;
  r.local_mask = 0;
  for (int s = 0; s < PQ_MAX_S; ++s) { r.coff[s] = -1; r.nterm[s] = -1; }
  if (d.type != 1 || d.within >= 0 || d.n_states < 2 || d.n_states > PQ_MAX_S || d.n_sched != 0) return r;
  int nrecv = 0;
  for (int s = 0; s < SG_MAX_STREAMS; ++s)
    if (d.recv_of_stream[s] >= 0) { ++nrecv; r.recv = d.recv_of_stream[s]; }
  if (nrecv != 1) return r;
  const sg_receiver_desc& rv = d.receivers[r.recv];
  if (!rv.multi || rv.n != d.n_states) return r;
  int starts = 0, h = 0;
  for (int s = 0; s < d.n_states; ++s) {
    const sg_state_desc& x = d.states[s];
    if (x.kind != SG_K_STREAM && x.kind != SG_K_COUNT && x.kind != SG_K_LOGICAL) return r;
    if (x.callback >= 0 || x.within_every >= 0) return r;
    if (x.local) r.local_mask |= 1u << s;
    else r.nterm[s] = pp_terms(d.code + x.prog_off, x.prog_len, r.term[s]);
    if (x.is_start) {
      ++starts;
      r.start = s;
      if (x.kind != SG_K_STREAM || x.next_every != s) return r;
    } else if (x.next_every >= 0) {
      return r;
    }
    if (x.kind == SG_K_COUNT) {
      if (x.min_count < 1 || x.max_count < x.min_count || x.max_count > 8) return r;
      r.coff[s] = r.chain;
      r.chain += x.max_count;
      h += x.max_count;
    } else {
      h += 1;
    }
    if (x.kind == SG_K_LOGICAL && (x.partner < 0 || d.states[x.partner].kind != SG_K_LOGICAL)) return r;
  }
  if (starts != 1 || r.chain > PQ_MAX_CHAIN) return r;
  // pool bound: one partial per non-start element's newAndEvery list, the start state's every-clone, and the one
  // allocated inside a step before the step's frees (logical partners share their partial: one element)
  int elements = 0;
  for (int s = 0; s < d.n_states; ++s)
    if (!(d.states[s].kind == SG_K_LOGICAL && d.states[s].partner >= 0 && d.states[s].partner < s)) ++elements;
  if (elements + 1 > PQ_MAX_P) return r;
  r.pool = elements + 1;
  r.horizon = h;
  r.ok = 1;
  return r;
}

// State geometry: S states, CH count-chain entries per partial, NP partials in the pool.  A lane's state lives in LDS,
// so its size sets how many lanes a CU holds; queries that fit the small geometry (C3's family: <= 4 states, <= 6 chain
// entries, <= 3 elements) run with 124-byte states instead of 236 (sg_seq_small).
template <int S_, int CH_, int NP_>
struct SqGeo {
  static constexpr int S = S_;
  static constexpr int CH = CH_;
  static constexpr int NP = NP_;
  static constexpr uint32_t all = (1u << NP_) - 1u;
};
using SqBig = SqGeo<PQ_MAX_S, PQ_MAX_CHAIN, PQ_MAX_P>;
using SqSmall = SqGeo<4, 6, 4>;

template <class G>
struct SeqPartialT {
  int8_t slot[G::S];              // stream / logical: row position (low 7 bits) or -1
  int8_t chain[G::CH];            // count chains (positions), inline: no two partials share one in this family
  int8_t clen[G::S];
  int8_t pts;                     // position whose timestamp is the partial's (StateEvent.timestamp), -1: none
};
template <class G>
struct SeqStateT {
  SeqPartialT<G> P[G::NP];
  int8_t list[G::S][2][PQ_MAX_L];
  int8_t llen_[G::S][2];
  uint32_t free_mask;   // pool entries free for allocation in this event
  uint32_t h_init;      // per-state processor flags (KeyMachine H_* words)
  uint32_t created;
  uint32_t fch, fret, fsuc;   // H_CHANGED / H_RETURNED / H_SUCCESS bits between runs (registers while running)
};
using SeqPartial = SeqPartialT<SqBig>;
using SeqState = SeqStateT<SqBig>;

SG_HD inline bool sg_seq_small(const SgSeqRule& r, const sg_nfa_desc& d) {
  return r.ok && d.n_states <= SqSmall::S && r.chain <= SqSmall::CH && r.pool <= SqSmall::NP;
}

// State table of one sequence family known at compile time (kinds, successors, logical pairs, reset / update / init
// orders, visit order): the machine's loops over the states unroll and its kind branches fold, as chain.h's PpShapeC3
// does for the partial lanes.  Counts and filters stay run-time values.  SqShapeAny reads the descriptor.
struct SqShapeAny {
  static constexpr bool known = false;
  static constexpr int n = 0, n_init = 0, n_reset = 0, n_update = 0;
  static constexpr int8_t kind[1] = {0}, next[1] = {0}, nevery[1] = {0}, partner[1] = {0}, ltype[1] = {0},
                          sel[1] = {0}, last[1] = {0}, coff[1] = {0}, init[1] = {0}, reset[1] = {0}, update[1] = {0},
                          pres[1] = {0};
};
// `every e1=S[..], e2=S[..]<m:n>, e3=S[..] or e4=S[..]` (C3b's family: one stream, a count state feeding an `or` pair
// whose members both select), as lowering.py lays it out
struct SqShapeC3b {
  static constexpr bool known = true;
  static constexpr int n = 4, n_init = 4, n_reset = 3, n_update = 3;
  static constexpr int8_t kind[4] = {SG_K_STREAM, SG_K_COUNT, SG_K_LOGICAL, SG_K_LOGICAL};
  static constexpr int8_t next[4] = {1, 3, -1, -1};
  static constexpr int8_t nevery[4] = {0, -1, -1, -1};
  static constexpr int8_t partner[4] = {-1, -1, 3, 2};
  static constexpr int8_t ltype[4] = {0, 0, 1, 1};
  static constexpr int8_t sel[4] = {0, 0, 1, 1};
  static constexpr int8_t last[4] = {2, 1, 2, 3};
  static constexpr int8_t coff[4] = {-1, 0, -1, -1};
  static constexpr int8_t init[4] = {0, 1, 2, 3};
  static constexpr int8_t reset[3] = {2, 1, 0};
  static constexpr int8_t update[3] = {0, 1, 2};
  static constexpr int8_t pres[4] = {0, 1, 2, 3};   // the receiver's processors (visited in reverse)
};
template <class SH>
SG_HD inline bool sg_sq_shape_is(const sg_nfa_desc& d, const SgSeqRule& r) {
  if (!SH::known || !r.ok || d.n_states != SH::n || r.start != 0) return false;
  if (d.n_init != SH::n_init || d.n_reset != SH::n_reset || d.n_update != SH::n_update) return false;
  for (int k = 0; k < SH::n_init; ++k) if (d.init_order[k] != SH::init[k]) return false;
  for (int k = 0; k < SH::n_reset; ++k) if (d.reset_ops[k] != SH::reset[k]) return false;
  for (int k = 0; k < SH::n_update; ++k) if (d.update_ops[k] != SH::update[k]) return false;
  const sg_receiver_desc& rv = d.receivers[r.recv];
  if (rv.n != SH::n) return false;
  for (int s = 0; s < SH::n; ++s) {
    const sg_state_desc& x = d.states[s];
    if (x.kind != SH::kind[s] || (x.is_start != 0) != (s == 0) || x.next_state != SH::next[s] ||
        x.next_every != SH::nevery[s] || x.partner != SH::partner[s] ||
        (x.kind == SG_K_LOGICAL && x.logical_type != SH::ltype[s]) || (x.has_selector != 0) != (SH::sel[s] != 0) ||
        x.this_last != SH::last[s] || (x.kind == SG_K_COUNT && r.coff[s] != SH::coff[s]) || rv.pres[s] != SH::pres[s])
      return false;
  }
  return true;
}

// Src: int64_t ts(int64_t pos); SgVal read(int64_t pos, int ret_slot, int type); int lbit(int s, int64_t pos) (-1: VM)
// Sink: void emit(int group, int64_t pts, ...) receives the machine itself (see SeqMachine::emit)
template <class Src, class G = SqBig, bool FAST = false, class SH = SqShapeAny>   // FAST: see chain.h sg_terms_fast
struct SeqMachine {
  const sg_nfa_desc* d;
  const SgSeqRule* ru;
  Src src;
  SeqStateT<G>* M;
  int64_t cur;            // position of the current row
  int failed;
  uint32_t f_changed, f_returned, f_success;

  SG_HD const sg_state_desc& st(int s) const { return d->states[s]; }
  static constexpr bool KN = SH::known;
  SG_HD int ns() const { if constexpr (KN) return SH::n; else return d->n_states; }
  SG_HD int kind_of(int s) const { if constexpr (KN) return SH::kind[s]; else return st(s).kind; }
  SG_HD bool start_of(int s) const { if constexpr (KN) return s == 0; else return st(s).is_start != 0; }
  SG_HD int next_of(int s) const { if constexpr (KN) return SH::next[s]; else return st(s).next_state; }
  SG_HD int nevery_of(int s) const { if constexpr (KN) return SH::nevery[s]; else return st(s).next_every; }
  SG_HD int partner_of(int s) const { if constexpr (KN) return SH::partner[s]; else return st(s).partner; }
  SG_HD int ltype_of(int s) const { if constexpr (KN) return SH::ltype[s]; else return st(s).logical_type; }
  SG_HD bool sel_of(int s) const { if constexpr (KN) return SH::sel[s] != 0; else return st(s).has_selector != 0; }
  SG_HD int last_of(int s) const { if constexpr (KN) return SH::last[s]; else return st(s).this_last; }
  SG_HD int coff_of(int s) const { if constexpr (KN) return SH::coff[s]; else return ru->coff[s]; }
  SG_HD static uint32_t bit(int s) { return 1u << s; }
  SG_HD void fail(int why = 1) { if (!failed) failed = why; }   // 1 pool, 2 list, 3 returned, 4 chain, 5 output

  SG_HD void begin() {   // a run resumes the state's processor flags
    f_changed = M->fch;
    f_returned = M->fret;
    f_success = M->fsuc;
    failed = 0;
  }
  SG_HD void finish() {
    M->fch = f_changed;
    M->fret = f_returned;
    M->fsuc = f_success;
  }
  SG_HD void reset_runtime() {
    M->created = 0;
    M->h_init = 0;
    for (int s = 0; s < G::S; ++s) { M->llen_[s][0] = 0; M->llen_[s][1] = 0; }
    M->free_mask = G::all;
    f_changed = f_returned = f_success = 0;
    failed = 0;
  }

  // ---- pool
  SG_HD void recompute_free() {   // KeyMachine::gc at a step boundary: roots are the lists
    uint32_t live = 0;
#pragma unroll
    for (int s = 0; s < (KN ? SH::n : G::S); ++s) {
      if (!KN && s >= d->n_states) break;
#pragma unroll
      for (int w = 0; w < 2; ++w)
        for (int i = 0; i < M->llen_[s][w]; ++i) live |= 1u << M->list[s][w][i];
    }
    M->free_mask = ~live & G::all;
  }
  SG_HD int alloc() {
    const uint32_t f = M->free_mask;
    if (!f) { fail(1); return 0; }
    int p = 0;
    while (!((f >> p) & 1u)) ++p;
    M->free_mask &= ~(1u << p);
    return p;
  }
  SG_HD int new_partial() {
    const int p = alloc();
    SeqPartialT<G>& x = M->P[p];
    x.pts = -1;
    for (int s = 0; s < G::S; ++s) { x.slot[s] = -1; x.clen[s] = 0; }
    return p;
  }
  SG_HD int clone_partial(int q) {   // shallow clone; chains are never shared here (sg_seq_rule), so copy them
    const int p = alloc();
    if (failed) return 0;
    M->P[p] = M->P[q];
    return p;
  }

  // ---- lists
  SG_HD int llen(int s, int w) const { return M->llen_[s][w]; }
  SG_HD void ladd(int s, int w, int p) {
    if (M->llen_[s][w] >= PQ_MAX_L) { fail(2); return; }
    M->list[s][w][M->llen_[s][w]++] = (int8_t)p;
  }
  SG_HD void lclear(int s, int w) { M->llen_[s][w] = 0; }

  // ---- events
  SG_HD int64_t get_event(int p, int s, int idx) {
    const SeqPartialT<G>& x = M->P[p];
    if (kind_of(s) != SG_K_COUNT) {
      if (x.slot[s] < 0) return -1;
      return (idx == 0 || idx == -1) ? dec(x.slot[s]) : -1;
    }
    const int n = x.clen[s];
    if (n == 0) return -1;
    int k;
    if (idx >= 0) k = idx;
    else if (idx == -1) k = n - 1;
    else if (idx == -2) k = n - 2;
    else k = n + idx;
    if (k < 0 || k >= n) return -1;
    return dec(x.chain[coff_of(s) + k]);
  }
  SG_HD int8_t enc(int64_t pos) const { return (int8_t)(pos & 0x7F); }
  SG_HD int64_t dec(int x) const { return x < 0 ? -1 : cur - (int64_t)(((uint32_t)(cur & 0x7F) - (uint32_t)x) & 0x7Fu); }
  SG_HD bool has_event(int p, int s) {
    const SeqPartialT<G>& x = M->P[p];
    return kind_of(s) == SG_K_COUNT ? x.clen[s] > 0 : x.slot[s] >= 0;
  }
  SG_HD int slot_pos(int p, int s) {
    const SeqPartialT<G>& x = M->P[p];
    return kind_of(s) == SG_K_COUNT ? x.chain[coff_of(s)] : x.slot[s];
  }
  struct Reader {
    SeqMachine* m;
    int p;
    SG_HD SgVal read(int s, int idx, int slotk, int type) {
      const int64_t r = m->get_event(p, s, idx);
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
  SG_HD void operand_bits(int p, const PpOperand& o, int64_t& bits, int& null) {
    if (o.kind == SG_OP_CONST) {
      bits = o.bits;
      null = 0;
      return;
    }
    const int64_t r = get_event(p, o.state, o.idx);
    if (r < 0) { bits = 0; null = 1; return; }
    src.read_bits(r, o.slot, o.type, bits, null);
  }
  SG_HD bool filter(int s, int p) {
    if ((ru->local_mask >> s) & 1u) {
      const int b = src.lbit(s, cur);
      if (b >= 0) return b != 0;
    }
    const int nt = ru->nterm[s];
    if (FAST) {
      for (int i = 0; i < nt; ++i) {
        const PpTerm& t = ru->term[s][i];
        int64_t a, b;
        int na, nb;
        operand_bits(p, t.l, a, na);
        operand_bits(p, t.r, b, nb);
        if (na || nb) {
          if (t.op != 1) return false;
          continue;
        }
        if (!(t.fast == 1 ? pp_cmp_i(t.op, a, b) : pp_cmp_f(t.op, pp_f32(a), pp_f32(b)))) return false;
      }
      return true;
    }
    Reader rd{this, p};
    if (nt >= 0) {
      for (int i = 0; i < nt; ++i) {
        const PpTerm& t = ru->term[s][i];
        if (t.fast) {   // same result as sg_cmp on the two values, without building SgVals
          int64_t a, b;
          int na, nb;
          operand_bits(p, t.l, a, na);
          operand_bits(p, t.r, b, nb);
          if (na || nb) {
            if (t.op != 1) return false;
            continue;
          }
          if (!(t.fast == 1 ? pp_cmp_i(t.op, a, b) : pp_cmp_f(t.op, pp_f32(a), pp_f32(b)))) return false;
          continue;
        }
        const SgVal l = t.l.kind == SG_OP_CONST ? sg_val_from_bits(t.l.bits, t.l.type, 0) : rd.read(t.l.state, t.l.idx, t.l.slot, t.l.type);
        const SgVal r = t.r.kind == SG_OP_CONST ? sg_val_from_bits(t.r.bits, t.r.type, 0) : rd.read(t.r.state, t.r.idx, t.r.slot, t.r.type);
        if (!sg_cmp(t.op, t.dom, l, r)) return false;
      }
      return true;
    }
    return sg_eval(d->code + st(s).prog_off, st(s).prog_len, rd);
  }

  // ---- posts (sequence branches)
  SG_HD void stream_post(int s, int p) {
    f_changed |= bit(s);
    M->P[p].pts = (int8_t)slot_pos(p, s);
    if (sel_of(s)) f_returned |= bit(s);
    if (next_of(s) >= 0) add_state(next_of(s), p);
    if (nevery_of(s) >= 0) add_every_state(nevery_of(s), p);
  }
  SG_HD void count_post(int s, int p) {
    const sg_state_desc& x = st(s);
    SeqPartialT<G>& y = M->P[p];
    const int n = y.clen[s];
    f_success |= bit(s);
    y.pts = y.chain[coff_of(s) + n - 1];
    if (n >= x.min_count) {
      if (next_of(s) >= 0) add_state(next_of(s), p);
      if (n != x.max_count) add_state(s, p);
      if (n == x.max_count) f_changed |= bit(s);
    }
  }
  SG_HD void logical_post(int s, int p) {
    const int q = partner_of(s);
    if (ltype_of(s) == 0) {
      if (M->P[p].slot[q] >= 0) stream_post(s, p);
      else f_changed |= bit(s);
    } else {
      stream_post(s, p);
      if (sel_of(q) && last_of(s) == q) f_returned |= bit(q);
    }
  }
  SG_HD void add_state(int s, int p) {
    if (kind_of(s) == SG_K_LOGICAL) {
      if (llen(s, 1) == 0) ladd(s, 1, p);
      if (llen(partner_of(s), 1) == 0) ladd(partner_of(s), 1, p);
      return;
    }
    if (llen(s, 1) == 0) ladd(s, 1, p);
  }
  SG_HD void add_every_state(int s, int p) {   // start state only (sg_seq_rule): a stream state
    const int c = clone_partial(p);
    if (failed) return;
    ladd(s, 1, c);
  }
  SG_HD void init_state(int s) {
    if (start_of(s) && (!((M->h_init >> s) & 1u) || nevery_of(s) >= 0)) {
      const int p = new_partial();
      if (failed) return;
      add_state(s, p);
      M->h_init |= bit(s);
    }
  }
  SG_HD void move_nae(int s) {
    for (int i = 0; i < M->llen_[s][1]; ++i) ladd(s, 0, M->list[s][1][i]);
    M->llen_[s][1] = 0;
  }
  SG_HD void update_state(int s) {
    move_nae(s);
    if (kind_of(s) == SG_K_LOGICAL) move_nae(partner_of(s));
  }
  SG_HD void reset_state(int s) {
    if (kind_of(s) == SG_K_LOGICAL) {
      const int q = partner_of(s);
      if (ltype_of(s) == 1 || llen(s, 0) == llen(q, 0)) {
        lclear(s, 0);
        lclear(q, 0);
        if (start_of(s) && llen(s, 1) == 0) init_state(s);
      }
      return;
    }
    lclear(s, 0);
    if (start_of(s) && llen(s, 1) == 0) init_state(s);
  }
  SG_HD void create_runtime() {
    M->created = 1;
    if constexpr (KN) {
#pragma unroll
      for (int k = 0; k < SH::n_init; ++k) if (!failed) init_state(SH::init[k]);
    } else {
      for (int k = 0; k < d->n_init && !failed; ++k) init_state(d->init_order[k]);
    }
  }

  // ---- processAndReturn (sequence); returned partials appended to ret
  SG_HD int process_and_return(int s, int* ret) {
    const int kind = kind_of(s);
    int nret = 0;
    const int n = llen(s, 0);
    int w = 0;
    const int last = last_of(s);
    for (int r = 0; r < n && !failed; ++r) {
      const int p = M->list[s][0][r];
      SeqPartialT<G>& y = M->P[p];
      bool remove = false;
      if (kind == SG_K_COUNT) {
        if ((s + 1 < ns() && has_event(p, s + 1)) || (s + 2 < ns() && has_event(p, s + 2))) continue;
        if (y.clen[s] >= st(s).max_count) { fail(4); break; }
        y.chain[coff_of(s) + y.clen[s]++] = enc(cur);
        f_success &= ~bit(s);
        f_changed &= ~bit(s);
        if (filter(s, p)) count_post(s, p);
        if ((f_returned >> last) & 1u) {
          f_returned &= ~bit(last);
          if (nret < PQ_MAX_RET) ret[nret++] = p; else fail(3);
        }
        if ((f_changed >> s) & 1u) remove = true;
        if (!((f_success >> s) & 1u)) {
          --y.clen[s];
          remove = true;
        }
      } else {
        if (kind == SG_K_LOGICAL && ltype_of(s) == 1 && y.slot[partner_of(s)] >= 0) continue;
        y.slot[s] = enc(cur);
        f_changed &= ~bit(s);
        if (filter(s, p)) {
          if (kind == SG_K_LOGICAL) logical_post(s, p);
          else stream_post(s, p);
        }
        if ((f_returned >> last) & 1u) {
          f_returned &= ~bit(last);
          if (nret < PQ_MAX_RET) ret[nret++] = p; else fail(3);
        }
        if ((f_changed >> s) & 1u) remove = true;
        else {
          y.slot[s] = -1;
          remove = true;
        }
      }
      if (!remove) M->list[s][0][w++] = (int8_t)p;
    }
    M->llen_[s][0] = (int8_t)w;
    return nret;
  }

  // Re-express the state's positions for the next push, where the row at position `from` becomes position 0 (the carried
  // rows are the key's rows from `from` on); `last` is the position of the key's last row.
  SG_HD void rebase(int64_t last, int64_t from) {
    cur = last;
    for (int p = 0; p < G::NP; ++p) {
      SeqPartialT<G>& x = M->P[p];
      for (int s = 0; s < G::S; ++s)
        if (x.slot[s] >= 0) x.slot[s] = enc(dec(x.slot[s]) - from);
      for (int c = 0; c < G::CH; ++c) x.chain[c] = enc(dec(x.chain[c]) - from);
      if (x.pts >= 0) x.pts = enc(dec(x.pts) - from);
    }
  }

  // ---- one row (KeyMachine::receive, multi receiver, sequence); emit(p, group) for every returned partial
  template <class Emit>
  SG_HD void receive(int64_t pos, Emit& emit) {
    cur = pos;
    recompute_free();
    if (!M->created) create_runtime();
    const sg_receiver_desc& rv = d->receivers[ru->recv];
    int ret[PQ_MAX_RET];
    if constexpr (KN) {
#pragma unroll
      for (int k = 0; k < SH::n_reset; ++k) if (!failed) reset_state(SH::reset[k]);
#pragma unroll
      for (int k = 0; k < SH::n_update; ++k) if (!failed) update_state(SH::update[k]);
      const bool selector = rv.selector != 0;
#pragma unroll
      for (int k = 0; k < SH::n; ++k) {
        if (failed) break;
        const int nr = process_and_return(SH::pres[SH::n - 1 - k], ret);
        if (selector)
          for (int i = 0; i < nr; ++i) emit(*this, ret[i], k);
      }
    } else {
      for (int k = 0; k < d->n_reset && !failed; ++k) reset_state(d->reset_ops[k]);
      for (int k = 0; k < d->n_update && !failed; ++k) update_state(d->update_ops[k]);
      for (int k = 0; k < rv.n && !failed; ++k) {
        const int s = rv.pres[rv.n - 1 - k];
        const int nr = process_and_return(s, ret);
        if (rv.selector)
          for (int i = 0; i < nr; ++i) emit(*this, ret[i], k);
      }
    }
  }
};

// Two machine states are the same runtime when their lists hold equal partials in equal order with the same sharing
// (pool slots may differ) and the same pending H_RETURNED bits.  Positions are compared encoded (absolute & 0x7F:
// both states are at the same row, and a live position is within H < 128 rows of it).
// Not compared, because nothing reads them before writing them: H_CHANGED / H_SUCCESS (cleared before every filter),
// H_INIT (only read for start states without `every`, outside sg_seq_rule).
template <class G>
SG_HD inline bool sg_seq_equiv(const SeqStateT<G>& A, const SeqStateT<G>& B, const sg_nfa_desc& d, const SgSeqRule& ru) {
  if (A.created != B.created || A.fret != B.fret) return false;
  int8_t a2b[G::NP], b2a[G::NP];
  for (int p = 0; p < G::NP; ++p) { a2b[p] = -1; b2a[p] = -1; }
  for (int s = 0; s < d.n_states; ++s)
    for (int w = 0; w < 2; ++w) {
      if (A.llen_[s][w] != B.llen_[s][w]) return false;
      for (int i = 0; i < A.llen_[s][w]; ++i) {
        const int pa = A.list[s][w][i], pb = B.list[s][w][i];
        if (a2b[pa] >= 0 || b2a[pb] >= 0) {
          if (a2b[pa] != pb || b2a[pb] != pa) return false;
          continue;
        }
        a2b[pa] = (int8_t)pb;
        b2a[pb] = (int8_t)pa;
        const SeqPartialT<G>& x = A.P[pa];
        const SeqPartialT<G>& y = B.P[pb];
        if (x.pts != y.pts) return false;
        for (int t = 0; t < d.n_states; ++t) {
          if (d.states[t].kind == SG_K_COUNT) {
            if (x.clen[t] != y.clen[t]) return false;
            for (int c = 0; c < x.clen[t]; ++c)
              if (x.chain[ru.coff[t] + c] != y.chain[ru.coff[t] + c]) return false;
          } else if (x.slot[t] != y.slot[t]) {
            return false;
          }
        }
      }
    }
  return true;
}
