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
// Positions are stored as their low 15 bits (-1: none) and decoded against the current row: a live partial's events
// are at most H rows back (a sequence partial advances on every event or dies).

struct SgSeqRule {
  int32_t ok;
  int32_t start;
  int32_t recv;
  int32_t horizon;                  // H: a partial is at most H events old
  int32_t coff[PQ_MAX_S];           // count state -> offset of its chain inside a partial's chain
  int32_t chain;                    // chain entries per partial
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
  r.horizon = h;
  r.ok = 1;
  return r;
}

// State geometry: S states, CH count-chain entries per partial.  A lane's state lives in LDS, so its size sets how
// many lanes a CU holds; queries that fit the small geometry (C3's family: <= 4 states, <= 6 chain entries) run with
// ~220-byte states instead of ~350 (sg_seq_small).
template <int S_, int CH_>
struct SqGeo {
  static constexpr int S = S_;
  static constexpr int CH = CH_;
};
using SqBig = SqGeo<PQ_MAX_S, PQ_MAX_CHAIN>;
using SqSmall = SqGeo<4, 6>;

template <class G>
struct SeqPartialT {
  int16_t slot[G::S];             // stream / logical: row position or -1
  int16_t chain[G::CH];           // count chains (positions), inline: no two partials share one in this family
  int8_t clen[G::S];
  int16_t pts;                    // position whose timestamp is the partial's (StateEvent.timestamp), -1: none
};
template <class G>
struct SeqStateT {
  SeqPartialT<G> P[PQ_MAX_P];
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
  return r.ok && d.n_states <= SqSmall::S && r.chain <= SqSmall::CH;
}

// Src: int64_t ts(int64_t pos); SgVal read(int64_t pos, int ret_slot, int type); int lbit(int s, int64_t pos) (-1: VM)
// Sink: void emit(int group, int64_t pts, ...) receives the machine itself (see SeqMachine::emit)
template <class Src, class G = SqBig, bool FAST = false>   // FAST: see chain.h sg_terms_fast
struct SeqMachine {
  const sg_nfa_desc* d;
  const SgSeqRule* ru;
  Src src;
  SeqStateT<G>* M;
  int64_t cur;            // position of the current row
  int failed;
  uint32_t f_changed, f_returned, f_success;

  SG_HD const sg_state_desc& st(int s) const { return d->states[s]; }
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
    M->free_mask = (1u << PQ_MAX_P) - 1u;
    f_changed = f_returned = f_success = 0;
    failed = 0;
  }

  // ---- pool
  SG_HD void recompute_free() {   // KeyMachine::gc at a step boundary: roots are the lists
    uint32_t live = 0;
    for (int s = 0; s < d->n_states; ++s)
      for (int w = 0; w < 2; ++w)
        for (int i = 0; i < M->llen_[s][w]; ++i) live |= 1u << M->list[s][w][i];
    M->free_mask = ~live & ((1u << PQ_MAX_P) - 1u);
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
    if (st(s).kind != SG_K_COUNT) {
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
    return dec(x.chain[ru->coff[s] + k]);
  }
  SG_HD int16_t enc(int64_t pos) const { return (int16_t)(pos & 0x7FFF); }
  SG_HD int64_t dec(int x) const { return x < 0 ? -1 : cur - (int64_t)(((uint32_t)(cur & 0x7FFF) - (uint32_t)x) & 0x7FFFu); }
  SG_HD bool has_event(int p, int s) {
    const SeqPartialT<G>& x = M->P[p];
    return st(s).kind == SG_K_COUNT ? x.clen[s] > 0 : x.slot[s] >= 0;
  }
  SG_HD int slot_pos(int p, int s) {
    const SeqPartialT<G>& x = M->P[p];
    return st(s).kind == SG_K_COUNT ? x.chain[ru->coff[s]] : x.slot[s];
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
    const sg_state_desc& x = st(s);
    f_changed |= bit(s);
    M->P[p].pts = (int16_t)slot_pos(p, s);
    if (x.has_selector) f_returned |= bit(s);
    if (x.next_state >= 0) add_state(x.next_state, p);
    if (x.next_every >= 0) add_every_state(x.next_every, p);
  }
  SG_HD void count_post(int s, int p) {
    const sg_state_desc& x = st(s);
    SeqPartialT<G>& y = M->P[p];
    const int n = y.clen[s];
    f_success |= bit(s);
    y.pts = y.chain[ru->coff[s] + n - 1];
    if (n >= x.min_count) {
      if (x.next_state >= 0) add_state(x.next_state, p);
      if (n != x.max_count) add_state(s, p);
      if (n == x.max_count) f_changed |= bit(s);
    }
  }
  SG_HD void logical_post(int s, int p) {
    const sg_state_desc& x = st(s);
    if (x.logical_type == 0) {
      if (M->P[p].slot[x.partner] >= 0) stream_post(s, p);
      else f_changed |= bit(s);
    } else {
      stream_post(s, p);
      if (st(x.partner).has_selector && st(s).this_last == x.partner) f_returned |= bit(x.partner);
    }
  }
  SG_HD void add_state(int s, int p) {
    const sg_state_desc& x = st(s);
    if (x.kind == SG_K_LOGICAL) {
      if (llen(s, 1) == 0) ladd(s, 1, p);
      if (llen(x.partner, 1) == 0) ladd(x.partner, 1, p);
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
    const sg_state_desc& x = st(s);
    if (x.is_start && (!((M->h_init >> s) & 1u) || x.next_every >= 0)) {
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
    if (st(s).kind == SG_K_LOGICAL) move_nae(st(s).partner);
  }
  SG_HD void reset_state(int s) {
    const sg_state_desc& x = st(s);
    if (x.kind == SG_K_LOGICAL) {
      const int q = x.partner;
      if (x.logical_type == 1 || llen(s, 0) == llen(q, 0)) {
        lclear(s, 0);
        lclear(q, 0);
        if (x.is_start && llen(s, 1) == 0) init_state(s);
      }
      return;
    }
    lclear(s, 0);
    if (x.is_start && llen(s, 1) == 0) init_state(s);
  }
  SG_HD void create_runtime() {
    M->created = 1;
    for (int k = 0; k < d->n_init && !failed; ++k) init_state(d->init_order[k]);
  }

  // ---- processAndReturn (sequence); returned partials appended to ret
  SG_HD int process_and_return(int s, int* ret) {
    const sg_state_desc& x = st(s);
    int nret = 0;
    const int n = llen(s, 0);
    int w = 0;
    const int last = x.this_last;
    for (int r = 0; r < n && !failed; ++r) {
      const int p = M->list[s][0][r];
      SeqPartialT<G>& y = M->P[p];
      bool remove = false;
      if (x.kind == SG_K_COUNT) {
        if ((s + 1 < d->n_states && has_event(p, s + 1)) || (s + 2 < d->n_states && has_event(p, s + 2))) continue;
        if (y.clen[s] >= x.max_count) { fail(4); break; }
        y.chain[ru->coff[s] + y.clen[s]++] = enc(cur);
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
        if (x.kind == SG_K_LOGICAL && x.logical_type == 1 && y.slot[x.partner] >= 0) continue;
        y.slot[s] = enc(cur);
        f_changed &= ~bit(s);
        if (filter(s, p)) {
          if (x.kind == SG_K_LOGICAL) logical_post(s, p);
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
    for (int p = 0; p < PQ_MAX_P; ++p) {
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
    for (int k = 0; k < d->n_reset && !failed; ++k) reset_state(d->reset_ops[k]);
    for (int k = 0; k < d->n_update && !failed; ++k) update_state(d->update_ops[k]);
    const sg_receiver_desc& rv = d->receivers[ru->recv];
    int ret[PQ_MAX_RET];
    for (int k = 0; k < rv.n && !failed; ++k) {
      const int s = rv.pres[rv.n - 1 - k];
      const int nr = process_and_return(s, ret);
      if (rv.selector)
        for (int i = 0; i < nr; ++i) emit(*this, ret[i], k);
    }
  }
};

// Two machine states are the same runtime when their lists hold equal partials in equal order with the same sharing
// (pool slots may differ) and the same pending H_RETURNED bits.  Positions are compared encoded (absolute & 0x7FFF).
// Not compared, because nothing reads them before writing them: H_CHANGED / H_SUCCESS (cleared before every filter),
// H_INIT (only read for start states without `every`, outside sg_seq_rule).
template <class G>
SG_HD inline bool sg_seq_equiv(const SeqStateT<G>& A, const SeqStateT<G>& B, const sg_nfa_desc& d, const SgSeqRule& ru) {
  if (A.created != B.created || A.fret != B.fret) return false;
  int8_t a2b[PQ_MAX_P], b2a[PQ_MAX_P];
  for (int p = 0; p < PQ_MAX_P; ++p) { a2b[p] = -1; b2a[p] = -1; }
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
