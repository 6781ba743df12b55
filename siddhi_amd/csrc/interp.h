// General per-key NFA machine for the MI355X state engine (SG_SHAPE_GENERAL).
//
// One partition key's cloned runtime (PartitionRuntime.clonePartition, C/partition/PartitionRuntime.java:
// 261-308) lives in a fixed-size HBM arena; one GPU thread advances it over that key's rows in arrival
// order.  Partial matches (StateEvent), retained event copies (StreamEvent data) and count-chain nodes
// live in per-key pools addressed by int32 indices, so the reference's aliasing rules carry over exactly:
//   * the same partial index sits in several per-state lists (next.addState passes the object itself,
//     StreamPostStateProcessor.java:53-72; logical partners share it, LogicalPreStateProcessor.java:62-83);
//   * addEveryState makes a shallow clone: slot values (event / chain-head indices) are copied, chains
//     stay shared (StateEventCloner.java:48-60), so a later append through one partial is visible through
//     the other (StateEvent.addEvent/removeLastEvent, StateEvent.java:212-236).
// Unreferenced pool entries are reclaimed by mark-and-sweep at step boundaries (roots: every list).
//
// Every method below restates one reference method; the citations name it.  The code is written as
// __host__ __device__ so tests/host_interp can run the identical logic on the CPU against the oracle.
#pragma once
#include <stdint.h>

#include "../../include/siddhi_gpu.h"

#ifndef SG_GLOBAL
#define SG_GLOBAL   // (sg_device.h: the global address space on the GPU, nothing on the host)
#endif

#ifndef SG_HD
#define SG_HD __host__ __device__
#endif

#define SG_NIL (-1)

struct SgGeo {
  int32_t S, R, P, E, C, L, Q, A, nsel;
  int32_t off_lists, off_part, off_ev, off_chain, off_timer;
  int32_t off_scratch;        // 3 lists' worth of step scratch (partials a state returns / emits / re-arms in one step)
  int32_t part_words, ev_words, list_words;
  int64_t key_words;
};

// per-state header words
enum { H_INIT = 0, H_CHANGED, H_RETURNED, H_SUCCESS, H_SRESET, H_ACTIVE, H_LST_LO, H_LST_HI, H_STATE_WORDS };
// key header
enum {
  K_CREATED = 0, K_OVERFLOW, K_POS_LO, K_POS_HI, K_FREE_P, K_FREE_E, K_FREE_C, K_NFREE_P, K_NFREE_E, K_NFREE_C,
  K_DEPTH, K_HDR_FIXED
};

SG_HD inline int32_t sg_hdr_words(int S) { return K_HDR_FIXED + S * H_STATE_WORDS; }

// Emission records (before global ordering): [u64 sortkey][match record of sg_match_records layout:
// u64 trigger; i64 ts; i32 key; u32 group; u32 vnull; u32 pad; i64 vals[n_select]]
SG_HD inline int32_t sg_emit_stride(int nsel) { return 8 + 32 + 8 * nsel; }

struct SgRow {          // one input row as the machine sees it
  int64_t ts;
  uint64_t index;       // global event index
  int32_t stream;
  int32_t nullmask;     // over retained slots
  int64_t vals[SG_MAX_RET];
};

struct SgEmitSink {     // where emissions go (device: atomic bump buffer; host: vector)
  char* buf;
  int64_t cap;
  unsigned long long* count;
  int32_t* overflow;
  int32_t stride;
  int32_t key_bits;     // sortkey = (trigger_local << (key_bits + 1)) | (phase << key_bits) | key
};

struct KeyMachine {
  const sg_nfa_desc* d;
  const SgGeo* g;
  SG_GLOBAL int32_t* a;   // this key's arena (global-address-space pointer: plain global loads, not flat ones)
  int32_t key;
  int clone;            // partition clones never get withinEvery (cloneProperties, StreamPreStateProcessor.java:190-200)
  SgEmitSink sink;
  uint64_t base_index;
  // current step
  uint64_t trigger;
  int64_t trig_local;   // batch row of the trigger (ordering key)
  int phase;
  uint32_t group;
  int64_t now;          // playback clock value (TimestampGeneratorImpl.currentTime)
  int failed;
  int silent;           // replaying a unit's horizon: state only, no emission
  // condition bits of the states whose filter reads only the arriving event (predicate-evaluation pass,
  // pred.h; row = trig_local), or null: evaluate the program here
  const uint64_t* const* lbits = nullptr;

  // ---------------------------------------------------------------- raw accessors
  SG_HD SG_GLOBAL int32_t* hdr() { return a; }
  SG_HD SG_GLOBAL int32_t* sth(int s) { return a + K_HDR_FIXED + s * H_STATE_WORDS; }
  SG_HD SG_GLOBAL int32_t* list(int s, int which) { return a + g->off_lists + (s * 2 + which) * (g->L + 1); }
  SG_HD SG_GLOBAL int32_t* part(int p) { return a + g->off_part + p * g->part_words; }
  SG_HD SG_GLOBAL int32_t* ev(int e) { return a + g->off_ev + e * g->ev_words; }
  SG_HD SG_GLOBAL int32_t* chain(int c) { return a + g->off_chain + c * 3; }
  SG_HD SG_GLOBAL int32_t* tq(int ai) { return a + g->off_timer + ai * (2 + 2 * g->Q); }
  // step scratch: a state's list can return / emit / re-arm all its partials in one step (the reference collects
  // them in unbounded chunks), so these buffers are list-sized and grow with the lists
  SG_HD SG_GLOBAL int32_t* scratch(int i) { return a + g->off_scratch + i * (g->L + 1); }
  SG_HD static int64_t rd64(const SG_GLOBAL int32_t* p) { return (int64_t)(((uint64_t)(uint32_t)p[1] << 32) | (uint32_t)p[0]); }
  SG_HD static void wr64(SG_GLOBAL int32_t* p, int64_t v) { p[0] = (int32_t)(uint32_t)v; p[1] = (int32_t)(uint32_t)((uint64_t)v >> 32); }
  SG_HD int64_t pts(int p) { return rd64(part(p)); }
  SG_HD void set_pts(int p, int64_t t) { wr64(part(p), t); }
  SG_HD SG_GLOBAL int32_t& slot(int p, int s) { return part(p)[3 + s]; }
  SG_HD int64_t ets(int e) { return rd64(ev(e)); }
  SG_HD const sg_state_desc& st(int s) { return d->states[s]; }

  SG_HD void fail(int code) {
    if (!failed) { failed = code; hdr()[K_OVERFLOW] = code; }
  }

  // ---------------------------------------------------------------- pools
  SG_HD void format() {
    SG_GLOBAL int32_t* h = hdr();
    for (int i = 0; i < (int)g->key_words && i < sg_hdr_words(g->S); ++i) h[i] = 0;
    for (int s = 0; s < g->S; ++s) { list(s, 0)[0] = 0; list(s, 1)[0] = 0; sth(s)[H_ACTIVE] = 1; }
    for (int p = 0; p < g->P; ++p) part(p)[2] = (p + 1 < g->P) ? p + 1 : SG_NIL;
    for (int e = 0; e < g->E; ++e) ev(e)[5] = (e + 1 < g->E) ? e + 1 : SG_NIL;
    for (int c = 0; c < g->C; ++c) chain(c)[2] = (c + 1 < g->C) ? c + 1 : SG_NIL;
    h[K_FREE_P] = g->P ? 0 : SG_NIL;
    h[K_FREE_E] = g->E ? 0 : SG_NIL;
    h[K_FREE_C] = g->C ? 0 : SG_NIL;
    h[K_NFREE_P] = g->P;
    h[K_NFREE_E] = g->E;
    h[K_NFREE_C] = g->C;
    for (int i = 0; i < g->A; ++i) { tq(i)[0] = 0; tq(i)[1] = 0; }
    h[K_CREATED] = 1;
    wr64(h + K_POS_LO, -1);
  }
  SG_HD int alloc_part() {
    SG_GLOBAL int32_t* h = hdr();
    int p = h[K_FREE_P];
    if (p == SG_NIL) { fail(SG_ECAPACITY); return 0; }
    h[K_FREE_P] = part(p)[2];
    h[K_NFREE_P]--;
    part(p)[2] = -2;  // in use
    return p;
  }
  SG_HD int alloc_ev() {
    SG_GLOBAL int32_t* h = hdr();
    int e = h[K_FREE_E];
    if (e == SG_NIL) { fail(SG_ECAPACITY); return 0; }
    h[K_FREE_E] = ev(e)[5];
    h[K_NFREE_E]--;
    ev(e)[5] = -2;
    return e;
  }
  SG_HD int alloc_chain(int e) {
    SG_GLOBAL int32_t* h = hdr();
    int c = h[K_FREE_C];
    if (c == SG_NIL) { fail(SG_ECAPACITY); return 0; }
    h[K_FREE_C] = chain(c)[2];
    h[K_NFREE_C]--;
    chain(c)[0] = e;
    chain(c)[1] = SG_NIL;
    chain(c)[2] = -2;
    return c;
  }
  SG_HD int new_partial() {   // StateEventPool.borrowEvent: all slots empty, ts -1
    int p = alloc_part();
    set_pts(p, -1);
    for (int s = 0; s < g->S; ++s) slot(p, s) = SG_NIL;
    return p;
  }
  SG_HD int clone_partial(int q) {   // StateEventCloner.copyStateEvent (shallow)
    int p = alloc_part();
    set_pts(p, pts(q));
    for (int s = 0; s < g->S; ++s) slot(p, s) = slot(q, s);
    return p;
  }

  // mark-and-sweep: roots are the per-state lists
  SG_HD void mark_chain(int c) {
    while (c != SG_NIL && chain(c)[2] != -3) {
      chain(c)[2] = -3;
      ev(chain(c)[0])[5] = -3;
      c = chain(c)[1];
    }
  }
  SG_HD void gc() {
    for (int p = 0; p < g->P; ++p) if (part(p)[2] == -2 || part(p)[2] == -3) part(p)[2] = -2;
    // clear marks
    for (int e = 0; e < g->E; ++e) if (ev(e)[5] == -3) ev(e)[5] = -2;
    for (int c = 0; c < g->C; ++c) if (chain(c)[2] == -3) chain(c)[2] = -2;
    for (int s = 0; s < g->S; ++s)
      for (int w = 0; w < 2; ++w) {
        SG_GLOBAL int32_t* l = list(s, w);
        for (int i = 0; i < l[0]; ++i) {
          int p = l[1 + i];
          if (part(p)[2] == -3) continue;
          part(p)[2] = -3;
          for (int k = 0; k < g->S; ++k) {
            int v = slot(p, k);
            if (v == SG_NIL) continue;
            if (st(k).kind == SG_K_COUNT) mark_chain(v);
            else ev(v)[5] = -3;
          }
        }
      }
    SG_GLOBAL int32_t* h = hdr();
    h[K_FREE_P] = SG_NIL; h[K_NFREE_P] = 0;
    for (int p = g->P - 1; p >= 0; --p) {
      if (part(p)[2] == -3) { part(p)[2] = -2; continue; }
      part(p)[2] = h[K_FREE_P]; h[K_FREE_P] = p; h[K_NFREE_P]++;
    }
    h[K_FREE_E] = SG_NIL; h[K_NFREE_E] = 0;
    for (int e = g->E - 1; e >= 0; --e) {
      if (ev(e)[5] == -3) { ev(e)[5] = -2; continue; }
      ev(e)[5] = h[K_FREE_E]; h[K_FREE_E] = e; h[K_NFREE_E]++;
    }
    h[K_FREE_C] = SG_NIL; h[K_NFREE_C] = 0;
    for (int c = g->C - 1; c >= 0; --c) {
      if (chain(c)[2] == -3) { chain(c)[2] = -2; continue; }
      chain(c)[2] = h[K_FREE_C]; h[K_FREE_C] = c; h[K_NFREE_C]++;
    }
  }
  SG_HD void maybe_gc() {
    int listed = 0;
    for (int s = 0; s < g->S; ++s) listed += list(s, 0)[0] + list(s, 1)[0];
    SG_GLOBAL int32_t* h = hdr();
    int need_p = 2 * listed + 2 * g->S + 4, need_c = listed + 4, need_e = 4 + (g->A ? listed : 0);
    if (h[K_NFREE_P] < need_p || h[K_NFREE_C] < need_c || h[K_NFREE_E] < need_e) {
      gc();
      if (h[K_NFREE_P] < need_p || h[K_NFREE_C] < need_c || h[K_NFREE_E] < need_e) fail(SG_ECAPACITY);
    }
  }

  // ---------------------------------------------------------------- lists (LinkedList<StateEvent>)
  SG_HD int llen(int s, int w) { return list(s, w)[0]; }
  SG_HD void ladd(int s, int w, int p) {
    SG_GLOBAL int32_t* l = list(s, w);
    if (l[0] >= g->L) { fail(SG_ECAPACITY); return; }
    l[1 + l[0]] = p;
    l[0]++;
  }
  SG_HD void lclear(int s, int w) { list(s, w)[0] = 0; }

  // ---------------------------------------------------------------- event access (StateEvent.getStreamEvent)
  // returns event-pool index or NIL for position (state, index_in_chain)
  SG_HD int get_event(int p, int s, int idx) {
    int v = slot(p, s);
    if (v == SG_NIL) return SG_NIL;
    if (st(s).kind != SG_K_COUNT) return (idx == 0 || idx == -1) ? v : SG_NIL;
    int c = v;
    if (idx >= 0) {
      for (int i = 1; i <= idx; ++i) { c = chain(c)[1]; if (c == SG_NIL) return SG_NIL; }
    } else if (idx == -1) {
      while (chain(c)[1] != SG_NIL) c = chain(c)[1];
    } else if (idx == -2) {
      if (chain(c)[1] == SG_NIL) return SG_NIL;
      while (chain(chain(c)[1])[1] != SG_NIL) c = chain(c)[1];
    } else {
      int n = 0;
      for (int x = c; x != SG_NIL; x = chain(x)[1]) ++n;
      int k = n + idx;
      if (k < 0) return SG_NIL;
      for (int i = 0; i < k; ++i) c = chain(c)[1];
    }
    return chain(c)[0];
  }
  SG_HD int chain_len(int c, int* last) {
    int n = 1;
    while (chain(c)[1] != SG_NIL) { c = chain(c)[1]; ++n; }
    *last = c;
    return n;
  }
  SG_HD void add_event(int p, int s, int e) {   // StateEvent.addEvent
    int c = alloc_chain(e);
    if (slot(p, s) == SG_NIL) { slot(p, s) = c; return; }
    int x = slot(p, s);
    while (chain(x)[1] != SG_NIL) x = chain(x)[1];
    chain(x)[1] = c;
  }
  SG_HD void remove_last_event(int p, int s) {   // StateEvent.removeLastEvent
    int x = slot(p, s);
    if (x == SG_NIL) return;
    while (chain(x)[1] != SG_NIL) {
      if (chain(chain(x)[1])[1] == SG_NIL) { chain(x)[1] = SG_NIL; return; }
      x = chain(x)[1];
    }
    slot(p, s) = SG_NIL;
  }
  SG_HD int64_t slot_ts(int p, int s) {   // timestamp of slot head (getStreamEvent(stateId))
    int v = slot(p, s);
    if (st(s).kind == SG_K_COUNT) v = chain(v)[0];
    return ets(v);
  }

  // ---------------------------------------------------------------- predicates
  struct PReader {
    KeyMachine* m;
    int p;
    SG_HD SgVal read(int s, int idx, int slotk, int type) {
      int e = m->get_event(p, s, idx);
      SgVal v;
      v.type = type;
      v.i = 0;
      v.d = 0;
      if (e == SG_NIL || ((m->ev(e)[4] >> slotk) & 1)) { v.null = 1; return v; }
      int64_t bits = rd64(m->ev(e) + 6 + 2 * slotk);
      return sg_val_from_bits(bits, type, 0);
    }
  };
  SG_HD bool filter(int s, int p) {
    if (lbits && lbits[s]) {   // (pred.h interleaved layout)
      const uint64_t r = (uint64_t)trig_local;
      return ((((const SG_GLOBAL uint64_t*)lbits[s])[(r >> 8) * 4 + (r & 3)] >> ((r >> 2) & 63)) & 1u) != 0;
    }
    PReader rd{this, p};
    return sg_eval(d->code + st(s).prog_off, st(s).prog_len, rd);
  }

  // ---------------------------------------------------------------- emission (QuerySelector)
  SG_HD void emit(int p) {
    if (failed || silent) return;
    unsigned long long o = atomic_bump(sink.count);
    if ((int64_t)o >= sink.cap) { *sink.overflow = 1; return; }
    char* r = sink.buf + (size_t)o * (size_t)sink.stride;
    uint64_t tl = (uint64_t)trig_local;
    uint64_t* h64 = (uint64_t*)r;
    h64[0] = (tl << (sink.key_bits + 1)) | ((uint64_t)(phase & 1) << sink.key_bits) | (uint32_t)key;
    h64[1] = trigger;
    h64[2] = (uint64_t)pts(p);
    uint32_t* h32 = (uint32_t*)(r + 24);
    h32[0] = (uint32_t)key;
    h32[1] = ((uint32_t)phase << 24) | group;
    uint32_t nm = 0;
    int64_t* vals = (int64_t*)(r + 40);
    for (int k = 0; k < d->n_select; ++k) {
      int e = get_event(p, d->sel_state[k], d->sel_index[k]);
      int rs = d->sel_ret[k];
      if (e == SG_NIL || ((ev(e)[4] >> rs) & 1)) { nm |= 1u << k; vals[k] = 0; continue; }
      vals[k] = rd64(ev(e) + 6 + 2 * rs);
    }
    h32[2] = nm;
    h32[3] = 0;
    if (phase == 0) group++;   // every timer emission is its own callback (sendEvent per partial)
  }
  SG_HD static unsigned long long atomic_bump(unsigned long long* c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return atomicAdd(c, 1ull);
#else
    return (*c)++;
#endif
  }

  // ================================================================ Pre/Post processors
  // StreamPostStateProcessor.process :53-72 (and Count/Logical/Absent overrides)
  SG_HD void post_process(int s, int p) {
    const sg_state_desc& x = st(s);
    switch (x.kind) {
      case SG_K_COUNT: count_post(s, p); return;
      case SG_K_LOGICAL: logical_post(s, p); return;
      case SG_K_ABSENT: absent_post(s, p); return;
      case SG_K_ALOGICAL: alogical_post(s, p); return;
      default: stream_post(s, p); return;
    }
  }
  SG_HD void stream_post(int s, int p) {
    const sg_state_desc& x = st(s);
    sth(s)[H_CHANGED] = 1;
    set_pts(p, slot_ts(p, s));
    if (x.has_selector) sth(s)[H_RETURNED] = 1;
    if (x.next_state >= 0) add_state(x.next_state, p);
    if (x.next_every >= 0) add_every_state(x.next_every, p);
    if (x.callback >= 0) count_start_state_reset(x.callback, 0);
  }
  // CountPostStateProcessor.process :45-71
  SG_HD void count_post(int s, int p) {
    const sg_state_desc& x = st(s);
    int last;
    int n = chain_len(slot(p, s), &last);
    sth(s)[H_SUCCESS] = 1;
    set_pts(p, ets(chain(last)[0]));
    if (n >= x.min_count) {
      if (d->type == 1) {
        if (x.next_state >= 0) add_state(x.next_state, p);
        if (n != x.max_count) add_state(s, p);
      } else if (n == x.min_count) {
        count_min_reached(s, p);
      }
      if (n == x.max_count) sth(s)[H_CHANGED] = 1;
    }
  }
  // CountPostStateProcessor.processMinCountReached :73-85
  SG_HD void count_min_reached(int s, int p) {
    const sg_state_desc& x = st(s);
    if (x.has_selector) { sth(s)[H_CHANGED] = 1; sth(s)[H_RETURNED] = 1; }
    if (x.next_state >= 0) add_state(x.next_state, p);
    if (x.next_every >= 0) add_every_state(x.next_every, p);
  }
  // LogicalPostStateProcessor.process :59-87
  SG_HD void logical_post(int s, int p) {
    const sg_state_desc& x = st(s);
    if (x.logical_type == 0) {
      const bool proceed = st(x.partner).kind == SG_K_ALOGICAL ? partner_can_proceed(x.partner, p)
                                                               : slot(p, x.partner) != SG_NIL;
      if (proceed) stream_post(s, p);
      else sth(s)[H_CHANGED] = 1;
    } else {
      stream_post(s, p);
      // partner post wired to the selector and our pre's thisLastProcessor is the partner post
      if (st(x.partner).has_selector && st(s).this_last == x.partner) sth(x.partner)[H_RETURNED] = 1;
    }
  }
  // AbsentStreamPostStateProcessor.process :36-56
  // AbsentLogicalPostStateProcessor.process :37-49 -- no forwarding, only the arrival is recorded
  SG_HD void alogical_post(int s, int p) {
    sth(s)[H_CHANGED] = 1;
    sth(s)[H_RETURNED] = 1;
    wr64(sth(s) + H_LST_LO, slot_ts(p, s));   // updateLastArrivalTime
  }
  SG_HD int64_t last_arrival(int s) { return rd64(sth(s) + H_LST_LO); }
  // AbsentLogicalPreStateProcessor.partnerCanProceed :353-383 (asked by the partner's AND post)
  SG_HD bool partner_can_proceed(int q, int p) {
    const sg_state_desc& x = st(q);
    if (d->type == 1 && x.next_every < 0 && last_arrival(q) > 0) return false;
    if (x.waiting_time == -1) {
      if (x.next_every < 0) return slot(p, q) == SG_NIL;
      if (last_arrival(q) > 0) {
        wr64(sth(q) + H_LST_LO, 0);
        init_state(q);
        return false;
      }
      return true;
    }
    return slot(p, q) != SG_NIL;
  }
  SG_HD void absent_post(int s, int p) {
    const sg_state_desc& x = st(s);
    sth(s)[H_CHANGED] = 1;
    int64_t t = slot_ts(p, s);
    set_pts(p, t);
    sth(s)[H_RETURNED] = 1;
    if (x.is_start && x.next_every == s) add_every_state(s, p);
    absent_update_last_arrival(s, t);
  }

  // ---- addState
  SG_HD void add_state(int s, int p) {
    const sg_state_desc& x = st(s);
    switch (x.kind) {
      case SG_K_ALOGICAL:    // AbsentLogicalPreStateProcessor.addState :83-105
        if (!sth(s)[H_ACTIVE]) return;
        logical_add(s, p);
        if (!x.is_start && x.waiting_time != -1) {
          tq_push(s, pts(p) + x.waiting_time);
          if (st(x.partner).kind == SG_K_ALOGICAL) tq_push(x.partner, pts(p) + st(x.partner).waiting_time);
        }
        return;
      case SG_K_LOGICAL:     // LogicalPreStateProcessor.addState :62-83
        logical_add(s, p);
        return;
      case SG_K_ABSENT: {    // AbsentStreamPreStateProcessor.addState :77-101
        if (!sth(s)[H_ACTIVE]) return;
        if (d->type == 1) { lclear(s, 1); ladd(s, 1, p); }
        else ladd(s, 1, p);
        if (!x.is_start) absent_schedule(s, pts(p) + x.waiting_time);
        return;
      }
      case SG_K_COUNT:       // CountPreStateProcessor.addState :109-132
        if (d->type == 1) { if (llen(s, 1) == 0) ladd(s, 1, p); }
        else ladd(s, 1, p);
        if (x.min_count == 0 && slot(p, s) == SG_NIL) count_min_reached(s, p);
        return;
      default:               // StreamPreStateProcessor.addState :203-216
        if (d->type == 1) { if (llen(s, 1) == 0) ladd(s, 1, p); }
        else ladd(s, 1, p);
        return;
    }
  }
  SG_HD void logical_add(int s, int p) {
    const sg_state_desc& x = st(s);
    int q = x.partner;
    if (x.is_start || d->type == 1) {
      if (llen(s, 1) == 0) ladd(s, 1, p);
      if (llen(q, 1) == 0) ladd(q, 1, p);
    } else {
      ladd(s, 1, p);
      ladd(q, 1, p);
    }
  }
  // ---- addEveryState
  SG_HD void add_every_state(int s, int p) {
    const sg_state_desc& x = st(s);
    int c = clone_partial(p);
    if (failed) return;
    switch (x.kind) {
      case SG_K_ALOGICAL:    // AbsentLogicalPreStateProcessor.addEveryState :107-120
        if (slot(c, s) != SG_NIL) set_pts(c, slot_ts(c, s));   // timestamp of the last arrived event
        slot(c, s) = SG_NIL;
        slot(c, x.partner) = SG_NIL;
        ladd(s, 1, c);
        ladd(x.partner, 1, c);
        return;
      case SG_K_LOGICAL:     // LogicalPreStateProcessor.addEveryState :86-92
        slot(c, s) = SG_NIL;
        ladd(s, 1, c);
        slot(c, x.partner) = SG_NIL;
        ladd(x.partner, 1, c);
        return;
      case SG_K_ABSENT:      // AbsentStreamPreStateProcessor.addEveryState :103-113
        ladd(s, 1, c);
        absent_schedule(s, pts(p) + x.waiting_time);
        return;
      default:               // StreamPreStateProcessor.addEveryState :219-227
        ladd(s, 1, c);
        return;
    }
  }
  // ---- init (StreamPreStateProcessor.init :157-166)
  SG_HD void init_state(int s) {
    const sg_state_desc& x = st(s);
    bool seq_abs = d->type == 1 && x.next_state >= 0 &&
                   (st(x.next_state).kind == SG_K_ABSENT || st(x.next_state).kind == SG_K_ALOGICAL);   // instanceof AbsentPreStateProcessor
    if (x.is_start && (!sth(s)[H_INIT] || x.next_every >= 0 || seq_abs)) {
      int p = new_partial();
      if (failed) return;
      add_state(s, p);
      sth(s)[H_INIT] = 1;
    }
  }
  // ---- updateState (StreamPreStateProcessor.updateState :281-289 / Logical :118-130 / Count :149-156)
  SG_HD void update_state(int s) {
    const sg_state_desc& x = st(s);
    if (x.kind == SG_K_COUNT && sth(s)[H_SRESET]) { sth(s)[H_SRESET] = 0; init_state(s); }
    move_nae(s);
    if (x.kind == SG_K_LOGICAL || x.kind == SG_K_ALOGICAL) move_nae(x.partner);
  }
  SG_HD void move_nae(int s) {
    SG_GLOBAL int32_t* n = list(s, 1);
    for (int i = 0; i < n[0]; ++i) ladd(s, 0, n[1 + i]);
    n[0] = 0;
  }
  // ---- resetState
  SG_HD bool seq_hold(int s) {   // SEQUENCE without every while the next state's pending is non-empty
    const sg_state_desc& x = st(s);
    if (d->type == 1 && x.next_every < 0) {
      if (x.next_state < 0) { fail(SG_EUNSUPPORTED); return true; }   // reference NPE
      if (llen(x.next_state, 0) != 0) return true;
    }
    return false;
  }
  SG_HD void reset_state(int s) {
    const sg_state_desc& x = st(s);
    if (x.kind == SG_K_LOGICAL || x.kind == SG_K_ALOGICAL) {   // LogicalPreStateProcessor.resetState :94-116
      int q = x.partner;
      if (x.logical_type == 1 || llen(s, 0) == llen(q, 0)) {
        lclear(s, 0);
        lclear(q, 0);
        if (x.is_start && llen(s, 1) == 0) {
          if (seq_hold(s)) return;
          init_state(s);
        }
      }
      return;
    }
    if (x.kind == SG_K_ABSENT) {    // AbsentStreamPreStateProcessor.resetState :115-133
      lclear(s, 0);
      if (x.is_start) {
        if (seq_hold(s)) return;
        init_state(s);
      }
      return;
    }
    lclear(s, 0);                   // StreamPreStateProcessor.resetState :262-278
    if (x.is_start && llen(s, 1) == 0) {
      if (seq_hold(s)) return;
      init_state(s);
    }
  }
  // CountPreStateProcessor.startStateReset :142-147
  SG_HD void count_start_state_reset(int s, int depth) {
    if (depth > 64) { fail(SG_EUNSUPPORTED); return; }   // reference StackOverflowError
    sth(s)[H_SRESET] = 1;
    if (st(s).callback >= 0) count_start_state_reset(s, depth + 1);
  }

  // ---- isExpired (StreamPreStateProcessor.isExpired :102-113)
  SG_HD bool is_expired(int s, int p, int64_t t) {
    if (st(s).is_start || d->within == -1) return false;
    for (int k = 0; k < d->n_start; ++k) {
      int id = d->start_ids[k];
      if (slot(p, id) == SG_NIL) continue;
      int64_t dt = slot_ts(p, id) - t;
      if (dt < 0) dt = -dt;
      if (dt > d->within) return true;
    }
    return false;
  }
  SG_HD int within_every(int s) { return clone ? -1 : st(s).within_every; }

  // ---- processAndReturn; returned partials are appended to ret[]
  SG_HD int process_and_return(int s, int e, SG_GLOBAL int32_t* ret, int retcap) {
    const sg_state_desc& x = st(s);
    if (x.kind == SG_K_ABSENT && !sth(s)[H_ACTIVE]) return 0;
    if (x.kind == SG_K_ALOGICAL) { alogical_process(s, e); return 0; }
    int nret = 0;
    SG_GLOBAL int32_t* l = list(s, 0);
    int n = l[0];
    int w = 0;
    int64_t t = ets(e);
    int last = x.this_last;
    for (int r = 0; r < n && !failed; ++r) {
      int p = l[1 + r];
      bool remove = false;
      if (x.kind == SG_K_COUNT) {
        // CountPreStateProcessor.processAndReturn :53-93 (no `within` check)
        if ((s + 1 < g->S && slot(p, s + 1) != SG_NIL) || (s + 2 < g->S && slot(p, s + 2) != SG_NIL)) continue;
        add_event(p, s, e);
        sth(s)[H_SUCCESS] = 0;
        sth(s)[H_CHANGED] = 0;
        if (filter(s, p)) post_process(s, p);
        if (sth(last)[H_RETURNED]) { sth(last)[H_RETURNED] = 0; if (nret < retcap) ret[nret++] = p; else fail(SG_ECAPACITY); }
        if (sth(s)[H_CHANGED]) remove = true;
        if (!sth(s)[H_SUCCESS]) {
          remove_last_event(p, s);
          if (d->type == 1) remove = true;
        }
      } else {
        // StreamPreStateProcessor.processAndReturn :292-337 (Logical :132-176, Absent via super)
        if (is_expired(s, p, t)) {
          int we = within_every(s);
          if (we >= 0) {
            // updateState on this very list while iterating it throws ConcurrentModificationException
            if (we == s || (st(we).kind == SG_K_LOGICAL && st(we).partner == s)) { fail(SG_EUNSUPPORTED); break; }
            add_every_state(we, p);
            update_state(we);
          }
          continue;   // removed
        }
        if (x.kind == SG_K_LOGICAL && x.logical_type == 1 && slot(p, x.partner) != SG_NIL) continue;  // removed
        slot(p, s) = e;
        sth(s)[H_CHANGED] = 0;
        if (filter(s, p)) post_process(s, p);
        if (sth(last)[H_RETURNED]) { sth(last)[H_RETURNED] = 0; if (nret < retcap) ret[nret++] = p; else fail(SG_ECAPACITY); }
        if (sth(s)[H_CHANGED]) remove = true;
        else {
          slot(p, s) = SG_NIL;
          if (d->type == 1) {
            if (x.kind != SG_K_ABSENT) remove = true;   // removeOnNoStateChange (absent: false)
            if (x.kind != SG_K_LOGICAL && x.callback >= 0) count_start_state_reset(x.callback, 0);
          }
        }
      }
      if (!remove) l[1 + w++] = p;
    }
    l[0] = w;
    if (x.kind == SG_K_ABSENT) return 0;   // AbsentStreamPreStateProcessor.processAndReturn: never returns
    return nret;
  }

  // AbsentLogicalPreStateProcessor.processAndReturn :244-305 (an S event on the absent side; returns nothing)
  SG_HD void alogical_process(int s, int e) {
    const sg_state_desc& x = st(s);
    if (!sth(s)[H_ACTIVE]) return;
    SG_GLOBAL int32_t* l = list(s, 0);
    int n = l[0], w = 0;
    const int64_t t = ets(e);
    for (int r = 0; r < n && !failed; ++r) {
      int p = l[1 + r];
      if (is_expired(s, p, t)) {
        int we = within_every(s);
        if (we >= 0) {
          if (we == s || we == x.partner) { fail(SG_EUNSUPPORTED); break; }   // CME in the reference
          add_every_state(we, p);
          update_state(we);
        }
        continue;
      }
      if (x.logical_type == 1 && slot(p, x.partner) != SG_NIL) continue;
      const int cur = slot(p, s);
      slot(p, s) = e;
      sth(s)[H_CHANGED] = 0;
      if (filter(s, p)) post_process(s, p);
      if (x.waiting_time != -1 || (d->type == 1 && x.logical_type == 0 && x.next_every >= 0)) slot(p, s) = cur;
      bool remove = false;
      if (sth(x.this_last)[H_RETURNED]) {   // passed the filter: no longer an absence candidate
        sth(x.this_last)[H_RETURNED] = 0;
        remove = true;
        if (d->type == 1) list_remove_first(x.partner, 0, p);
      }
      if (!sth(s)[H_CHANGED]) {
        slot(p, s) = cur;
        if (d->type == 1) {
          if (remove) { fail(SG_EUNSUPPORTED); break; }   // double iterator.remove() in the reference
          remove = true;
        }
      }
      if (!remove) l[1 + w++] = p;
    }
    if (!failed) l[0] = w;
  }
  SG_HD void list_remove_first(int s, int which, int p) {   // LinkedList.remove(Object)
    SG_GLOBAL int32_t* l = list(s, which);
    for (int i = 0; i < l[0]; ++i)
      if (l[1 + i] == p) {
        for (int j = i + 1; j < l[0]; ++j) l[j] = l[1 + j];
        l[0]--;
        return;
      }
  }
  // a fresh pooled StreamEvent (StreamEventPool.borrowEvent): timestamp -1, every attribute null
  SG_HD int blank_event() {
    int e = alloc_ev();
    if (failed) return 0;
    SG_GLOBAL int32_t* x = ev(e);
    wr64(x, -1);
    wr64(x + 2, 0);
    x[4] = -1;
    for (int k = 0; k < g->R; ++k) wr64(x + 6 + 2 * k, 0);
    return e;
  }
  // AbsentLogicalPreStateProcessor.process(ComplexEventChunk) :122-210 for one TIMER event at currentTime
  SG_HD void alogical_timer(int s, int64_t current) {
    const sg_state_desc& x = st(s);
    if (!sth(s)[H_ACTIVE]) return;
    bool not_processed = true;
    if (current >= last_arrival(s) + x.waiting_time) {
      if (x.is_start && d->type == 1 && llen(s, 1) == 0 && llen(s, 0) == 0) {
        int p = new_partial();
        if (failed) return;
        add_state(s, p);
      } else if (d->type == 1 && llen(s, 1) != 0) {
        reset_state(s);
      }
      update_state(s);
      SG_GLOBAL int32_t* l = list(s, 0);
      int n = l[0], w = 0;
      SG_GLOBAL int32_t* emitted = scratch(1);
      int ne = 0;
      for (int r = 0; r < n && !failed; ++r) {
        int p = l[1 + r];
        if (is_expired(s, p, current)) {
          int we = within_every(s);
          if (we >= 0) {
            if (we == s || we == x.partner) { fail(SG_EUNSUPPORTED); break; }
            add_every_state(we, p);
            update_state(we);
          }
          continue;
        }
        const int own = slot(p, s);
        const bool passed = own == SG_NIL ? current >= pts(p) + x.waiting_time : current >= ets(own) + x.waiting_time;
        if (passed) {
          const bool partner_bound = slot(p, x.partner) != SG_NIL;
          if (x.logical_type == 0 && partner_bound) {              // AND: partner received but did not send out
            if (ne < g->L) emitted[ne++] = p; else fail(SG_ECAPACITY);
          } else if (!partner_bound) {                               // OR: partner not received; AND: let it process
            if (own != SG_NIL) { fail(SG_EUNSUPPORTED); break; }     // (a chained absent slot is not representable)
            slot(p, s) = blank_event();
            if (x.logical_type == 1) { if (ne < g->L) emitted[ne++] = p; else fail(SG_ECAPACITY); }
          }
          continue;   // removed
        }
        l[1 + w++] = p;
      }
      if (failed) return;
      l[0] = w;
      not_processed = ne == 0;
      for (int i = 0; i < ne && !failed; ++i) {   // sendEvent :222-242
        int p = emitted[i];
        if (x.has_selector) emit(p);
        if (x.next_state >= 0) add_state(x.next_state, p);
        if (x.next_every >= 0) add_every_state(x.next_every, p);
        else if (x.is_start) {
          sth(s)[H_ACTIVE] = 0;
          if (x.logical_type == 1 && st(x.partner).kind == SG_K_ALOGICAL) sth(x.partner)[H_ACTIVE] = 0;
        }
        if (x.callback >= 0) count_start_state_reset(x.callback, 0);
      }
      wr64(sth(s) + H_LST_LO, 0);
    }
    if (x.next_every >= 0 || (not_processed && x.is_start)) {   // schedule again :199-209
      const int64_t la = last_arrival(s);
      tq_push(s, (la == 0 ? now : la) + x.waiting_time);
    }
  }

  // ---------------------------------------------------------------- absence timers (Scheduler FIFO)
  SG_HD int absent_index(int s) {   // this state's scheduler (sg_nfa_desc.sched_state: creation order)
    for (int k = 0; k < d->n_sched; ++k) if (d->sched_state[k] == s) return k;
    return 0;
  }
  SG_HD void tq_push(int s, int64_t t) {   // scheduler.notifyAt(t)
    SG_GLOBAL int32_t* q = tq(absent_index(s));
    if (q[1] >= g->Q) { fail(SG_ECAPACITY); return; }
    int pos = (q[0] + q[1]) % g->Q;
    wr64(q + 2 + 2 * pos, t);
    q[1]++;
  }
  SG_HD void absent_schedule(int s, int64_t t) {   // lastScheduledTime = t; scheduler.notifyAt(t)
    wr64(sth(s) + H_LST_LO, t);
    tq_push(s, t);
  }
  SG_HD void absent_update_last_arrival(int s, int64_t ts) { absent_schedule(s, ts + st(s).waiting_time); }
  SG_HD bool tq_empty(int ai) { return tq(ai)[1] == 0; }
  SG_HD int64_t tq_head(int ai) { SG_GLOBAL int32_t* q = tq(ai); return rd64(q + 2 + 2 * q[0]); }
  SG_HD void tq_pop(int ai) { SG_GLOBAL int32_t* q = tq(ai); q[0] = (q[0] + 1) % g->Q; q[1]--; }

  // AbsentStreamPreStateProcessor.process(ComplexEventChunk) :140-210 for one TIMER event at currentTime
  SG_HD void absent_timer(int s, int64_t current) {
    const sg_state_desc& x = st(s);
    if (!sth(s)[H_ACTIVE]) return;
    int64_t lst = rd64(sth(s) + H_LST_LO);
    bool initialize = x.is_start && llen(s, 1) == 0 && llen(s, 0) == 0;
    if (initialize && d->type == 1 && x.next_every < 0 && lst > 0) initialize = false;
    if (initialize) {
      int p = new_partial();
      if (failed) return;
      add_state(s, p);
    } else if (d->type == 1 && llen(s, 1) != 0) {
      reset_state(s);
    }
    move_nae(s);
    SG_GLOBAL int32_t* l = list(s, 0);
    int n = l[0], w = 0;
    SG_GLOBAL int32_t* emitted = scratch(1);
    int ne = 0;
    SG_GLOBAL int32_t* reevery = scratch(2);
    int nre = 0;
    lst = rd64(sth(s) + H_LST_LO);
    int we = within_every(s);
    for (int r = 0; r < n; ++r) {
      int p = l[1 + r];
      if (is_expired(s, p, current)) {
        if (we >= 0 && x.next_every != s) { if (nre < g->L) reevery[nre++] = p; else fail(SG_ECAPACITY); }
        continue;
      }
      int64_t t = pts(p);
      if ((t == -1 && current >= lst) || (t != -1 && current >= t + x.waiting_time)) {
        set_pts(p, current);
        if (ne < g->L) emitted[ne++] = p; else fail(SG_ECAPACITY);
        continue;
      }
      l[1 + w++] = p;
    }
    l[0] = w;
    for (int i = 0; i < nre; ++i) {
      if (x.next_every < 0) { fail(SG_EUNSUPPORTED); break; }
      add_every_state(x.next_every, reevery[i]);
    }
    if (we >= 0) update_state(we);
    bool not_processed = ne == 0;
    for (int i = 0; i < ne; ++i) {   // sendEvent :212-228
      int p = emitted[i];
      if (x.has_selector) emit(p);
      if (x.next_state >= 0) add_state(x.next_state, p);
      if (x.next_every >= 0) add_every_state(x.next_every, p);
      else if (x.is_start) sth(s)[H_ACTIVE] = 0;
      if (x.callback >= 0) count_start_state_reset(x.callback, 0);
    }
    lst = rd64(sth(s) + H_LST_LO);
    if (now > x.waiting_time + current) { lst = now + x.waiting_time; wr64(sth(s) + H_LST_LO, lst); }
    if (not_processed && lst < current) absent_schedule(s, current + x.waiting_time);
  }

  // ---------------------------------------------------------------- runtime-level operations
  SG_HD void create_runtime() {   // QueryRuntime.clone -> init (StreamInnerStateRuntime.init per state)
    format();
    for (int k = 0; k < d->n_init && !failed; ++k) init_state(d->init_order[k]);
    if (!clone) {   // SiddhiAppRuntime.start -> Absent{Stream,Logical}PreStateProcessor.start (not for clones)
      for (int s = 0; s < g->S; ++s) {
        if (st(s).kind == SG_K_ABSENT && st(s).is_start && sth(s)[H_ACTIVE]) absent_schedule(s, now + st(s).waiting_time);
        if (st(s).kind == SG_K_ALOGICAL && st(s).is_start && st(s).waiting_time != -1 && sth(s)[H_ACTIVE])
          tq_push(s, now + st(s).waiting_time);   // :334-345
      }
    }
  }
  SG_HD void reset_and_update() {   // StateStreamRuntime.resetAndUpdate :96-99
    for (int k = 0; k < d->n_reset && !failed; ++k) reset_state(d->reset_ops[k]);
    for (int k = 0; k < d->n_update && !failed; ++k) update_state(d->update_ops[k]);
  }
  // ProcessStreamReceiver family: one input row of this key's runtime (MultiProcessStreamReceiver.receive
  // :271-309 / SingleProcessStreamReceiver.processAndClear :54-81)
  SG_HD void receive(int stream, int e) {
    int ri = d->recv_of_stream[stream];
    if (ri < 0) return;
    const sg_receiver_desc& r = d->receivers[ri];
    phase = 1;
    SG_GLOBAL int32_t* ret = scratch(0);
    const int retcap = g->L;
    if (r.multi) {
      if (d->type == 0) { for (int k = 0; k < r.n; ++k) update_state(r.stab[k]); }
      else reset_and_update();
      for (int k = 0; k < r.n && !failed; ++k) {
        int s = r.pres[r.n - 1 - k];
        int nr = process_and_return(s, e, ret, retcap);
        group = (uint32_t)k;
        if (r.selector) for (int i = 0; i < nr; ++i) emit(ret[i]);
      }
    } else {
      if (d->type == 0) update_state(r.stab[0]);
      else reset_and_update();
      int nr = process_and_return(r.pres[0], e, ret, retcap);
      for (int i = 0; i < nr; ++i) {
        group = 0x800000u | (uint32_t)i;
        if (r.selector) emit(ret[i]);
      }
    }
  }
  // A PATTERN row on a stream whose receiver visits only states with empty lists changes nothing: updateState moves
  // nothing and processAndReturn walks nothing (MultiProcessStreamReceiver.receive :271-309).  Without absence (no
  // timers on the playback clock) such a row is skipped before its event is even copied -- e.g. the Stream1 rows after
  // a non-`every` e1 of PatternPartitionTestCase's shape has bound.
  SG_HD bool lists_empty(int s) {
    if (list(s, 0)[0] || list(s, 1)[0]) return false;
    const sg_state_desc& x = st(s);
    return !(x.kind == SG_K_LOGICAL && x.partner >= 0 && (list(x.partner, 0)[0] || list(x.partner, 1)[0]));
  }
  SG_HD bool stream_idle(int stream) {
    const int ri = d->recv_of_stream[stream];
    if (ri < 0) return true;
    const sg_receiver_desc& r = d->receivers[ri];
    for (int k = 0; k < r.n; ++k)
      if (!lists_empty(r.stab[k]) || !lists_empty(r.pres[k])) return false;
    return true;
  }
  // store one row's retained values in the event pool
  SG_HD int copy_row(const SgRow& row) {
    int e = alloc_ev();
    if (failed) return 0;
    SG_GLOBAL int32_t* x = ev(e);
    wr64(x, row.ts);
    wr64(x + 2, (int64_t)row.index);
    x[4] = row.nullmask;
    for (int k = 0; k < g->R; ++k) wr64(x + 6 + 2 * k, row.vals[k]);
    return e;
  }
  // A PATTERN without `every` and without absence never gets a new partial once its first one has left the start
  // state (StreamPreStateProcessor.init arms a start state only once unless an every re-arms it, :157-166): when every
  // list is empty the runtime has ended, and the key's remaining rows change nothing.
  SG_HD bool can_end() {
    if (d->type != 0 || d->n_sched != 0) return false;
    for (int s = 0; s < g->S; ++s)
      if (st(s).next_every >= 0 || st(s).within_every >= 0 || st(s).kind == SG_K_ABSENT || st(s).kind == SG_K_ALOGICAL)
        return false;
    return true;
  }
  SG_HD bool ended() {
    if (!hdr()[K_CREATED]) return false;
    for (int s = 0; s < g->S; ++s)
      if (list(s, 0)[0] || list(s, 1)[0]) return false;
    return true;
  }
  SG_HD int64_t pos() { return rd64(hdr() + K_POS_LO); }
  SG_HD void set_pos(int64_t v) { wr64(hdr() + K_POS_LO, v); }
};

// ------------------------------------------------------------------------------------------------
// Drive one key over this push: its own rows in arrival order, interleaved with the absence timers
// that fire on the global playback clock.  Timer semantics: InputHandler.send -> setCurrentTimestamp
// (C/stream/input/InputHandler.java:57-65, TimestampGeneratorImpl.java:106-125) notifies every
// Scheduler in registration order before the row is dispatched; a Scheduler fires while its FIFO head
// <= clock (Scheduler.java:74-86,179-214).  The clock is the largest timestamp so far: a row whose time goes
// back leaves it where it is and notifies no scheduler (setCurrentTimestamp returns early), but is still
// processed.  So the first row that fires a head value h after position `pos` is the first row at or after it
// that advances (or repeats) the clock to a value >= h.
//
// Rows interface:  n_own(), own_local(i) (local row index of the i-th own row), fill(local, SgRow&),
//                  ts(local), clock_at(local) (the clock once the row has set it), find_ge(from_local, value) ->
//                  first local row >= from_local that notifies the schedulers with the clock at >= value (or
//                  n_rows), n_rows(), plus has_receiver(stream).
//
// emit_from: own rows before this index only rebuild state (a chunked unit's replay window, see
// interp.hip): their matches are not emitted.
template <class Rows>
SG_HD void sg_run_key(KeyMachine& m, Rows& rows, int create_at_start, int64_t emit_from = 0) {
  const int A = m.g->A;
  const int32_t* abs_state = m.d->sched_state;   // scheduler order
  if (create_at_start && !m.hdr()[K_CREATED]) m.create_runtime();
  int64_t nown = rows.n_own();
  int64_t nrows = rows.n_rows();
  int64_t i = 0;
  const bool can_end = m.can_end();
  const bool skip_idle = m.d->type == 0 && m.d->n_sched == 0 && A == 0;
  while (!m.failed) {
    if (can_end && m.ended()) break;   // (no timers either: nothing left to fire)
    int64_t lev = (i < nown) ? rows.own_local(i) : nrows;
    // earliest timer trigger of this key's schedulers
    int64_t ltim = nrows;
    if (A > 0 && m.hdr()[K_CREATED]) {
      int64_t from = rows.first_after(m.pos());   // first local row with global index > pos
      for (int ai = 0; ai < A; ++ai) {
        if (m.tq_empty(ai)) continue;
        int64_t r = rows.find_ge(from, m.tq_head(ai));
        if (r < ltim) ltim = r;
      }
    }
    m.silent = i < emit_from ? 1 : 0;
    if (ltim < nrows && ltim <= lev) {
      m.now = rows.clock_at(ltim);
      m.trigger = rows.index_of(ltim);
      m.trig_local = ltim;
      m.phase = 0;
      for (int ai = 0; ai < A && !m.failed; ++ai) {
        m.group = (uint32_t)ai << 16;
        while (!m.failed && !m.tq_empty(ai) && m.tq_head(ai) <= m.now) {
          int64_t t = m.tq_head(ai);
          m.tq_pop(ai);
          m.maybe_gc();
          if (m.failed) break;
          if (m.st(abs_state[ai]).kind == SG_K_ALOGICAL) m.alogical_timer(abs_state[ai], t);
          else m.absent_timer(abs_state[ai], t);
        }
      }
      m.set_pos((int64_t)rows.index_of(ltim));
      if (ltim < lev) continue;
    }
    if (i >= nown) break;
    if (skip_idle && m.hdr()[K_CREATED] && m.stream_idle(rows.stream_at(lev))) {   // (stream_idle)
      m.set_pos((int64_t)rows.index_of(lev));
      ++i;
      continue;
    }
    SgRow row;
    rows.fill(lev, row);
    m.now = rows.clock_at(lev);
    m.trigger = row.index;
    m.trig_local = lev;
    if (!m.hdr()[K_CREATED]) m.create_runtime();
    if (m.failed) break;
    m.maybe_gc();
    if (m.failed) break;
    int e = m.copy_row(row);
    if (m.failed) break;
    m.receive(row.stream, e);
    m.set_pos((int64_t)row.index);
    ++i;
  }
}

// ------------------------------------------------------------------------------------------------
// Chunked units.  A key's rows can be cut into units that run in parallel when the state reached before
// a unit's first row is a function of a bounded suffix of the key's history (the "horizon"); each unit
// then starts from a fresh runtime and replays that suffix without emitting:
//   patterns with `within T` whose start states all re-arm themselves with `every` (and no
//   withinEvery re-arm outside partition clones): a partial started more than T before a row is expired
//   at that row (StreamPreStateProcessor.isExpired, C/query/input/stream/state/
//   StreamPreStateProcessor.java:102-113) and can neither advance nor emit again, so the rows with
//   ts >= ts(first) - T rebuild every live partial;
// Absence (timers on the global clock) is never chunked.
struct SgChunkRule {
  int kind;            // 0 none, 1 time horizon, 2 event horizon
  int64_t within;      // kind 1
  int64_t events;      // kind 2
};
SG_HD inline SgChunkRule sg_chunk_rule(const sg_nfa_desc& d) {
  SgChunkRule r{0, 0, 0};
  int starts = 0;
  for (int s = 0; s < d.n_states; ++s) {
    if (d.states[s].kind == SG_K_ABSENT || d.states[s].kind == SG_K_ALOGICAL) return r;
    if (d.states[s].is_start) {
      if (d.states[s].next_every != s) return r;
      ++starts;
    }
  }
  if (!starts) return r;
  if (d.type == 0) {
    if (d.within < 0) return r;
    if (!d.partitioned)
      for (int s = 0; s < d.n_states; ++s) if (d.states[s].within_every >= 0) return r;
    // CountPreStateProcessor.processAndReturn never checks `within` (CountPreStateProcessor.java:53-93): a count
    // state that emits itself, or hands over to another count state, keeps advancing an expired partial
    for (int s = 0; s < d.n_states; ++s) {
      const sg_state_desc& x = d.states[s];
      if (x.kind != SG_K_COUNT) continue;
      if (x.has_selector || (x.next_state >= 0 && d.states[x.next_state].kind == SG_K_COUNT)) return r;
    }
    r.kind = 1;
    r.within = d.within;
    return r;
  }
  // Sequences are never cut: a partial lives at most sum(max counts) events, but addState admits one partial per
  // newAndEvery list (StreamPreStateProcessor.addState :203-216), so whether a partial exists can depend on an older
  // one that occupied the list, and that on an older one still -- the state is not a function of a bounded suffix
  // (tests/test_partial_lanes.py::test_sequence_state_is_not_a_bounded_suffix).
  return r;
}
// First own row a unit starting at own row p0 (> 0) must replay from; ts_at(i) = timestamp of own row i.
template <class TsAt>
SG_HD int64_t sg_replay_start(const SgChunkRule& r, int64_t p0, TsAt ts_at) {
  if (r.kind == 2) return p0 > r.events ? p0 - r.events : 0;
  const int64_t lo_ts = ts_at(p0) - r.within;
  int64_t lo = 0, hi = p0;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (ts_at(mid) < lo_ts) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Arena geometry for a descriptor and pool capacities (words of int32 per key).
inline SgGeo sg_make_geo(const sg_nfa_desc& d, int P, int E, int C, int L, int Q) {
  SgGeo g;
  g.S = d.n_states;
  g.R = d.n_ret;
  g.P = P;
  g.E = E;
  g.C = C;
  g.L = L;
  g.Q = Q;
  g.A = 0;
  g.A = d.n_sched;   // one timer FIFO per absent state (Scheduler)
  g.nsel = d.n_select;
  g.part_words = 3 + g.S;
  g.ev_words = 6 + 2 * g.R;
  g.list_words = 2 * g.S * (L + 1);
  int32_t off = sg_hdr_words(g.S);
  g.off_lists = off;
  off += g.list_words;
  g.off_part = off;
  off += P * g.part_words;
  g.off_ev = off;
  off += E * g.ev_words;
  g.off_chain = off;
  off += C * 3;
  g.off_timer = off;
  off += g.A * (2 + 2 * Q);
  g.off_scratch = off;
  off += 3 * (L + 1);
  off = (off + 3) & ~3;
  g.key_words = off;
  return g;
}
