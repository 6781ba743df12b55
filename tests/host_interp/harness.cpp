// TEST HARNESS ONLY: runs the engine's per-key NFA machine (siddhi_amd/csrc/interp.h, the exact code the
// MI355X kernel executes) on the CPU so its logic can be compared with the oracle without a GPU.
// Not linked into libsiddhi_gpu.so and not reachable from the product path.
#define SG_HOST_ONLY 1
#define SG_HD
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../siddhi_amd/csrc/sg_device.h"
#include "../../siddhi_amd/csrc/interp.h"
#include "../../siddhi_amd/csrc/chain.h"
#include "../../siddhi_amd/csrc/seq.h"

struct HiHandle {
  sg_nfa_desc d;
  SgGeo g;
  std::vector<std::vector<int32_t>> arenas;
  std::vector<std::vector<char>> out;
  int err = 0;
  int chunk_rows = 0;   // >0: cut each key's rows into units replaying their horizon (as interp.hip does)
  // partial lanes (chain.h, as partial.hip runs them): carried rows per push, values as retained-slot bits
  int pp = 0;
  int pp_active = 1;
  struct CRow { int64_t ts; int32_t key; int64_t vals[SG_MAX_RET]; int32_t nullmask; uint8_t start; };
  std::vector<CRow> carried;
  std::vector<SeqState> seq_state;   // sequence lanes: per key (partial.hip's geometry choice: big ...)
  std::vector<SeqStateT<SqSmall>> seq_state_s;   // (... or small, sg_seq_small)
  int64_t spec_rows = 0, spec_warm = 0, spec_reruns = 0;   // speculative units (0: one run per key)
  int64_t pp_steps = 0, pp_lanes = 0, pp_skipped = 0;      // partial lanes: rows stepped, lanes started, rows skipped
  int64_t clock = 0;   // playback clock after the last push (TimestampGeneratorImpl.lastEventTimestamp)
};

struct HostRows {
  const sg_batch* b;
  const sg_nfa_desc* d;
  const std::vector<int64_t>* own;
  uint64_t index_of(int64_t r) { return b->index ? b->index[r] : b->base_index + (uint64_t)r; }
  int64_t first_after(int64_t pos) {
    if (!b->index) { int64_t p = pos - (int64_t)b->base_index + 1; return p < 0 ? 0 : (p > b->n ? b->n : p); }
    return std::upper_bound(b->index, b->index + b->n, (uint64_t)pos, [](uint64_t v, uint64_t x) { return v < x; }) - b->index;
  }
  int64_t n_own() { return (int64_t)own->size(); }
  int64_t own_local(int64_t i) { return (*own)[i]; }
  int stream_at(int64_t r) { return b->stream ? b->stream[r] : 0; }
  int64_t n_rows() { return b->n; }
  int64_t ts(int64_t r) { return b->ts[r]; }
  // playback clock: clk[r] = the clock once row r has set it, nf[r] = first row >= r that notifies the schedulers
  const std::vector<int64_t>* clk;
  const std::vector<int64_t>* nf;
  int64_t clock_at(int64_t r) { return (*clk)[r]; }
  int64_t find_ge(int64_t from, int64_t v) {
    const int64_t lo = std::lower_bound(clk->begin() + from, clk->end(), v) - clk->begin();
    return lo >= b->n ? b->n : (*nf)[lo];
  }
  void fill(int64_t r, SgRow& row) {
    row.ts = b->ts[r];
    row.index = index_of(r);
    row.stream = b->stream ? b->stream[r] : 0;
    row.nullmask = 0;
    for (int k = 0; k < d->n_ret; ++k) {
      int c = d->ret_col[k];
      int t = d->ret_type[k];
      if (b->nulls && b->nulls[c] && b->nulls[c][r]) { row.nullmask |= 1 << k; row.vals[k] = 0; continue; }
      const void* col = b->cols[c];
      int64_t bits;
      switch (t) {
        case SG_T_LONG: bits = ((const int64_t*)col)[r]; break;
        case SG_T_DOUBLE: memcpy(&bits, (const double*)col + r, 8); break;
        case SG_T_FLOAT: { uint32_t u; memcpy(&u, (const float*)col + r, 4); bits = u; break; }
        default: bits = ((const int32_t*)col)[r]; break;
      }
      row.vals[k] = bits;
    }
  }
};

static int64_t read_bits_col(const sg_batch* b, const sg_nfa_desc* d, int k, int64_t r, int* null) {
  int c = d->ret_col[k];
  int t = d->ret_type[k];
  *null = (b->nulls && b->nulls[c] && b->nulls[c][r]) ? 1 : 0;
  if (*null) return 0;
  const void* col = b->cols[c];
  int64_t bits;
  switch (t) {
    case SG_T_LONG: bits = ((const int64_t*)col)[r]; break;
    case SG_T_DOUBLE: memcpy(&bits, (const double*)col + r, 8); break;
    case SG_T_FLOAT: { uint32_t u; memcpy(&u, (const float*)col + r, 4); bits = u; break; }
    default: bits = ((const int32_t*)col)[r]; break;
  }
  return bits;
}

struct HostPpSrc {
  const sg_batch* b;
  const sg_nfa_desc* d;
  const std::vector<HiHandle::CRow>* c;
  int64_t nc;
  int64_t ts(int64_t x) const { return x < nc ? (*c)[x].ts : b->ts[x - nc]; }
  SgVal read(int64_t x, int slotk, int type) const {
    int null = 0;
    int64_t bits;
    if (x < nc) {
      null = ((*c)[x].nullmask >> slotk) & 1;
      bits = (*c)[x].vals[slotk];
    } else {
      bits = read_bits_col(b, d, slotk, x - nc, &null);
    }
    return sg_val_from_bits(bits, type, null);
  }
  int lbit(int, int64_t) const { return -1; }
  void read_bits(int64_t x, int slotk, int type, int64_t& bits, int& null) const {
    if (x < nc) {
      null = ((*c)[x].nullmask >> slotk) & 1;
      bits = (*c)[x].vals[slotk];
    } else {
      bits = read_bits_col(b, d, slotk, x - nc, &null);
    }
    if (type == SG_T_INT) bits = (int64_t)(int32_t)bits;
  }
};

// partial-lane push (partial.hip restated on the host); returns -1 when a lane outgrows its arrays
template <class G, class SH = PpShapeAny>
static int pp_push(HiHandle* h, const sg_batch* b, std::vector<char>& recs, std::vector<uint64_t>& k1,
                   std::vector<uint64_t>& th, std::vector<uint64_t>& tl) {
  const sg_nfa_desc& d = h->d;
  const SgPpRule ru = sg_pp_rule(d);
  const int64_t n = b->n;
  const int64_t nc = (int64_t)h->carried.size();
  int kmax = 0;
  for (auto& r : h->carried) kmax = std::max(kmax, r.key + 1);
  for (int64_t i = 0; i < n; ++i) if (d.partitioned && b->key && b->key[i] >= 0) kmax = std::max(kmax, b->key[i] + 1);
  std::vector<std::vector<int64_t>> own((size_t)std::max(kmax, 1));
  for (int64_t c = 0; c < nc; ++c) own[d.partitioned ? h->carried[c].key : 0].push_back(c);
  for (int64_t i = 0; i < n; ++i) {
    int s = b->stream ? b->stream[i] : 0;
    if (s < 0 || d.recv_of_stream[s] < 0) continue;
    int k = d.partitioned ? (b->key ? b->key[i] : -1) : 0;
    if (k < 0) continue;
    own[k].push_back(nc + i);
  }
  HostPpSrc src{b, &d, &h->carried, nc};
  // keys whose time goes back somewhere in this push, carried rows included (k_pp_segments)
  std::vector<uint8_t> kback(own.size(), 0);
  for (size_t k = 0; k < own.size(); ++k)
    for (size_t p = 1; p < own[k].size(); ++p)
      if (src.ts(own[k][p - 1]) > src.ts(own[k][p])) kback[k] = 1;
  std::vector<uint8_t> keep((size_t)(nc + n), 0), kstart((size_t)(nc + n), 0);
  const int rstride = 32 + 8 * d.n_select;
  for (size_t k = 0; k < own.size(); ++k) {
    const auto& rows = own[k];
    for (size_t p = 0; p < rows.size(); ++p) {
      PpLane<HostPpSrc, G, false, SH> L;   // (SH: the compile-time state table when the query has one, as on the GPU)
      PpArraysT<G> arr;
      L.d = &d;
      L.ru = &ru;
      L.src = src;
      L.A = &arr;
      if (rows[p] < nc && !h->carried[rows[p]].start) continue;   // a carried row starts only its pending partial
      if (!L.start_ok(rows[p])) continue;
      L.start(rows[p]);
      ++h->pp_lanes;
      bool emitted = false, finished = false;
      for (size_t q = p + 1; q < rows.size(); ++q) {
        const int64_t c = rows[q];
        const int64_t dt = src.ts(c) - L.e1_ts;
        if ((dt > d.within || -dt > d.within) && !L.waiting_count()) { finished = true; break; }
        {   // wait skipping (chain.h PpLane::wait_on): here every row the wait term rejects is skipped, the GPU skips
            // whole 8-row blocks that cannot pass it (on a key whose time goes back, only in a count state)
          int ws, wop, wf;
          int64_t wc;
          if (L.wait_on(ws, wop, wf, wc) && (L.wait_count || !kback[k])) {
            int64_t rb;
            int rn;
            src.read_bits(c, ws, wf == 1 ? SG_T_INT : SG_T_FLOAT, rb, rn);
            const bool pass = rn ? wop == 1 : (wf == 1 ? pp_cmp_i(wop, rb, wc) : pp_cmp_f(wop, pp_f32(rb), pp_f32(wc)));
            if (!pass) {
              ++h->pp_skipped;
              continue;
            }
          }
        }
        const int em = L.step(c);
        ++h->pp_steps;
        if (L.overflow) return -1;
        if (em >= 0 && c >= nc) {
          emitted = true;
          const int64_t r = c - nc;
          k1.push_back(((uint64_t)r << 8) | (uint32_t)em);
          uint64_t a, z;
          L.tie(a, z);
          th.push_back(a);
          tl.push_back(z);
          const size_t o = recs.size();
          recs.resize(o + rstride);
          char* rec = recs.data() + o;
          uint64_t trig = b->index ? b->index[r] : b->base_index + (uint64_t)r;
          memcpy(rec, &trig, 8);
          int64_t pts = L.pts;
          memcpy(rec + 8, &pts, 8);
          uint32_t h32[4] = {(uint32_t)k, (1u << 24) | (uint32_t)em, 0, 0};
          for (int s = 0; s < d.n_select; ++s) {
            int64_t v = 0;
            const int64_t ev = L.get_event(d.sel_state[s], d.sel_index[s]);
            if (ev < 0) { h32[2] |= 1u << s; }
            else {
              SgVal x = src.read(ev, d.sel_ret[s], d.ret_type[d.sel_ret[s]]);
              if (x.null) h32[2] |= 1u << s; else v = sg_val_bits(x);
            }
            memcpy(rec + 32 + 8 * s, &v, 8);
          }
          memcpy(rec + 16, h32, 16);
        }
        if (L.dead()) { finished = true; break; }
      }
      // pending after the key's last row: the rows the partial holds are carried, its e1 flagged as a start
      if (!finished && !emitted && !L.dead() && (L.waiting_count() || L.live_other()))
        L.witnesses([&](int64_t c, bool st) {
          keep[(size_t)c] = 1;
          if (st) kstart[(size_t)c] = 1;
        });
    }
  }
  // carry: the marked rows, key by key in arrival order (k_pp_carry)
  std::vector<HiHandle::CRow> next;
  for (size_t k = 0; k < own.size(); ++k) {
    for (int64_t c : own[k]) {
      if (!keep[(size_t)c]) continue;
      HiHandle::CRow cr;
      memset(&cr, 0, sizeof(cr));
      cr.ts = src.ts(c);
      cr.key = (int32_t)k;
      if (c < nc) cr = h->carried[c];
      else {
        for (int j = 0; j < d.n_ret; ++j) {
          int null = 0;
          cr.vals[j] = read_bits_col(b, &d, j, c - nc, &null);
          if (null) cr.nullmask |= 1 << j;
        }
      }
      cr.start = kstart[(size_t)c];
      next.push_back(cr);
    }
  }
  h->carried.swap(next);
  return 1;
}

// sequence-lane push (partial.hip's sequence route restated on the host): one compact machine per key, resumed from the
// key's carried state over its carried rows (the last H) + this push's rows; returns 0 when the machine overflows
struct HostSeqSrc {
  HostPpSrc base_src;
  const std::vector<int64_t>* rows;   // combined ids of this key's rows
  int64_t ts(int64_t pos) const { return base_src.ts((*rows)[pos]); }
  SgVal read(int64_t pos, int slotk, int type) const { return base_src.read((*rows)[pos], slotk, type); }
  int lbit(int, int64_t) const { return -1; }
  void read_bits(int64_t pos, int slotk, int type, int64_t& bits, int& null) const {
    base_src.read_bits((*rows)[pos], slotk, type, bits, null);
  }
};

template <class G, class SH = SqShapeAny>
static int seq_push(HiHandle* h, std::vector<SeqStateT<G>>& states, const sg_batch* b, std::vector<char>& recs,
                    std::vector<uint64_t>& k1) {
  const sg_nfa_desc& d = h->d;
  const SgSeqRule ru = sg_seq_rule(d);
  const int64_t n = b->n;
  const int64_t nc = (int64_t)h->carried.size();
  int kmax = 0;
  for (auto& r : h->carried) kmax = std::max(kmax, r.key + 1);
  for (int64_t i = 0; i < n; ++i) if (d.partitioned && b->key && b->key[i] >= 0) kmax = std::max(kmax, b->key[i] + 1);
  std::vector<std::vector<int64_t>> own((size_t)std::max(kmax, 1));
  for (int64_t c = 0; c < nc; ++c) own[d.partitioned ? h->carried[c].key : 0].push_back(c);
  std::vector<int64_t> ncar(own.size(), 0);
  for (size_t k = 0; k < own.size(); ++k) ncar[k] = (int64_t)own[k].size();
  for (int64_t i = 0; i < n; ++i) {
    int s = b->stream ? b->stream[i] : 0;
    if (s < 0 || d.recv_of_stream[s] < 0) continue;
    int k = d.partitioned ? (b->key ? b->key[i] : -1) : 0;
    if (k < 0) continue;
    own[k].push_back(nc + i);
  }
  if (states.size() < own.size()) states.resize(own.size());
  std::vector<SeqStateT<G>> next_state = states;
  HostPpSrc src{b, &d, &h->carried, nc};
  const int rstride = 32 + 8 * d.n_select;
  const int64_t H = ru.horizon;
  std::vector<HiHandle::CRow> next;
  for (size_t k = 0; k < own.size(); ++k) {
    const auto& rows = own[k];
    const int64_t nk = (int64_t)rows.size();
    if (!nk) continue;
    SeqStateT<G>& st = next_state[k];
    SeqMachine<HostSeqSrc, G, false, SH> m;
    m.d = &d;
    m.ru = &ru;
    m.src = HostSeqSrc{src, &rows};
    m.M = &st;
    m.failed = 0;
    m.f_changed = m.f_returned = m.f_success = 0;
    if (ncar[k] == 0) { memset(&st, 0, sizeof(st)); next_state[k] = st; }   // a key without state starts zeroed
    uint32_t seq = 0;
    int64_t crow = -1;
    auto emit = [&](SeqMachine<HostSeqSrc, G, false, SH>& mm, int p, int grp) {
      const int64_t r = crow;
      k1.push_back(((uint64_t)r << 16) | seq++);
      const size_t o = recs.size();
      recs.resize(o + rstride);
      char* rec = recs.data() + o;
      uint64_t trig = b->index ? b->index[r] : b->base_index + (uint64_t)r;
      memcpy(rec, &trig, 8);
      const int64_t pp = mm.dec(mm.M->P[p].pts);
      int64_t pts = pp >= 0 ? mm.src.ts(pp) : -1;
      memcpy(rec + 8, &pts, 8);
      uint32_t h32[4] = {(uint32_t)k, (1u << 24) | (uint32_t)grp, 0, 0};
      for (int s = 0; s < d.n_select; ++s) {
        int64_t v = 0;
        const int64_t ev = mm.get_event(p, d.sel_state[s], d.sel_index[s]);
        if (ev < 0) h32[2] |= 1u << s;
        else {
          SgVal x = mm.src.read(ev, d.sel_ret[s], d.ret_type[d.sel_ret[s]]);
          if (x.null) h32[2] |= 1u << s; else v = sg_val_bits(x);
        }
        memcpy(rec + 32 + 8 * s, &v, 8);
      }
      memcpy(rec + 16, h32, 16);
    };
    auto noemit = [&](SeqMachine<HostSeqSrc, G, false, SH>&, int, int) {};
    // run rows [a, b) from the state in `st` (the machine's M), emitting or not
    auto run = [&](int64_t a, int64_t b2, bool emitting) {
      m.begin();
      for (int64_t q = a; q < b2 && !m.failed; ++q) {
        crow = rows[q] - nc;
        seq = 0;
        if (emitting) m.receive(q, emit);
        else m.receive(q, noemit);
      }
      if (m.failed && getenv("SG_DEBUG_SEQ")) fprintf(stderr, "seq machine failed: %d\n", m.failed);
      m.finish();
      return !m.failed;
    };
    const int64_t R = h->spec_rows;
    if (R <= 0 || nk - ncar[k] <= R) {
      if (!run(ncar[k], nk, true)) return 0;
    } else {
      // speculative units (partial.hip's scheme): unit c > 0 starts from a zeroed state warmed up over the W rows before
      // it; a unit whose warmed-up start differs from its predecessor's end is rerun from that end; then every unit
      // runs again from its verified start, emitting
      const int64_t U = (nk - ncar[k] + R - 1) / R;
      std::vector<SeqStateT<G>> start((size_t)U), fin((size_t)U);
      for (int64_t c = 0; c < U; ++c) {
        const int64_t s0 = ncar[k] + c * R, s1 = std::min(nk, s0 + R);
        if (c == 0) st = next_state[k];
        else {
          memset(&st, 0, sizeof(st));
          if (!run(std::max<int64_t>(0, s0 - h->spec_warm), s0, false)) return 0;
        }
        start[c] = st;
        if (!run(s0, s1, false)) return 0;
        fin[c] = st;
      }
      for (int64_t c = 1; c < U; ++c) {
        if (sg_seq_equiv(start[c], fin[c - 1], d, ru)) continue;
        ++h->spec_reruns;
        const int64_t s0 = ncar[k] + c * R, s1 = std::min(nk, s0 + R);
        start[c] = fin[c - 1];
        st = start[c];
        if (!run(s0, s1, false)) return 0;
        fin[c] = st;
      }
      for (int64_t c = 0; c < U; ++c) {
        const int64_t s0 = ncar[k] + c * R, s1 = std::min(nk, s0 + R);
        st = start[c];
        if (!run(s0, s1, true)) return 0;
      }
    }
    // carry: the last H rows and the state re-expressed over them
    const int64_t from = nk > H ? nk - H : 0;
    m.rebase(nk - 1, from);
    for (int64_t q = from; q < nk; ++q) {
      const int64_t c = rows[q];
      HiHandle::CRow cr;
      memset(&cr, 0, sizeof(cr));
      if (c < nc) cr = h->carried[c];
      else {
        cr.ts = src.ts(c);
        cr.key = (int32_t)k;
        for (int j = 0; j < d.n_ret; ++j) {
          int null = 0;
          cr.vals[j] = read_bits_col(b, &d, j, c - nc, &null);
          if (null) cr.nullmask |= 1 << j;
        }
      }
      next.push_back(cr);
    }
  }
  states.swap(next_state);
  h->carried.swap(next);
  return 1;
}

extern "C" {

void hi_set_pp(HiHandle* h, int on) { h->pp = on; }
void hi_set_spec(HiHandle* h, int64_t rows, int64_t warm) { h->spec_rows = rows; h->spec_warm = warm; }
int64_t hi_spec_reruns(HiHandle* h) { return h->spec_reruns; }
int64_t hi_pp_steps(HiHandle* h, int64_t* lanes) { *lanes = h->pp_lanes; return h->pp_steps; }
int64_t hi_pp_skipped(HiHandle* h) { return h->pp_skipped; }
int hi_seq_rule(const sg_nfa_desc* d) { return sg_seq_rule(*d).ok; }
int hi_pp_rule(const sg_nfa_desc* d) { return sg_pp_rule(*d).ok; }
int hi_pp_shape_c3(const sg_nfa_desc* d) { return sg_pp_shape_is<PpShapeC3>(*d, sg_pp_rule(*d)) ? 1 : 0; }
int hi_sq_shape_c3b(const sg_nfa_desc* d) { return sg_sq_shape_is<SqShapeC3b>(*d, sg_seq_rule(*d)) ? 1 : 0; }
// the lane kernels' FAST variant applies (chain.h sg_terms_fast): seq = 1 for the sequence-lane rule
int hi_terms_fast(const sg_nfa_desc* d, int seq) {
  return seq ? sg_terms_fast(sg_seq_rule(*d), d->n_states) : sg_terms_fast(sg_pp_rule(*d), d->n_states);
}

HiHandle* hi_open(const sg_nfa_desc* d, int P, int E, int C, int L) {
  HiHandle* h = new HiHandle();
  h->d = *d;
  h->g = sg_make_geo(*d, P, E, C, L, L);
  return h;
}

void hi_close(HiHandle* h) { delete h; }

void hi_set_chunk(HiHandle* h, int chunk_rows) { h->chunk_rows = chunk_rows; }

int hi_chunk_rule(const sg_nfa_desc* d, int64_t* horizon) {
  SgChunkRule r = sg_chunk_rule(*d);
  *horizon = r.kind == 2 ? r.events : r.within;
  return r.kind;
}

static int machine_push(HiHandle* h, const sg_batch* b, bool silent);

int hi_push(HiHandle* h, const sg_batch* b) {
  if (h->pp && h->pp_active && sg_seq_rule(h->d).ok) {
    std::vector<char> recs;
    std::vector<uint64_t> k1;
    const std::vector<HiHandle::CRow> before = h->carried;
    const std::vector<SeqState> before_st = h->seq_state;
    const std::vector<SeqStateT<SqSmall>> before_s = h->seq_state_s;
    const bool small = sg_seq_small(sg_seq_rule(h->d), h->d);
    // (partial.hip's kernel choice: the specialised machine for C3b's family in the small geometry)
    const bool c3b = small && sg_sq_shape_is<SqShapeC3b>(h->d, sg_seq_rule(h->d));
    if (c3b ? seq_push<SqSmall, SqShapeC3b>(h, h->seq_state_s, b, recs, k1)
            : small ? seq_push(h, h->seq_state_s, b, recs, k1) : seq_push(h, h->seq_state, b, recs, k1)) {
      const int rstride = 32 + 8 * h->d.n_select;
      std::vector<size_t> idx(k1.size());
      for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
      std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return k1[x] < k1[y]; });
      for (size_t i : idx) h->out.emplace_back(recs.begin() + i * rstride, recs.begin() + (i + 1) * rstride);
      return 0;
    }
    // a key outgrew the compact machine: only a fresh stream can move to the per-key machine exactly
    if (!before.empty()) { h->err = SG_ECAPACITY; return SG_ECAPACITY; }
    h->carried = before;
    h->seq_state = before_st;
    h->seq_state_s = before_s;
  }
  if (h->pp && h->pp_active && (sg_pp_rule(h->d).ok || sg_seq_rule(h->d).ok)) {
   if (sg_pp_rule(h->d).ok) {
    std::vector<char> recs;
    std::vector<uint64_t> k1, th, tl;
    const SgPpRule pr = sg_pp_rule(h->d);
    const int rc = !sg_pp_small(pr, h->d)                  ? pp_push<PpBig>(h, b, recs, k1, th, tl)
                   : sg_pp_shape_is<PpShapeC3>(h->d, pr) ? pp_push<PpSmall, PpShapeC3>(h, b, recs, k1, th, tl)
                                                          : pp_push<PpSmall>(h, b, recs, k1, th, tl);
    if (rc < 0) { h->err = SG_EUNSUPPORTED; return SG_EUNSUPPORTED; }
    if (rc == 1) {
      const int rstride = 32 + 8 * h->d.n_select;
      std::vector<size_t> idx(k1.size());
      for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
      std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) {
        if (k1[x] != k1[y]) return k1[x] < k1[y];
        if (th[x] != th[y]) return th[x] < th[y];
        return tl[x] < tl[y];
      });
      for (size_t i : idx) h->out.emplace_back(recs.begin() + i * rstride, recs.begin() + (i + 1) * rstride);
      return 0;
    }
   }
    // leave the route: replay the carried rows through the machine without emitting
    h->pp_active = 0;
    const size_t nc = h->carried.size();
    if (nc) {
      std::vector<int64_t> ts(nc), colv[SG_MAX_COLS];
      const int recv = sg_pp_rule(h->d).ok ? sg_pp_rule(h->d).recv : sg_seq_rule(h->d).recv;
      std::vector<int32_t> key(nc), stream(nc, h->d.receivers[recv].stream);
      std::vector<uint8_t> nul[SG_MAX_COLS];
      const void* cols[SG_MAX_COLS] = {};
      const uint8_t* nuls[SG_MAX_COLS] = {};
      for (int j = 0; j < h->d.n_ret; ++j) {
        const int c = h->d.ret_col[j];
        colv[c].resize(nc);
        nul[c].resize(nc);
        for (size_t i = 0; i < nc; ++i) {
          int64_t bits = h->carried[i].vals[j];
          const int t = h->d.ret_type[j];
          if (t == SG_T_LONG || t == SG_T_DOUBLE) colv[c][i] = bits;
          else { int32_t w = (int32_t)(uint32_t)bits; memcpy(&colv[c][i], &w, 4); }
          nul[c][i] = (h->carried[i].nullmask >> j) & 1;
        }
        // 4-byte columns are read as int32/float from the start of each 8-byte cell: pack them densely
        if (!(h->d.ret_type[j] == SG_T_LONG || h->d.ret_type[j] == SG_T_DOUBLE)) {
          std::vector<int64_t> packed((nc + 1) / 2);
          for (size_t i = 0; i < nc; ++i) memcpy((char*)packed.data() + 4 * i, &colv[c][i], 4);
          colv[c].swap(packed);
        }
        cols[c] = colv[c].data();
        nuls[c] = nul[c].data();
      }
      for (size_t i = 0; i < nc; ++i) { ts[i] = h->carried[i].ts; key[i] = h->carried[i].key; }
      sg_batch cb;
      memset(&cb, 0, sizeof(cb));
      cb.n = (int64_t)nc;
      cb.ts = ts.data();
      cb.stream = stream.data();
      cb.key = key.data();
      cb.cols = cols;
      cb.nulls = nuls;
      h->carried.clear();
      if (int f = machine_push(h, &cb, true)) return f;
    }
  }
  return machine_push(h, b, false);
}

static int machine_push(HiHandle* h, const sg_batch* b, bool silent) {
  const sg_nfa_desc& d = h->d;
  int64_t n = b->n;
  int32_t kmax = -1;
  for (int64_t i = 0; i < n; ++i) if (b->key && b->key[i] > kmax) kmax = b->key[i];
  if (!d.partitioned) kmax = 0;
  if ((int64_t)h->arenas.size() < kmax + 1) h->arenas.resize(kmax + 1);
  std::vector<std::vector<int64_t>> own(h->arenas.size());
  for (int64_t i = 0; i < n; ++i) {
    int s = b->stream ? b->stream[i] : 0;
    if (s < 0 || d.recv_of_stream[s] < 0) continue;
    int k = d.partitioned ? b->key[i] : 0;
    if (k < 0) continue;
    own[k].push_back(i);
  }
  unsigned long long count = 0;
  int32_t overflow = 0;
  int stride = sg_emit_stride(d.n_select);
  size_t cap = 4 * (size_t)n + 4096;
  std::vector<char> buf(cap * stride);
  int kb = 1;
  while ((1ull << kb) <= (uint64_t)h->arenas.size()) ++kb;
  // the playback clock over this push (TimestampGeneratorImpl.setCurrentTimestamp: a row whose time goes back does not
  // move it and notifies nobody)
  std::vector<int64_t> clk((size_t)n), nf((size_t)n + 1);
  {
    int64_t c = h->clock;
    std::vector<char> fires((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
      fires[i] = b->ts[i] >= c;
      c = std::max(c, b->ts[i]);
      clk[i] = c;
    }
    nf[n] = n;
    for (int64_t i = n - 1; i >= 0; --i) nf[i] = fires[i] ? i : nf[i + 1];
    h->clock = c;
  }
  for (size_t k = 0; k < h->arenas.size(); ++k) {
    if (h->arenas[k].empty()) {
      if (own[k].empty() && d.partitioned) continue;
      h->arenas[k].assign((size_t)h->g.key_words, 0);
    }
    auto run = [&](int32_t* arena, const std::vector<int64_t>* rws, int64_t emit_from) {
      KeyMachine m;
      memset(&m, 0, sizeof(m));
      m.d = &d;
      m.g = &h->g;
      m.a = arena;
      m.key = (int32_t)k;
      m.clone = d.partitioned;
      m.sink = SgEmitSink{buf.data(), (int64_t)cap, &count, &overflow, stride, kb};
      m.base_index = b->base_index;
      HostRows rows{b, &d, rws, &clk, &nf};
      sg_run_key(m, rows, !d.partitioned, emit_from);
      return m.failed;
    };
    const SgChunkRule rule = sg_chunk_rule(d);
    const int64_t nown = (int64_t)own[k].size();
    const int64_t R = h->chunk_rows;
    if (R <= 0 || rule.kind == 0 || nown <= R) {
      if (int f = run(h->arenas[k].data(), &own[k], 0)) { h->err = f; return f; }
      continue;
    }
    // chunked units: unit 0 continues the key's state; unit c > 0 replays its horizon from a fresh runtime
    // (or from the state at the push start when the horizon reaches the key's first row of this push)
    const std::vector<int32_t> snap = h->arenas[k];
    std::vector<int32_t> last;
    for (int64_t p0 = 0; p0 < nown; p0 += R) {
      const int64_t p1 = std::min(nown, p0 + R);
      if (p0 == 0) {
        std::vector<int64_t> sub(own[k].begin(), own[k].begin() + p1);
        if (int f = run(h->arenas[k].data(), &sub, 0)) { h->err = f; return f; }
        continue;
      }
      const int64_t q = sg_replay_start(rule, p0, [&](int64_t i) { return b->ts[own[k][i]]; });
      std::vector<int32_t> arena = q == 0 ? snap : std::vector<int32_t>((size_t)h->g.key_words, 0);
      std::vector<int64_t> sub(own[k].begin() + q, own[k].begin() + p1);
      if (int f = run(arena.data(), &sub, p0 - q)) { h->err = f; return f; }
      if (p1 == nown) last.swap(arena);
    }
    h->arenas[k].swap(last);
  }
  if (overflow) { h->err = SG_ECAPACITY; return SG_ECAPACITY; }
  if (silent) return 0;
  std::vector<size_t> idx(count);
  for (size_t i = 0; i < count; ++i) idx[i] = i;
  auto sk = [&](size_t i) { uint64_t v; memcpy(&v, buf.data() + i * stride, 8); return v; };
  std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return sk(x) < sk(y); });
  for (size_t i : idx) h->out.emplace_back(buf.begin() + i * stride + 8, buf.begin() + (i + 1) * stride);
  return 0;
}

int64_t hi_count(HiHandle* h) { return (int64_t)h->out.size(); }

void hi_fetch(HiHandle* h, uint64_t* trig, int64_t* ts, int32_t* key, uint32_t* group, int64_t* vals, uint32_t* vnull) {
  int ns = h->d.n_select;
  for (size_t i = 0; i < h->out.size(); ++i) {
    const char* r = h->out[i].data();
    memcpy(trig + i, r, 8); memcpy(ts + i, r + 8, 8); memcpy(key + i, r + 16, 4); memcpy(group + i, r + 20, 4);
    memcpy(vnull + i, r + 24, 4);
    if (ns) memcpy(vals + i * ns, r + 32, 8 * (size_t)ns);
  }
  h->out.clear();
}

}
