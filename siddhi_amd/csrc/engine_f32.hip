// Instantiation of the closed-form every->next pipeline (engine_impl.h) for float compared values.
#include "engine_impl.h"

void sg_every_next_f32(SgHandle* h, const BatchView& bv, int64_t n) { dispatch_np<float>(h, bv, n); }

void sg_run_every_next(SgHandle* h, const BatchView& bv, int64_t n) {
  switch (h->desc.shape_args[5]) {
    case SG_T_FLOAT: sg_every_next_f32(h, bv, n); break;
    case SG_T_DOUBLE: sg_every_next_f64(h, bv, n); break;
    case SG_T_LONG: sg_every_next_i64(h, bv, n); break;
    default: sg_every_next_i32(h, bv, n); break;
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

// Snapshot of the closed form's state: the carried rows (per key, the rows still inside `within` of the key's
// last event -- they rebuild e2's pending list, StreamPreStateProcessor.currentState
// C/query/input/stream/state/StreamPreStateProcessor.java:352-359) and the null history of the columns.
static int col_bytes(const sg_nfa_desc& d, int c) {
  return (d.col_type[c] == SG_T_LONG || d.col_type[c] == SG_T_DOUBLE) ? 8 : 4;
}

void sg_every_next_snapshot(SgHandle* h, SnapW& w) {
  const sg_nfa_desc& d = h->desc;
  EveryNextState* es = (h->state && h->state_kind == 1) ? (EveryNextState*)h->state : nullptr;
  const int64_t n = es ? es->carry[es->cur].n : 0;
  w.pod(n);
  for (int c = 0; c < SG_MAX_COLS; ++c) w.pod((uint8_t)(es && es->nul_seen[c]));
  if (!n) return;
  const CarrySet& cs = es->carry[es->cur];
  w.dev(cs.ts, n * 8, h->stream);
  w.dev(cs.key, n * 4, h->stream);
  w.dev(cs.flags, n, h->stream);
  for (int c = 0; c < d.n_cols; ++c) {
    w.dev(cs.col[c], n * col_bytes(d, c), h->stream);
    w.dev(cs.nul[c], n, h->stream);
  }
}

void sg_every_next_restore(SgHandle* h, SnapR& r) {
  const sg_nfa_desc& d = h->desc;
  if (!h->state) { h->state = new EveryNextState(); h->state_kind = 1; }
  EveryNextState* es = (EveryNextState*)h->state;
  const int64_t n = r.pod<int64_t>();
  if (n < 0 || n >= (1ll << 30)) throw SgError(SG_EINVAL, "snapshot: bad carried-row count");
  for (int c = 0; c < SG_MAX_COLS; ++c) es->nul_seen[c] = r.pod<uint8_t>() != 0;
  es->carry[0].n = es->carry[1].n = 0;
  CarrySet& cs = es->carry[es->cur];
  if (!n) return;
  cs.ensure(n, d.n_cols, d.col_type);
  r.dev(cs.ts, n * 8, h->stream);
  r.dev(cs.key, n * 4, h->stream);
  r.dev(cs.flags, n, h->stream);
  for (int c = 0; c < d.n_cols; ++c) {
    r.dev(cs.col[c], n * col_bytes(d, c), h->stream);
    r.dev(cs.nul[c], n, h->stream);
  }
  cs.n = n;
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
