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

void sg_every_next_release(SgHandle* h) {
  if (h->state_kind != 1) return;
  EveryNextState* es = (EveryNextState*)h->state;
  es->carry[0].release();
  es->carry[1].release();
  delete es;
  h->state = nullptr;
  h->state_kind = 0;
}
