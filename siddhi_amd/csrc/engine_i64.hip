// Instantiation of the closed-form every->next pipeline (engine_impl.h) for int64_t compared values.
#include "engine_impl.h"

void sg_every_next_i64(SgHandle* h, const BatchView& bv, int64_t n) { dispatch_np<int64_t>(h, bv, n); }
