// Instantiation of the closed-form every->next pipeline (engine_impl.h) for int32_t compared values.
#include "engine_impl.h"

void sg_every_next_i32(SgHandle* h, const BatchView& bv, int64_t n) { dispatch_np<int32_t>(h, bv, n); }
