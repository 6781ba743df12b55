// Instantiation of the closed-form every->next pipeline (engine_impl.h) for double compared values.
#include "engine_impl.h"

void sg_every_next_f64(SgHandle* h, const BatchView& bv, int64_t n) { dispatch_np<double>(h, bv, n); }
