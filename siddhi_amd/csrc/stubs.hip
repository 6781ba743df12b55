// Absence closed form (SG_SHAPE_EVERY_ABSENT_EQ) not built yet in this revision: such queries run on the
// general per-key machine (interp.hip), which is exact but sequential per key.
#include "sg_engine.h"
void sg_run_every_absent(SgHandle* h, const BatchView& bv, int64_t n) { sg_run_general(h, bv, n); }
