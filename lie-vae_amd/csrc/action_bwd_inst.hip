// Explicit instantiation of one backward degree-range kernel (LV_BWD_R in
// [0, kNumBwdRanges)), one object per range.
#include "action_bwd.h"

#ifndef LV_BWD_R
#error "compile with -DLV_BWD_R=<range>"
#endif

namespace lv {
template struct BwdLauncher<LV_BWD_R>;
}  // namespace lv
