// Explicit instantiation of the backward group-action kernels for one l_max
// (LV_INST_L), one object per l so that the large-l variants compile in parallel.
#include "action_bwd.h"

#ifndef LV_INST_L
#error "compile with -DLV_INST_L=<l_max>"
#endif

namespace lv {
template struct BwdLauncher<LV_INST_L>;
}  // namespace lv
