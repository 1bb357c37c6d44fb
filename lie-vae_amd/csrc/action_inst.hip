// Explicit instantiation of the forward group-action kernels for one l_max (LV_INST_L)
// and the Wigner-D kernel of degree LV_INST_L, one object per l so that the large-l
// variants compile in parallel.
#include "action_fwd.h"

#ifndef LV_INST_L
#error "compile with -DLV_INST_L=<l_max>"
#endif

namespace lv {
template struct FwdLauncher<LV_INST_L>;
template struct WigLauncher<LV_INST_L>;
}  // namespace lv
