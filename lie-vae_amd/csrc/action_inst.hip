// Explicit instantiation of the group-action kernels for one l_max (LV_INST_L).
#include "action_kernels.h"

#ifndef LV_INST_L
#error "compile with -DLV_INST_L=<l_max>"
#endif

namespace lv {
template struct FwdLauncher<LV_INST_L>;
template struct BwdLauncher<LV_INST_L>;
template struct WigLauncher<LV_INST_L>;
}  // namespace lv
