// Explicit instantiation of the group-action kernels for one l_max (LV_INST_L), one part
// per object (LV_INST_PART 0 = forward kernels, 1 = backward + Wigner-D) so that the
// large-l variants compile in parallel.
#include "action_kernels.h"

#ifndef LV_INST_L
#error "compile with -DLV_INST_L=<l_max>"
#endif
#ifndef LV_INST_PART
#define LV_INST_PART 0
#endif

namespace lv {
#if LV_INST_PART == 0
template struct FwdLauncher<LV_INST_L>;
#else
template struct BwdLauncher<LV_INST_L>;
template struct WigLauncher<LV_INST_L>;
#endif
}  // namespace lv
