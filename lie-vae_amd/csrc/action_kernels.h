#pragma once
// All group-action kernels (forward + backward); host code in action.hip includes this.
#include "action_bwd.h"
#include "action_fwd.h"
