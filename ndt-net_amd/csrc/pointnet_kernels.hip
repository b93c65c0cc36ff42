// pointnet_kernels.hip -- placeholder until the MFMA forward lands.
#include <hip/hip_runtime.h>
#include "pointnet.h"
