// woq_chain.h -- the persistent decode chain (woq_chain.hip): a list of decode GEMV ops run in one launch.
#pragma once
#include <hip/hip_runtime.h>

#include "woq_kernels.h"

namespace nad {
// LDS bytes one op needs inside the chain (sets a.part_off)
size_t chain_lds_layout(GemvArgs& a, int waves, int grid);
// dev_ops: n_ops GemvArgs in device memory; flags[grid] must be 0 at launch; status[0] set on a barrier timeout
hipError_t launch_chain(const GemvArgs* dev_ops, int n_ops, int hilo, int asym, int waves, int grid, size_t lds,
                        unsigned* flags, unsigned* status, int npre, hipStream_t st);
}  // namespace nad
