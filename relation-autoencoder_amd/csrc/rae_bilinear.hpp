// RESCAL / RESCAL+SP decoders (Bilinear.py, BilinearPlusSP.py) -- placeholder until the
// MFMA path lands; the host refuses these decoders for now.
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

template <bool V4>
__device__ void bilinear_example(const StepArgs& a, int64_t g, int bl, char* smem, bool hybrid) {
    __builtin_trap();
}

template <int OPT>
__device__ void task_bilinear_tile(const StepArgs& a, int i0, int k0, int slot, int lane) {
    __builtin_trap();
}

}  // namespace rae
