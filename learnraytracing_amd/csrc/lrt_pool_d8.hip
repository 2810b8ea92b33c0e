// pool kernel instances for max_depth <= 8 (lrt_pool_launch.h).
#include "lrt_pool_launch.h"

namespace lrt {

int launch_pool_d8(const KernelArgs& a, bool lds, int xc, int rows, int frames, int pix_cap, hipStream_t s) {
    return launch_pool_split<8>(a, lds, xc, rows, frames, pix_cap, s);
}

}  // namespace lrt
