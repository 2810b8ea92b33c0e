// pool kernel instances for max_depth <= 64 (lrt_pool_launch.h).
#include "lrt_pool_launch.h"

namespace lrt {

int launch_pool_d64(const KernelArgs& a, bool lds, int xc, int rows, int frames, int pix_cap, hipStream_t s) {
    return launch_pool_split<64>(a, lds, xc, rows, frames, pix_cap, s);
}

}  // namespace lrt
