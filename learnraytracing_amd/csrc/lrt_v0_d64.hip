// v0 instances for max_depth <= 64 (lrt_v0.h): levels beyond 8 in a global overflow stack.
#include "lrt_v0.h"

namespace lrt {

int launch_v0_d64(const KernelArgs& a, bool lds, int xc, int rows, int frames, bool feat, bool colours, hipStream_t s) {
    if (colours) return launch_depth<64, 1>(a, lds, xc, rows, s);
    return launch_split<64>(a, lds, xc, rows, frames, feat, s);
}

}  // namespace lrt
