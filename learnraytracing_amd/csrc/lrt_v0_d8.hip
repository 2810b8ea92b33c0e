// v0 instances for max_depth <= 8 (lrt_v0.h): the 8 recursion levels live in LDS.
#include "lrt_v0.h"

namespace lrt {

int launch_v0_d8(const KernelArgs& a, bool lds, int xc, int rows, int frames, bool feat, bool colours, hipStream_t s) {
    if (colours) return launch_depth<8, 1>(a, lds, xc, rows, s);
    return launch_split<8>(a, lds, xc, rows, frames, feat, s);
}

}  // namespace lrt
