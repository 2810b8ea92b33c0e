// The tile order's sort on the device (lrt_hip.hip tile_order): tiles by recorded cost,
// heaviest first, ties by tile index -- rocPRIM's radix sort is stable, so the permutation is
// the one std::stable_sort on the host gave (round 2-3), without the host round trip (a
// blocking D2H of the costs, the sort, a blocking H2D of the permutation: ~0.6 ms of host
// latency on the launch that flipped the order, profiles/r3_p). Its own translation unit:
// rocPRIM's templates stay out of the kernels' file.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

namespace lrt {

// tile ids 0..n-1 (the sort's values input)
__global__ void iota_kernel(int* v, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// tmp == nullptr: *tmp_bytes = the scratch the sort needs for n keys. Otherwise enqueues on s:
// perm_out = tile ids ordered by cost_in descending (stable), keys_out = the sorted costs.
hipError_t sort_tiles_desc(const unsigned* cost_in, unsigned* keys_out, const int* ids_in, int* perm_out, int n,
                           void* tmp, size_t* tmp_bytes, hipStream_t s, unsigned end_bit) {
    return rocprim::radix_sort_pairs_desc(tmp, *tmp_bytes, cost_in, keys_out, ids_in, perm_out, (unsigned)n, 0u,
                                          end_bit, s);
}

hipError_t fill_iota(int* v, int n, hipStream_t s) {
    iota_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(v, n);
    return hipGetLastError();
}

}  // namespace lrt
