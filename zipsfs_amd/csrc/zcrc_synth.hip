// zcrc_synth.hip -- on-device synthetic payload generator (bench/test data).
//
// Not a CRC path: fills buffers with the counter-based payload of SURVEY.md
// 8(d) so that multi-GiB batches never cross PCIe and the CPU oracle can
// regenerate any buffer to check it:
//   word j of buffer with payload index I = splitmix64(seed ^ (I<<32 | j)),
//   little-endian, truncated at the buffer length.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zcrc_internal.h"

namespace zcrc {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// One workgroup walks buffers blockIdx.x, blockIdx.x + gridDim.x, ...; threads
// write 16 B (two words) per step; the ragged tail is written bytewise.
__global__ __launch_bounds__(256) void fill_synthetic_kernel(const uint64_t *ptrs, const uint64_t *lens,
                                                             uint64_t n, uint64_t index0, uint64_t index_step,
                                                             uint64_t seed) {
  for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
    uint8_t *dst = reinterpret_cast<uint8_t *>(ptrs[b]);
    const uint64_t len = lens[b];
    const uint64_t key = (index0 + b * index_step) << 32;
    const bool aligned16 = (reinterpret_cast<uintptr_t>(dst) & 15u) == 0;
    const uint64_t npairs = aligned16 ? len / 16 : 0;
    for (uint64_t p = threadIdx.x; p < npairs; p += blockDim.x) {
      const uint64_t w0 = mix64(seed ^ (key + 2 * p)), w1 = mix64(seed ^ (key + 2 * p + 1));
      ulonglong2 v;
      v.x = w0;
      v.y = w1;
      reinterpret_cast<ulonglong2 *>(dst)[p] = v;
    }
    for (uint64_t k = npairs * 16 + threadIdx.x; k < len; k += blockDim.x) {
      const uint64_t w = mix64(seed ^ (key + k / 8));
      dst[k] = (uint8_t)(w >> (8 * (k % 8)));
    }
  }
}

hipError_t launch_fill_synthetic(const uint64_t *d_ptrs, const uint64_t *d_lens, uint64_t n, uint64_t index0,
                                 uint64_t index_step, uint64_t seed, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t grid = n < 65536 ? n : 65536;
  hipLaunchKernelGGL(fill_synthetic_kernel, dim3((unsigned)grid), dim3(256), 0, stream, d_ptrs, d_lens, n, index0,
                     index_step, seed);
  return hipGetLastError();
}

}  // namespace zcrc
