// tools/hbm_probe.hip -- HBM read-bandwidth probe for MI355X (measurement only).
//
// Measures the practical pure-read ceiling that the CRC kernel is compared
// against, for several access shapes:
//   grid    : classic grid-stride, lane-interleaved over the whole buffer
//   wave    : each wave owns a contiguous range (the CRC kernel's shape)
//   wg      : each workgroup owns a contiguous range, its waves interleaved
// Each variant xor-reduces 16-B loads (buffer_load_dwordx4) so nothing is
// written but one word per thread.  Usage: hbm_probe [GiB] [reps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <int D>
__device__ __forceinline__ void consume(const uint4 *v, uint4 &acc) {
#pragma unroll
  for (int u = 0; u < D; u++) {
    acc.x ^= v[u].x;
    acc.y ^= v[u].y;
    acc.z ^= v[u].z;
    acc.w ^= v[u].w;
  }
}

// grid-stride: block b, iteration k reads chunk (k*grid + b)*blockDim*16*D
template <int D>
__global__ void read_grid(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * D;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * D; base + (uint64_t)blockDim.x * D <= n16;
       base += stride) {
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = p[base + (uint64_t)u * blockDim.x + threadIdx.x];
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// wave-contiguous: wave w owns [w*per, (w+1)*per) 16-B chunks
template <int D>
__global__ void read_wave(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const uint64_t per = n16 / waves;
  const uint32_t lane = threadIdx.x & 63;
  const uint4 *q = p + w * per;
  for (uint64_t base = 0; base + 64 * D <= per; base += 64 * D) {
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = q[base + u * 64 + lane];
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// workgroup-contiguous: block b owns [b*per, (b+1)*per), threads interleaved
template <int D>
__global__ void read_wg(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t per = n16 / gridDim.x;
  const uint4 *q = p + (uint64_t)blockIdx.x * per;
  for (uint64_t base = 0; base + (uint64_t)blockDim.x * D <= per; base += (uint64_t)blockDim.x * D) {
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = q[base + (uint64_t)u * blockDim.x + threadIdx.x];
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// workgroup range, waves take C-byte chunks round-robin (wave j: chunks j, j+nw, ...)
template <int D, int CKIB>
__global__ void read_wgchunk(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t per = n16 / gridDim.x;
  const uint4 *q = p + (uint64_t)blockIdx.x * per;
  const uint32_t nw = blockDim.x / 64, wv = threadIdx.x / 64, lane = threadIdx.x & 63;
  const uint64_t c16 = (uint64_t)CKIB * 64;  // 16-B chunks per C
  const uint64_t nchunks = per / c16;
  for (uint64_t c = wv; c < nchunks; c += nw) {
    const uint4 *r = q + c * c16;
    for (uint64_t base = 0; base + 64 * D <= c16; base += 64 * D) {
      uint4 v[D];
#pragma unroll
      for (int u = 0; u < D; u++) v[u] = r[base + u * 64 + lane];
      consume<D>(v, acc);
    }
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// wave-contiguous with a per-wave rotation of the start: wave w reads its
// range from a pseudo-random 1 KiB-aligned offset, wrapping around
template <int D>
__global__ void read_wave_skew(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const uint64_t per = n16 / waves;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nblk = per / 64;
  const uint64_t rot = (uint64_t)(hash32((uint32_t)w) % (uint32_t)(nblk / D)) * D * 64;
  const uint4 *q = p + w * per;
  for (uint64_t base = 0; base + 64 * D <= per; base += 64 * D) {
    uint64_t b = base + rot;
    if (b >= per) b -= per;
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = q[b + u * 64 + lane];
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// workgroup-contiguous with per-WG rotation
template <int D>
__global__ void read_wg_skew(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t per = n16 / gridDim.x;
  const uint64_t step = (uint64_t)blockDim.x * D;
  const uint64_t rot = (uint64_t)(hash32(blockIdx.x) % (uint32_t)(per / step)) * step;
  const uint4 *q = p + (uint64_t)blockIdx.x * per;
  for (uint64_t base = 0; base + step <= per; base += step) {
    uint64_t b = base + rot;
    if (b >= per) b -= per;
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = q[b + (uint64_t)u * blockDim.x + threadIdx.x];
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// workgroup range processed in 16 KiB rows (wave j: 1 KiB j of each row),
// range rotated per WG at ROTK-KiB granularity
template <int D, int ROTK>
__global__ void read_wg_rot(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t per = n16 / gridDim.x;
  const uint64_t step = (uint64_t)blockDim.x * D;
  const uint64_t g16 = (uint64_t)ROTK * 64;
  const uint64_t rot = (uint64_t)(hash32(blockIdx.x) % (uint32_t)(per / g16)) * g16;
  const uint4 *q = p + (uint64_t)blockIdx.x * per;
  for (uint64_t base = 0; base + step <= per; base += step) {
    uint64_t b = base + rot;
    if (b >= per) b -= per;
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = q[b + (uint64_t)u * blockDim.x + threadIdx.x];
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// chunk sweep: chunk c (CK KiB) -> workgroup c % grid, read in 16 KiB rows
template <int D, int CK>
__global__ void read_chunk_sweep(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t c16 = (uint64_t)CK * 64, step = (uint64_t)blockDim.x * D;
  const uint64_t nch = n16 / c16;
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint4 *q = p + c * c16;
    for (uint64_t base = 0; base + step <= c16; base += step) {
      uint4 v[D];
#pragma unroll
      for (int u = 0; u < D; u++) v[u] = q[base + (uint64_t)u * blockDim.x + threadIdx.x];
      consume<D>(v, acc);
    }
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// the same two shapes with non-temporal (nt) loads
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntload(const uint4 *a) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(a));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

template <int D>
__global__ void read_grid_nt(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * D;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * D; base + (uint64_t)blockDim.x * D <= n16;
       base += stride) {
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = ntload(&p[base + (uint64_t)u * blockDim.x + threadIdx.x]);
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int D>
__global__ void read_wave_nt(const uint4 *p, uint64_t n16, uint32_t *out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const uint64_t per = n16 / waves;
  const uint32_t lane = threadIdx.x & 63;
  const uint4 *q = p + w * per;
  for (uint64_t base = 0; base + 64 * D <= per; base += 64 * D) {
    uint4 v[D];
#pragma unroll
    for (int u = 0; u < D; u++) v[u] = ntload(&q[base + u * 64 + lane]);
    consume<D>(v, acc);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

typedef void (*kfn)(const uint4 *, uint64_t, uint32_t *);

static double run(const char *name, kfn k, int grid, int block, const uint4 *p, uint64_t n16, uint32_t *out, int reps,
                  uint64_t bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, p, n16, out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, p, n16, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double gbs = (double)bytes * reps / (ms * 1e-3) / 1e9;
  printf("%-34s grid=%5d block=%4d  %8.1f GB/s  (%.3f ms/launch)\n", name, grid, block, gbs, ms / reps);
  fflush(stdout);
  return gbs;
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 16.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  const uint64_t n16 = bytes / 16;
  uint4 *p;
  uint32_t *out;
  CHECK(hipMalloc(&p, bytes));
  CHECK(hipMalloc(&out, 64ull << 20));
  CHECK(hipMemset(p, 0x5A, bytes));
  CHECK(hipDeviceSynchronize());
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("hbm_probe: %.1f GiB, %d CUs, %d reps\n", gib, cus, reps);
  if (cus != 256 || (n16 % (1ull << 20)) != 0) {
    fprintf(stderr, "probe expects 256 CUs and a multiple of 16 MiB\n");
    return 1;
  }
  // every (grid, block, D) below tiles the 16 GiB range exactly, so the byte
  // count per launch is exact (n16 is a multiple of 2^20 chunks)
  for (int round = 0; round < 2; round++) {
    printf("-- round %d\n", round);
    run("grid-stride D=4 (1024 thr, 1/CU)", read_grid<4>, cus, 1024, p, n16, out, reps, bytes);
    run("grid-stride D=4 nt", read_grid_nt<4>, cus, 1024, p, n16, out, reps, bytes);
    run("grid-stride D=8 nt", read_grid_nt<8>, cus, 1024, p, n16, out, reps, bytes);
    run("wave-contig D=4", read_wave<4>, cus, 1024, p, n16, out, reps, bytes);
    run("wave-contig D=4 nt", read_wave_nt<4>, cus, 1024, p, n16, out, reps, bytes);
    if (getenv("PROBE_ALL") == nullptr) continue;
    run("wg-rot 64K D=4", read_wg_rot<4, 64>, cus, 1024, p, n16, out, reps, bytes);
    run("wg-rot 1M D=4", read_wg_rot<4, 1024>, cus, 1024, p, n16, out, reps, bytes);
    run("wg-rot 4M D=4", read_wg_rot<4, 4096>, cus, 1024, p, n16, out, reps, bytes);
    run("wg-rot 1M D=2", read_wg_rot<2, 1024>, cus, 1024, p, n16, out, reps, bytes);
    run("chunk-sweep 64K D=4", read_chunk_sweep<4, 64>, cus, 1024, p, n16, out, reps, bytes);
    run("chunk-sweep 256K D=4", read_chunk_sweep<4, 256>, cus, 1024, p, n16, out, reps, bytes);
    run("chunk-sweep 1M D=4", read_chunk_sweep<4, 1024>, cus, 1024, p, n16, out, reps, bytes);
    run("chunk-sweep 1M D=2", read_chunk_sweep<2, 1024>, cus, 1024, p, n16, out, reps, bytes);
  }
  CHECK(hipFree(p));
  CHECK(hipFree(out));
  return 0;
}
