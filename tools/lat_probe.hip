// tools/lat_probe.hip -- single-wave latency of the instruction chains the
// inflate literal loop is built from (measurement only).  Each variant runs
// a dependent chain N times in one wave and reports cycles per iteration
// (s_memtime, shader clock).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int V>
__global__ void probe(uint32_t *out, uint32_t n, uint32_t seed) {
  uint64_t t0 = 0, t1 = 0;
  uint32_t s = seed;
  uint32_t lut = threadIdx.x * 0x9E3779B1u;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (uint32_t i = 0; i < n; i++) {
    if (V == 0) {  // dependent SALU chain: 4 ops
      asm volatile("s_add_u32 %0, %0, 1\n\ts_xor_b32 %0, %0, 5\n\ts_lshr_b32 %0, %0, 1\n\ts_add_u32 %0, %0, 3" : "+s"(s) :: "scc");
    } else if (V == 1) {  // readlane (VALU->SGPR) then SALU use
      asm volatile("v_readlane_b32 %0, %1, %0\n\ts_and_b32 %0, %0, 63" : "+s"(s) : "v"(lut) : "scc");
    } else if (V == 2) {  // gpr_idx lookup + readlane + SALU use
      asm volatile(
          "s_and_b32 s70, %0, 15\n\t"
          "s_set_gpr_idx_on s70, gpr_idx(SRC0)\n\t"
          "v_mov_b32 v56, v40\n\t"
          "s_set_gpr_idx_off\n\t"
          "v_readlane_b32 %0, v56, %0\n\t"
          "s_and_b32 %0, %0, 63"
          : "+s"(s) : "v"(lut) : "s70", "v56", "scc");
    } else if (V == 3) {  // s_cbranch taken each iteration
      asm volatile(
          "s_add_u32 %0, %0, 1\n\t"
          "s_cmp_eq_u32 %0, 0\n\t"
          "s_cbranch_scc0 L_a_%=\n\t"
          "s_add_u32 %0, %0, 7\n\t"
          "L_a_%=:"
          : "+s"(s) :: "scc");
    } else if (V == 4) {  // VALU op then readlane of its result
      asm volatile("v_add_u32 v56, %1, %0\n\tv_readlane_b32 %0, v56, %0\n\ts_and_b32 %0, %0, 63" : "+s"(s) : "v"(lut) : "v56", "scc");
    } else if (V == 6) {  // 4 independent SALU
      uint32_t a = s, b = s + 1, c = s + 2, d = s + 3;
      asm volatile("s_add_u32 %0, %0, 1\n\ts_xor_b32 %1, %1, 5\n\ts_lshr_b32 %2, %2, 1\n\ts_add_u32 %3, %3, 3"
                   : "+s"(a), "+s"(b), "+s"(c), "+s"(d) :: "scc");
      s = a ^ b ^ c ^ d;
    } else if (V == 7) {  // 8 independent SALU
      uint32_t a = s, b = s + 1, c = s + 2, d = s + 3;
      asm volatile("s_add_u32 %0, %0, 1\n\ts_xor_b32 %1, %1, 5\n\ts_lshr_b32 %2, %2, 1\n\ts_add_u32 %3, %3, 3\n\t"
                   "s_add_u32 %0, %0, 1\n\ts_xor_b32 %1, %1, 5\n\ts_lshr_b32 %2, %2, 1\n\ts_add_u32 %3, %3, 3"
                   : "+s"(a), "+s"(b), "+s"(c), "+s"(d) :: "scc");
      s = a ^ b ^ c ^ d;
    } else if (V == 8) {  // 8 dependent SALU
      asm volatile("s_add_u32 %0, %0, 1\n\ts_xor_b32 %0, %0, 5\n\ts_lshr_b32 %0, %0, 1\n\ts_add_u32 %0, %0, 3\n\t"
                   "s_add_u32 %0, %0, 1\n\ts_xor_b32 %0, %0, 5\n\ts_lshr_b32 %0, %0, 1\n\ts_add_u32 %0, %0, 3" : "+s"(s) :: "scc");
    } else if (V == 5) {  // ds_write_b8 + SALU (no dependence)
      asm volatile("v_mov_b32 v57, %0\n\tds_write_b8 v57, v57\n\ts_add_u32 %0, %0, 1\n\ts_and_b32 %0, %0, 255" : "+s"(s) :: "v57", "scc");
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) {
    out[0] = (uint32_t)(t1 - t0);
    out[1] = s;
  }
}

int main() {
  uint32_t *d;
  CHECK(hipMalloc(&d, 64));
  const uint32_t n = 100000;
  const char *names[] = {"4 dependent SALU", "v_readlane + s_and", "gpr_idx lookup (6 instr)",
                         "SALU + taken branch (3-4 instr)", "v_add + v_readlane + s_and", "v_mov + ds_write_b8 + 2 SALU",
                         "4 independent SALU (+3 xor)", "8 independent SALU (+3 xor)", "8 dependent SALU"};
  void (*ks[])(uint32_t *, uint32_t, uint32_t) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>,
                                                  probe<6>, probe<7>, probe<8>};
  for (int rep = 0; rep < 1; rep++)
    for (int v = 0; v < 9; v++) {
      hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, d, n, 12345u);
      CHECK(hipDeviceSynchronize());
      uint32_t h[2];
      CHECK(hipMemcpy(h, d, 8, hipMemcpyDeviceToHost));
      printf("%-36s %7.2f cycles/iter (s_memtime)\n", names[v], (double)h[0] / n);
      fflush(stdout);
    }
  return 0;
}
