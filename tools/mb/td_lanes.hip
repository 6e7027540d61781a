// Microbenchmark (not shipped): cost of a wave's dwordx4 gather on MI355X as a
// function of active lanes and of distinct 128-B lines per instruction.
//   mode 0: each active lane gathers 7 x 16 B of its own random 128-B record
//   mode 1: cooperative: 8 lanes share one record (lane i reads chunk i % 8 of
//           record i / 8 of the group), so one instruction touches 8 lines
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(64) k(const f4 *__restrict__ tab, uint32_t nrec, int active, int iters, int mode,
                                        float *out) {
  uint32_t lane = threadIdx.x;
  uint32_t s = (blockIdx.x * 64 + lane) * 2654435761u + 12345u;
  uint32_t sg = blockIdx.x * 2654435761u + 777u + (lane >> 3) * 40503u;  // same for 8 lanes
  f4 acc = (f4){0, 0, 0, 0};
  if ((int)lane < active) {
    for (int i = 0; i < iters; ++i) {
      if (mode == 0) {
        s = s * 1103515245u + 12345u;
        const f4 *p = tab + (size_t)((s >> 8) % nrec) * 8;
        f4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4], f = p[5], g = p[6];
        acc += a + b + c + d + e + f + g;
      } else {
        // 7 instructions, each touching 8 records (one per 8-lane group)
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          sg = sg * 1103515245u + 12345u;
          acc += tab[(size_t)((sg >> 8) % nrec) * 8 + (lane & 7)];
        }
      }
    }
  }
  if (acc.x == 1.2345f) out[0] = acc.y;
}
int main() {
  uint32_t nrec = 16384;  // 2 MB of 128-B records (L2 resident)
  f4 *tab;
  float *out;
  (void)hipMalloc(&tab, (size_t)nrec * 128);
  (void)hipMemset(tab, 0, (size_t)nrec * 128);
  (void)hipMalloc(&out, 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int grid = 256 * 16;  // 16 waves per CU
  for (int mode = 0; mode < 2; ++mode)
    for (int active : {64, 32, 16, 8}) {
      int iters = 200;
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, tab, nrec, active, iters, mode, out);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, tab, nrec, active, iters, mode, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      double insts = (double)grid * iters * 7;
      printf("mode %d active %2d: %.3f ms, %.2f ns per wave-gather-instr per CU\n", mode, active, ms,
             ms * 1e6 / (insts / 256));
    }
  return 0;
}
