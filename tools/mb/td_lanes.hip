// Microbenchmark (not shipped; tools/profile.py runs it as the TD-model
// calibration): the cost of one wave's dwordx4 gather instruction on MI355X as
// a function of the active lanes and of the distinct 128-B lines it touches.
// Every pattern gathers from a 2 MB table of 128-B records (L2 resident, like
// C2's scene) with 16 waves per CU issuing back to back, so the time per
// instruction is the vector-memory path's throughput (TA/TD), not latency.
//
//   mode 0: each active lane gathers 7 x 16 B of its own random record
//           (one line per active lane per instruction: k_render's node step)
//   mode 1: 8 lanes share one record (lane i reads chunk i % 8 of record i / 8
//           of its 8-lane group): active / 8 lines per instruction
//   mode 2: 4 lanes share one 64-B half record: active / 4 lines
//   mode 3: every lane reads the same record (1 line per instruction)
//
// Output, one JSON line per pattern: mode, active lanes, lines per
// instruction (by construction), ms, shader clock (s_memtime over
// s_memrealtime, 100 MHz), cycles per wave-instruction per CU.
// tools/profile.py fits cycles = a + b * lines and reports k_render's TD
// floor as (a * SQ_INSTS_VMEM_RD + b * TCP_TOTAL_CACHE_ACCESSES) / CUs.
//   td_lanes [--json]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(64) k(const f4 *__restrict__ tab, uint32_t nrec, int active, int iters, int mode,
                                        float *out, unsigned long long *clk) {
  const uint32_t lane = threadIdx.x;
  uint32_t s = (blockIdx.x * 64 + lane) * 2654435761u + 12345u;
  const uint32_t grp = mode == 1 ? (lane >> 3) : (mode == 2 ? (lane >> 2) : 0u);
  uint32_t sg = blockIdx.x * 2654435761u + 777u + grp * 40503u;  // the same for the lanes of a group
  unsigned long long t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && lane == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f4 acc = (f4){0, 0, 0, 0};
  if ((int)lane < active) {
    for (int i = 0; i < iters; ++i) {
      if (mode == 0) {
        s = s * 1103515245u + 12345u;
        const f4 *p = tab + (size_t)((s >> 8) % nrec) * 8;
        f4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4], f = p[5], g = p[6];
        acc += a + b + c + d + e + f + g;
      } else {
        // 7 instructions, each touching one line per lane group
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          sg = sg * 1103515245u + 12345u;
          const uint32_t chunk = mode == 1 ? (lane & 7u) : (mode == 2 ? (lane & 3u) : (lane & 7u));
          acc += tab[(size_t)((sg >> 8) % nrec) * 8 + chunk];
        }
      }
    }
  }
  if (acc.x == 1.2345f) out[0] = acc.y;
  if (blockIdx.x == 0 && lane == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}
int main(int argc, char **argv) {
  const bool json = argc > 1 && std::strcmp(argv[1], "--json") == 0;
  uint32_t nrec = 16384;  // 2 MB of 128-B records (L2 resident)
  f4 *tab;
  float *out;
  unsigned long long *clk;
  if (hipMalloc(&tab, (size_t)nrec * 128) != hipSuccess || hipMemset(tab, 0, (size_t)nrec * 128) != hipSuccess ||
      hipMalloc(&out, 64) != hipSuccess || hipMalloc(&clk, 16) != hipSuccess) {
    std::fprintf(stderr, "setup failed\n");
    return 1;
  }
  int n_cu = 0;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = n_cu * 16;  // 16 waves per CU
  struct P {
    int mode, active;
  };
  const P pats[] = {{0, 64}, {0, 48}, {0, 32}, {0, 16}, {0, 8}, {0, 1}, {1, 64}, {1, 32}, {1, 16},
                    {1, 8},  {2, 64}, {2, 32}, {3, 64}};
  for (const P &p : pats) {
    const int iters = 200;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, tab, nrec, p.active, iters, p.mode, out, clk);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, tab, nrec, p.active, iters, p.mode, out, clk);
    (void)hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) {
      std::fprintf(stderr, "kernel failed\n");
      return 1;
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0.0;  // s_memrealtime: 100 MHz
    const double insts_per_cu = (double)grid * iters * 7 / n_cu;
    const int lines = p.mode == 0 ? p.active : (p.mode == 1 ? (p.active + 7) / 8 : (p.mode == 2 ? (p.active + 3) / 4 : 1));
    const double cyc = ms * 1e-3 * ghz * 1e9 / insts_per_cu;
    if (json)
      std::printf("{\"mode\": %d, \"active\": %d, \"lines\": %d, \"ms\": %.4f, \"clock_GHz\": %.4f, "
                  "\"insts_per_cu\": %.0f, \"cycles_per_inst\": %.3f}\n",
                  p.mode, p.active, lines, ms, ghz, insts_per_cu, cyc);
    else
      std::printf("mode %d active %2d lines %2d: %.3f ms at %.3f GHz, %.2f ns = %.1f cycles per wave-gather per CU\n",
                  p.mode, p.active, lines, ms, ghz, ms * 1e6 / insts_per_cu, cyc);
  }
  return 0;
}
