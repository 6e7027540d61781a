// mcpt_treelet_gpu.hip — TreeletBVH<GPU>: the reference's GPU treelet pass
// (MCPT/BVH/treeletBVH.cpp:413-438 launching MCPT/kernels/treeletBVH.cl:230-531),
// restated deterministically for gfx950.
//
// Why it matters: SceneCL's ctor falls through into its `GPUBVH:` block for
// EVERY bvhtype (MCPT/scenebuild.cpp:66-95: "hlbvh" and "treelet" upload their
// tree, then fall through; "treeletGPU" jumps there), so the tree the
// reference's intersect kernel reads (:125) is always a fresh HLBVH
// restructured in place by this kernel.  Traversal order decides near-tie
// winners (objdef.h:213), so rendering the reference's image needs this tree.
//
// The kernel's result depends on warp-synchronous behaviour; the semantics
// restated here (DESIGN.md §3.9 has the full list; the CPU restatement
// oracle/mcpt_oracle_treelet_gpu.cpp follows the kernel line by line):
//  * the result is schedule-independent: a node is processed once, after its
//    subtree, and its processing touches only its subtree (whose node-id set a
//    rebuild keeps), so the 32-lane group per leaf walking up with atomic flags
//    becomes one launch per ORIGINAL depth, deepest first, one wave per node;
//  * SAH at arrival (:269-270) = (s_l + s_r) + (Cinn*AREA)/rootArea, leaves
//    AREA/rootArea (:261); the refit (:524-525) = fma(Cinn, AREA, s_l + s_r),
//    WITHOUT /rootArea, so rebuilt nodes carry un-normalised costs that later
//    treelet choices compare against normalised ones;
//  * pickNode's argmax (:93-113): lanes 0..3 reduce in lockstep, then each
//    compares ITS OWN partial maximum with ITS OWN queue entry; zero, one or
//    several store maxNodeID (highest lane's store lands; none keeps the
//    previous value); the queue is a plain array (expanded entry replaced by
//    the left child, right child appended);
//  * subset DP: masks of <= 5 leaves as the CPU pass (first strict minimum
//    in the (p - delta) & s order); 6 leaves: the 31 partitions without the
//    mask's lowest bit, wave min, the highest tying lane's partition; 7: the
//    63 even masks two per lane (4l+2 before 4l+4), same tie rule;
//  * FP as ROCm's OpenCL compiler builds the kernel for gfx950 (the rule for
//    every reference kernel here): AREA = 2*fma(y,z,fma(x,y,x*z)), DP costs
//    fma(Cinn, a, cs), min/max = v_min/v_max, x / rootArea =
//    ldexp(frexp_mant(x) * v_rcp(frexp_mant(rootArea)), ex - er).
// Compiled with the device flags (Makefile DEVFLAGS); every fused operation
// is written as an explicit fma, so no contraction decides a bit here.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <string>
#include <vector>

#include "../../include/mcpt_hip.h"

namespace mcpt {
int fail(int code, const std::string &msg);  // mcpt_host.cpp
int tree_levels(const mcpt_bvh_node *nodes, int64_t n, hipStream_t st, int32_t *lv, uint32_t *cnt,
                std::vector<uint32_t> &off);  // mcpt_build.hip
}  // namespace mcpt

namespace {

constexpr int TG_MAX = 7;          // treeletBVH.cl:6
constexpr float TG_CINN = 1.2f;    // :2 (Ctri + Cleaf = 1.0f)

struct RootDiv {
  float root_area;  // AREA(nodes[0]) (:245)
  float rcp_mant;   // v_rcp_f32(frexp_mant(rootArea))
  int exp;          // frexp_exp(rootArea)
  int err;          // layout check result
};

__device__ inline float tg_area(const float *mn, const float *mx) {  // AREA (:12-15), contracted
  const float x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
  return 2.0f * __builtin_fmaf(y, z, __builtin_fmaf(x, y, x * z));
}
__device__ inline float tg_div(const RootDiv &r, float x) {  // x / rootArea, OpenCL 2.5-ulp '/'
  const float m = __builtin_amdgcn_frexp_mantf(x);
  const int e = __builtin_amdgcn_frexp_expf(x);
  return __builtin_amdgcn_ldexpf(m * r.rcp_mant, e - r.exp);
}
__device__ inline int pdep5(int k, int mask) {  // k-th (1-based) subset of `mask`, increasing order
  int r = 0;
  for (int b = 0; b < 7; ++b)
    if (mask & (1 << b)) {
      if (k & 1) r |= 1 << b;
      k >>= 1;
    }
  return r;
}
__device__ inline float wave_min(float v) {
  for (int o = 32; o > 0; o >>= 1) v = __builtin_fminf(v, __shfl_xor(v, o, 64));
  return v;
}

// the 2n-1 HLBVH layout the kernel assumes: internal [0, n-2], leaves [n-1, 2n-2]
__global__ void k_tg_check(const mcpt_bvh_node *__restrict__ nodes, int64_t n, RootDiv *rd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * n - 1) return;
  const mcpt_bvh_node &b = nodes[i];
  const bool leaf = b.left == b.right;
  bool bad = leaf != (i >= n - 1);
  if (!leaf) bad |= b.left < 0 || b.left >= 2 * n - 1 || b.right < 0 || b.right >= 2 * n - 1;
  if (bad) atomicOr(&rd->err, 1);
}

__global__ void k_tg_init(const mcpt_bvh_node *__restrict__ nodes, RootDiv *rd) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float ra = tg_area(nodes[0].bbmin, nodes[0].bbmax);
  rd->root_area = ra;
  rd->rcp_mant = __builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(ra));
  rd->exp = __builtin_amdgcn_frexp_expf(ra);
}

__global__ void k_tg_leaves(const mcpt_bvh_node *__restrict__ nodes, int64_t n, const RootDiv *__restrict__ rdp,
                            float *sah) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + n - 1;  // [n-1, 2n-2] (:259-261)
  if (i > 2 * n - 2) return;
  sah[i] = tg_div(*rdp, tg_area(nodes[i].bbmin, nodes[i].bbmax));
}

// one depth of internal nodes, one 64-lane wave per node: the loop body of
// reconstructTreelet (:265-528) run by the group that arrives second
__global__ __launch_bounds__(64) void k_tg_level(const int32_t *__restrict__ lvl, uint32_t count, mcpt_bvh_node *nodes,
                                                 float *sah, const RootDiv *__restrict__ rdp) {
  __shared__ int qid[TG_MAX];
  __shared__ int freeN[TG_MAX - 1];
  __shared__ int size_s;
  __shared__ float a[128], copt[128];
  __shared__ int popt[128];
  __shared__ float bmn[TG_MAX][4], bmx[TG_MAX][4];
  if (blockIdx.x >= count) return;
  const int lane = threadIdx.x;
  const int X = lvl[blockIdx.x];
  const RootDiv rd = *rdp;

  if (lane == 0) {
    const mcpt_bvh_node &b = nodes[X];
    sah[X] = (sah[b.left] + sah[b.right]) + tg_div(rd, TG_CINN * tg_area(b.bbmin, b.bbmax));  // :269-270
    // pickNode (:65-142) as its 32 lanes run it
    int id_[TG_MAX];
    float sv[TG_MAX];
    for (int i = 0; i < TG_MAX; ++i) id_[i] = 0, sv[i] = 0.0f;  // `= {}` (:281)
    id_[0] = X;
    sv[0] = sah[X];
    int sp = 1, m = 0, nf = 0;
    while (sp < TG_MAX) {
      if (sp == 1) {
        m = 0;
      } else {
        float s[TG_MAX + 1];
        for (int i = 0; i <= TG_MAX; ++i) s[i] = i < sp ? sv[i] : -FLT_MAX;
        const int ns = sp < 4 ? 2 : 3;
        int sd = sp < 4 ? 2 : 4;
        for (int k = 0; k < ns; ++k, sd >>= 1) {  // lockstep: reads before writes
          float nv[4];
          for (int l = 0; l < 4; ++l) nv[l] = __builtin_fmaxf(s[l], s[l + sd]);
          for (int l = 0; l < 4; ++l) s[l] = nv[l];
        }
        for (int l = 0; l < 4; ++l)  // each lane vs its own entry; the highest store lands
          if (s[l] == sv[l]) m = l;
      }
      if (sv[m] < 0.0f) break;
      const int id = id_[m];
      const int l = nodes[id].left, r = nodes[id].right;
      if (l == r) {
        sv[m] = -1.0f;
        continue;
      }
      id_[m] = l;
      sv[m] = sah[l];
      id_[sp] = r;
      sv[sp] = sah[r];
      ++sp;
      freeN[nf++] = id;
    }
    for (int i = 0; i < TG_MAX; ++i) qid[i] = id_[i];
    size_s = sp;
  }
  __syncthreads();
  const int N = size_s;
  if (N < 3) return;  // :289-292
  const int NB = (1 << N) - 1;
  if (lane < N) {
    const mcpt_bvh_node &q = nodes[qid[lane]];
    for (int k = 0; k < 4; ++k) bmn[lane][k] = q.bbmin[k], bmx[lane][k] = q.bbmax[k];
    copt[1 << lane] = sah[qid[lane]];  // :304-306: bit l <-> entry l
  }
  __syncthreads();
  for (int s = lane + 1; s <= NB; s += 64) {  // calcUnionArea (:144-165): bit j <-> entry N-1-j
    float mn[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX}, mx[4] = {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    int mask = s, now = N - 1;
    while (mask > 0 && now >= 0) {
      if (mask & 1)
        for (int k = 0; k < 4; ++k) {
          mn[k] = __builtin_fminf(bmn[now][k], mn[k]);
          mx[k] = __builtin_fmaxf(bmx[now][k], mx[k]);
        }
      --now;
      mask >>= 1;
    }
    a[s] = tg_area(mn, mx);
  }
  __syncthreads();
  const int kmax = N < 5 ? N : 5;
  for (int k = 2; k <= kmax; ++k) {  // (:310-330), one popcount class per step
    for (int part = lane + 1; part <= NB; part += 64) {
      if (__builtin_popcount(part) != k) continue;
      float cs = FLT_MAX;
      int ps = 0;
      const int delta = (part - 1) & part;
      int p = (-delta) & part;
      do {
        const float c = copt[p] + copt[part ^ p];
        if (c < cs) {
          cs = c;
          ps = p;
        }
        p = (p - delta) & part;
      } while (p != 0);
      copt[part] = __builtin_fmaf(TG_CINN, a[part], cs);
      popt[part] = ps;
    }
    __syncthreads();
  }
  if (N >= 6) {  // 6 leaves (:336-359)
    for (int M = 63; M <= NB; ++M) {
      if (__builtin_popcount(M) != 6) continue;
      const int rest = M & (M - 1);  // the mask without its lowest bit
      const int part = lane < 31 ? pdep5(lane + 1, rest) : 0;
      const float c = lane < 31 ? copt[part] + copt[part ^ M] : FLT_MAX;
      const float mn = wave_min(c);
      const unsigned long long tie = __ballot(lane < 31 && c == mn);
      const int w = 63 - __builtin_clzll(tie);
      if (lane == 0) {
        copt[M] = __builtin_fmaf(TG_CINN, a[M], mn);
        popt[M] = pdep5(w + 1, rest);
      }
    }
    __syncthreads();
  }
  if (N == 7) {  // 7 leaves (:364-392)
    const int t1 = 4 * lane + 2, t2 = 4 * lane + 4;
    const float c1 = lane < 32 ? copt[t1] + copt[127 - t1] : FLT_MAX;
    const float c2 = lane < 31 ? copt[t2] + copt[127 - t2] : FLT_MAX;
    const float mn = wave_min(__builtin_fminf(c1, c2));
    const unsigned long long m1 = __ballot(lane < 32 && c1 == mn);
    const unsigned long long m2 = __ballot(lane < 31 && c2 == mn);
    const int w = 63 - __builtin_clzll(m1 | m2);
    if (lane == 0) {
      copt[127] = __builtin_fmaf(TG_CINN, a[127], mn);
      popt[127] = ((m1 >> w) & 1) ? 4 * w + 2 : 4 * w + 4;
    }
    __syncthreads();
  }
  if (lane != 0) return;
  // reconstruct (:438-501)
  struct Split {
    int parent_code, self_code, parent_id;
  };
  Split b1[TG_MAX], b2[TG_MAX];
  Split *cur = b1, *nxt = b2;
  int ncur = 1, nnxt = 0, fnow = 1;
  cur[0] = Split{NB, popt[NB], freeN[0]};
  while (ncur > 0) {
    for (int x = 0; x < ncur; ++x) {
      const Split i = cur[x];
      const int lcode = popt[i.self_code], rcode = popt[i.self_code ^ i.parent_code];
      const int pid = i.parent_id;
      if (__builtin_popcount(i.self_code) == 1) {
        const int node = qid[N - (31 - __builtin_clz((unsigned)i.self_code)) - 1];
        nodes[pid].left = node;
        nodes[node].parent = pid;
      } else {
        const int f = freeN[fnow++];
        nxt[nnxt++] = Split{i.self_code, lcode, f};
        nodes[pid].left = f;
        nodes[f].parent = pid;
      }
      const int rc = i.self_code ^ i.parent_code;
      if (__builtin_popcount(rc) == 1) {
        const int node = qid[N - (31 - __builtin_clz((unsigned)rc)) - 1];
        nodes[pid].right = node;
        nodes[node].parent = pid;
      } else {
        const int f = freeN[fnow++];
        nxt[nnxt++] = Split{rc, rcode, f};
        nodes[pid].right = f;
        nodes[f].parent = pid;
      }
    }
    Split *t = cur;
    cur = nxt;
    nxt = t;
    ncur = nnxt;
    nnxt = 0;
  }
  for (int i = N - 2; i >= 0; --i) {  // refit (:519-527)
    mcpt_bvh_node &P = nodes[freeN[i]];
    const mcpt_bvh_node &A = nodes[P.left], &B = nodes[P.right];
    for (int k = 0; k < 4; ++k) {
      P.bbmin[k] = __builtin_fminf(A.bbmin[k], B.bbmin[k]);
      P.bbmax[k] = __builtin_fmaxf(A.bbmax[k], B.bbmax[k]);
    }
    sah[freeN[i]] = __builtin_fmaf(TG_CINN, tg_area(P.bbmin, P.bbmax), sah[P.left] + sah[P.right]);
  }
}

inline unsigned tg_blocks(int64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

#define TG_OK(expr)                                                                                  \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) {                                                                          \
      rc = mcpt::fail(MCPT_ERR_HIP, std::string("treelet_gpu_device: ") + #expr + ": " + hipGetErrorString(e_)); \
      goto done;                                                                                     \
    }                                                                                                \
  } while (0)

extern "C" int mcpt_treelet_gpu_device(mcpt_bvh_node *nodes, int64_t n_nodes, void *stream) {
  if (!nodes || n_nodes <= 0 || (n_nodes & 1) == 0)
    return mcpt::fail(MCPT_ERR_ARG, "treelet_gpu_device: expected a 2n-1-node BVH");
  const int64_t n = (n_nodes + 1) / 2;
  if (n < 2) return MCPT_OK;  // one leaf: its group finds no parent (:262-264)
  if (n > (int64_t)0x3FFFFFFF) return mcpt::fail(MCPT_ERR_LIMIT, "treelet_gpu_device: too many triangles");
  hipStream_t st = (hipStream_t)stream;
  int rc = MCPT_OK;
  float *sah = nullptr;
  int32_t *lv = nullptr;
  uint32_t *cnt = nullptr;
  RootDiv *rd = nullptr;
  RootDiv rd_h;
  std::vector<uint32_t> off;

  TG_OK(hipMalloc(&sah, n_nodes * sizeof(float)));
  TG_OK(hipMalloc(&lv, (n - 1) * sizeof(int32_t)));
  TG_OK(hipMalloc(&cnt, sizeof(uint32_t)));
  TG_OK(hipMalloc(&rd, sizeof(RootDiv)));
  TG_OK(hipMemsetAsync(rd, 0, sizeof(RootDiv), st));
  hipLaunchKernelGGL(k_tg_check, dim3(tg_blocks(n_nodes, 256)), dim3(256), 0, st, nodes, n, rd);
  TG_OK(hipGetLastError());
  TG_OK(hipMemcpyAsync(&rd_h, rd, sizeof(RootDiv), hipMemcpyDeviceToHost, st));
  TG_OK(hipStreamSynchronize(st));
  if (rd_h.err) {
    rc = mcpt::fail(MCPT_ERR_ARG,
                    "treelet_gpu_device: not an HLBVH layout (internal nodes [0, n-2], leaves [n-1, 2n-2])");
    goto done;
  }
  rc = mcpt::tree_levels(nodes, n, st, lv, cnt, off);  // depth groups, top-down
  if (rc != MCPT_OK) goto done;
  hipLaunchKernelGGL(k_tg_init, dim3(1), dim3(64), 0, st, nodes, rd);
  TG_OK(hipGetLastError());
  hipLaunchKernelGGL(k_tg_leaves, dim3(tg_blocks(n, 256)), dim3(256), 0, st, nodes, n, rd, sah);
  TG_OK(hipGetLastError());
  for (size_t k = off.size() - 1; k-- > 0;) {  // deepest depth first
    const uint32_t a = off[k], b = off[k + 1];
    if (b == a) continue;
    hipLaunchKernelGGL(k_tg_level, dim3(b - a), dim3(64), 0, st, lv + a, b - a, nodes, sah, rd);
    TG_OK(hipGetLastError());
  }
  TG_OK(hipStreamSynchronize(st));
done:
  for (void *p : {(void *)sah, (void *)lv, (void *)cnt, (void *)rd})
    if (p) (void)hipFree(p);
  return rc;
}

// TreeletBVH<GPU>(bvhBuffer, trBuffer) as a reference host calls it on host
// data (scenebuild.cpp:89-94, bvhtest.cpp:503-511): upload, restructure in
// HBM, read back, on the calling thread's current device.
extern "C" int mcpt_treelet_gpu(mcpt_bvh_node *nodes, int64_t n_nodes) {
  if (!nodes || n_nodes <= 0) return mcpt::fail(MCPT_ERR_ARG, "treelet_gpu: bad argument");
  int rc = MCPT_OK;
  mcpt_bvh_node *d = nullptr;
  const size_t bytes = (size_t)n_nodes * sizeof(mcpt_bvh_node);
  TG_OK(hipMalloc(&d, bytes));
  TG_OK(hipMemcpy(d, nodes, bytes, hipMemcpyHostToDevice));
  rc = mcpt_treelet_gpu_device(d, n_nodes, nullptr);
  if (rc != MCPT_OK) goto done;
  TG_OK(hipMemcpy(nodes, d, bytes, hipMemcpyDeviceToHost));
done:
  if (d) (void)hipFree(d);
  return rc;
}
