/* mcpt_oracle_treelet_gpu.cpp — TEST INFRASTRUCTURE ONLY: a sequential CPU
 * restatement of the reference's GPU treelet pass, TreeletBVH<GPU>
 * (MCPT/BVH/treeletBVH.cpp:413-438 launching MCPT/kernels/treeletBVH.cl:230-531
 * with one 32-lane work-group per triangle).  This is the tree every reference
 * render traverses: SceneCL's ctor falls through into its `GPUBVH:` block for
 * every bvhtype (MCPT/scenebuild.cpp:66-95), re-uploading a fresh HLBVH and
 * restructuring it in place with this kernel before intersect reads it
 * (:125).  The product's restatement is csrc/mcpt_treelet_gpu.hip; tests
 * compare the two node arrays bit for bit.
 *
 * PARITY UNPINNED: treeletBVH.cl does not compile with clang (`__local`
 * variables declared inside the non-kernel function pickNode, :80-81), so no
 * reference output exists to pin this restatement; DESIGN.md §3.9 lists the
 * assumptions below.
 *
 * Schedule.  Group g starts at leaf g+n-1 (:259-262) and walks up the CURRENT
 * parent links; at each node the first of the two arriving groups stops
 * (atomic_cmpxchg on flags, :273-277) and the second one processes it.  A
 * node's processing reads and writes only its own subtree, whose node-id set
 * a rebuild preserves (the treelet root keeps its id, freeBVHNode[0] = idx),
 * so every schedule in which a node follows its subtree gives the same tree.
 * Here: groups 0..n-1 one after the other, each running until it stops.
 *
 * Semantics taken from the kernel source, with the GPU's FP rules (ROCm's
 * OpenCL compiler for gfx950, the convention of every other reference kernel
 * in this repo: FP_CONTRACT on, min/max = IEEE minNum/maxNum, 2.5-ulp '/'):
 *  - AREA (:12-15) = 2 * fma(y, z, fma(x, y, x*z))   (clang's fmuladd chain);
 *  - x / rootArea = ldexp(frexp_mant(x) * rcp(frexp_mant(rootArea)), ex - er)
 *    (v_frexp_mant / v_rcp_f32 / v_mul / v_ldexp); rcp(mant(rootArea)) is a
 *    parameter because v_rcp_f32's rounding is the hardware's (the GPU tests
 *    pass the device's own value; CPU-only tests use the correctly rounded one);
 *  - leaf SAH (:261) = AREA / rootArea; SAH at arrival (:269-270) =
 *    (s_l + s_r) + (Cinn*AREA) / rootArea; the refit (:524-525) =
 *    fma(Cinn, AREA, s_l + s_r) — no /rootArea there;
 *  - subset DP (:310-330) for masks of <= 5 leaves: each mask's first strictly
 *    smaller cost in the (p - delta) & s enumeration, copt = fma(Cinn, a, cs);
 *    the kernel's round tables order every mask after its subsets (checked
 *    once against the tables);
 *  - 6-leaf masks (:336-359): the 31 partitions without the mask's lowest bit,
 *    one per lane, min-reduced; 7 leaves (:364-392): the 63 even masks, two per
 *    lane (4l+2 then 4l+4), min-reduced; lane 31's second candidate (mask 0,
 *    copt[0] never written) is taken never to equal the minimum.
 * Warp-synchronous semantics (the kernel's __local reductions have no barriers
 * and rely on 32 lanes in lockstep: every lane reads its operands before any
 * lane of the same instruction stores):
 *  - pickNode's argmax (:93-113) reduces sahvbuffer with lanes 0..3 only and
 *    then lets EACH of those lanes compare its own partial maximum with its
 *    own queue entry, so zero, one or several lanes store maxNodeID; with none
 *    it keeps the previous iteration's value;
 *  - when several lanes of one store instruction write the same __local word
 *    (maxNodeID, popt[63..127]), the highest lane's value lands (option bit 0
 *    set: the lowest lane's, for sensitivity tests).
 * Option bit 1 divides the refit SAH by rootArea like TreeletBVH<CPU>
 * (treeletBVH.cpp:292-293): NOT the reference kernel, a test knob that shows
 * what the missing /rootArea (treeletBVH.cl:524-525) changes.
 * Memory: sequentially consistent (the first arriver's SAH store is followed
 * by the second's); flags start at zero.
 */
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "mcpt_oracle.h"

namespace {

constexpr float Cinn = 1.2f;  // treeletBVH.cl:2-4 (Ctri + Cleaf = 1.0f)
constexpr int MAX_NODE = 7;   // :6

struct G {
  mcpt_bvh_node *nodes;
  std::vector<float> sah;
  float R;   // rcp(frexp_mant(rootArea)) as the GPU rounds it
  int er;    // frexp exponent of rootArea
  int lane_rule;
  bool refit_normalised;
  int64_t *st;
};

// IEEE minNum / maxNum on non-NaN inputs; an equal +-0 pair is counted (st[6])
// and resolved -0 for min, +0 for max.
float cl_min(G &g, float a, float b) {
  if (a < b) return a;
  if (b < a) return b;
  if (std::signbit(a) != std::signbit(b)) {
    if (g.st) ++g.st[6];
    return std::signbit(a) ? a : b;
  }
  return b;
}
float cl_max(G &g, float a, float b) {
  if (a > b) return a;
  if (b > a) return b;
  if (std::signbit(a) != std::signbit(b)) {
    if (g.st) ++g.st[6];
    return std::signbit(a) ? b : a;
  }
  return b;
}

float area(const float *mn, const float *mx) {  // AREA, :12-15, contracted
  const float x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
  return 2.0f * std::fma(y, z, std::fma(x, y, x * z));
}

float div_root(const G &g, float x) {  // x / rootArea, OpenCL 2.5-ulp division
  if (x == 0.0f || !std::isfinite(x)) return x == 0.0f ? x * g.R : x;
  int ex;
  const float m = std::frexp(x, &ex);
  return std::ldexp(m * g.R, ex - g.er);
}

struct Q {
  int id;
  float sah;
};

// pickNode (:65-142) as its 32 lanes execute it.  Returns sp; q[0..sp) and
// freeN[0..sp-1) filled.
int pick_node(G &g, int idx, Q *q, int *freeN) {
  for (int i = 0; i < MAX_NODE; ++i) q[i] = Q{0, 0.0f};  // `= {}` at :281
  int sp = 1;
  q[0] = Q{idx, g.sah[idx]};
  int maxNodeID = -1;  // __local, written below before its first read
  int nextFree = 0;
  while (sp < MAX_NODE) {
    if (sp == 1) {
      maxNodeID = 0;  // lane 0 (:88-91); lanes 1..3 never match (their window is -FLT_MAX, q[lid] 0)
    } else {
      float s[MAX_NODE + 1];
      for (int i = 0; i <= MAX_NODE; ++i) s[i] = i < sp ? q[i].sah : -FLT_MAX;  // :93-98
      // lanes 0..3 in lockstep: each statement reads before it writes (:100-109)
      const int strides3[3] = {4, 2, 1}, strides2[2] = {2, 1};
      const int *sd = sp < 4 ? strides2 : strides3;
      const int ns = sp < 4 ? 2 : 3;
      for (int k = 0; k < ns; ++k) {
        float nv[4];
        for (int l = 0; l < 4; ++l) nv[l] = cl_max(g, s[l], s[l + sd[k]]);
        for (int l = 0; l < 4; ++l) s[l] = nv[l];
      }
      int writers = 0, w = -1;
      for (int l = 0; l < 4; ++l) {  // :110-112, each lane against ITS OWN entry
        if (s[l] == q[l].sah) {
          ++writers;
          if (g.lane_rule == 0 || w < 0) w = l;
        }
      }
      if (writers > 0) maxNodeID = w;
      if (g.st) {
        if (writers > 1) ++g.st[1];
        if (writers == 0) ++g.st[2];
      }
    }
    if (q[maxNodeID].sah < 0.0f) break;  // :117-119
    const int id = q[maxNodeID].id;
    const int left = g.nodes[id].left, right = g.nodes[id].right;
    if (left == right) {  // :124-127
      q[maxNodeID].sah = -1.0f;
      continue;
    }
    q[maxNodeID] = Q{left, g.sah[left]};  // :129-134
    q[sp] = Q{right, g.sah[right]};
    ++sp;
    freeN[nextFree++] = id;
  }
  return sp;
}

// the rest of the loop body of reconstructTreelet (:286-527) for node idx
void rebuild(G &g, int idx) {
  Q q[MAX_NODE];
  int freeN[MAX_NODE - 1];
  const int size = pick_node(g, idx, q, freeN);
  if (size < 3) {  // :289-292
    if (g.st) ++g.st[5];
    return;
  }
  if (g.st) ++g.st[0];
  const int N = size, NB = (1 << N) - 1;
  float bmn[MAX_NODE][4], bmx[MAX_NODE][4];
  for (int i = 0; i < N; ++i) {  // :137-140
    std::memcpy(bmn[i], g.nodes[q[i].id].bbmin, 16);
    std::memcpy(bmx[i], g.nodes[q[i].id].bbmax, 16);
  }
  float a[128] = {}, copt[128] = {};
  int popt[128] = {};
  for (int m = 1; m <= NB; ++m) {  // calcUnionArea (:144-165): bit j <-> entry N-1-j
    float mn[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX}, mx[4] = {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    int mask = m, nowID = N - 1;
    while (mask > 0 && nowID >= 0) {
      if (mask & 1)
        for (int k = 0; k < 4; ++k) {
          mn[k] = cl_min(g, bmn[nowID][k], mn[k]);
          mx[k] = cl_max(g, bmx[nowID][k], mx[k]);
        }
      --nowID;
      mask >>= 1;
    }
    a[m] = area(mn, mx);
  }
  for (int l = 0; l < N; ++l) copt[1 << l] = g.sah[q[l].id];  // :304-306: bit l <-> entry l
  // masks of 2..min(N,5) leaves (:310-330), in popcount order (= the rounds' dependency order)
  for (int k = 2; k <= (N < 5 ? N : 5); ++k)
    for (int part = 1; part <= NB; ++part) {
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
      copt[part] = std::fma(Cinn, a[part], cs);
      popt[part] = ps;
    }
  if (N >= 6) {  // 6 leaves (:336-359)
    for (int M = 63; M <= NB; ++M) {
      if (__builtin_popcount(M) != 6) continue;
      const int low = M & -M;
      int parts[31], np = 0;
      for (int u = 1; u < M; ++u)
        if ((u & M) == u && !(u & low)) parts[np++] = u;  // roundSixPart: increasing, lane = rank
      float c[31], mn = FLT_MAX;
      for (int l = 0; l < 31; ++l) {
        c[l] = copt[parts[l]] + copt[parts[l] ^ M];
        mn = cl_min(g, mn, c[l]);
      }
      int w = -1, ties = 0;
      for (int l = 0; l < 31; ++l)
        if (c[l] == mn) {
          ++ties;
          if (g.lane_rule == 0 || w < 0) w = l;
        }
      if (g.st && ties > 1) ++g.st[3];
      copt[M] = std::fma(Cinn, a[M], mn);
      popt[M] = parts[w];
    }
  }
  if (N == 7) {  // 7 leaves (:364-392)
    float c1[32], c2[32], mn = FLT_MAX;
    for (int l = 0; l < 32; ++l) {
      const int t1 = 4 * l + 2, t2 = 4 * l + 4;
      c1[l] = copt[t1] + copt[127 - t1];
      mn = cl_min(g, mn, c1[l]);
      if (l < 31) {
        c2[l] = copt[t2] + copt[127 - t2];
        mn = cl_min(g, mn, c2[l]);
      }
    }
    int w = -1, wm = 0, ties = 0;
    for (int l = 0; l < 32; ++l) {
      int m = 0;
      if (c1[l] == mn) m = 4 * l + 2;
      else if (l < 31 && c2[l] == mn) m = 4 * l + 4;
      if (m) {
        ++ties;
        if (g.lane_rule == 0 || w < 0) w = l, wm = m;
      }
    }
    if (g.st && ties > 1) ++g.st[4];
    copt[127] = std::fma(Cinn, a[127], mn);
    popt[127] = wm;
  }
  // reconstruct (:438-501), lane 0
  struct Split {
    int parentCode, selfCode, parentID;
  };
  Split b1[MAX_NODE], b2[MAX_NODE];
  Split *toSplit = b1, *back = b2;
  toSplit[0] = Split{NB, popt[NB], freeN[0]};
  int toSP = 1, toSPBack = 0, freeNodeNow = 1;
  mcpt_bvh_node *nodes = g.nodes;
  while (toSP > 0) {
    for (int x = 0; x < toSP; ++x) {
      const Split i = toSplit[x];
      const int leftCode = popt[i.selfCode];
      const int rightCode = popt[i.selfCode ^ i.parentCode];
      const int pid = i.parentID;
      if (__builtin_popcount(i.selfCode) == 1) {
        const int node = q[N - (31 - __builtin_clz((unsigned)i.selfCode)) - 1].id;
        nodes[pid].left = node;
        nodes[node].parent = pid;
      } else {
        const int f = freeN[freeNodeNow++];
        back[toSPBack++] = Split{i.selfCode, leftCode, f};
        nodes[pid].left = f;
        nodes[f].parent = pid;
      }
      const int rc = i.selfCode ^ i.parentCode;
      if (__builtin_popcount(rc) == 1) {
        const int node = q[N - (31 - __builtin_clz((unsigned)rc)) - 1].id;
        nodes[pid].right = node;
        nodes[node].parent = pid;
      } else {
        const int f = freeN[freeNodeNow++];
        back[toSPBack++] = Split{rc, rightCode, f};
        nodes[pid].right = f;
        nodes[f].parent = pid;
      }
    }
    Split *t = toSplit;
    toSplit = back;
    back = t;
    toSP = toSPBack;
    toSPBack = 0;
  }
  // refit (:519-527): no /rootArea
  for (int i = N - 2; i >= 0; --i) {
    mcpt_bvh_node &P = nodes[freeN[i]];
    const mcpt_bvh_node &L = nodes[P.left], &Rn = nodes[P.right];
    for (int k = 0; k < 4; ++k) {
      P.bbmin[k] = cl_min(g, L.bbmin[k], Rn.bbmin[k]);
      P.bbmax[k] = cl_max(g, L.bbmax[k], Rn.bbmax[k]);
    }
    if (g.refit_normalised)  // option bit 1 (not the kernel): treeletBVH.cpp:292-293's form
      g.sah[freeN[i]] = g.sah[P.left] + g.sah[P.right] + div_root(g, Cinn * area(P.bbmin, P.bbmax));
    else
      g.sah[freeN[i]] = std::fma(Cinn, area(P.bbmin, P.bbmax), g.sah[P.left] + g.sah[P.right]);
  }
}

}  // namespace

/* stats (optional, 8 entries): [0] treelets rebuilt, [1] pickNode steps where
 * several lanes stored maxNodeID, [2] steps where none did (stale value kept),
 * [3] 6-leaf masks with tied partitions, [4] 7-leaf roots with ties, [5] nodes
 * skipped (treelet < 3 leaves), [6] +-0 min/max ties, [7] unused. */
extern "C" int oracle_treelet_gpu(mcpt_bvh_node *nodes, int64_t n_nodes, uint32_t rcp_mant_root_bits,
                                  int32_t options, int64_t *stats) {
  if (!nodes || n_nodes <= 0 || (n_nodes & 1) == 0 || (options & ~3)) return -2;
  const int64_t n = (n_nodes + 1) / 2;
  if (stats) std::memset(stats, 0, 8 * sizeof(int64_t));
  G g;
  g.nodes = nodes;
  g.lane_rule = options & 1;
  g.refit_normalised = (options & 2) != 0;
  g.st = stats;
  g.sah.assign(n_nodes, 0.0f);
  const float rootArea = area(nodes[0].bbmin, nodes[0].bbmax);  // :245
  const float m = std::frexp(rootArea, &g.er);
  if (rcp_mant_root_bits) std::memcpy(&g.R, &rcp_mant_root_bits, 4);
  else g.R = (float)(1.0L / (long double)m);
  std::vector<int> flags(n, 0);  // flags[] indexed by internal node id (< n-1)
  for (int64_t grp = 0; grp < n; ++grp) {
    int idx = (int)(grp + n - 1);
    g.sah[idx] = div_root(g, area(nodes[idx].bbmin, nodes[idx].bbmax));  // :261 (1.0f * AREA)
    idx = nodes[idx].parent;
    while (idx != -1) {
      if (idx < 0 || idx >= n - 1) return -1;  // not a 2n-1 LBVH layout
      const mcpt_bvh_node &b = nodes[idx];
      g.sah[idx] = (g.sah[b.left] + g.sah[b.right]) + div_root(g, Cinn * area(b.bbmin, b.bbmax));  // :269-270
      if (flags[idx] != 1) {  // atomic_cmpxchg(flags+idx, 0, 1) != 1: first arrival stops
        flags[idx] = 1;
        break;
      }
      rebuild(g, idx);
      idx = nodes[idx].parent;  // :528
    }
  }
  return 0;
}

/* frexp mantissa of AREA(nodes[0]) (treeletBVH.cl:245), for the caller that
 * asks the GPU for its v_rcp_f32 of it. */
extern "C" float oracle_treelet_gpu_root_mant(const mcpt_bvh_node *root) {
  int e;
  return std::frexp(area(root->bbmin, root->bbmax), &e);
}
