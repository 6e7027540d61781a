// Binned-SAH search tree for the EXACT path (see mcpt_bvh4.h).
//
// The reference searches its HLBVH (Morton-order median splits) left-first;
// the EXACT kernels search this tree nearest-first instead and prove, per
// ray, that the order cannot change the reference's answer (falling back to
// the reference tree when it could).  Only the search cost depends on this
// tree, so it is built for that: surface-area-heuristic splits over 32
// centroid bins per axis, collapsed to 4-wide nodes by an SAH-optimal
// dynamic programme, one reference leaf per slot.
#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <functional>
#include <thread>

#include "mcpt_bvh4.h"

#ifndef MCPT_SAH_BINS  // centroid bins per axis (A/B builds only: mcpt_upload.hip's GPU build uses 32 too)
#define MCPT_SAH_BINS 32
#endif
#ifndef MCPT_COLLAPSE_CTRI  // cost of a triangle test per node step in the collapse (A/B builds only)
#define MCPT_COLLAPSE_CTRI 1.7
#endif

namespace mcpt {
namespace {

struct BinNode {
  float box[6];
  int32_t left, right;  // children (binary node ids); -1 for a leaf
  int32_t item;         // leaf: index into the leaf list
};

struct Builder {
  const std::vector<LeafRef> &L;
  std::vector<float> cen;  // 3 per leaf
  std::vector<int32_t> idx;
  std::vector<BinNode> nodes;  // 2m-1, subtree of [lo,hi) at [base, base + 2(hi-lo)-1)
  int max_threads;

  explicit Builder(const std::vector<LeafRef> &l) : L(l) {}

  static void grow(float *b, const float *x) {
    for (int a = 0; a < 3; ++a) {
      b[2 * a] = std::min(b[2 * a], x[2 * a]);
      b[2 * a + 1] = std::max(b[2 * a + 1], x[2 * a + 1]);
    }
  }
  static void empty(float *b) {
    for (int a = 0; a < 3; ++a) b[2 * a] = FLT_MAX, b[2 * a + 1] = -FLT_MAX;
  }
  static double area(const float *b) {
    double dx = (double)b[1] - b[0], dy = (double)b[3] - b[2], dz = (double)b[5] - b[4];
    if (dx < 0) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }

  // returns the split position in idx (lo < mid < hi)
  int64_t split(int64_t lo, int64_t hi) {
    constexpr int NB = MCPT_SAH_BINS;
    float cmin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, cmax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = lo; i < hi; ++i) {
      const float *c = &cen[3 * (size_t)idx[i]];
      for (int a = 0; a < 3; ++a) cmin[a] = std::min(cmin[a], c[a]), cmax[a] = std::max(cmax[a], c[a]);
    }
    double best = DBL_MAX;
    int best_axis = -1, best_bin = -1;
    for (int a = 0; a < 3; ++a) {
      const float ext = cmax[a] - cmin[a];
      if (!(ext > 0)) continue;
      const float scale = NB / ext;
      float bb[NB][6];
      int64_t bc[NB];
      for (int k = 0; k < NB; ++k) empty(bb[k]), bc[k] = 0;
      for (int64_t i = lo; i < hi; ++i) {
        const int32_t it = idx[i];
        int k = std::min(NB - 1, (int)((cen[3 * (size_t)it + a] - cmin[a]) * scale));
        grow(bb[k], L[it].box);
        ++bc[k];
      }
      double left_cost[NB];
      float acc[6];
      empty(acc);
      int64_t cnt = 0;
      for (int k = 0; k < NB - 1; ++k) {
        grow(acc, bb[k]);
        cnt += bc[k];
        left_cost[k] = cnt ? area(acc) * (double)cnt : -1.0;
      }
      empty(acc);
      cnt = 0;
      for (int k = NB - 1; k > 0; --k) {
        grow(acc, bb[k]);
        cnt += bc[k];
        if (!cnt || left_cost[k - 1] < 0) continue;
        const double c = left_cost[k - 1] + area(acc) * (double)cnt;
        if (c < best) best = c, best_axis = a, best_bin = k;
      }
    }
    int64_t mid = (lo + hi) / 2;
    if (best_axis >= 0) {
      const int a = best_axis;
      const float scale = NB / (cmax[a] - cmin[a]);
      auto it = std::stable_partition(idx.begin() + lo, idx.begin() + hi, [&](int32_t t) {
        return std::min(NB - 1, (int)((cen[3 * (size_t)t + a] - cmin[a]) * scale)) < best_bin;
      });
      const int64_t m = it - idx.begin();
      if (m > lo && m < hi) mid = m;
    }
    return mid;
  }

  void build(int64_t lo, int64_t hi, int64_t base, int depth) {
    BinNode &n = nodes[base];
    if (hi - lo == 1) {
      std::memcpy(n.box, L[idx[lo]].box, sizeof(n.box));
      n.left = n.right = -1;
      n.item = idx[lo];
      return;
    }
    const int64_t mid = split(lo, hi);
    const int64_t lbase = base + 1, rbase = base + 2 * (mid - lo);
    // the two halves touch disjoint idx ranges and node ranges: safe to run in parallel
    if (depth < 16 && (1 << (depth + 1)) <= max_threads && hi - lo > 65536) {  // depth bound: no shift overflow (UBSan)
      std::thread t([&] { build(lo, mid, lbase, depth + 1); });
      build(mid, hi, rbase, depth + 1);
      t.join();
    } else {
      build(lo, mid, lbase, depth + 1);
      build(mid, hi, rbase, depth + 1);
    }
    n.left = (int32_t)lbase;
    n.right = (int32_t)rbase;
    n.item = -1;
    std::memcpy(n.box, nodes[lbase].box, sizeof(n.box));
    grow(n.box, nodes[rbase].box);
  }
};

}  // namespace

int build_sah4(const std::vector<LeafRef> &leaves, std::vector<Node4Rec> &out, int32_t *stack_need, int threads) {
  const int64_t m = (int64_t)leaves.size();
  out.clear();
  *stack_need = 1;
  if (m <= 0) return -1;
  Builder B(leaves);
  B.max_threads = std::max(1, threads);
  B.cen.resize(3 * (size_t)m);
  B.idx.resize((size_t)m);
  for (int64_t i = 0; i < m; ++i) {
    for (int a = 0; a < 3; ++a) B.cen[3 * i + a] = 0.5f * (leaves[i].box[2 * a] + leaves[i].box[2 * a + 1]);
    B.idx[i] = (int32_t)i;
  }
  B.nodes.resize(2 * (size_t)m - 1);
  B.build(0, m, 0, 0);
  if (m == 1) return 0;  // a single leaf: the kernels handle it without a node

  const std::vector<BinNode> &N = B.nodes;
  // collapse to 4-wide nodes, SAH-optimally (dynamic programme over the binary
  // tree): f[x][k] = the least cost of x's subtree as at most k slot entries,
  // where a wide node costs area x C_STEP plus its entries and a leaf entry
  // area x C_TRI (the ratio of the measured per-step and per-test times,
  // DESIGN.md §3.3).  Measured against opening the largest child greedily:
  // C2 -2.2 %, C4 -1.7 %, C3 / C5 unchanged (profiles/r02_quant_ab.txt).
  constexpr double C_STEP = 1.0, C_TRI = MCPT_COLLAPSE_CTRI;
  const size_t nn = N.size();
  std::vector<std::array<double, 5>> f(nn);
  std::vector<std::array<int8_t, 5>> cut(nn);  // split of f[x][k]: a entries left (0 = x itself is the entry)
  std::vector<std::array<int8_t, 2>> wide(nn);  // x as a wide node: entries from the left / right child
  for (int64_t x = (int64_t)nn - 1; x >= 0; --x) {  // children have larger ids than their parent
    const double sa = Builder::area(N[x].box);
    if (N[x].item >= 0) {
      for (int k = 1; k <= 4; ++k) f[x][k] = sa * C_TRI, cut[x][k] = 0;
      continue;
    }
    const int32_t l = N[x].left, r = N[x].right;
    double bw = DBL_MAX;
    for (int a = 1; a <= 3; ++a)
      for (int b = 1; a + b <= 4; ++b)
        if (f[l][a] + f[r][b] < bw) bw = f[l][a] + f[r][b], wide[x] = {(int8_t)a, (int8_t)b};
    f[x][1] = sa * C_STEP + bw;
    cut[x][1] = 0;
    for (int k = 2; k <= 4; ++k) {
      f[x][k] = f[x][k - 1];
      cut[x][k] = cut[x][k - 1];
      for (int a = 1; a < k; ++a)
        if (f[l][a] + f[r][k - a] < f[x][k]) f[x][k] = f[l][a] + f[r][k - a], cut[x][k] = (int8_t)a;
    }
  }
  // the entries (subtree roots) of x's subtree as at most k slots, left to right
  std::function<void(int32_t, int, int32_t *, int &)> entries = [&](int32_t x, int k, int32_t *e, int &ne) {
    const int a = cut[x][k];
    if (a == 0) {
      e[ne++] = x;
      return;
    }
    entries(N[x].left, a, e, ne);
    entries(N[x].right, k - a, e, ne);
  };
  // emit nodes in depth-first preorder
  struct Pending {
    int32_t bin, out;
  };
  std::vector<Pending> todo(1, Pending{0, 0});
  out.emplace_back();
  while (!todo.empty()) {
    const Pending p = todo.back();
    todo.pop_back();
    int32_t kids[4] = {-1, -1, -1, -1};
    int nk = 0;
    entries(N[p.bin].left, wide[p.bin][0], kids, nk);
    entries(N[p.bin].right, wide[p.bin][1], kids, nk);
    Node4Rec rec;
    std::memset(&rec, 0, sizeof(rec));
    int32_t child_out[4] = {-1, -1, -1, -1};
    for (int k = 0; k < 4; ++k) {
      if (k >= nk) {
        rec.link[k] = kEmptySlot4;
        continue;
      }
      const BinNode &c = N[kids[k]];
      std::memcpy(rec.q + 6 * k, c.box, sizeof(c.box));
      if (c.item >= 0) {
        rec.link[k] = ~leaves[c.item].tri;
      } else {
        child_out[k] = (int32_t)out.size();
        rec.link[k] = child_out[k];
        out.emplace_back();
      }
    }
    out[p.out] = rec;
    for (int k = nk - 1; k >= 0; --k)  // preorder: slot 0's subtree next
      if (child_out[k] >= 0) todo.push_back(Pending{kids[k], child_out[k]});
  }
  // children are allocated when their parent is emitted: ids only grow down the tree
  std::vector<int32_t> need(out.size(), 0);
  for (int64_t k = (int64_t)out.size() - 1; k >= 0; --k) {
    int ns = 0, below = 0;
    for (int s = 0; s < 4; ++s) {
      if (out[k].link[s] == kEmptySlot4) continue;
      ++ns;
      if (out[k].link[s] >= 0) below = std::max(below, need[out[k].link[s]]);
    }
    need[k] = ns - 1 + below;
  }
  *stack_need = std::max(need[0], 1);
  return 0;
}

// ------------------------------------------------------------ quantization
namespace {
// the device's decode: one fused multiply-add, one rounding
inline float qdec(int q, float s, float o) { return std::fma((float)q, s, o); }
inline bool normal_or_zero(float x) { return x == 0.0f || (std::isfinite(x) && std::fabs(x) >= FLT_MIN); }
}  // namespace

int quantize_node4(const Node4Rec &in, Node4Q &out) {
  std::memset(&out, 0, sizeof(out));
  float scale[3];
  for (int a = 0; a < 3; ++a) {
    float lo = FLT_MAX, hi = -FLT_MAX;
    for (int k = 0; k < 4; ++k) {
      if (in.link[k] == kEmptySlot4) continue;
      lo = std::min(lo, in.q[6 * k + 2 * a]);
      hi = std::max(hi, in.q[6 * k + 2 * a + 1]);
    }
    if (lo > hi) lo = hi = 0.0f;  // no slot (cannot happen for built trees)
    // origin strictly below every lower plane (q = 0 decodes to it exactly),
    // a normal float or zero (below 0 the next float down would be subnormal)
    float org = std::nextafter(lo, -FLT_MAX);
    if (!normal_or_zero(org)) org = -FLT_MIN;
    if (!normal_or_zero(org) || !std::isfinite(hi)) return -1;
    // the smallest power of two s with fma(255, s, org) > hi
    const double span = (double)hi - (double)org;
    int e = span > 0 ? (int)std::ceil(std::log2(span / 255.0)) : -126;
    e = std::max(-126, std::min(e, 127));
    while (e > -126 && qdec(255, std::ldexp(1.0f, e - 1), org) > hi) --e;
    while (e <= 127 && !(qdec(255, std::ldexp(1.0f, e), org) > hi)) ++e;
    if (e > 127) return -1;
    const float s = std::ldexp(1.0f, e);
    out.org[a] = org;
    scale[a] = s;
    for (int k = 0; k < 4; ++k) {
      uint8_t &ql = out.q[6 * k + 2 * a], &qh = out.q[6 * k + 2 * a + 1];
      if (in.link[k] == kEmptySlot4) {
        ql = 0;
        qh = 0;
        continue;
      }
      const float bl = in.q[6 * k + 2 * a], bh = in.q[6 * k + 2 * a + 1];
      // lo: the largest q whose decoded plane lies strictly below bl (q = 0 does)
      int q = (int)std::max(0.0, std::min(255.0, std::floor(((double)bl - (double)org) / s)));
      while (q > 0 && !(qdec(q, s, org) < bl)) --q;
      while (q < 255 && qdec(q + 1, s, org) < bl) ++q;
      while (q > 0 && !normal_or_zero(qdec(q, s, org))) --q;
      if (!(qdec(q, s, org) < bl) || !normal_or_zero(qdec(q, s, org))) return -1;
      ql = (uint8_t)q;
      // hi: the smallest q whose decoded plane lies strictly above bh (q = 255 does)
      q = (int)std::max(0.0, std::min(255.0, std::ceil(((double)bh - (double)org) / s)));
      while (q < 255 && !(qdec(q, s, org) > bh)) ++q;
      while (q > 0 && qdec(q - 1, s, org) > bh) --q;
      while (q < 255 && !normal_or_zero(qdec(q, s, org))) ++q;
      if (!(qdec(q, s, org) > bh) || !normal_or_zero(qdec(q, s, org))) return -1;
      qh = (uint8_t)q;
    }
  }
  out.sx = scale[0];
  out.sy = scale[1];
  out.sz = scale[2];
  for (int k = 0; k < 4; ++k) out.link[k] = in.link[k];
  return 0;
}

}  // namespace mcpt
