// tools/wide8.h — the 8-wide search tree of the round-6 experiment (DESIGN.md
// §3.3 "An 8-wide search tree: built, bit-exact, slower; removed"): not part of
// the product.  The library shipped it as a node format for one build (commit
// 609e80b: DevNode8, step8, mcpt_tuning.wide_nodes); it measured slower on every
// workload and was taken out.  Kept here for tools/wide_order_sim.cpp.
#pragma once
#include <algorithm>
#include <array>
#include <cfloat>
#include <cstring>
#include <functional>
#include <vector>

#include "mcpt_bvh4.h"

namespace mcpt {
namespace wide8 {

inline double area(const float *b) {
  double dx = (double)b[1] - b[0], dy = (double)b[3] - b[2], dz = (double)b[5] - b[4];
  if (dx < 0) return 0.0;
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}

// 256-B 8-wide node of the same search tree (DevNode8): slot k's box is
// q[6k..6k+5] in Node4Rec's plane order, link as Node4Rec's.  Fourteen 16-B
// gathers per step (the last 32 B are padding: two 128-B lines per node).
struct Node8Rec {
  float q[48];
  int32_t link[8];
  float pad[8];
};
static_assert(sizeof(Node8Rec) == 256, "DevNode8 layout");

// The 4-wide search tree widened to 8 slots: an SAH-optimal choice of which
// internal slots of each 4-wide node to open (splice their slots in place), a
// dynamic programme over the 4-wide tree with build_sah4's costs.  Every slot
// keeps the 4-wide slot's box bit for bit, so each leaf keeps the reference
// leaf's own box and every internal box is still a union of leaf boxes
// (DESIGN.md §3.3); slots stay in the 4-wide tree's left-to-right order.
// A pure function of the 4-wide tree: both upload paths, whose 4-wide trees
// are byte-identical, get the same 8-wide bytes.  Nodes in depth-first
// preorder (root = 0); *stack_need as build_sah4's.  Returns 0, or -1 for an
// empty input.
inline int widen_sah8(const std::vector<Node4Rec> &in, std::vector<Node8Rec> &out, int32_t *stack_need) {
  constexpr int K = 8;
  const int64_t n = (int64_t)in.size();
  out.clear();
  *stack_need = 1;
  if (n <= 0) return -1;
  auto slot_area = [&](int64_t y, int s) { return area(in[(size_t)y].q + 6 * s); };
  auto slots_of = [&](int64_t y) {
    int ns = 0;
    while (ns < 4 && in[(size_t)y].link[ns] != kEmptySlot4) ++ns;
    return ns;
  };
  for (int64_t y = 0; y < n; ++y)  // children after their parent (preorder ids), no empty slot before a used one
    for (int s = 0; s < 4; ++s) {
      const int32_t l = in[(size_t)y].link[s];
      if (l >= 0 && (l <= y || l >= n)) return -1;
      if (l == kEmptySlot4 && s + 1 < 4 && in[(size_t)y].link[s + 1] != kEmptySlot4) return -1;
    }
  // open[y][k]: the least cost of 4-wide node y's slots spliced into a parent
  // as at most k entries (INF below y's slot count); whole[c][k]: the cost of
  // the subtree under a slot whose child is c as at most k entries -- c kept
  // as one entry (an 8-wide node of its own: its area, one step, plus
  // open[c][K]) or opened.  Leaf entries cost the same in every choice (each
  // leaf is one entry exactly once), so only the node steps' areas are summed:
  // the SAH expectation of 8-wide node visits.
  constexpr double INF = DBL_MAX / 4;
  std::vector<std::array<double, K + 1>> open((size_t)n), whole((size_t)n);
  std::vector<std::array<uint16_t, K + 1>> allot((size_t)n);  // 4 bits per slot: entries given to it
  for (int64_t y = n - 1; y >= 0; --y) {
    const Node4Rec &r = in[(size_t)y];
    const int ns = slots_of(y);
    // whole[] of y's internal children: the slot box is the child's box
    for (int s = 0; s < ns; ++s) {
      const int32_t c = r.link[s];
      if (c < 0) continue;
      const double kept = slot_area(y, s) + open[(size_t)c][K];
      for (int k = 1; k <= K; ++k) whole[(size_t)c][k] = std::min(kept, open[(size_t)c][k]);
    }
    // cost[s][k] of slot s given at most k entries
    double cost[4][K + 1];
    for (int s = 0; s < ns; ++s)
      for (int k = 1; k <= K; ++k) cost[s][k] = r.link[s] < 0 ? 0.0 : whole[(size_t)r.link[s]][k];
    // knapsack over the slots in order: best[j][k] = slots 0..j-1 in at most k entries
    double best[5][K + 1];
    uint16_t how[5][K + 1];
    for (int k = 0; k <= K; ++k) best[0][k] = 0.0, how[0][k] = 0;
    for (int j = 1; j <= ns; ++j)
      for (int k = 0; k <= K; ++k) {
        best[j][k] = INF;
        how[j][k] = 0;
        for (int a = 1; a <= k - (j - 1); ++a) {
          const double c = best[j - 1][k - a] + cost[j - 1][a];
          if (c < best[j][k]) best[j][k] = c, how[j][k] = (uint16_t)(how[j - 1][k - a] | (a << (4 * (j - 1))));
        }
      }
    for (int k = 1; k <= K; ++k) open[(size_t)y][k] = best[ns][k], allot[(size_t)y][k] = how[ns][k];
  }
  // emit: an 8-wide node per kept 4-wide node, in depth-first preorder
  struct Entry {
    const float *box;
    int32_t link;  // leaf (~tri), or a 4-wide node kept as one entry
  };
  std::function<void(int64_t, int, std::vector<Entry> &)> entries = [&](int64_t y, int k, std::vector<Entry> &e) {
    const Node4Rec &r = in[(size_t)y];
    const uint16_t al = allot[(size_t)y][k];
    for (int s = 0; s < slots_of(y); ++s) {
      const int ks = (al >> (4 * s)) & 15;
      const int32_t c = r.link[s];
      if (c < 0 || ks == 1 || !(open[(size_t)c][ks] < slot_area(y, s) + open[(size_t)c][K]))
        e.push_back(Entry{r.q + 6 * s, c});
      else
        entries(c, ks, e);
    }
  };
  struct Pending {
    int64_t y4;
    int32_t out;
  };
  std::vector<Pending> todo(1, Pending{0, 0});
  out.emplace_back();
  std::vector<Entry> e;
  while (!todo.empty()) {
    const Pending p = todo.back();
    todo.pop_back();
    e.clear();
    entries(p.y4, K, e);
    Node8Rec rec;
    std::memset(&rec, 0, sizeof(rec));
    int32_t child_out[K];
    for (int k = 0; k < K; ++k) {
      child_out[k] = -1;
      if (k >= (int)e.size()) {
        rec.link[k] = kEmptySlot4;
        continue;
      }
      std::memcpy(rec.q + 6 * k, e[k].box, 6 * sizeof(float));
      if (e[k].link < 0) {
        rec.link[k] = e[k].link;
      } else {
        child_out[k] = (int32_t)out.size();
        rec.link[k] = child_out[k];
        out.emplace_back();
      }
    }
    out[(size_t)p.out] = rec;
    for (int k = (int)e.size() - 1; k >= 0; --k)  // preorder: slot 0's subtree next
      if (child_out[k] >= 0) todo.push_back(Pending{e[k].link, child_out[k]});
  }
  std::vector<int32_t> need(out.size(), 0);
  for (int64_t k = (int64_t)out.size() - 1; k >= 0; --k) {
    int ns = 0, below = 0;
    for (int s = 0; s < K; ++s) {
      if (out[(size_t)k].link[s] == kEmptySlot4) continue;
      ++ns;
      if (out[(size_t)k].link[s] >= 0) below = std::max(below, need[(size_t)out[(size_t)k].link[s]]);
    }
    need[(size_t)k] = ns - 1 + below;
  }
  *stack_need = std::max(need[0], 1);
  return 0;
}


}  // namespace wide8
}  // namespace mcpt
