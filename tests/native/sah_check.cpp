// CPU check of the EXACT path's SAH search tree (montecarlopathtracing_amd/csrc/mcpt_sah.cpp),
// built and run by tests/test_cpu.py::test_sah_search_tree_invariants.
//   sah_check <n_leaves> <seed> <clustered 0|1>
// Prints "ok nodes=<k> need=<s>" or the first violated invariant.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <random>
#include <vector>

#include "mcpt_bvh4.h"

using mcpt::LeafRef;
using mcpt::Node4Rec;

static int fail(const char *what, long a, long b) {
  std::printf("FAIL %s %ld %ld\n", what, a, b);
  return 1;
}

int main(int argc, char **argv) {
  const int n = std::atoi(argv[1]);
  std::mt19937 g((unsigned)std::atoi(argv[2]));
  const bool clustered = std::atoi(argv[3]) != 0;
  std::uniform_real_distribution<float> u(-50.0f, 50.0f), e(0.0f, 0.5f);
  std::vector<LeafRef> L(n);
  for (int i = 0; i < n; ++i) {
    float c[3] = {u(g), u(g), u(g)};
    if (clustered && i % 3 == 0) c[0] = c[1] = c[2] = 1.0f;  // identical centroids: no SAH split
    for (int a = 0; a < 3; ++a) {
      L[i].box[2 * a] = c[a] - e(g);
      L[i].box[2 * a + 1] = c[a] + e(g);
    }
    if (i % 5 == 1) L[i].box[2 * (i % 3)] = L[i].box[2 * (i % 3) + 1];  // flat on one axis (axis-aligned triangle)
    if (i % 11 == 2) L[i].box[2 * (i % 3)] = 0.0f, L[i].box[2 * (i % 3) + 1] = std::max(0.0f, L[i].box[2 * (i % 3) + 1]);
    if (i % 13 == 3) L[i].box[2 * (i % 3) + 1] = 0.0f, L[i].box[2 * (i % 3)] = std::min(0.0f, L[i].box[2 * (i % 3)]);
    L[i].tri = (int)(((long)i * 7919) % n);  // a permutation (n is not a multiple of 7919)
  }
  std::vector<int> leaf_of(n);
  for (int i = 0; i < n; ++i) leaf_of[L[i].tri] = i;
  std::vector<Node4Rec> t1, t8;
  int need1 = 0, need8 = 0;
  if (mcpt::build_sah4(L, t1, &need1, 1) || mcpt::build_sah4(L, t8, &need8, 8)) return fail("build", 0, 0);
  if (n == 1) return t1.empty() ? (std::printf("ok nodes=0 need=%d\n", need1), 0) : fail("single", 0, 0);
  // deterministic whatever the thread count
  if (t1.size() != t8.size() || need1 != need8 || std::memcmp(t1.data(), t8.data(), t1.size() * sizeof(Node4Rec)))
    return fail("thread-dependent tree", (long)t1.size(), (long)t8.size());
  // every leaf exactly once with its own box; every slot box = union of its subtree
  std::vector<int> seen(n, 0);
  std::vector<int> visited(t1.size(), 0);
  int max_need = 0;
  std::vector<int> need(t1.size(), -1);
  // recompute the stack bound bottom-up (children have larger ids)
  for (long k = (long)t1.size() - 1; k >= 0; --k) {
    int ns = 0, below = 0;
    for (int s = 0; s < 4; ++s) {
      const int32_t l = t1[k].link[s];
      if (l == mcpt::kEmptySlot4) continue;
      ++ns;
      if (l >= 0) {
        if (l <= k || l >= (long)t1.size()) return fail("child id order", k, l);
        below = below > need[l] ? below : need[l];
      }
    }
    if (ns < 2) return fail("node with < 2 slots", k, ns);
    need[k] = ns - 1 + below;
  }
  max_need = need[0] > 1 ? need[0] : 1;
  if (max_need != need1) return fail("stack need", max_need, need1);
  // union check: walk every node, compare each internal slot's box with the union of the child's slots
  for (size_t k = 0; k < t1.size(); ++k) {
    for (int s = 0; s < 4; ++s) {
      const int32_t l = t1[k].link[s];
      if (l == mcpt::kEmptySlot4) continue;
      const float *b = t1[k].q + 6 * s;
      if (l < 0) {
        const int tri = ~l;
        if (tri < 0 || tri >= n) return fail("leaf id", (long)k, tri);
        if (seen[tri]++) return fail("leaf twice", (long)k, tri);
        if (std::memcmp(b, L[leaf_of[tri]].box, sizeof(float) * 6)) return fail("leaf box", (long)k, tri);
      } else {
        if (visited[l]++) return fail("node twice", (long)k, l);
        float un[6] = {1e30f, -1e30f, 1e30f, -1e30f, 1e30f, -1e30f};
        for (int c = 0; c < 4; ++c) {
          if (t1[l].link[c] == mcpt::kEmptySlot4) continue;
          for (int a = 0; a < 3; ++a) {
            un[2 * a] = std::min(un[2 * a], t1[l].q[6 * c + 2 * a]);
            un[2 * a + 1] = std::max(un[2 * a + 1], t1[l].q[6 * c + 2 * a + 1]);
          }
        }
        if (std::memcmp(un, b, sizeof(un))) return fail("slot box != union of child", (long)k, l);
      }
    }
  }
  for (int i = 0; i < n; ++i)
    if (seen[i] != 1) return fail("leaf missing", i, seen[i]);
  for (size_t k = 1; k < t1.size(); ++k)
    if (visited[k] != 1) return fail("unreachable node", (long)k, visited[k]);
  // the 64-B quantized nodes (mcpt::quantize_node4): every decoded slot box
  // strictly contains the exact one, links unchanged, and the slab test
  // (objdef.h:223-237, NaN-ignoring fmin/fmax like v_min/v_max_f32) passes on
  // the decoded box whenever it passes on the exact one -- rays include zero
  // direction components with the origin exactly on a box plane.
  std::mt19937 rg(12345u);
  long slab_checks = 0;
  for (size_t k = 0; k < t1.size(); ++k) {
    mcpt::Node4Q qn;
    if (mcpt::quantize_node4(t1[k], qn) != 0) return fail("quantize", (long)k, 0);
    const float s[3] = {qn.sx, qn.sy, qn.sz};
    for (int c = 0; c < 4; ++c) {
      if (qn.link[c] != t1[k].link[c]) return fail("quantized link", (long)k, c);
      if (t1[k].link[c] == mcpt::kEmptySlot4) continue;
      const float *b = t1[k].q + 6 * c;
      float dq[6];
      for (int i = 0; i < 6; ++i) dq[i] = std::fma((float)qn.q[6 * c + i], s[i / 2], qn.org[i / 2]);
      for (int a = 0; a < 3; ++a)
        if (!(dq[2 * a] < b[2 * a]) || !(dq[2 * a + 1] > b[2 * a + 1])) return fail("not strictly contained", (long)k, c);
      for (int r = 0; r < 24; ++r) {
        float o[3], d[3];
        for (int a = 0; a < 3; ++a) {
          const int pick = (int)(rg() % 6);  // origin on a plane, inside, or anywhere
          o[a] = pick == 0 ? b[2 * a] : pick == 1 ? b[2 * a + 1] : pick == 2 ? 0.5f * (b[2 * a] + b[2 * a + 1])
                                                                              : (float)((int)(rg() % 200) - 100);
          const int dz = (int)(rg() % 4);  // +0, -0, or a random component
          d[a] = dz == 0 ? 0.0f : dz == 1 ? -0.0f : (float)((int)(rg() % 2001) - 1000) / 1000.0f;
        }
        auto pass = [&](const float *bx) {
          float tn = -INFINITY, tf = INFINITY;
          for (int a = 0; a < 3; ++a) {
            const float ri = 1.0f / d[a];
            const float t1 = (bx[2 * a] - o[a]) * ri, t2 = (bx[2 * a + 1] - o[a]) * ri;
            const float mn = std::fmin(t1, t2), mx = std::fmax(t1, t2);
            tn = a == 0 ? mn : std::fmax(tn, mn);
            tf = a == 0 ? mx : std::fmin(tf, mx);
          }
          return !(tf < tn || tf < 0.001f);
        };
        ++slab_checks;
        if (pass(b) && !pass(dq)) return fail("decoded box fails where the exact box passes", (long)k, c);
      }
    }
  }
  std::printf("ok nodes=%zu need=%d slab_checks=%ld\n", t1.size(), need1, slab_checks);
  return 0;
}
