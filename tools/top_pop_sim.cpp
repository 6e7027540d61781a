// tools/top_pop_sim.cpp — CPU estimate of where the EXACT search's node steps
// fall once the search tree's top L levels live in LDS (design aid for
// DESIGN.md §3.4; not a parity tool: plain Moller-Trumbore, a uniform
// hemisphere bounce).  Per segment: the steps `begin_segment` takes from LDS
// (the nearest-first descent while the entered child is a top node), the
// T-phase steps of top nodes popped from the stack later (siblings pushed on
// the way down: still 7 global gathers each as shipped), and the deeper ones.
//   g++ -O2 -std=c++17 -pthread -I montecarlopathtracing_amd/csrc tools/top_pop_sim.cpp \
//       montecarlopathtracing_amd/csrc/mcpt_host.cpp montecarlopathtracing_amd/csrc/mcpt_sah.cpp -o /tmp/tps
//   /tmp/tps scenes/cbox/ cbox.obj 278 273 -800  278 273 -799  39.3077  [rays]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <utility>
#include <vector>

#include "../include/mcpt_hip.h"
#include "mcpt_bvh4.h"

namespace {
struct V {
  float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V norm(V a) {
  const float l = std::sqrt(dot(a, a));
  return {a.x / l, a.y / l, a.z / l};
}
struct Ray {
  V o, d, ri;
};
bool slab(const float *b, const Ray &r, float tmin, float lim, float &tn) {
  float t0 = -INFINITY, t1 = INFINITY;
  const float o[3] = {r.o.x, r.o.y, r.o.z}, ri[3] = {r.ri.x, r.ri.y, r.ri.z};
  for (int a = 0; a < 3; ++a) {
    const float u = (b[2 * a] - o[a]) * ri[a], v = (b[2 * a + 1] - o[a]) * ri[a];
    t0 = std::fmax(t0, std::fmin(u, v));
    t1 = std::fmin(t1, std::fmax(u, v));
  }
  tn = t0;
  return !(t1 < t0 || t1 < tmin) && !(t0 > lim);
}
float tri_hit(const mcpt_triangle &t, const Ray &r) {
  const V v0{t.v[0][0], t.v[0][1], t.v[0][2]}, v1{t.v[1][0], t.v[1][1], t.v[1][2]}, v2{t.v[2][0], t.v[2][1], t.v[2][2]};
  const V e1 = sub(v1, v0), e2 = sub(v2, v0), p = cross(r.d, e2);
  const float det = dot(e1, p);
  if (std::fabs(det) < 1e-12f) return INFINITY;
  const float inv = 1.0f / det;
  const V s = sub(r.o, v0);
  const float u = dot(s, p) * inv;
  if (u < 0 || u > 1) return INFINITY;
  const V q = cross(s, e1);
  const float v = dot(r.d, q) * inv;
  if (v < 0 || u + v > 1) return INFINITY;
  const float tt = dot(e2, q) * inv;
  return tt > 1e-3f ? tt : INFINITY;
}

struct Counts {
  long s_steps = 0, t_top = 0, t_deep = 0, pops_top_all_pruned = 0;
  long pops = 0, cull_node = 0, cull_leaf = 0, cull_node_q = 0, cull_leaf_q = 0;  // pop-time culling by t_near
};
float g_qstep = 0;  // 7-bit linear t_near quantum (scene diagonal / 127)

// nearest first, the other passing slots pushed in slot order (as step4q);
// entries carry their depth.  Top nodes: depth < L.
float trace(const std::vector<mcpt::Node4Rec> &N, const std::vector<mcpt_triangle> &T, const Ray &r, float margin, int L,
            Counts &c, int &hit) {
  float best = INFINITY;
  hit = -1;
  struct E {
    int link, depth;
    float tn;
  };
  std::vector<E> st;
  int cur = 0, depth = 0;
  bool in_s = L > 0;  // begin_segment's descent
  for (;;) {
    if (cur < 0 && cur != mcpt::kEmptySlot4) {
      const float t = tri_hit(T[~cur], r);
      if (t < best) best = t, hit = ~cur;
      cur = mcpt::kEmptySlot4;
    }
    if (cur == mcpt::kEmptySlot4) {
      if (st.empty()) break;
      const E e = st.back();
      st.pop_back();
      cur = e.link, depth = e.depth;
      ++c.pops;
      // would a stored t_near have culled it (no step / no test)?
      if (e.tn > best + margin) ++(cur < 0 ? c.cull_leaf : c.cull_node);
      const float tq = std::floor(std::max(e.tn, 0.0f) / g_qstep) * g_qstep;  // rounded down: conservative
      if (tq > best + margin) ++(cur < 0 ? c.cull_leaf_q : c.cull_node_q);
      in_s = false;
      continue;
    }
    if (in_s && depth < L)
      ++c.s_steps;
    else if (depth < L)
      ++c.t_top;
    else
      ++c.t_deep;
    const mcpt::Node4Rec &n = N[cur];
    std::pair<float, int> h[4];
    int nh = 0;
    for (int s = 0; s < 4; ++s) {
      if (n.link[s] == mcpt::kEmptySlot4) continue;
      float tn;
      if (slab(n.q + 6 * s, r, 1e-3f, best + margin, tn)) h[nh++] = {tn, s};
    }
    if (!nh) {
      if (!in_s && depth < L) ++c.pops_top_all_pruned;
      cur = mcpt::kEmptySlot4;
      in_s = false;
      continue;
    }
    int sel = 0;
    for (int i = 1; i < nh; ++i)
      if (h[i].first < h[sel].first) sel = i;
    for (int i = nh - 1; i >= 0; --i)
      if (i != sel) st.push_back({n.link[h[i].second], depth + 1, h[i].first});
    cur = n.link[h[sel].second];
    ++depth;
    if (cur < 0) in_s = false;  // a leaf: the L phase
  }
  return best;
}
}  // namespace

int main(int argc, char **argv) {
  if (argc < 10) {
    std::fprintf(stderr, "usage: dir obj px py pz lx ly lz fov [rays]\n");
    return 2;
  }
  int64_t n = 0;
  int32_t nm = 0;
  if (mcpt_load_obj(argv[1], argv[2], nullptr, nullptr, &n, nullptr, &nm)) return 1;
  std::vector<mcpt_triangle> T(n);
  std::vector<int32_t> mid(n);
  std::vector<mcpt_material> M(nm);
  if (mcpt_load_obj(argv[1], argv[2], T.data(), mid.data(), &n, M.data(), &nm)) return 1;
  mcpt_pack_triangles(T.data(), mid.data(), n);
  std::vector<mcpt_bvh_node> B(2 * n - 1);
  mcpt_build_hlbvh(T.data(), n, B.data());
  std::vector<mcpt::LeafRef> Ls;
  for (auto &b : B)
    if (b.left == b.right) {
      mcpt::LeafRef r;
      const float bx[6] = {b.bbmin[0], b.bbmax[0], b.bbmin[1], b.bbmax[1], b.bbmin[2], b.bbmax[2]};
      std::memcpy(r.box, bx, sizeof bx);
      r.tri = b.left;
      Ls.push_back(r);
    }
  std::vector<mcpt::Node4Rec> t4;
  int32_t need4;
  mcpt::build_sah4(Ls, t4, &need4, 8);
  const mcpt_bvh_node &root = B[0];
  const float dx = root.bbmax[0] - root.bbmin[0], dy = root.bbmax[1] - root.bbmin[1], dz = root.bbmax[2] - root.bbmin[2];
  const float margin = std::ldexp(std::sqrt(dx * dx + dy * dy + dz * dz), -10);
  g_qstep = std::sqrt(dx * dx + dy * dy + dz * dz) / 127.0f;
  const V eye{(float)atof(argv[3]), (float)atof(argv[4]), (float)atof(argv[5])};
  const V at{(float)atof(argv[6]), (float)atof(argv[7]), (float)atof(argv[8])};
  const float fov = (float)atof(argv[9]) * 3.14159265f / 180.0f;
  const int rays = argc > 10 ? atoi(argv[10]) : 20000;
  const V fw = norm(sub(at, eye)), rt = norm(cross(fw, V{0, 1, 0})), up = cross(rt, fw);
  std::printf("{\"tris\": %ld, \"nodes4\": %zu, \"rays\": %d, \"levels\": [", (long)n, t4.size(), rays);
  for (int L = 0; L <= 5; ++L) {
    Counts c;
    std::mt19937 g(1);
    std::uniform_real_distribution<float> u01(0.0f, 1.0f);
    long segs = 0;
    for (int k = 0; k < rays; ++k) {
      const float a = (u01(g) - 0.5f) * 2 * std::tan(fov / 2), b = (u01(g) - 0.5f) * 2 * std::tan(fov / 2);
      Ray r;
      r.o = eye;
      r.d = norm(V{fw.x + a * rt.x + b * up.x, fw.y + a * rt.y + b * up.y, fw.z + a * rt.z + b * up.z});
      for (int bounce = 0; bounce < 8; ++bounce) {
        r.ri = {1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
        int h;
        const float t = trace(t4, T, r, margin, L, c, h);
        ++segs;
        if (h < 0) break;
        const V p{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
        V nn{T[h].normal[0], T[h].normal[1], T[h].normal[2]};
        if (dot(nn, r.d) > 0) nn = {-nn.x, -nn.y, -nn.z};
        V d;
        do {
          d = {u01(g) * 2 - 1, u01(g) * 2 - 1, u01(g) * 2 - 1};
        } while (dot(d, d) > 1 || dot(d, d) < 1e-6f);
        d = norm(d);
        if (dot(d, nn) < 0) d = {-d.x, -d.y, -d.z};
        r.o = {p.x + 1e-3f * d.x, p.y + 1e-3f * d.y, p.z + 1e-3f * d.z};
        r.d = d;
      }
    }
    std::printf("%s\n {\"L\": %d, \"segments\": %ld, \"s_steps\": %.3f, \"t_top_popped\": %.3f, \"t_top_all_pruned\": %.3f, "
                "\"t_deep\": %.3f, \"pops\": %.3f, \"cull_node\": %.3f, \"cull_leaf\": %.3f, \"cull_node_q7\": %.3f, "
                "\"cull_leaf_q7\": %.3f}",
                L ? "," : "", L, segs, (double)c.s_steps / segs, (double)c.t_top / segs,
                (double)c.pops_top_all_pruned / segs, (double)c.t_deep / segs, (double)c.pops / segs,
                (double)c.cull_node / segs, (double)c.cull_leaf / segs, (double)c.cull_node_q / segs,
                (double)c.cull_leaf_q / segs);
  }
  std::printf("]}\n");
  return 0;
}
