// tools/wide_order_sim.cpp — CPU estimate of the EXACT search's node steps per
// segment for the 4-wide and 8-wide search trees and for the order in which a
// node's other passing slots are pushed (design aid for DESIGN.md §3.3; not
// a parity tool: the triangle test is plain Moller-Trumbore, the bounce a
// cosine-free uniform hemisphere draw).
//   g++ -O2 -std=c++17 -pthread -I montecarlopathtracing_amd/csrc -I tools tools/wide_order_sim.cpp \
//       montecarlopathtracing_amd/csrc/mcpt_host.cpp montecarlopathtracing_amd/csrc/mcpt_sah.cpp -o /tmp/wos
//   /tmp/wos scenes/cbox/ cbox.obj 278 273 -800  278 273 -799  39.3077  [rays]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../include/mcpt_hip.h"
#include "mcpt_bvh4.h"
#include "wide8.h"

namespace {
struct V {
  float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V norm(V a) {
  float l = std::sqrt(dot(a, a));
  return {a.x / l, a.y / l, a.z / l};
}

struct Ray {
  V o, d, ri;
};
bool slab(const float *b, const Ray &r, float tmin, float lim, float &tn) {
  float t0 = -INFINITY, t1 = INFINITY;
  const float o[3] = {r.o.x, r.o.y, r.o.z}, ri[3] = {r.ri.x, r.ri.y, r.ri.z};
  for (int a = 0; a < 3; ++a) {
    float u = (b[2 * a] - o[a]) * ri[a], v = (b[2 * a + 1] - o[a]) * ri[a];
    t0 = std::fmax(t0, std::fmin(u, v));
    t1 = std::fmin(t1, std::fmax(u, v));
  }
  tn = t0;
  return !(t1 < t0 || t1 < tmin) && !(t0 > lim);
}
float tri_hit(const mcpt_triangle &t, const Ray &r) {
  V v0{t.v[0][0], t.v[0][1], t.v[0][2]}, v1{t.v[1][0], t.v[1][1], t.v[1][2]}, v2{t.v[2][0], t.v[2][1], t.v[2][2]};
  V e1 = sub(v1, v0), e2 = sub(v2, v0), p = cross(r.d, e2);
  float det = dot(e1, p);
  if (std::fabs(det) < 1e-12f) return INFINITY;
  float inv = 1.0f / det;
  V s = sub(r.o, v0);
  float u = dot(s, p) * inv;
  if (u < 0 || u > 1) return INFINITY;
  V q = cross(s, e1);
  float v = dot(r.d, q) * inv;
  if (v < 0 || u + v > 1) return INFINITY;
  float tt = dot(e2, q) * inv;
  return tt > 1e-3f ? tt : INFINITY;
}

template <int K, class Node>
struct Search {
  const std::vector<Node> &N;
  const std::vector<mcpt_triangle> &T;
  int order;  // 0: nearest first, rest in slot order; 1: all by distance
  long steps = 0, tests = 0;
  float trace(const Ray &r, float margin, int &hit) {
    float best = INFINITY;
    hit = -1;
    std::vector<int> st;
    st.push_back(0);
    while (!st.empty()) {
      int cur = st.back();
      st.pop_back();
      if (cur < 0) {
        ++tests;
        float t = tri_hit(T[~cur], r);
        if (t < best) best = t, hit = ~cur;
        continue;
      }
      ++steps;
      const Node &n = N[cur];
      std::pair<float, int> h[K];
      int nh = 0;
      for (int s = 0; s < K; ++s) {
        if (n.link[s] == mcpt::kEmptySlot4) continue;
        float tn;
        if (slab(n.q + 6 * s, r, 1e-3f, best + margin, tn)) h[nh++] = {tn, s};
      }
      if (!nh) continue;
      if (order == 1) {
        std::stable_sort(h, h + nh, [](auto a, auto b) { return a.first < b.first; });
        for (int i = nh - 1; i >= 0; --i) st.push_back(n.link[h[i].second]);
      } else {
        int sel = 0;
        for (int i = 1; i < nh; ++i)
          if (h[i].first < h[sel].first) sel = i;
        for (int i = nh - 1; i >= 0; --i)
          if (i != sel) st.push_back(n.link[h[i].second]);
        st.push_back(n.link[h[sel].second]);
      }
    }
    return best;
  }
};
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
  std::vector<mcpt::LeafRef> L;
  for (auto &b : B)
    if (b.left == b.right) {
      mcpt::LeafRef r;
      const float bx[6] = {b.bbmin[0], b.bbmax[0], b.bbmin[1], b.bbmax[1], b.bbmin[2], b.bbmax[2]};
      std::memcpy(r.box, bx, sizeof bx);
      r.tri = b.left;
      L.push_back(r);
    }
  std::vector<mcpt::Node4Rec> t4;
  std::vector<mcpt::wide8::Node8Rec> t8;
  int32_t need4, need8;
  mcpt::build_sah4(L, t4, &need4, 8);
  mcpt::wide8::widen_sah8(t4, t8, &need8);
  const mcpt_bvh_node &root = B[0];
  float dx = root.bbmax[0] - root.bbmin[0], dy = root.bbmax[1] - root.bbmin[1], dz = root.bbmax[2] - root.bbmin[2];
  const float margin = std::ldexp(std::sqrt(dx * dx + dy * dy + dz * dz), -10);
  V eye{(float)atof(argv[3]), (float)atof(argv[4]), (float)atof(argv[5])};
  V at{(float)atof(argv[6]), (float)atof(argv[7]), (float)atof(argv[8])};
  const float fov = (float)atof(argv[9]) * 3.14159265f / 180.0f;
  const int rays = argc > 10 ? atoi(argv[10]) : 20000;
  V fw = norm(sub(at, eye)), rt = norm(cross(fw, V{0, 1, 0})), up = cross(rt, fw);
  Search<4, mcpt::Node4Rec> s4{t4, T, 0};
  Search<8, mcpt::wide8::Node8Rec> s8a{t8, T, 0}, s8b{t8, T, 1};
  Search<4, mcpt::Node4Rec> s4b{t4, T, 1};
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
      int h4, h8, hx, hy;
      const float t = s4.trace(r, margin, h4);
      s8a.trace(r, margin, h8);
      s8b.trace(r, margin, hx);
      s4b.trace(r, margin, hy);
      ++segs;
      if (h4 < 0) break;
      V p{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
      V nn{T[h4].normal[0], T[h4].normal[1], T[h4].normal[2]};
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
  std::printf("{\"tris\": %ld, \"nodes4\": %zu, \"nodes8\": %zu, \"need4\": %d, \"need8\": %d, \"segments\": %ld,\n"
              " \"steps4_nearest\": %.3f, \"steps4_sorted\": %.3f, \"steps8_nearest\": %.3f, \"steps8_sorted\": %.3f,\n"
              " \"tests4\": %.3f, \"tests8\": %.3f}\n",
              (long)n, t4.size(), t8.size(), need4, need8, segs, (double)s4.steps / segs, (double)s4b.steps / segs,
              (double)s8a.steps / segs, (double)s8b.steps / segs, (double)s4.tests / segs, (double)s8a.tests / segs);
  return 0;
}
