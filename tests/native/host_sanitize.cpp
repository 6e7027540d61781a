// host_sanitize.cpp — TEST INFRASTRUCTURE.  Drives every host-side entry
// point of libmcpt_hip.so (csrc/mcpt_host.cpp: OBJ/MTL loader, material
// classification, packing, HLBVH, stack depth, SAH metric, camera, RGBE
// writer; csrc/mcpt_sah.cpp: the multi-threaded SAH search-tree builder) on
// the committed scenes, synthetic meshes and edge cases.  Built by
// tests/native/Makefile as
//   host_asan  -fsanitize=address,undefined (no recovery: the first report fails the run)
//   host_tsan  -fsanitize=thread (the 16-thread SAH builder and the HLBVH on 16 host threads)
// and run by tests/test_cpu.py::test_host_code_under_sanitizers.
//   host_sanitize <repo root> <threads>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mcpt_hip.h"
#include "mcpt_bvh4.h"

static int failures = 0;
#define CHECK(cond, what)                                  \
  do {                                                     \
    if (!(cond)) {                                         \
      std::printf("FAIL %s (%s)\n", what, mcpt_last_error()); \
      ++failures;                                          \
    }                                                      \
  } while (0)

static std::vector<mcpt_triangle> mesh(int n, unsigned seed, bool dup, bool flat) {
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> u(-3.0f, 3.0f);
  std::vector<mcpt_triangle> t(n);
  for (int i = 0; i < n; ++i) {
    std::memset(&t[i], 0, sizeof(mcpt_triangle));
    for (int k = 0; k < 3; ++k)
      for (int a = 0; a < 3; ++a) t[i].v[k][a] = (dup && i % 2) ? t[i - 1].v[k][a] : u(g);
    if (flat)
      for (int k = 0; k < 3; ++k) t[i].v[k][2] = 0.0f;
  }
  return t;
}

static void tree_checks(std::vector<mcpt_triangle> tris, int threads) {
  const int64_t n = (int64_t)tris.size();
  std::vector<int32_t> mid(n, 0);
  CHECK(mcpt_pack_triangles(tris.data(), mid.data(), n) == MCPT_OK, "pack");
  std::vector<mcpt_bvh_node> nodes(2 * n - 1);
  CHECK(mcpt_build_hlbvh(tris.data(), n, nodes.data()) == MCPT_OK, "hlbvh");
  int32_t depth = 0;
  CHECK(mcpt_bvh_stack_depth(nodes.data(), (int64_t)nodes.size(), &depth) == MCPT_OK, "stack depth");
  double sah = 0.0;
  CHECK(mcpt_bvh_sah(nodes.data(), (int64_t)nodes.size(), &sah) == MCPT_OK && std::isfinite(sah), "sah");
  // the EXACT path's search tree over the reference leaves, multi-threaded
  std::vector<mcpt::LeafRef> leaves;
  for (const auto &b : nodes)
    if (b.left == b.right) {
      mcpt::LeafRef L;
      const float bx[6] = {b.bbmin[0], b.bbmax[0], b.bbmin[1], b.bbmax[1], b.bbmin[2], b.bbmax[2]};
      std::memcpy(L.box, bx, sizeof(bx));
      L.tri = b.left;
      leaves.push_back(L);
    }
  std::vector<mcpt::Node4Rec> a, b;
  int32_t na = 0, nb = 0;
  CHECK(mcpt::build_sah4(leaves, a, &na, 1) == 0, "sah4 1 thread");
  CHECK(mcpt::build_sah4(leaves, b, &nb, threads) == 0, "sah4 threads");
  CHECK(a.size() == b.size() && na == nb &&
            (a.empty() || std::memcmp(a.data(), b.data(), a.size() * sizeof(mcpt::Node4Rec)) == 0),
        "sah4 thread-independent");
}

int main(int argc, char **argv) {
  const std::string root = argc > 1 ? argv[1] : ".";
  const int threads = argc > 2 ? std::atoi(argv[2]) : 16;
  // scenes through the loader (thirdpartywrapper.cpp:25-99)
  const char *scenes[][2] = {{"scenes/cbox/", "cbox.obj"}, {"scenes/veach_mis/", "mis.obj"},
                             {"scenes/diningroom/", "diningroom.obj"}};
  for (auto &sc : scenes) {
    const std::string dir = root + "/" + sc[0];
    int64_t n = 0;
    int32_t nm = 0;
    CHECK(mcpt_load_obj(dir.c_str(), sc[1], nullptr, nullptr, &n, nullptr, &nm) == MCPT_OK && n > 0, "load sizes");
    std::vector<mcpt_triangle> tris(n);
    std::vector<int32_t> mid(n);
    std::vector<mcpt_material> mats(nm);
    CHECK(mcpt_load_obj(dir.c_str(), sc[1], tris.data(), mid.data(), &n, mats.data(), &nm) == MCPT_OK, "load");
    tree_checks(tris, threads);
  }
  // loader error paths
  int64_t n = 0;
  int32_t nm = 0;
  CHECK(mcpt_load_obj((root + "/scenes/").c_str(), "missing.obj", nullptr, nullptr, &n, nullptr, &nm) == MCPT_ERR_IO,
        "missing file");
  // synthetic meshes and edge cases of the HLBVH (one, two, three triangles,
  // duplicate Morton codes, a flat axis)
  for (int k : {1, 2, 3, 17, 1000, 100000}) tree_checks(mesh(k, (unsigned)k, false, false), threads);
  tree_checks(mesh(600, 5, true, false), threads);
  tree_checks(mesh(600, 6, false, true), threads);
  // camera, classification, RGBE encoder
  mcpt_camera cam;
  const double p[3] = {278, 273, -800}, l[3] = {278, 273, -799}, up[3] = {0, 1, 0};
  CHECK(mcpt_parse_camera(p, l, up, 39.3077, &cam) == MCPT_OK, "camera");
  mcpt_material m;
  const float z[3] = {0, 0, 0}, kd[3] = {0.5f, 0.5f, 0.5f}, ka[3] = {10, 10, 10};
  CHECK(mcpt_classify_material(1.0f, z, kd, z, 1.0f, &m) == MCPT_OK && m.type == MCPT_DIFFUSE, "diffuse");
  CHECK(mcpt_classify_material(1.0f, ka, z, z, 1.0f, &m) == MCPT_OK && m.type == MCPT_LIGHT, "light");
  CHECK(mcpt_classify_material(1.5f, z, z, z, 1.0f, &m) == MCPT_OK && m.type == MCPT_TRANSPARENT, "glass");
  CHECK(mcpt_classify_material(1.0f, z, kd, kd, 50.0f, &m) == MCPT_OK && m.type == MCPT_GLOSSY, "glossy");
  for (int w : {1, 7, 8, 33, 300}) {  // RLE runs and the short-row path of stb's writer
    const int h = 5;
    std::vector<float> img((size_t)w * h * 4);
    for (size_t i = 0; i < img.size(); ++i) img[i] = (i % 7 == 0) ? 0.0f : (float)((i * 37) % 101) / 13.0f;
    const int64_t bytes = mcpt_encode_hdr(w, h, img.data(), 1, nullptr, 0);
    CHECK(bytes > 0, "hdr size");
    std::vector<uint8_t> out((size_t)bytes);
    CHECK(mcpt_encode_hdr(w, h, img.data(), 1, out.data(), bytes) == bytes, "hdr encode");
    CHECK(mcpt_encode_hdr(w, h, img.data(), 1, out.data(), bytes - 1) < 0, "hdr short buffer");
  }
  std::printf("%s %d failures\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
