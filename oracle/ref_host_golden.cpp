// ref_host_golden.cpp — TEST INFRASTRUCTURE ONLY (never linked into the
// product).  A command-line driver over the reference's OWN host C++,
// compiled unmodified from /root/reference by oracle/Makefile (flags and the
// forced include oracle/ref_prelude.h only):
//   MCPT/auxiliary.cpp          Auxiliary::parseCamera        (auxiliary.cpp:20-71)
//   MCPT/thirdpartywrapper.cpp  ThirdPartyWrapper::loadObject (thirdpartywrapper.cpp:25-99,
//                               tinyobjloader + the material classification)
//   MCPT/BVH/treeletBVH.cpp     TreeletBVH<CPU>               (treeletBVH.cpp:30-372)
//   MCPT/bvhtest.cpp            BVH::TEST::SAH / LCV          (bvhtest.cpp:104-115, 324-444)
// tools/make_host_goldens.py runs it in the build container and commits its
// outputs as fixtures under tests/golden/ (it never travels to the GPU box).
//
//   ref_host_golden camera <out> px py pz lx ly lz ux uy uz fov
//   ref_host_golden load <dir/> <obj> <out_tris> <out_mats> <out_ids>
//   ref_host_golden treelet <in_nodes> <out_nodes>
//   ref_host_golden sah <in_nodes>                    (prints the float's bits)
//   ref_host_golden lcv <in_nodes> <camera.bin>       (prints the float's bits; W/H from ./config.json)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "auxiliary.h"
#include "bvhtest.h"
#include "thirdpartywrapper.h"
#include "treeletBVH.h"

using namespace MCPT;

template <class T>
static std::vector<T> read_vec(const char *path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  std::vector<T> v(s.size() / sizeof(T));
  std::memcpy(v.data(), s.data(), v.size() * sizeof(T));
  return v;
}

template <class T>
static void write_vec(const char *path, const std::vector<T> &v) {
  FILE *f = std::fopen(path, "wb");
  std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
}

static uint32_t bits(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  return u;
}

int main(int argc, char **argv) {
  static_assert(sizeof(Camera) == 80 && sizeof(Triangle) == 64 && sizeof(Material) == 48 && sizeof(BVHNode) == 64,
                "objdef.h record sizes");
  if (argc < 2) return 2;
  const std::string cmd = argv[1];
  if (cmd == "camera" && argc == 13) {
    json j;
    j["position"] = {std::atof(argv[3]), std::atof(argv[4]), std::atof(argv[5])};
    j["lookat"] = {std::atof(argv[6]), std::atof(argv[7]), std::atof(argv[8])};
    j["up"] = {std::atof(argv[9]), std::atof(argv[10]), std::atof(argv[11])};
    j["fov"] = std::atof(argv[12]);
    const Camera c = Auxiliary::parseCamera(j);
    write_vec(argv[2], std::vector<Camera>{c});
    return 0;
  }
  if (cmd == "load" && argc == 7) {
    auto [tris, mats, ids] = ThirdPartyWrapper::loadObject(argv[2], argv[3]);
    write_vec(argv[4], tris);
    write_vec(argv[5], mats);
    write_vec(argv[6], ids);
    return 0;
  }
  if (cmd == "treelet" && argc == 4) {
    const auto nodes = read_vec<BVHNode>(argv[2]);
    BVH::TreeletBVH<BVH::CPU> t(nodes);
    write_vec(argv[3], t.getBVH());
    return 0;
  }
  if (cmd == "sah" && argc == 3) {
    std::printf("%u\n", bits(BVH::TEST::SAH(read_vec<BVHNode>(argv[2]))));
    return 0;
  }
  if (cmd == "lcv" && argc == 4) {
    const auto cam = read_vec<Camera>(argv[3]);
    std::printf("%u\n", bits(BVH::TEST::LCV(read_vec<BVHNode>(argv[2]), cam.at(0))));
    return 0;
  }
  std::fprintf(stderr, "bad command\n");
  return 2;
}
