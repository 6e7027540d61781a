// ref_io_shim.cpp — TEST INFRASTRUCTURE ONLY.  A C entry point over the
// reference's vendored, unmodified third-party I/O code (compiled from
// /root/reference by oracle/Makefile): tinyobjloader 2.0.0rc as
// ThirdPartyWrapper::loadObject drives it (MCPT/thirdpartywrapper.cpp:25-63)
// and stb_image_write v1.13 as outputPicture drives it (:14-23).  Used to pin
// the product's OBJ/MTL loader and RGBE writer byte for byte.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "stb_image_write.h"
#include "tiny_obj_loader.h"

extern "C" {

// Fills, per triangle, 9 floats (v0 v1 v2 xyz) and the face material id, and
// per material: ior, ambient[3], diffuse[3], specular[3], shininess (11 floats).
// Call with null outputs to get the counts.
int ref_load_obj(const char *directory, const char *objname, float *verts, int32_t *matids, int64_t *ntri,
                 float *mats, int32_t *nmat) {
  tinyobj::attrib_t attrib;
  std::vector<tinyobj::shape_t> shapes;
  std::vector<tinyobj::material_t> materials;
  std::string dir(directory), obj(objname);
  bool ok = tinyobj::LoadObj(&attrib, &shapes, &materials, nullptr, nullptr, (dir + obj).c_str(), dir.c_str());
  if (!ok) return -1;
  int64_t k = 0;
  for (auto &s : shapes) {
    for (size_t i = 0; i < s.mesh.num_face_vertices.size(); ++i) {
      if (verts) {
        for (int v = 0; v < 3; ++v) {
          size_t vi = (size_t)s.mesh.indices[i * 3 + v].vertex_index;
          for (int j = 0; j < 3; ++j) verts[k * 9 + v * 3 + j] = attrib.vertices[vi * 3 + j];
        }
        matids[k] = s.mesh.material_ids[i];
      }
      ++k;
    }
  }
  if (mats) {
    for (size_t m = 0; m < materials.size(); ++m) {
      float *o = mats + 11 * m;
      o[0] = materials[m].ior;
      for (int j = 0; j < 3; ++j) {
        o[1 + j] = materials[m].ambient[j];
        o[4 + j] = materials[m].diffuse[j];
        o[7 + j] = materials[m].specular[j];
      }
      o[10] = materials[m].shininess;
    }
  }
  *ntri = k;
  *nmat = (int32_t)materials.size();
  return 0;
}

int ref_write_hdr(const char *path, int w, int h, const float *rgba, int flip) {
  stbi_flip_vertically_on_write(flip);
  return stbi_write_hdr(path, w, h, 4, rgba) ? 0 : -1;
}

}  // extern "C"
