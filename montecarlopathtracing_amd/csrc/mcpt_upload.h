// mcpt_upload.h — internal interface between the GPU scene build
// (mcpt_upload.hip) and mcpt_scene_upload_device (mcpt_device.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mcpt_hip.h"

namespace mcpt {

// Device arrays of a scene built on the GPU, in the byte layouts of
// mcpt_device.hip's DevNode4 (near4, nodes4), DevNode4Q (near4q), DevNode
// (nodes), DevTri (tris) and DevTriQ (triq).  The caller owns (hipFree) them.
struct DeviceScene {
  void *near4, *near4q, *nodes4, *nodes, *tris, *triq;
  int64_t n_near4, n_nodes4, n_int;
  int32_t stack_depth;  // the reference tree's DFS stack bound (mcpt_bvh_stack_depth)
  int32_t depth4;       // max of both 4-wide trees' stack needs
  bool quant;           // near4q / triq built
  mcpt_bvh_node root;   // host copy of node 0
};

// tris (n) and nodes (2n-1, the HLBVH layout) are DEVICE arrays; on failure
// the arrays already allocated in *out are left for the caller to free.
int build_scene_device(const mcpt_triangle *tris, int64_t n, const mcpt_bvh_node *nodes, int32_t n_mats,
                       hipStream_t st, DeviceScene *out);

}  // namespace mcpt
