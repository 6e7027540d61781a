// Host-side builder of the EXACT path's search tree (mcpt_sah.cpp), shared
// with mcpt_device.hip.  The record layout is DevNode4's.
#pragma once
#include <cstdint>
#include <vector>

namespace mcpt {

constexpr int32_t kEmptySlot4 = INT32_MIN + 2;  // == kEmptySlot in mcpt_device.hip

// 128-B 4-wide node: slot k's box is q[6k..6k+5] = (minx,maxx,miny,maxy,minz,maxz);
// link >= 0 another node, < 0 a leaf (~triangle), kEmptySlot4 unused.
struct Node4Rec {
  float q[24];
  int32_t link[4];
  float pad[4];
};
static_assert(sizeof(Node4Rec) == 128, "DevNode4 layout");

// One leaf of the reference HLBVH: its triangle and its box exactly as the
// reference stores it (the box the reference's slab test sees).
struct LeafRef {
  float box[6];  // minx maxx miny maxy minz maxz
  int32_t tri;
};

// Binned-SAH 4-wide tree over the reference's leaves, one leaf per slot, so
// every leaf keeps the reference's own box and every internal box is a union
// of them.  Nodes come out in depth-first preorder (root = 0).  *stack_need
// bounds the stack entries any visiting order can hold (k-1 per k-slot node
// on a root-to-leaf path).  Deterministic for a given input; threads only
// split the work.  Returns 0, or -1 for an empty input.
int build_sah4(const std::vector<LeafRef> &leaves, std::vector<Node4Rec> &out, int32_t *stack_need, int threads);

}  // namespace mcpt
