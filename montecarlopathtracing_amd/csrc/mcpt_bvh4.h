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

// 64-B quantized form of a Node4Rec, the search-tree node k_render reads with
// four 16-B gathers instead of seven.  Per axis a float origin o_a and a
// power-of-two scale s_a; every slot plane is one byte q, decoded on the GPU as
// fma((float)q, s_a, o_a) (one rounding, = std::fma).  The bytes are chosen so
// that every decoded box STRICTLY contains the slot's exact box on every side
// (lo' < lo, hi' > hi), and every decoded value is a normal float or zero.  The
// slab test is monotone in the box, so a strictly larger box passes whenever
// the exact one does -- also when a direction component is +-0 and the origin
// lies on a box plane, the case where a merely non-strict container can fail
// (DESIGN.md §3.3).  Layout = the four loads:
//   [o.x o.y o.z s.x] [q 0..15] [q 16..23, s.y, s.z] [link 0..3]
// q value i belongs to slot i/6, plane i%6 (minx maxx miny maxy minz maxz),
// i.e. Node4Rec::q's order.  Empty slots keep their link (kEmptySlot4).
struct Node4Q {
  float org[3];
  float sx;
  uint8_t q[24];
  float sy, sz;
  int32_t link[4];
};
static_assert(sizeof(Node4Q) == 64, "four 16-B loads");

// Returns 0, or -1 when some axis cannot be quantized within the float range
// (the scene then keeps the 128-B nodes).
int quantize_node4(const Node4Rec &in, Node4Q &out);

}  // namespace mcpt
