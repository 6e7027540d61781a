/* mcpt_oracle_treelet.cpp — TEST INFRASTRUCTURE ONLY: literal CPU restatement
 * of the reference's TreeletBVH<CPU> (MCPT/BVH/treeletBVH.cpp:1-387), the
 * Karras & Aila 2013 treelet restructuring the reference applies for
 * config "bvhtype": "treelet" (MCPT/scenebuild.cpp:70-73).
 *
 * Written the way the reference is: the same std::vector / std::push_heap /
 * std::pop_heap / std::sort calls (libstdc++ here, MSVC's STL there: both
 * implement pop_heap as Floyd's hole descent + sift-up and push_heap as a
 * sift-up, so the heap's array layout — which decides the treelet's leaf
 * order — is the same), the same float expression trees (this file is
 * compiled with -ffp-contract=off, the reference host's plain IEEE math),
 * std::min/std::max for box unions (oclbasic.h:196-226).  The product's GPU
 * restatement (csrc/mcpt_build.hip, mcpt_treelet_device) writes the heap out
 * by hand; tests compare the two node arrays bit for bit.
 *
 * Quirks kept (they decide the output):
 *  - getInformation's leaf test is `id > size/2` (treeletBVH.cpp:327), so the
 *    first leaf n-1 is treated as an internal node whose two children are
 *    node `left` (its triangle index, read as a node index);
 *  - leaf costs are seeded as cost[1<<i] = SAH[pq[i]] (:125-127) while the
 *    union boxes map bit k to pq[n-1-k] (:106-118) and the rebuild maps bit k
 *    to pq[size-1-k] (:259,271);
 *  - the parent walk reads the ORIGINAL tree's parent links (:352-366);
 *  - refit SAH divides by rootArea, captured once before any rebuild.
 * If the first-leaf quirk makes the reference's recursion cycle (the triangle
 * index of leaf n-1 names one of its ancestors, or itself) the reference
 * overflows its stack; here that is reported as -1.
 */
#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <vector>

#include "mcpt_oracle.h"

namespace {

constexpr int MAX_NODE = 7;                    // treeletBVH.cpp:14
constexpr int TOTAL_BIT = (1 << MAX_NODE) - 1;  // :15
constexpr float Cinn = 1.2f, Cleaf = 0.0f, Ctri = 1.0f;  // auxiliary.h:9-11

struct V4 {
  float s[4];
};
struct Box {
  V4 bbmin, bbmax;
};

V4 ld(const float *p) { return V4{{p[0], p[1], p[2], p[3]}}; }
V4 vmin(const V4 &a, const V4 &b) {  // oclbasic.h:196-201
  V4 r;
  for (int i = 0; i < 4; ++i) r.s[i] = std::min(a.s[i], b.s[i]);
  return r;
}
V4 vmax(const V4 &a, const V4 &b) {  // oclbasic.h:214-219
  V4 r;
  for (int i = 0; i < 4; ++i) r.s[i] = std::max(a.s[i], b.s[i]);
  return r;
}
float AREA(const V4 &bbmin, const V4 &bbmax) {  // auxiliary.cpp:15-18
  V4 arg;
  for (int i = 0; i < 4; ++i) arg.s[i] = bbmax.s[i] - bbmin.s[i];
  return 2.0f * (arg.s[0] * arg.s[1] + arg.s[0] * arg.s[2] + arg.s[1] * arg.s[2]);
}
Box unionBox(const Box &a, const Box &b) {  // auxiliary.cpp:5-10
  Box r;
  r.bbmax = vmax(a.bbmax, b.bbmax);
  r.bbmin = vmin(a.bbmin, b.bbmin);
  return r;
}

struct State {
  mcpt_bvh_node *bvh;
  std::vector<float> SAHValue;
  std::vector<char> onStack;  // cycle detection for the recursion quirk
  float rootArea;
  bool cycle = false;
  V4 bmin(int i) const { return ld(bvh[i].bbmin); }
  V4 bmax(int i) const { return ld(bvh[i].bbmax); }
};

// treeletBVH.cpp:321-341 recurseGet, on the ORIGINAL tree (`orig`)
void recurseGet(State &S, const mcpt_bvh_node *orig, size_t size, int rootID, float rootArea) {
  if (S.SAHValue[rootID] == -1.0f) {
    if ((size_t)rootID > (size >> 1)) {
      S.SAHValue[rootID] = (Ctri + Cleaf) * AREA(ld(orig[rootID].bbmin), ld(orig[rootID].bbmax)) / rootArea;
      return;
    }
    if (S.onStack[rootID]) {  // the reference recurses forever here
      S.cycle = true;
      return;
    }
    S.onStack[rootID] = 1;
    const int left = orig[rootID].left, right = orig[rootID].right;
    recurseGet(S, orig, size, left, rootArea);
    if (S.cycle) return;
    recurseGet(S, orig, size, right, rootArea);
    if (S.cycle) return;
    S.SAHValue[rootID] = S.SAHValue[left] + S.SAHValue[right] +
                         Cinn * (AREA(ld(orig[rootID].bbmin), ld(orig[rootID].bbmax))) / rootArea;
    S.onStack[rootID] = 0;
  }
}

// treeletBVH.cpp:30-318
void reconstructTreelet(State &S, int rootID) {
  mcpt_bvh_node *bvh = S.bvh;
  struct QueueNode {
    int id;
    float value;
    bool operator<(const QueueNode &ano) const {
      if (value < ano.value) return true;
      else if (value == ano.value && id < ano.id) return true;
      return false;
    }
  };
  std::vector<QueueNode> pq;
  std::vector<int> freeBVHNode;
  pq.push_back({rootID, S.SAHValue[rootID]});

  while (pq.size() < (size_t)MAX_NODE) {
    auto maxNode = pq.front();
    auto maxNodeID = maxNode.id;
    std::pop_heap(pq.begin(), pq.end());
    pq.pop_back();
    if (maxNode.value < 0.0f) {
      pq.push_back({maxNodeID, -1.0f});
      break;
    }
    auto lid = bvh[maxNodeID].left;
    auto rid = bvh[maxNodeID].right;
    if (lid == rid) {
      pq.push_back({maxNodeID, maxNodeID * (-1.0f)});
      std::push_heap(pq.begin(), pq.end());
      continue;
    } else {
      pq.push_back({lid, S.SAHValue[lid]});
      std::push_heap(pq.begin(), pq.end());
      pq.push_back({rid, S.SAHValue[rid]});
      std::push_heap(pq.begin(), pq.end());
      freeBVHNode.push_back(maxNodeID);
    }
  }

  int NOW_NODE, NOW_TOTAL_BIT;
  if (pq.size() < 3) return;
  if (pq.size() < (size_t)MAX_NODE) {
    NOW_NODE = (int)pq.size();
    NOW_TOTAL_BIT = (1 << NOW_NODE) - 1;
  } else {
    NOW_NODE = MAX_NODE;
    NOW_TOTAL_BIT = TOTAL_BIT;
  }

  std::vector<float> areaOfUnion(1 << NOW_NODE);
  for (int i = 1; i < (1 << NOW_NODE); ++i) {
    std::vector<int> x(NOW_NODE, 0);
    int temp = NOW_NODE - 1, s = i;
    while (s > 0) {
      x[temp] = s & 0x1;
      s >>= 1;
      --temp;
    }
    Box box = {{{FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX}}, {{-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX}}};
    for (int j = 0; j < NOW_NODE; ++j)
      if (x[j]) box = unionBox(box, {S.bmin(pq[j].id), S.bmax(pq[j].id)});
    areaOfUnion[i] = AREA(box.bbmin, box.bbmax);
  }

  std::vector<float> cost(1 << NOW_NODE);
  for (int i = 0; i < NOW_NODE; ++i) cost[(1 << i)] = S.SAHValue[pq[i].id];

  struct Node {
    int count, value;
    bool operator<(const Node &ano) const {
      if (count < ano.count) return true;
      else if (count == ano.count && value < ano.value) return true;
      return false;
    }
  };
  std::vector<Node> bitsVector;
  for (int s = 1; s < (1 << NOW_NODE); ++s) bitsVector.push_back({__builtin_popcount(s), s});
  std::sort(bitsVector.begin(), bitsVector.end());

  std::vector<int> partitionPos(1 << NOW_NODE);
  size_t startFrom;
  for (startFrom = 0; startFrom < bitsVector.size(); ++startFrom)
    if (bitsVector[startFrom].count == 2) break;
  // the k loop with its goto (:168-198) visits every entry of count >= 2 in order
  for (; startFrom < bitsVector.size(); ++startFrom) {
    float cs = FLT_MAX;
    float ps = 0;
    int s = bitsVector[startFrom].value;
    int delta = (s - 1) & s;
    int p = (-delta) & s;
    do {
      float c = cost[p] + cost[s ^ p];
      if (c < cs) {
        cs = c;
        ps = p;
      }
      p = (p - delta) & s;
    } while (p != 0);
    cost[s] = Cinn * areaOfUnion[s] + cs;
    partitionPos[s] = ps;
  }

  // rebuild (:201-291)
  struct SplitInnerNode {
    int parentCode, selfCode, parentID;
  };
  auto leafOf = [&](int code) {  // toRight = 31 - CLZ(code): the bit index
    int toRight = 31 - __builtin_clz((unsigned)code);
    return pq[pq.size() - toRight - 1].id;
  };
  std::vector<SplitInnerNode> toSplit, answer;
  int freeNodeNow = 0;
  toSplit.push_back({NOW_TOTAL_BIT, partitionPos[NOW_TOTAL_BIT], freeBVHNode[freeNodeNow]});
  ++freeNodeNow;
  while (!toSplit.empty()) {
    for (auto i : toSplit) {
      auto leftCode = partitionPos[i.selfCode];
      auto rightCode = partitionPos[i.selfCode ^ i.parentCode];
      auto parentNodeID = i.parentID;
      if (__builtin_popcount(i.selfCode) == 1) {
        int node = leafOf(i.selfCode);
        bvh[parentNodeID].left = node;
        bvh[node].parent = parentNodeID;
      } else {
        int freeNext = bvh[parentNodeID].left = freeBVHNode[freeNodeNow++];
        answer.push_back({i.selfCode, leftCode, freeNext});
        bvh[freeNext].parent = parentNodeID;
      }
      if (__builtin_popcount(i.parentCode ^ i.selfCode) == 1) {
        int node = leafOf(i.parentCode ^ i.selfCode);
        bvh[parentNodeID].right = node;
        bvh[node].parent = parentNodeID;
      } else {
        int freeNext = bvh[parentNodeID].right = freeBVHNode[freeNodeNow++];
        answer.push_back({i.selfCode ^ i.parentCode, rightCode, freeNext});
        bvh[freeNext].parent = parentNodeID;
      }
    }
    toSplit = std::move(answer);
    answer.clear();
  }

  // refit (:293-302)
  for (int i = (int)freeBVHNode.size() - 1; i >= 0; --i) {
    auto &node = bvh[freeBVHNode[i]];
    V4 mx = vmax(S.bmax(node.left), S.bmax(node.right));
    V4 mn = vmin(S.bmin(node.left), S.bmin(node.right));
    std::memcpy(node.bbmax, mx.s, 16);
    std::memcpy(node.bbmin, mn.s, 16);
    S.SAHValue[freeBVHNode[i]] = S.SAHValue[node.left] + S.SAHValue[node.right] +
                                 Cinn * (AREA(S.bmin(freeBVHNode[i]), S.bmax(freeBVHNode[i]))) / S.rootArea;
  }
}

}  // namespace

extern "C" int oracle_treelet(mcpt_bvh_node *nodes, int64_t n_nodes) {
  if (!nodes || n_nodes <= 0) return -2;
  const std::vector<mcpt_bvh_node> orig(nodes, nodes + n_nodes);  // `bvh` in the ctor (:346)
  State S;
  S.bvh = nodes;  // `bvhnode`, the copy that is rebuilt
  S.SAHValue.assign(n_nodes, -1.0f);
  S.onStack.assign(n_nodes, 0);
  const size_t size = (size_t)n_nodes;
  {
    float rootArea = AREA(ld(orig[0].bbmin), ld(orig[0].bbmax));  // getInformation :343-347
    recurseGet(S, orig.data(), size, 0, rootArea);
    if (S.cycle) return -1;
  }
  S.rootArea = AREA(ld(orig[0].bbmin), ld(orig[0].bbmax));  // :351
  std::vector<int> flag(size >> 1);
  for (size_t i = (size >> 1); i < size; ++i) {  // :358-371
    auto nowParent = orig[i].parent;
    while (nowParent != -1) {
      if (!flag[nowParent]) {
        flag[nowParent] = 1;
        break;
      }
      reconstructTreelet(S, nowParent);
      nowParent = orig[nowParent].parent;
    }
  }
  return 0;
}
