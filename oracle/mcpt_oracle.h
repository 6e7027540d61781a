/* mcpt_oracle.h — TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg).  Never linked into libmcpt_hip.so.
 *
 * A plain-C CPU restatement of the reference's per-sample path (records from
 * include/mcpt_hip.h, byte-identical to MCPT/objdef.h).  Each function cites
 * the reference lines it restates.  Floating point: IEEE binary32, with an
 * explicit fmaf() exactly where OpenCL's default FP_CONTRACT fuses an
 * expression in the reference kernels, libm for the transcendentals; the
 * GPU's OpenCL built-ins (hardware rcp/rsq/sqrt, ocml cos/sin/pow) round some
 * results differently by an ulp, so kernel outputs agree to a few ulp and
 * chaotic paths diverge — tests compare with stated tolerances.
 * Pinned against the reference kernels' own outputs: tests/golden/.
 */
#ifndef MCPT_ORACLE_H
#define MCPT_ORACLE_H
#include <stdint.h>

#include "../include/mcpt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

int oracle_parse_camera(const double pos[3], const double look[3], const double up[3], double fov, mcpt_camera *out);
int oracle_pack_triangles(mcpt_triangle *tris, const int32_t *mat_index, int64_t n);
int oracle_build_hlbvh(const mcpt_triangle *tris, int64_t n, mcpt_bvh_node *nodes);
void oracle_generate(const mcpt_camera *cam, int32_t w, int32_t h, mcpt_ray *rays);
void oracle_intersect(const mcpt_triangle *tris, const mcpt_bvh_node *nodes, const mcpt_ray *rays, int64_t n,
                      mcpt_hit *hits, float tmin);
void oracle_shade(const mcpt_material *mats, mcpt_ray *rays, const mcpt_hit *hits, float *colors, uint32_t *seeds,
                  int64_t n, int32_t max_depth);
void oracle_accumulate(float *colors, float *hist, int32_t *count, int64_t n, int32_t max_attempt);
/* Whole frame loop per pixel (OpenCLApp.cpp:57-82 + colorout.cpp:40-73) over
 * `frames` frames starting at frame index frame_begin, OpenMP over pixels
 * with `threads` threads (<= 0: all).  stats[4] (optional): segments, node
 * visits, triangle tests, unknown-material hits. */
void oracle_render(const mcpt_camera *cam, const mcpt_triangle *tris, const mcpt_bvh_node *nodes,
                   const mcpt_material *mats, int32_t w, int32_t h, int32_t max_depth, int32_t frame_begin,
                   int32_t frames, int32_t max_attempt, uint32_t *seeds, float *hist, int32_t *count,
                   int32_t threads, uint64_t *stats);
/* Same, restricted to a pixel subset (indices into W*H), for bounded samples. */
void oracle_render_pixels(const mcpt_camera *cam, const mcpt_triangle *tris, const mcpt_bvh_node *nodes,
                          const mcpt_material *mats, int32_t w, int32_t h, const int32_t *pixels, int64_t npix,
                          int32_t max_depth, int32_t frame_begin, int32_t frames, int32_t max_attempt,
                          uint32_t *seeds, float *hist, int32_t *count, int32_t threads, uint64_t *stats);
/* Counting mode for SURVEY §8(d)'s E_node/E_tri: 1 = t-pruned traversal
 * (skip a node whose box starts beyond the current hit).  Default 0 =
 * the reference's exhaustive traversal. */
void oracle_set_prune(int on);
/* TreeletBVH<CPU> (MCPT/BVH/treeletBVH.cpp:343-372) in place on a 2n-1-node
 * HLBVH; mcpt_oracle_treelet.cpp.  0 ok, -1 the reference's recursion would
 * not terminate on this tree, -2 bad argument. */
int oracle_treelet(mcpt_bvh_node *nodes, int64_t n_nodes);
/* TreeletBVH<GPU> (treeletBVH.cpp:413-438 + kernels/treeletBVH.cl:230-531), the
 * tree every reference render traverses (scenebuild.cpp:87-95), in place on a
 * 2n-1-node HLBVH; mcpt_oracle_treelet_gpu.cpp (PARITY UNPINNED: the kernel
 * does not compile).  rcp_mant_root_bits: v_rcp_f32(frexp_mant(rootArea)) as
 * float bits (0: the correctly rounded reciprocal); options 0 = the kernel
 * (bit 0: the lowest lane's store lands instead of the highest's; bit 1:
 * refit SAH divided by rootArea — sensitivity knobs, not the reference);
 * stats[8] optional.  0 ok, -1 not an HLBVH layout, -2 bad argument. */
int oracle_treelet_gpu(mcpt_bvh_node *nodes, int64_t n_nodes, uint32_t rcp_mant_root_bits, int32_t options,
                       int64_t *stats);
float oracle_treelet_gpu_root_mant(const mcpt_bvh_node *root);
/* testbvh metrics (bvhtest.cpp): SAH :97-108, LCV :324-444 (counts optional,
 * index i*H + j), EPO_GPU's kernel EPO.cl:133-197 per triangle. */
float oracle_bvh_sah(const mcpt_bvh_node *nodes, int64_t n_nodes);
float oracle_bvh_lcv(const mcpt_bvh_node *nodes, int64_t n_nodes, const mcpt_camera *cam, int32_t w, int32_t h,
                     uint32_t *counts);
void oracle_bvh_epo(const mcpt_bvh_node *nodes, const mcpt_triangle *tris, int64_t n_tris, float *epo, float *area);
int64_t oracle_encode_hdr(int32_t w, int32_t h, const float *rgba, int32_t flip, uint8_t *out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
