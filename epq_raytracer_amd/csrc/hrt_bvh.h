// hrt_bvh.h -- host-built bounding volume hierarchy for bounce segments (HRT_KERNEL_BUNDLE_BVH).
//
// The reference scans every triangle of every mesh whose AABB test passes (raytracing.glsl:278-286);
// the BVH only lets the trace kernel skip triangles it can PROVE the reference rejects for a given
// ray, so results stay byte-identical (DESIGN.md "BVH cull" has the error analysis).  Each entry is
// one (mesh m, triangle i) of the reference's scan with key = 1 + its scan position, which breaks
// equal-distance ties exactly like the reference's strict '<' in scan order.
#pragma once

#include <stdint.h>

#include <vector>

#include "hip_raytrace.h"

namespace hrt {

// 16 floats per node:
//   [0..2]  box lo (vertices a, a+e1, a+e2 of every triangle below, rounded outward)
//   [3]     margin a: the box grows by a + b R for a lane whose origin is within R of every vertex
//   [4..6]  box hi
//   [7]     margin b (from tri_ext = the largest per-axis triangle extent below and G = max |e|/|n|)
//   [8..10] normal-cone axis c (unit)
//   [11]    cos(phi)   (phi >= angle(c, n_i / |n_i|) for every triangle; (0, 1) = no cone)
//   [12]    sin(phi)
//   [13]    rho = max |n_i - e1_i x e2_i| / |n_i|   (record normal vs exact cross product)
//   [14]    bits: leaf ? first_prim | count << 27 : right child (the left child is the next node)
//   [15]    bits: escape node (preorder successor that is not a descendant; n_nodes = end)
// 16 floats per prim: (a, key bits) (e1, mesh bits) (e2, triangle index bits) (n, 0).
//
// Grazing band: the box cull's error bound needs |d.n^| >= kBandTau for front-facing triangles, so
// every triangle with d.n^ in (-kBandTau, +2e-5) ("in the band" of d) is tested separately.  Ray
// directions are binned on a cube map (face, iu, iv), dir_res x dir_res cells per face; band_list of a
// cell holds every leaf prim that is in the band of SOME direction of that cell.
struct BvhHost {
  std::vector<float> nodes;
  std::vector<float> prims;      // leaf-ordered regular triangles
  std::vector<float> irregular;  // entries the analysis does not cover: tested for every bounce ray
  std::vector<uint32_t> entries;    // per leaf prim: triangle index | mesh << 26
  std::vector<uint32_t> key_base;   // per mesh: scan key of (m, i) = key_base[m] + i (mod 2^32)
  std::vector<uint32_t> band_off;   // 6 dir_res^2 + 1 offsets into band_list
  uint32_t dir_res = 64;            // direction cells per face edge (dir_res_for)
  double sah_tri_frac = 0.0;        // expected leaf triangle tests of a uniform random ray / entries
  double margin_frac = 0.0;         // mean over nodes of (a + b R_scene) / the box's largest extent
  std::vector<uint32_t> band_list;  // per entry: its prim's index (uploaded as 16-bit words, band_wide())
  std::vector<float> band_nhat;     // per prim: n / |n| in binary32, n^.a (the entries' pre-check normal and plane)
  float band_a1 = 0.0f;             // max over prims of |a|_1 (the plane filter's tolerance)
  bool band_wide() const { return n_prims > 65536u; }  // entries of 32 bits instead of 16
  std::vector<float> wq_nodes;      // BUNDLE_WQ's 48 B node image (make_wq_nodes)
  bool wq_ok = false;               // the image exists (fewer than 65536 nodes)
  uint32_t wq_n_nodes = 0;          // its nodes (the binary nodes a group collapse keeps)
  uint32_t wq_width = 2;            // its largest group (children tested per node pop)
  uint32_t n_nodes = 0, n_prims = 0, n_irregular = 0, n_never = 0;  // never = zero normal (dn == 0)
  double rho_max = 0.0;
  float abs_coef = 0.0f, rel_t = 0.0f;  // box-test t-slack: [-abs_coef R, best (1 + rel_t) + abs_coef R]
  float band_tau = 0.0f;            // the grazing band's width tau_g this hierarchy was built for
};

// auto HRT_OPT_WQ_NODE_RADIUS: per-node R above this HRT_SCENE_BVH_MARGIN_MILLI (island 26 / island@4 69:
// scene-wide R; cave 197: per node, 8.54 -> 7.38 ms per frame; island with per-node R 2.33 -> 2.39 ms)
constexpr uint32_t kNodeRadiusMarginMilli = 100;

#ifndef HRT_BAND_TAU
#define HRT_BAND_TAU 3e-3f
#endif
constexpr float kBandTau = HRT_BAND_TAU;
// (tau_g trades the nodes' box margins, ~ 1 / tau_g, against the band lists' length, ~ cell + tau_g.
// r03: 4.5e-3 / 6e-3 / 9e-3: 6.36 / 6.43 / 6.62 ms per frame on cave (profiles/r03/r03f_*) -- measured
// while the band's owner search lost list starts (fixed in r03v); with every band entry tested for its
// own ray a band test is the dearer side: 3e-3, island 2.132 -> 2.109, cave 6.041 -> 5.945 ms with 256
// cells per face edge (512 cells: 2.089 / 5.827 ms but 3x the counter bytes, below; 2e-3 and 1.5e-3
// measure the same; profiles/r03/r03w_*, r03x_*, r03z_*).  The node margins cost little
// (tools/margin_emul.py: 7.1 -> 7.5 leaf tests per cave bounce ray at 2e-3).
// build_bvh takes it as a parameter, the kernels read it from
// TraceParams::bvh_band_tau.)
// Grazing-band entries: the prim index alone, 2 B (4 B above 65536 prims); the pre-check reads the
// prim's unit normal from BvhHost::band_nhat (a few KB, cache-resident) instead of carrying a quantized
// copy in every entry (r03: 8 B entries with fixed-point normals made the lists 29 MB on island, and
// their reads most of the kernel's fetched bytes).  n^ in binary32 is within 2^-24 per component of
// n / |n|, so d.n^ is off by < 4e-7 for |d| = 1, far inside the pre-check's 1e-5 widening.
// Direction cells per cube-map face edge: finer cells mean shorter per-ray lists (a ray scans its
// cell's list on every bounce) but ~linearly more entries per triangle (a triangle's band is a
// great-circle strip).  256 up to 8K entries (island: 9 entries per list, 29 MB), 128 up to 32K, 64
// above (profiles/r01p_*).
#ifndef HRT_DIR_RES_SMALL
// r03z (tau 3e-3): 256 / 384 / 512 cells -- island 2.109 / 2.101 / 2.089 ms, FETCH_SIZE x2 0.32 / 0.76 /
// 1.06 GB per frame; cave 5.945 / 5.871 / 5.827 ms, 0.40 / 0.64 / 0.80 GB: the finer lists are 1-2%
// faster but no longer fit the L2 (island 512: 16.5 MB of entries + 6.3 MB of offsets), 256 kept then.
// r05 (20-frame launches at bench.py's shape, profiles/r05/r05q-t_*): 256 / 512 / 1024 / 1536 / 2048
// cells -- island 1.760 / 1.745 / 1.719 / 1.717 / 1.712 ms, cave 5.436 / 5.316 / 5.260 / 5.257 / 5.292 ms;
// a bounce lane scans ~13 band entries per lookup at 256 on cave, 6.4 at 1024.  The time is worth more
// than the L2 residency; 1024 (island 24 M entries + 25 MB of offsets, ~74 MB on the device; cave ~106
// MB; tau_g 1.5e-3 / 2e-3 / 4e-3 / 5e-3 at 1024 were no better).
#define HRT_DIR_RES_SMALL 1024
#endif
constexpr int kDirResMax = HRT_DIR_RES_SMALL;
inline int dir_res_for(uint64_t entries) { return entries <= 8192 ? HRT_DIR_RES_SMALL : entries <= 32768 ? 128 : 64; }

// Leaf size when HRT_OPT_BVH_LEAF_SIZE is 0 (auto): 2 for scenes BUNDLE_WQ takes (grouped nodes test
// 4 children per visit, so smaller leaves cost few extra steps and save triangle pairs: island 3.42 ->
// 3.34 ms, profiles/r02j_wq_groups_ab.jsonl), 4 above (fewer nodes for the LDS-resident hierarchy).
inline uint32_t auto_leaf_size(uint64_t entries) { return entries <= 8192 ? 2u : 4u; }

constexpr uint32_t kBvhMaxMeshes = 64;     // per-lane mesh filter is a 64-bit mask
constexpr uint32_t kBvhMaxLeafCount = 16;  // leaf count lives in bits 27..31 of node word 14
// The grazing-band lists hold ~450 entries (16 B) per triangle on the reference's meshes, so the
// hierarchy is not built above this many (mesh, triangle) entries (~1.9 GB of band lists).
constexpr uint64_t kBvhMaxEntries = 1u << 18;

// BUNDLE_WQ node image, 12 floats per node (48 B instead of 64, so cave-sized hierarchies leave
// room for the pair stacks in LDS).  A wide tree over a subset of the binary nodes: the children of an
// inner node are a GROUP of 2..width kept nodes stored side by side at fc .. fc + count - 1 (the binary
// children, the larger-area inner ones replaced by their own children while the group has room), so
// a (ray, group) stack entry tests the whole group with no parent record.  Root at 0.
//   [0..2] box lo, [3] margin a, [4..6] box hi, [7] margin b   (the kept binary node's, unchanged)
//   [8]  bits: cone axis x | axis y << 16   (binary16, nearest: |error| <= 2^-12 per component)
//   [9]  bits: cone axis z | cos(phi) << 16 (cos rounded down)
//   [10] bits: S = sin(phi)^2 x 1.00001 (rounded up; the kernel's squared back-face test multiplies by it,
//        the unsquared ones use sqrt(S)) | escape << 16 (the next member of its group; the last member:
//        its parent's escape; root: the node count -- a stackless walk continues there after the subtree)
//   [11] bits: leaf ? first_prim | count << 27 : fc | (group count - 1) << 16
// The kernel widens its back-face cone test by the axis error, so the image only ever keeps more;
// skipping a collapsed node's own box test only keeps more as well.
constexpr float kWqAxisErr = 5e-4f;  // >= sqrt(3) 2^-12: bound on |d.axis_16 - d.axis| for |d| = 1
constexpr uint32_t kWqMaxWidth = 4;  // widest group an image may have (HRT_OPT_BVH_WIDTH; the kernel's slots)
constexpr uint32_t kWqDefaultWidth = 4;
bool make_wq_nodes(const BvhHost& b, std::vector<float>& out, uint32_t width, uint32_t* n_out, uint32_t* w_out);

// Builds the hierarchy over every (mesh, triangle) entry of the scene.  Returns false (and leaves
// `out` empty) when the scene has more than kBvhMaxMeshes meshes, kBvhMaxEntries entries or 2^26
// triangles.  bands = false leaves the grazing-band lists to a later build_bands (hrt_set_scene picks
// the leaf size from the hierarchy first; the lists are most of the build's time).
bool build_bvh(const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes, uint32_t n_meshes,
               uint32_t leaf_size, BvhHost& out, uint32_t wq_width = kWqDefaultWidth, float band_tau = kBandTau,
               bool bands = true);
// The grazing-band lists (band_off, band_list, band_nhat, band_a1) of a hierarchy built without them.
void build_bands(BvhHost& out);
// Drops the process-wide band-list cache of build_bands; returns the host bytes it held.
uint64_t release_band_cache();

}  // namespace hrt
