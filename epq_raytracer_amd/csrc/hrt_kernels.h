// hrt_kernels.h -- launch interface between the C-ABI layer (hrt_api.cpp) and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hip_raytrace.h"

namespace hrt {

constexpr uint32_t kSchedWords = 1024;  // TraceParams::sched (hrt_kernels.hip kSchedHist ...)

// Kernel argument block (passed by value; lives in the kernarg segment, read through SGPRs).
struct TraceParams {
  const float4* rays;            // W*H sample centres, indexed by global pixel id
  const hrt_sphere* spheres;
  const hrt_triangle* tris;
  const hrt_mesh* meshes;
  const float4* tri_nhat;        // per triangle: normalize(normal) (tri_normals at hrt_set_scene)
  uint32_t* img8;                // local_rows x W packed RGBA8 (RGBA8 mode) or nullptr
  float4* img32;                 // local_rows x W float4 (RGBA32F mode) or nullptr
  unsigned long long* counters;  // [0] segments, [1] triangle tests, [2] wave steps; nullptr = off
  unsigned long long* diag;      // HRT_OPT_COUNTERS = 2: cull diagnostics (HRT_DIAG_*), else nullptr
  unsigned long long* tile_cycles;  // HRT_OPT_COUNTERS = 2: per 8x8 tile {clocks, bounce iterations,
                                    // bounce survivors, bounce clocks}, else nullptr
  hrt_push_constants pc;
  uint32_t local_rows, row_tile, part_index, part_count;
  uint32_t n_tris;               // uploaded triangle count (LDS staging)
  // Bundle variants: per-frame compacted camera-facing triangles (camera_lists kernel).
  uint32_t* cam_start;           // num_meshes: first compacted record of mesh m
  uint32_t* cam_count;           // num_meshes: its number of camera-facing triangles
  uint32_t cam_list_capacity;    // sum of the meshes' len (record capacity)
  float4* cam_tris;              // 4 float4 per record: (ao, num_t) (e1, index bits) (e2, -) (n, -)
  float4* cam_cull;              // 5 float4 per record: bundle-cull linear forms + margins
  uint32_t sec_batch;            // bounce segments run once this many lanes of a wave wait (1..64)
  // Persistent (LDS) variants' scheduler: sched[0] work counter, [1] item count, [2] heavy tiles,
  // [3] first heavy cost bucket, [5] cooperative-item counter, [6..7] u64 sum of tile costs,
  // [8..) planner histogram / offsets / cursors (kSchedWords in all); tile_cost per 8x8 tile (shader clocks / 16, this trace);
  // item_buf (tiles x 8) the planned items; items = item_buf when this trace follows a plan.
  uint32_t* sched;
  uint32_t* tile_cost;
  uint32_t* item_buf;
  const uint32_t* items;
  uint32_t split_k;              // items per heavy tile (1 = no splitting; 2, 4, 8)
  int32_t split_factor;          // heavy: cost > split_factor x a resident wave's share (-1: auto)
  uint32_t split_prio;           // heavy items run at raised wave priority (s_setprio 3)
  uint32_t coop;                 // heavy tiles run cooperatively by a whole workgroup (BUNDLE_CULL_LDS)
  uint32_t plan_valid;           // tile_cost holds the previous trace's costs of this context
  uint32_t probe;                // a 1-sample planning probe (HRT_OPT_PROBE): launched as the diagnostics
                                 // instantiation (<.., true>, all diagnostics pointers null) so that
                                 // profilers list it apart from the frame's trace kernel
  uint32_t num_cus;              // compute units of the device (persistent grid size)
  // BUNDLE_BVH: bounce-segment hierarchy built by hrt_set_scene (hrt_bvh.h records); nullptr = none.
  const float4* bvh_nodes;       // 4 float4 per node, preorder with escape indices
  const float4* bvh_wq_nodes;    // 3 float4 per node: BUNDLE_WQ's image (hrt_bvh.h make_wq_nodes), or nullptr
  uint32_t bvh_wq_n_nodes;       // its nodes
  uint32_t bvh_wq_width;         // its largest group (children per node-stack entry)
  const float4* bvh_prims;       // 4 float4 per leaf triangle
  const float4* bvh_irregular;   // 4 float4 per entry outside the analysis (tested for every ray)
  const uint32_t* bvh_band_off;  // 6 bvh_dir_res^2 + 1 offsets: grazing-band prims per direction cell
  uint32_t bvh_dir_res;          // direction cells per cube-map face edge
  uint32_t bvh_sah_milli;        // hierarchy quality (HRT_SCENE_BVH_SAH_MILLI)
  const void* bvh_band;          // grazing-band entries: prim indices, 16-bit (32-bit when bvh_band_wide)
  const float4* bvh_band_nhat;   // per prim: its unit normal (the entries' pre-check)
  const uint32_t* bvh_band_rec;  // BUNDLE_WQ: 8 dwords per direction cell (start, length, 12 first entries), or null
  uint32_t bvh_band_wide;
  uint32_t bvh_band_bits;        // bit width of the longest band list
  uint32_t cam_lists_ready;      // (host) cam_tris / cam_cull / cam_meta already hold this camera's lists
  const uint32_t* bvh_entries;   // per leaf prim: triangle index | mesh << 26 (BUNDLE_BVH_LDS)
  const uint32_t* bvh_keybase;   // per mesh: key = keybase[m] + triangle index
  uint32_t bvh_n_nodes, bvh_n_irregular, bvh_n_prims, bvh_n_meshes;
  float bvh_abs_coef, bvh_rel_t;  // box-test t-slack (hrt_bvh.h)
  uint32_t bvh_max_leaf;         // largest leaf triangle count of the hierarchy
  uint32_t wq_ncap, wq_tcap;     // BUNDLE_WQ: per-wave node / triangle pair stack capacities (launch_trace)
  // Frames per launch (persistent variants, hrt_compute_n): frame f (0 <= f < n_frames) uses
  // rng_offset + f and writes img8 / img32 + f * frame_stride pixels.  0 or 1: one frame.
  uint32_t n_frames;
  size_t frame_stride;
  uint32_t bvh_node_r;  // BUNDLE_WQ: trace_bundle_wq_nr, box margins with a per-node R (HRT_OPT_WQ_NODE_RADIUS)
  float bvh_band_tau;   // the grazing band's width tau_g the hierarchy and band lists were built for
  float bvh_band_a1;    // max over prims of |a|_1: the band's plane filter tolerance (bvh_band_nhat .w = n^.a)
  uint32_t grab_always; // (debug, HRT_DEBUG_OPT_GRAB_RUNS) persistent waves take kGrab items per atomic to the end
  // (builds with -DHRT_TIMELINE=1, HRT_DEBUG_OPT_TIMELINE) per executed work item of the persistent kernels:
  // {s_memrealtime at its start, when its tile list was built, at its end, tile | log2 k << 22 | s << 25 |
  // hot << 31 | frame << 32 | run << 40 | sky << 47 | resident wave << 48}; timeline_count counts the records (capacity timeline_cap)
  unsigned long long* timeline;
  uint32_t* timeline_count;
  uint32_t timeline_cap;
  // persistent kernels (HRT_TL_PREPASS): per 8x8 tile of this launch, the wave's primary triangle list and
  // octant table as build_tile_list makes them (kTlRecWords words: list entries per lane, octant test sums
  // per lane, n, ok, aabb lo / hi, aabb_ok), filled by the tile_lists kernel before the trace; nullptr = off
  uint32_t* tl_cache;
  uint32_t tl_lists_ready;  // tl_cache already holds this camera's lists (hrt_api.cpp launch_frames): no tile_lists
  uint32_t split_factor4;   // (host side, launch_trace) the heavy threshold in quarters of a wave's share; 0: split_factor
};
constexpr uint32_t kTlRecWords = 136;

// Per device, once: the dynamic-LDS limits of the persistent kernels (hipFuncSetAttribute).
hipError_t ensure_kernel_attributes(int device);
// Launches the trace kernel(s); *ran / *block receive the resolved hrt_kernel and workgroup size.
hipError_t launch_trace(const TraceParams& p, int variant, hipStream_t stream, int* ran, int* block);
int resolve_variant(const TraceParams& p, int variant);  // the kernel an HRT_KERNEL_* request runs
// Ray centres (first + px * x) + py * y for every pixel of a width x height image (hrt_generate_rays).
hipError_t launch_make_rays(float4* rays, uint32_t width, uint32_t height, const float first[3], const float px[3],
                            const float py[3], hipStream_t stream);
hipError_t launch_clear(uint32_t* img8, float4* img32, size_t npix, hipStream_t stream);
// the nf frames of a stack (image f at f * npix) folded into the accumulator as frames frame0 + f
hipError_t launch_accumulate_frames(uint32_t* cur8, const uint32_t* stack8, float4* cur32, const float4* stack32,
                                   size_t npix, uint32_t nf, uint32_t frame0, hipStream_t stream);
hipError_t launch_tri_normals(const hrt_triangle* tris, float4* nhat, uint32_t n, hipStream_t stream);
// BUNDLE_WQ's per-cell band records from the offsets and the 16-bit lists (hrt_kernels.hip band_cell).
hipError_t launch_band_records(const uint32_t* off, const uint32_t* band16, uint32_t* rec, uint32_t cells,
                               hipStream_t stream);
hipError_t launch_accumulate(uint32_t* cur8, const uint32_t* new8, float4* cur32, const float4* new32, size_t npix,
                             uint32_t frame, hipStream_t stream);
// Row-tile framebuffer assembly: gathered = parts x local_rows rows (rank-major), frame = height rows of
// row_words 4-byte words; global row y comes from part (y / row_tile) % parts (hip_raytrace.h partition).
hipError_t launch_assemble_rows(const uint32_t* gathered, uint32_t* frame, uint32_t row_words, uint32_t height,
                                uint32_t local_rows, uint32_t row_tile, uint32_t parts, hipStream_t stream);
// hrt_debug_math_check: fast division / sqrt paths vs the IEEE sequences (out[4] device counters).
hipError_t launch_math_check(uint32_t n, uint32_t seed, unsigned long long* out, hipStream_t stream);
hipError_t launch_band_flatten_check(const uint32_t* n, const uint32_t* b0, uint32_t rounds, uint32_t* out,
                                     hipStream_t stream);  // BandFlat on 64 given lists
hipError_t launch_math_check_rng(unsigned long long* out, hipStream_t stream);  // all 2^32 RNG states
// the pair traversal's LDS handoff protocol on a scripted wave (hrt_debug_wq_protocol)
hipError_t launch_wq_protocol_check(uint32_t rounds, const uint32_t* cnt, const uint32_t* take, const uint32_t* tgt,
                                    const unsigned long long* val, const unsigned long long* seed, uint32_t* popped,
                                    unsigned long long* seen, unsigned long long* slots, uint32_t* depth,
                                    hipStream_t stream);
// BUNDLE_WQ's per-wave node-stack capacity for an image of n_nodes records with groups of `width` and
// leaves of at most max_leaf triangles (0: does not fit the LDS)
uint32_t wq_stack_cap(uint32_t n_nodes, uint32_t width, uint32_t max_leaf);
constexpr uint32_t kAutoLeafWqStack = 512;  // auto leaf size: the smallest leaf whose image leaves this much
hipError_t launch_convert(const uint32_t* src8, float4* dst32, const float4* src32, uint32_t* dst8, size_t npix,
                          hipStream_t stream);

}  // namespace hrt
