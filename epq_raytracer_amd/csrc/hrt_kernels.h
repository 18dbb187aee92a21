// hrt_kernels.h -- launch interface between the C-ABI layer (hrt_api.cpp) and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hip_raytrace.h"

namespace hrt {

// Kernel argument block (passed by value; lives in the kernarg segment, read through SGPRs).
struct TraceParams {
  const float4* rays;            // W*H sample centres, indexed by global pixel id
  const hrt_sphere* spheres;
  const hrt_triangle* tris;
  const hrt_mesh* meshes;
  uint32_t* img8;                // local_rows x W packed RGBA8 (RGBA8 mode) or nullptr
  float4* img32;                 // local_rows x W float4 (RGBA32F mode) or nullptr
  unsigned long long* counters;  // [0] segments, [1] triangle tests; nullptr = off
  hrt_push_constants pc;
  uint32_t local_rows, row_tile, part_index, part_count;
  uint32_t n_tris;               // uploaded triangle count (LDS staging)
  // Camera-facing lists (variant 8): per mesh m, the triangles of [first_index, first_index+len) with
  // dot(cam_pos - a, n) > 0 in buffer order -- the only ones a primary ray (origin = cam_pos) can accept.
  uint32_t* cam_list;            // sum(len) entries; mesh m's list starts at cam_start[m]
  uint32_t* cam_start;           // num_meshes
  uint32_t* cam_count;           // num_meshes
  uint32_t cam_list_capacity;
  float4* cam_tris;              // variant 10: compacted camera-facing records (a.w = original index bits)
  uint32_t cam_layout;
  float4* cam_cull;              // variant 14: 5 float4 bundle-cull records per compacted triangle
  uint32_t sec_batch;            // variant 14: run the bounce path once this many lanes wait (1..64)           // 0: (a,idx)(e1)(e2)(n); 1 (variant 11): (ao,num_t)(e1,idx)(e2)(n)
};

hipError_t launch_trace(const TraceParams& p, int variant, hipStream_t stream);
bool variant_uses_camera_lists(const TraceParams& p, int variant);
hipError_t launch_clear(uint32_t* img8, float4* img32, size_t npix, hipStream_t stream);
hipError_t launch_accumulate(uint32_t* cur8, const uint32_t* new8, float4* cur32, const float4* new32, size_t npix,
                             uint32_t frame, hipStream_t stream);
hipError_t launch_convert(const uint32_t* src8, float4* dst32, const float4* src32, uint32_t* dst8, size_t npix,
                          hipStream_t stream);

}  // namespace hrt
