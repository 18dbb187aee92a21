/*
 * hrt_host.h -- host-side helpers of libhip_raytrace.so: the C++ mirror of the reference's host prep
 * that feeds the kernels (the part of src/raytrace_pipeline.rs that stays on the CPU) and of the
 * external load_obj it consumes.  The arithmetic follows the reference's Rust exactly as written
 * (no contraction, DESIGN.md numerics spec S8), so the records match the Rust host byte for byte
 * under the documented assumptions on rust_maths.
 *
 *   hrt_host_create_rays       create_ray_subbuffer   src/raytrace_pipeline.rs:289-338
 *   hrt_host_ray_grid          its per-image constants (:298-316, :337); hrt_generate_rays
 *                              (hip_raytrace.h) evaluates the per-pixel loop :319-326 on the device
 *   hrt_host_view_matrix       get_view_matrix        src/raytrace_pipeline.rs:269-285
 *   hrt_host_transform_meshes  transform_meshes       src/raytrace_pipeline.rs:377-428
 *                              (+ create_mesh_subbuffer :363-374 first_index bookkeeping)
 *   hrt_obj_*                  graphics::load_obj (rust_vulkan_graphics@b3c6a9c4, external):
 *                              one mesh per `o` record, file order, face winding preserved
 *                              (called at src/main.rs:131,237,283)
 */
#ifndef HRT_HOST_H
#define HRT_HOST_H

#include "hip_raytrace.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Writes width*height rays (row-major, id = x + y*width) and the default jitter
 * max(|pixel_x|, |pixel_y|) * 0.5 (src/raytrace_pipeline.rs:337).  Returns the ray count
 * (0 for a zero-sized image, like the reference's zero-length protection :298-303). */
uint32_t hrt_host_create_rays(uint32_t width, uint32_t height, float camera_focal_length, float viewport_height,
                              const float up[3], hrt_ray* out, float* default_jitter);

/* The grid behind hrt_host_create_rays: ray (x, y) = (first + px * x) + py * y, each operation
 * rounded as written.  Any output pointer may be NULL.  Returns width*height (0: zero-sized). */
uint32_t hrt_host_ray_grid(uint32_t width, uint32_t height, float camera_focal_length, float viewport_height,
                           const float up[3], float first[3], float px[3], float py[3], float* default_jitter);

/* Host-only inspection of the hierarchy hrt_set_scene builds for BUNDLE_BVH (tests; no GPU).
 * counts = {nodes, prims, irregular, never, built, band entries, direction cells per face edge R};
 * each array (capacity in elements: floats for nodes/prims/irregular = 16 per record, u32 for
 * band_off = 6*R*R+1 (R <= 256) and band_list = 1 prim index per entry) is filled when non-NULL and large
 * enough.  Returns 1 (filled), 0 (not built), -1 (a capacity too small). */
int hrt_debug_bvh_build(const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes, uint32_t n_meshes,
                        uint32_t leaf_size, uint32_t counts[7], float* nodes, uint64_t nodes_cap, float* prims,
                        uint64_t prims_cap, float* irregular, uint64_t irregular_cap, uint32_t* band_off,
                        uint64_t band_off_cap, uint32_t* band_list, uint64_t band_list_cap);

/* Host-only: the 48-byte node image BUNDLE_WQ stages in LDS (12 floats per node, layout in
 * epq_raytracer_amd/csrc/hrt_bvh.h make_wq_nodes) for the hierarchy hrt_set_scene would build with
 * groups of up to `width` children (HRT_OPT_BVH_WIDTH).  Returns the node count (out filled), 0 (not
 * built / 65536 nodes or more), -1 (cap too small). */
int64_t hrt_debug_bvh_wq_nodes(const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes, uint32_t n_meshes,
                               uint32_t leaf_size, uint32_t width, float* out, uint64_t cap);

/* Column-major mat4 for push_constants.cam_alignment_mat: columns = normalised direction,
 * new_y, new_z (so mat3(M) * (1,0,0) = direction / |direction|), 4th column (0,0,0,1). */
void hrt_host_view_matrix(const float direction[3], const float up[3], float out[16]);

/* Flatten meshes into triangle and mesh records.  For mesh m: positions_m (n_verts_m * 3 floats),
 * indices_m (n_idx_m, a multiple of 3, 0-based into positions_m), material_m.
 * tris_out must hold sum(n_idx_m)/3 records (tri_capacity).  Returns HRT_ERR_INVALID_ARGUMENT on an
 * out-of-range index or insufficient capacity. */
hrt_status hrt_host_transform_meshes(uint32_t n_meshes, const float* const* positions, const uint32_t* n_verts,
                                     const uint32_t* const* indices, const uint32_t* n_idx,
                                     const hrt_material* materials, hrt_triangle* tris_out, uint32_t tri_capacity,
                                     hrt_mesh* meshes_out);

/* ---- Wavefront OBJ (load_obj semantics) ---------------------------------------------------- */
typedef struct hrt_obj hrt_obj;

hrt_status hrt_obj_load(const char* path, hrt_obj** out);
uint32_t hrt_obj_num_meshes(const hrt_obj* obj);
/* positions: the file's full vertex list (n_verts * 3 floats); indices: this mesh's triangles
 * (0-based into positions; polygons are fan-triangulated v0,vi,vi+1). Pointers live until free. */
hrt_status hrt_obj_mesh(const hrt_obj* obj, uint32_t i, const char** name, const float** positions,
                        uint32_t* n_verts, const uint32_t** indices, uint32_t* n_idx);
void hrt_obj_free(hrt_obj* obj);

#ifdef __cplusplus
}
#endif

#endif /* HRT_HOST_H */
