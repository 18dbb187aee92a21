// hrt_host.cpp -- host-side prep of the reference's RayTracePipeline (src/raytrace_pipeline.rs:269-428)
// and a Wavefront OBJ reader with graphics::load_obj semantics.  Compiled with -ffp-contract=off:
// the reference host is Rust, which never contracts, so every expression below is evaluated as
// written (DESIGN.md numerics spec S8).
#include "hrt_host.h"

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct V3 {
  float x, y, z;
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
// rust_maths Vector3::cross / magnitude / normalised (S8)
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float magnitude(V3 a) { return __builtin_sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
inline V3 normalised(V3 a) { return a / magnitude(a); }
inline float fmin_rs(float a, float b) { return __builtin_fminf(a, b); }  // f32::min (NaN-ignoring)
inline float fmax_rs(float a, float b) { return __builtin_fmaxf(a, b); }  // f32::max

constexpr float kF32Max = 3.40282347e+38f;

}  // namespace

extern "C" uint32_t hrt_host_ray_grid(uint32_t width, uint32_t height, float camera_focal_length,
                                      float viewport_height, const float up[3], float first[3], float px[3],
                                      float py[3], float* default_jitter) {
  // zero length protection, src/raytrace_pipeline.rs:298-303
  if (width == 0 || height == 0) {
    if (default_jitter) *default_jitter = 0.0f;
    return 0;
  }
  const float vw = viewport_height * ((float)width / (float)height);           // :307
  const V3 X{1.0f, 0.0f, 0.0f};
  const V3 vx = normalised(cross(V3{up[0], up[1], up[2]}, X));                 // :309
  const V3 vy = normalised(cross(vx, X));                                      // :310
  const V3 ul = (V3{0.0f, 0.0f, 0.0f} + X * camera_focal_length) - (vx * vw + vy * viewport_height) * 0.5f;  // :311
  const V3 dx = vx * vw / (float)width;                                        // :313
  const V3 dy = vy * viewport_height / (float)height;                          // :314
  const V3 f = ul + (dx + dy) * 0.5f;                                          // :316
  const float fv[3] = {f.x, f.y, f.z}, xv[3] = {dx.x, dx.y, dx.z}, yv[3] = {dy.x, dy.y, dy.z};
  for (int k = 0; k < 3; ++k) {
    if (first) first[k] = fv[k];
    if (px) px[k] = xv[k];
    if (py) py[k] = yv[k];
  }
  if (default_jitter) *default_jitter = fmax_rs(magnitude(dx), magnitude(dy)) * 0.5f;  // :337
  return width * height;
}

extern "C" uint32_t hrt_host_create_rays(uint32_t width, uint32_t height, float camera_focal_length,
                                         float viewport_height, const float up[3], hrt_ray* out,
                                         float* default_jitter) {
  float f[3], dx[3], dy[3];
  const uint32_t n = hrt_host_ray_grid(width, height, camera_focal_length, viewport_height, up, f, dx, dy,
                                       default_jitter);
  if (n == 0 || !out) return n;
  const V3 first{f[0], f[1], f[2]}, px{dx[0], dx[1], dx[2]}, py{dy[0], dy[1], dy[2]};
  for (uint32_t y = 0; y < height; ++y) {                                      // :319-326
    for (uint32_t x = 0; x < width; ++x) {
      const V3 r = first + px * (float)x + py * (float)y;
      hrt_ray& o = out[(size_t)y * width + x];
      o.sample_centre[0] = r.x;
      o.sample_centre[1] = r.y;
      o.sample_centre[2] = r.z;
      o.sample_centre[3] = 1.0f;  // extend(); unused by the kernel
    }
  }
  return n;
}

extern "C" void hrt_host_view_matrix(const float direction[3], const float up[3], float out[16]) {
  const V3 d{direction[0], direction[1], direction[2]};
  const V3 u{up[0], up[1], up[2]};
  const V3 nx = normalised(d);                  // :273
  const V3 nz = -normalised(cross(d, u));       // :274  (unary minus binds after the method calls)
  const V3 ny = -normalised(cross(nx, nz));     // :275
  // Matrix3::from_columns(nx, ny, nz).transposed(), rows uploaded as mat4 columns (:278-284).
  const float m[16] = {nx.x, nx.y, nx.z, 0.0f, ny.x, ny.y, ny.z, 0.0f, nz.x, nz.y, nz.z, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f};
  std::memcpy(out, m, sizeof m);
}

extern "C" hrt_status hrt_host_transform_meshes(uint32_t n_meshes, const float* const* positions,
                                                const uint32_t* n_verts, const uint32_t* const* indices,
                                                const uint32_t* n_idx, const hrt_material* materials,
                                                hrt_triangle* tris_out, uint32_t tri_capacity,
                                                hrt_mesh* meshes_out) {
  if (n_meshes && (!positions || !n_verts || !indices || !n_idx || !materials || !meshes_out))
    return HRT_ERR_INVALID_ARGUMENT;
  uint32_t tri_count = 0;
  for (uint32_t m = 0; m < n_meshes; ++m) {  // :384-425
    const float* P = positions[m];
    const uint32_t* I = indices[m];
    const uint32_t ni = n_idx[m];
    if (ni % 3 != 0) return HRT_ERR_INVALID_ARGUMENT;
    const uint32_t num_tris = ni / 3;
    if ((uint64_t)tri_count + num_tris > tri_capacity) return HRT_ERR_INVALID_ARGUMENT;
    float min_x = kF32Max, min_y = kF32Max, min_z = kF32Max;       // :388
    float max_x = -kF32Max, max_y = -kF32Max, max_z = -kF32Max;    // :389 (f32::MIN)
    for (uint32_t i = 0; i < ni; i += 3) {
      const uint32_t ia = I[i], ib = I[i + 1], ic = I[i + 2];
      if (ia >= n_verts[m] || ib >= n_verts[m] || ic >= n_verts[m]) return HRT_ERR_INVALID_ARGUMENT;
      const V3 a{P[3 * ia], P[3 * ia + 1], P[3 * ia + 2]};
      const V3 b{P[3 * ib], P[3 * ib + 1], P[3 * ib + 2]};
      const V3 c{P[3 * ic], P[3 * ic + 1], P[3 * ic + 2]};
      const V3 e1 = b - a, e2 = c - a;                                // :396-397
      const V3 n = cross(e1, e2);                                     // :398
      min_x = fmin_rs(min_x, fmin_rs(a.x, fmin_rs(b.x, c.x)));        // :400-406
      min_y = fmin_rs(min_y, fmin_rs(a.y, fmin_rs(b.y, c.y)));
      min_z = fmin_rs(min_z, fmin_rs(a.z, fmin_rs(b.z, c.z)));
      max_x = fmax_rs(max_x, fmax_rs(a.x, fmax_rs(b.x, c.x)));
      max_y = fmax_rs(max_y, fmax_rs(a.y, fmax_rs(b.y, c.y)));
      max_z = fmax_rs(max_z, fmax_rs(a.z, fmax_rs(b.z, c.z)));
      hrt_triangle& t = tris_out[tri_count + i / 3];
      const float rec[16] = {a.x, a.y, a.z, 1.0f, e1.x, e1.y, e1.z, 1.0f, e2.x, e2.y, e2.z, 1.0f, n.x, n.y, n.z, 1.0f};
      std::memcpy(&t, rec, sizeof rec);
    }
    hrt_mesh& out = meshes_out[m];                                    // :417-423
    out.min_point[0] = min_x; out.min_point[1] = min_y; out.min_point[2] = min_z;
    out.max_point[0] = max_x; out.max_point[1] = max_y; out.max_point[2] = max_z;
    out.first_index = tri_count;
    out.len = num_tris;
    out.material = materials[m];
    tri_count += num_tris;                                            // :424
  }
  return HRT_OK;
}

// ------------------------------------------------------------------------------------------------
// OBJ reader.  load_obj (external crate) semantics as inferred in SURVEY.md 8(c)(1): one mesh per
// `o` record in file order; `v` positions are global and 1-based (negative = relative); face
// vertex order is kept (winding matters: triangles are single-sided, raytracing.glsl:217).
// Faces before the first `o` form an unnamed mesh.  Normals/texcoords are ignored (`v//n`, `v/t/n`).
// ------------------------------------------------------------------------------------------------
struct hrt_obj {
  std::vector<float> positions;
  struct Mesh {
    std::string name;
    std::vector<uint32_t> indices;
  };
  std::vector<Mesh> meshes;
};

namespace {

bool parse_face_index(const char*& p, long nverts, uint32_t* out) {
  char* end = nullptr;
  errno = 0;
  long v = std::strtol(p, &end, 10);
  if (end == p || errno) return false;
  p = end;
  while (*p && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n') ++p;  // skip /t/n
  long idx = v > 0 ? v - 1 : nverts + v;
  if (v == 0 || idx < 0 || idx >= nverts) return false;
  *out = (uint32_t)idx;
  return true;
}

}  // namespace

extern "C" hrt_status hrt_obj_load(const char* path, hrt_obj** out) {
  if (!path || !out) return HRT_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  FILE* f = std::fopen(path, "rb");
  if (!f) return HRT_ERR_IO;
  auto* obj = new hrt_obj();
  // whole lines of any length (getline grows the buffer): a long 'f' n-gon or 'o' name is never split
  char* buf = nullptr;
  size_t cap = 0;
  bool ok = true;
  while (ok && getline(&buf, &cap, f) != -1) {
    const char* p = buf;
    while (*p == ' ' || *p == '\t') ++p;
    if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
      float x, y, z;
      if (std::sscanf(p + 2, "%f %f %f", &x, &y, &z) != 3) { ok = false; break; }
      obj->positions.push_back(x);
      obj->positions.push_back(y);
      obj->positions.push_back(z);
    } else if (p[0] == 'o' && (p[1] == ' ' || p[1] == '\t')) {
      std::string name(p + 2);
      while (!name.empty() && (name.back() == '\n' || name.back() == '\r' || name.back() == ' ')) name.pop_back();
      obj->meshes.push_back({name, {}});
    } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
      if (obj->meshes.empty()) obj->meshes.push_back({"", {}});
      std::vector<uint32_t> poly;
      const char* q = p + 2;
      const long nv = (long)(obj->positions.size() / 3);
      while (true) {
        while (*q == ' ' || *q == '\t') ++q;
        if (!*q || *q == '\n' || *q == '\r') break;
        uint32_t idx;
        if (!parse_face_index(q, nv, &idx)) { ok = false; break; }
        poly.push_back(idx);
      }
      if (!ok || poly.size() < 3) { ok = false; break; }
      auto& ind = obj->meshes.back().indices;
      for (size_t k = 1; k + 1 < poly.size(); ++k) {
        ind.push_back(poly[0]);
        ind.push_back(poly[k]);
        ind.push_back(poly[k + 1]);
      }
    }
  }
  std::free(buf);
  std::fclose(f);
  if (!ok) {
    delete obj;
    return HRT_ERR_IO;
  }
  *out = obj;
  return HRT_OK;
}

extern "C" uint32_t hrt_obj_num_meshes(const hrt_obj* obj) { return obj ? (uint32_t)obj->meshes.size() : 0; }

extern "C" hrt_status hrt_obj_mesh(const hrt_obj* obj, uint32_t i, const char** name, const float** positions,
                                   uint32_t* n_verts, const uint32_t** indices, uint32_t* n_idx) {
  if (!obj || i >= obj->meshes.size()) return HRT_ERR_INVALID_ARGUMENT;
  const auto& m = obj->meshes[i];
  if (name) *name = m.name.c_str();
  if (positions) *positions = obj->positions.data();
  if (n_verts) *n_verts = (uint32_t)(obj->positions.size() / 3);
  if (indices) *indices = m.indices.data();
  if (n_idx) *n_idx = (uint32_t)m.indices.size();
  return HRT_OK;
}

extern "C" void hrt_obj_free(hrt_obj* obj) { delete obj; }
