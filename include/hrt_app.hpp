/*
 * hrt_app.hpp -- the reference's host-side interface for the path-trace hot path, in C++ over the
 * C ABI of libhip_raytrace.so (hip_raytrace.h, hrt_host.h).  The reference host is Rust, whose
 * toolchain this image lacks, so this header mirrors its public surface with the same names,
 * argument meaning and error behaviour (a failed call throws, where the Rust code would panic on
 * `.unwrap()`); epq_raytracer_amd/app.py + pipeline.py are the Python mirror of the same surface.
 *
 *   CustomMaterial .. InvisLightMaterial   src/materials.rs:4-94   (Into<RayTracingMaterial>)
 *   Sphere, get_null_sphere                src/objects.rs:8-30
 *   Mesh, RayTracingMesh, get_null_mesh    src/objects.rs:35-47 (graphics::Mesh reduced to what the
 *                                          path reads: positions and triangle indices)
 *   Camera                                 graphics::Camera's fields the path reads
 *   RayTracerSettings                      src/raytracing_app.rs:17-29
 *   RayTracePipeline                       src/raytrace_pipeline.rs:31-266 (new / image / compute / init)
 *   DiffusePipeline                        src/diffuse.rs:22-136 (new / image / next_frame)
 *   RayTracingApp, compute_then_render,    src/raytracing_app.rs:32-227 (without the window: a render
 *   compute_n_then_render                  callback receives the accumulated image)
 *   load_obj                               graphics::load_obj (one mesh per `o` record)
 *
 * Header-only; link with -lhip_raytrace.  Nothing here runs on the CPU in place of the device: a
 * missing device makes the first context constructor throw (HRT_ERR_NO_DEVICE).
 */
#ifndef HRT_APP_HPP
#define HRT_APP_HPP

#include <array>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "hip_raytrace.h"
#include "hrt_host.h"

namespace epq {

using Vec3 = std::array<float, 3>;

// A failed library call: the status and hrt_last_error's text.
class HrtError : public std::runtime_error {
 public:
  HrtError(hrt_status s, const std::string& what) : std::runtime_error(what), status(s) {}
  hrt_status status;
};

inline void check(hrt_status s, const char* where, const hrt_context* ctx = nullptr) {
  if (s == HRT_OK) return;
  std::string msg = std::string(where) + ": status " + std::to_string((int)s);
  if (ctx) {
    const char* e = hrt_last_error(ctx);
    if (e && *e) msg += std::string(" (") + e + ")";
  }
  throw HrtError(s, msg);
}

// ---- materials, src/materials.rs ---------------------------------------------------------------
using RayTracingMaterial = hrt_material;

inline RayTracingMaterial make_material(std::array<float, 4> colour, std::array<float, 4> emission,
                                        std::array<float, 4> settings) {
  RayTracingMaterial m{};
  for (int i = 0; i < 4; ++i) {
    m.colour[i] = colour[i];
    m.emission[i] = emission[i];
    m.settings[i] = settings[i];
  }
  return m;
}

struct CustomMaterial {  // :4-34 (Default: colour 0.5, no emission, smoothness / fuzz / spec prob 0)
  Vec3 colour{0.5f, 0.5f, 0.5f};
  Vec3 emission_colour{0.0f, 0.0f, 0.0f};
  float emission_strength = 0.0f;
  float smoothness = 0.0f;
  float fuzz = 0.0f;
  float specular_probability = 0.0f;
  operator RayTracingMaterial() const {
    return make_material({colour[0], colour[1], colour[2], 0.0f},
                         {emission_colour[0], emission_colour[1], emission_colour[2], emission_strength},
                         {specular_probability, smoothness, fuzz, 0.0f});
  }
};
struct LambertianMaterial {  // :38-50
  Vec3 colour;
  operator RayTracingMaterial() const {
    return make_material({colour[0], colour[1], colour[2], 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}, {1.0f, 0.0f, 0.0f, 0.0f});
  }
};
struct MetalMaterial {  // :52-66
  Vec3 colour;
  float smoothness;
  float fuzz;
  operator RayTracingMaterial() const {
    return make_material({colour[0], colour[1], colour[2], 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f},
                         {1.0f, smoothness, fuzz, 0.0f});
  }
};
struct LightMaterial {  // :68-80
  std::array<float, 4> emission;
  operator RayTracingMaterial() const {
    return make_material({1.0f, 1.0f, 1.0f, 1.0f}, emission, {1.0f, 1.0f, 0.0f, 0.0f});
  }
};
struct InvisLightMaterial {  // :82-94 (settings[3] == 1: the invisible-light flag)
  std::array<float, 4> emission;
  operator RayTracingMaterial() const {
    return make_material({1.0f, 1.0f, 1.0f, 1.0f}, emission, {0.0f, 1.0f, 0.0f, 1.0f});
  }
};

// ---- objects, src/objects.rs --------------------------------------------------------------------
struct Sphere {  // :8-22
  Vec3 centre;
  float radius;
  RayTracingMaterial material;
  operator hrt_sphere() const {
    hrt_sphere s{};
    for (int i = 0; i < 3; ++i) s.centre[i] = centre[i];
    s.radius = radius;
    s.material = material;
    return s;
  }
};
inline Sphere get_null_sphere() { return Sphere{{0.0f, 0.0f, 0.0f}, 0.0f, LambertianMaterial{{1.0f, 1.0f, 1.0f}}}; }

struct Mesh {  // graphics::Mesh: positions (x, y, z per vertex) and 0-based triangle indices
  std::vector<float> positions;
  std::vector<uint32_t> indices;
  std::string name;
};
struct RayTracingMesh {  // :35-38
  Mesh mesh;
  RayTracingMaterial material;
};
inline RayTracingMesh get_null_mesh() {  // :40-47
  return RayTracingMesh{Mesh{{0.0f, 0.0f, 0.0f}, {0u, 0u, 0u}, ""}, LambertianMaterial{{1.0f, 1.0f, 1.0f}}};
}

// graphics::load_obj: one Mesh per `o` record, file order, winding kept (hrt_obj_*).
inline std::vector<Mesh> load_obj(const std::string& path) {
  hrt_obj* obj = nullptr;
  check(hrt_obj_load(path.c_str(), &obj), "hrt_obj_load");
  std::unique_ptr<hrt_obj, void (*)(hrt_obj*)> guard(obj, hrt_obj_free);
  std::vector<Mesh> out;
  for (uint32_t i = 0; i < hrt_obj_num_meshes(obj); ++i) {
    const char* name = nullptr;
    const float* pos = nullptr;
    const uint32_t* idx = nullptr;
    uint32_t nv = 0, ni = 0;
    check(hrt_obj_mesh(obj, i, &name, &pos, &nv, &idx, &ni), "hrt_obj_mesh");
    out.push_back(Mesh{std::vector<float>(pos, pos + 3 * (size_t)nv), std::vector<uint32_t>(idx, idx + ni),
                       name ? name : ""});
  }
  return out;
}

// ---- camera, settings ---------------------------------------------------------------------------
struct Camera {  // graphics::Camera: default up (0, 1, 0), direction stored as given
  Vec3 position{0.0f, 0.0f, 0.0f};
  Vec3 direction{1.0f, 0.0f, 0.0f};
  Vec3 up{0.0f, 1.0f, 0.0f};
  void do_move(float /*frame_time*/) {}  // src/raytracing_app.rs:169 (the app's camera is not controllable)
};

struct RayTracerSettings {  // src/raytracing_app.rs:17-29
  std::optional<float> sample_jitter;
  uint32_t num_samples = 1;
  uint32_t max_bounces = 0;
  bool use_environment_lighting = true;
  std::vector<Sphere> sphere_data;
  std::vector<RayTracingMesh> mesh_data;
  float camera_focal_length = 1.0f;
  float viewport_height = 2.0f;
  Vec3 up{0.0f, 1.0f, 0.0f};
};

// ---- the device context: the trace image and the accumulated image of one hrt_context -----------
class Context {
 public:
  // partition = {row_tile, part_index, part_count} (multi-GPU row tiles) or all zero: the whole image
  Context(uint32_t width, uint32_t height, int device = -1, hrt_mode mode = HRT_MODE_RGBA8,
          std::array<uint32_t, 3> partition = {0u, 0u, 1u}) {
    hrt_create_info info{width, height, device, (uint32_t)mode, partition[0], partition[1], partition[2]};
    hrt_context* c = nullptr;
    check(hrt_create(&info, &c), "hrt_create");
    ctx_.reset(c);
    check(hrt_get_layout(c, &layout_), "hrt_get_layout", c);
  }
  hrt_context* get() const { return ctx_.get(); }
  const hrt_layout& layout() const { return layout_; }
  void set_option(hrt_option key, int64_t value) { check(hrt_set_option(get(), key, value), "hrt_set_option", get()); }
  hrt_stats stats() const {
    hrt_stats s{};
    check(hrt_get_stats(get(), &s), "hrt_get_stats", get());
    return s;
  }
  void synchronize() { check(hrt_synchronize(get()), "hrt_synchronize", get()); }
  // the context's own pixel format (rgba8 or rgba32f): what checkpoints hold
  hrt_format native_format() const { return layout_.mode == HRT_MODE_RGBA8 ? HRT_FMT_RGBA8 : HRT_FMT_RGBA32F; }
  // checkpoint / resume: restore the accumulator from bytes read(HRT_IMG_ACCUM, native_format()) returned
  void load_accumulator(const std::vector<uint8_t>& img) {
    check(hrt_load_accumulator(get(), native_format(), img.data(), img.size()), "hrt_load_accumulator", get());
  }
  void load_accumulator_rgba8(const std::vector<uint8_t>& img) {
    check(hrt_load_accumulator(get(), HRT_FMT_RGBA8, img.data(), img.size()), "hrt_load_accumulator", get());
  }
  // the context's local rows of an image in fmt (local_rows x width x 4 channels of 1 or 4 bytes); never
  // the collective gather (HRT_IMG_LOCAL), also on a context joined to a communicator
  std::vector<uint8_t> read(hrt_image_id image, hrt_format fmt) const {
    std::vector<uint8_t> out((size_t)layout_.local_rows * layout_.width * (fmt == HRT_FMT_RGBA8 ? 4 : 16));
    check(hrt_read_image(get(), (uint32_t)image | HRT_IMG_LOCAL, fmt, out.data(), out.size()), "hrt_read_image", get());
    return out;
  }
  std::vector<uint8_t> read_rgba8(hrt_image_id image) const { return read(image, HRT_FMT_RGBA8); }

 private:
  struct Del {
    void operator()(hrt_context* c) const { hrt_destroy(c); }
  };
  std::unique_ptr<hrt_context, Del> ctx_;
  hrt_layout layout_{};
};

// What RayTracePipeline::image / DiffusePipeline::image hand to the presenter.
struct Image {
  Context* ctx;
  hrt_image_id id;
  std::vector<uint8_t> read_rgba8() const { return ctx->read_rgba8(id); }
};

// ---- pipelines ---------------------------------------------------------------------------------
class RayTracePipeline {  // src/raytrace_pipeline.rs:31-266
 public:
  RayTracePipeline(Context& ctx, std::array<uint32_t, 2> image_size, const RayTracerSettings& settings)
      : ctx_(&ctx), size_(image_size) {
    // create_ray_subbuffer (:289-338)
    std::vector<hrt_ray> rays((size_t)image_size[0] * image_size[1] + 1);
    float jitter = 0.0f;
    const uint32_t n_rays = hrt_host_create_rays(image_size[0], image_size[1], settings.camera_focal_length,
                                                 settings.viewport_height, settings.up.data(), rays.data(), &jitter);
    // create_sphere_subbuffer (:342-360): the spheres as given (an empty list uploads none)
    std::vector<hrt_sphere> spheres(settings.sphere_data.begin(), settings.sphere_data.end());
    // transform_meshes (:377-428); an empty list flattens the null mesh and uploads zero meshes
    const std::vector<RayTracingMesh> null_list{get_null_mesh()};
    const std::vector<RayTracingMesh>& ml = settings.mesh_data.empty() ? null_list : settings.mesh_data;
    std::vector<const float*> pos;
    std::vector<const uint32_t*> idx;
    std::vector<uint32_t> nv, ni;
    std::vector<hrt_material> mats;
    size_t ntri = 0;
    for (const RayTracingMesh& m : ml) {
      pos.push_back(m.mesh.positions.data());
      idx.push_back(m.mesh.indices.empty() ? nullptr : m.mesh.indices.data());
      nv.push_back((uint32_t)(m.mesh.positions.size() / 3));
      ni.push_back((uint32_t)m.mesh.indices.size());
      mats.push_back(m.material);
      ntri += m.mesh.indices.size() / 3;
    }
    std::vector<hrt_triangle> tris(ntri ? ntri : 1);
    std::vector<hrt_mesh> meshes(ml.size());
    check(hrt_host_transform_meshes((uint32_t)ml.size(), pos.data(), nv.data(), idx.data(), ni.data(), mats.data(),
                                    tris.data(), (uint32_t)ntri, meshes.data()),
          "hrt_host_transform_meshes");
    ray_count_ = n_rays;
    sphere_count_ = (int32_t)settings.sphere_data.size();
    mesh_count_ = (int32_t)settings.mesh_data.size();
    num_samples_ = settings.num_samples > 1 ? (int32_t)settings.num_samples : 1;  // :88
    max_bounces_ = (int32_t)settings.max_bounces;                                // :89
    use_env_ = settings.use_environment_lighting;
    jitter_ = settings.sample_jitter ? *settings.sample_jitter : jitter;
    check(hrt_set_scene(ctx.get(), rays.data(), n_rays, spheres.data(), (uint32_t)spheres.size(), tris.data(),
                        (uint32_t)ntri, meshes.data(), (uint32_t)mesh_count_),
          "hrt_set_scene", ctx.get());
  }
  Image image() const { return Image{ctx_, HRT_IMG_TRACE}; }  // :156
  // the 124-byte block of dispatch() (:243-257)
  hrt_push_constants push_constants(const Camera& camera, uint32_t rng_offset, bool init) const {
    hrt_push_constants pc{};
    pc.cam_pos[0] = camera.position[0];
    pc.cam_pos[1] = camera.position[1];
    pc.cam_pos[2] = camera.position[2];
    pc.cam_pos[3] = 1.0f;
    hrt_host_view_matrix(camera.direction.data(), camera.up.data(), pc.cam_alignment_mat);
    pc.num_rays = (int32_t)ray_count_;
    pc.num_spheres = sphere_count_;
    pc.num_meshes = mesh_count_;
    pc.num_samples = num_samples_;
    pc.jitter_size = jitter_;
    pc.max_bounces = max_bounces_;
    pc.use_environment_light = use_env_ ? 1u : 0u;
    pc.rng_offset = rng_offset;
    pc.init = init ? 1u : 0u;
    pc.width = size_[0];
    pc.height = size_[1];
    return pc;
  }
  void compute(const Camera& camera, uint32_t rng_offset) {  // :162-187
    const hrt_push_constants pc = push_constants(camera, rng_offset, false);
    check(hrt_trace(ctx_->get(), &pc), "hrt_trace", ctx_->get());
  }
  void init() {  // :190-213: clear the trace image
    const hrt_push_constants pc = push_constants(Camera{}, 0u, true);
    check(hrt_trace(ctx_->get(), &pc), "hrt_trace", ctx_->get());
  }
  Context& context() const { return *ctx_; }
  std::array<uint32_t, 2> image_size() const { return size_; }

 private:
  Context* ctx_;
  std::array<uint32_t, 2> size_;
  uint32_t ray_count_ = 0;
  int32_t sphere_count_ = 0, mesh_count_ = 0, num_samples_ = 1, max_bounces_ = 0;
  bool use_env_ = true;
  float jitter_ = 0.0f;
};

class DiffusePipeline {  // src/diffuse.rs:22-136 (image_combiner.glsl)
 public:
  DiffusePipeline(Context& ctx, std::array<uint32_t, 2> image_size) : ctx_(&ctx), size_(image_size) {}
  Image image() const { return Image{ctx_, HRT_IMG_ACCUM}; }  // :69
  std::array<uint32_t, 2> image_size() const { return size_; }
  void next_frame(uint32_t frame_num, const Image& next_image) {  // :73-136
    if (next_image.ctx != ctx_ || next_image.id != HRT_IMG_TRACE)
      throw HrtError(HRT_ERR_INVALID_ARGUMENT, "next_frame: next_image must be the trace image of the same context");
    check(hrt_accumulate(ctx_->get(), frame_num), "hrt_accumulate", ctx_->get());
  }

 private:
  Context* ctx_;
  std::array<uint32_t, 2> size_;
};

// ---- the app, src/raytracing_app.rs -----------------------------------------------------------
class RayTracingApp {
 public:
  using Render = std::function<void(const Image&)>;  // the presenter (RenderPassOverFrame) hook
  RayTracingApp(Camera camera, RayTracerSettings settings, int device = -1, hrt_mode mode = HRT_MODE_RGBA8)
      : camera(std::move(camera)), settings_(std::move(settings)), device_(device), mode_(mode) {}  // :46-71

  // :74-140: build the pipelines, clear both images with frame 0, frame -> 1
  void open(std::array<uint32_t, 2> image_size, Render render = nullptr) {
    ctx_ = std::make_unique<Context>(image_size[0], image_size[1], device_, mode_);
    raytrace_ = std::make_unique<RayTracePipeline>(*ctx_, image_size, settings_);
    diffuse_ = std::make_unique<DiffusePipeline>(*ctx_, image_size);
    render_ = std::move(render);
    raytrace_->init();                                // :128
    diffuse_->next_frame(frame_, raytrace_->image());  // :129
    if (render_) render_(diffuse_->image());          // :131-136
    frame_ += 1;                                      // :139
  }
  bool is_open() const { return ctx_ != nullptr; }
  uint32_t frame() const { return frame_; }

  // Checkpoint / resume (not a reference feature): the accumulator in the context's own
  // format plus the frame counter are the whole state of a progressive render (frame k traces with
  // rng_offset = k), so resuming on an open app of the same size and mode continues it byte for byte.
  struct Checkpoint {
    std::vector<uint8_t> accum;
    uint32_t frame = 0;
    hrt_layout layout{};
  };
  Checkpoint checkpoint() const {
    require_open();
    return Checkpoint{ctx_->read(HRT_IMG_ACCUM, ctx_->native_format()), frame_, ctx_->layout()};
  }
  void resume(const Checkpoint& c) {
    require_open();
    const hrt_layout& l = ctx_->layout();
    if (std::memcmp(&l, &c.layout, sizeof l) != 0)
      throw HrtError(HRT_ERR_INVALID_ARGUMENT, "RayTracingApp::resume: checkpoint of another size, mode or partition");
    ctx_->load_accumulator(c.accum);
    frame_ = c.frame;
  }
  RayTracePipeline& raytrace() { return *raytrace_; }
  DiffusePipeline& diffuse() { return *diffuse_; }
  Context& context() { return *ctx_; }

  Camera camera;

 private:
  friend void compute_then_render(RayTracingApp& app, float frame_time);
  friend void compute_n_then_render(RayTracingApp& app, uint32_t num_renders);
  void require_open() const {
    if (!ctx_) throw HrtError(HRT_ERR_INVALID_ARGUMENT, "RayTracingApp: open() has not been called");
  }
  RayTracerSettings settings_;
  int device_;
  hrt_mode mode_;
  std::unique_ptr<Context> ctx_;
  std::unique_ptr<RayTracePipeline> raytrace_;
  std::unique_ptr<DiffusePipeline> diffuse_;
  Render render_;
  uint32_t frame_ = 0;
};

// src/raytracing_app.rs:156-194: one traced frame, accumulate, present
inline void compute_then_render(RayTracingApp& app, float frame_time) {
  app.require_open();
  app.camera.do_move(frame_time);
  app.raytrace_->compute(app.camera, app.frame_);
  app.diffuse_->next_frame(app.frame_, app.raytrace_->image());
  if (app.render_) app.render_(app.diffuse_->image());
  app.frame_ += 1;
}

// src/raytracing_app.rs:196-227: num_renders frames chained without a host wait (one hrt_compute_n:
// the same traces and accumulates byte for byte), then one present
inline void compute_n_then_render(RayTracingApp& app, uint32_t num_renders) {
  app.require_open();
  if (num_renders > 0) {
    const hrt_push_constants pc = app.raytrace_->push_constants(app.camera, app.frame_, false);
    check(hrt_compute_n(app.ctx_->get(), &pc, num_renders), "hrt_compute_n", app.ctx_->get());
    app.frame_ += num_renders;
  }
  if (app.render_) app.render_(app.diffuse_->image());
}

}  // namespace epq

#endif  // HRT_APP_HPP
