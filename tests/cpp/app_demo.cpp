// The reference's host flow (src/main.rs -> RayTracingApp::open -> compute_then_render /
// compute_n_then_render) written against include/hrt_app.hpp, the C++ mirror of its public surface.
// tests/test_cpp_app.py renders the same scene through the Python mirror and compares the frames.
//
//   app_demo <out.bin> <width> <height> <spp> <bounces> <frames> <loop|batch|resume|resume32> [obj path]
//
// resume / resume32 (rgba8 / rgba32f mode): frames / 2 frames through compute_n_then_render, a
// checkpoint, a NEW app that resumes from it, the remaining frames through compute_then_render.
//
// Scene (fixed here, mirrored in tests/test_cpp_app.py::demo_settings): a ground sphere, a metal and
// a light sphere, an invisible light, and a two-triangle quad with a custom material (plus every mesh
// of the OBJ file, Lambertian, when a path is given).  Output: u64 segments, u64 triangle tests, u32
// final frame counter, then the accumulated rgba8 image (height x width x 4).  A library error prints
// its message and exits with 10 + the hrt_status.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "hrt_app.hpp"

static epq::RayTracerSettings demo_settings(uint32_t spp, uint32_t bounces, const char* obj) {
  epq::RayTracerSettings s;
  s.num_samples = spp;
  s.max_bounces = bounces;
  s.use_environment_lighting = true;
  s.sphere_data = {
      epq::Sphere{{0.0f, -100.5f, -1.0f}, 100.0f, epq::LambertianMaterial{{0.8f, 0.8f, 0.0f}}},
      epq::Sphere{{0.0f, 0.0f, -1.2f}, 0.5f, epq::MetalMaterial{{0.8f, 0.6f, 0.2f}, 0.9f, 0.05f}},
      epq::Sphere{{-1.0f, 0.3f, -1.0f}, 0.3f, epq::LightMaterial{{1.0f, 0.9f, 0.7f, 4.0f}}},
      epq::Sphere{{1.2f, 1.5f, -0.5f}, 0.4f, epq::InvisLightMaterial{{0.9f, 0.9f, 1.0f, 6.0f}}},
  };
  epq::CustomMaterial quad_mat;
  quad_mat.colour = {0.2f, 0.5f, 0.8f};
  quad_mat.smoothness = 0.3f;
  quad_mat.specular_probability = 0.25f;
  s.mesh_data.push_back(epq::RayTracingMesh{
      epq::Mesh{{0.5f, -0.5f, -2.0f, 1.5f, -0.5f, -2.0f, 1.5f, 0.8f, -2.0f, 0.5f, 0.8f, -2.0f}, {0, 1, 2, 0, 2, 3}, "quad"},
      quad_mat});
  if (obj) {
    for (epq::Mesh& m : epq::load_obj(obj)) s.mesh_data.push_back(epq::RayTracingMesh{m, epq::LambertianMaterial{{0.6f, 0.6f, 0.6f}}});
  }
  return s;
}

int main(int argc, char** argv) {
  if (argc < 8) {
    std::fprintf(stderr, "usage: %s out.bin width height spp bounces frames loop|batch [obj]\n", argv[0]);
    return 2;
  }
  const uint32_t w = (uint32_t)std::atoi(argv[2]), h = (uint32_t)std::atoi(argv[3]);
  const uint32_t spp = (uint32_t)std::atoi(argv[4]), bounces = (uint32_t)std::atoi(argv[5]);
  const uint32_t frames = (uint32_t)std::atoi(argv[6]);
  const bool batch = std::strcmp(argv[7], "batch") == 0;
  const bool resume = std::strncmp(argv[7], "resume", 6) == 0;
  const hrt_mode mode = std::strcmp(argv[7], "resume32") == 0 ? HRT_MODE_RGBA32F : HRT_MODE_RGBA8;
  try {
    epq::Camera cam;
    cam.position = {0.0f, 0.3f, 1.5f};
    cam.direction = {0.0f, -0.1f, -1.0f};
    const epq::RayTracerSettings settings = demo_settings(spp, bounces, argc > 8 ? argv[8] : nullptr);
    auto app = std::make_unique<epq::RayTracingApp>(cam, settings, -1, mode);
    uint32_t presented = 0;
    app->open({w, h}, [&](const epq::Image&) { ++presented; });
    uint64_t seg = 0, tt = 0;
    if (batch) {
      epq::compute_n_then_render(*app, frames);
    } else if (resume) {
      epq::compute_n_then_render(*app, frames / 2);
      const epq::RayTracingApp::Checkpoint ck = app->checkpoint();
      const hrt_stats s1 = app->context().stats();
      seg += s1.segments;
      tt += s1.tri_tests;
      app = std::make_unique<epq::RayTracingApp>(cam, settings, -1, mode);  // a restart
      app->open({w, h});
      app->resume(ck);
      for (uint32_t k = frames / 2; k < frames; ++k) epq::compute_then_render(*app, 1.0f / 60.0f);
    } else {
      for (uint32_t k = 0; k < frames; ++k) epq::compute_then_render(*app, 1.0f / 60.0f);
    }
    epq::RayTracingApp& app_ = *app;
    const hrt_stats st = app_.context().stats();
    const std::vector<uint8_t> img = app_.diffuse().image().read_rgba8();
    FILE* f = std::fopen(argv[1], "wb");
    if (!f) return 3;
    seg += st.segments;
    tt += st.tri_tests;
    const uint32_t fr = app_.frame();
    std::fwrite(&seg, 8, 1, f);
    std::fwrite(&tt, 8, 1, f);
    std::fwrite(&fr, 4, 1, f);
    std::fwrite(img.data(), 1, img.size(), f);
    std::fclose(f);
    std::printf("app_demo: %ux%u %u spp %u bounces, %u frames (%s), %u presents, %llu segments\n", w, h, spp, bounces,
                frames, batch ? "compute_n_then_render" : resume ? "checkpoint + resume" : "compute_then_render", presented,
                (unsigned long long)seg);
    return 0;
  } catch (const epq::HrtError& e) {
    std::fprintf(stderr, "app_demo: %s\n", e.what());
    return 10 + (int)e.status;
  }
}
