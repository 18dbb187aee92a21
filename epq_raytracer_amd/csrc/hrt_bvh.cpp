// hrt_bvh.cpp -- binned-SAH build of the bounce-segment BVH (hrt_bvh.h).  Host C++, run by
// hrt_set_scene; all bounds are computed in double and rounded outward to float so that the trace
// kernel's cull tests are conservative (DESIGN.md "BVH cull").
#include "hrt_bvh.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>

#ifndef HRT_BVH_SWEEP
#define HRT_BVH_SWEEP 1  // full-sweep SAH splits (0: 16 bins per axis)
#endif
#ifndef HRT_BVH_SAH_R
#define HRT_BVH_SAH_R 0.25  // the SAH costs boxes grown by their triangles' margins at this x the scene diagonal (0: plain boxes)
#endif

namespace hrt {
namespace {

struct V3 {
  double x, y, z;
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double norm(V3 a) { return std::sqrt(dot(a, a)); }
inline double comp(V3 a, int k) { return k == 0 ? a.x : (k == 1 ? a.y : a.z); }
inline V3 ld(const float* p) { return {p[0], p[1], p[2]}; }

struct Box {
  V3 lo{HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi{-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  void grow(V3 p) {
    lo = {std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z)};
    hi = {std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z)};
  }
  void grow(const Box& b) {
    grow(b.lo);
    grow(b.hi);
  }
  double area() const {
    if (lo.x > hi.x) return 0.0;
    const V3 e = hi - lo;
    return 2.0 * (e.x * e.y + e.y * e.z + e.z * e.x);
  }
};

// One regular (mesh, triangle) entry.
struct Entry {
  Box box;
  Box sbox;        // what the SAH sees: box grown by the triangle's own margin at R = kSahR x the scene diagonal
  V3 centroid;
  V3 nhat;         // n_rec / |n_rec|
  double g;        // max(|e1|, |e2|) / |n_rec|
  double rho;      // |n_rec - e1 x e2| / |n_rec|
  double ext;      // largest per-axis extent of the triangle
  uint32_t key, mesh, index;
};

float round_down(double v) {
  float f = (float)v;
  if ((double)f > v) f = std::nextafter(f, -HUGE_VALF);
  return f;
}
float round_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = std::nextafter(f, HUGE_VALF);
  return f;
}
float bits_f(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

struct Builder {
  std::vector<Entry>& e;
  uint32_t leaf_size;
  BvhHost& out;

  void emit_prim(const Entry& en, const hrt_triangle* tris) {
    const hrt_triangle& t = tris[en.index];
    const float rec[16] = {t.a[0], t.a[1], t.a[2], bits_f(en.key),
                           t.edge_one[0], t.edge_one[1], t.edge_one[2], bits_f(en.mesh),
                           t.edge_two[0], t.edge_two[1], t.edge_two[2], bits_f(en.index),
                           t.normal[0], t.normal[1], t.normal[2], 0.0f};
    out.prims.insert(out.prims.end(), rec, rec + 16);
    out.entries.push_back(en.index | (en.mesh << 26));
  }

  void build(uint32_t b, uint32_t n, const hrt_triangle* tris) {
    const uint32_t node = out.n_nodes++;
    out.nodes.resize((size_t)out.n_nodes * 16, 0.0f);
    Box box, cbox;
    V3 axis{0, 0, 0};
    // box margin for a lane whose origin is within R of every vertex below: each triangle i needs
    // 2 eta_i ext_i = a_i + b_i R, eta_i = 6e + (1.01 rho_i + 3.2e + 18.4e G_i R) / (tau_g - rho_i - 4e-7)
    // (DESIGN.md "BVH cull"), so the node takes max_i a_i and max_i b_i -- per triangle, not the
    // product of the subtree's largest extent and largest G (r02 and before), which charged a big
    // triangle with a small triangle's G (cave: 2x wider margins)
    const double eps = 5.9604644775390625e-08;
    double rho = 0, a_tri = 0, b_tri = 0;
    for (uint32_t i = b; i < b + n; ++i) {
      box.grow(e[i].box);
      cbox.grow(e[i].centroid);
      axis = axis + e[i].nhat;
      rho = std::max(rho, e[i].rho);
      const double inv_tpi = 1.02 / ((double)out.band_tau - e[i].rho - 4e-7);
      a_tri = std::max(a_tri, 2.02 * e[i].ext * (6 * eps + (1.01 * e[i].rho + 3.2 * eps) * inv_tpi));
      b_tri = std::max(b_tri, 2.02 * e[i].ext * 18.4 * eps * e[i].g * inv_tpi);
    }
    // normal cone around the mean direction
    double cphi = 0.0, sphi = 1.0;
    const double an = norm(axis);
    if (an > 1e-9) {
      axis = axis * (1.0 / an);
      double phi = 0.0;
      for (uint32_t i = b; i < b + n; ++i) phi = std::max(phi, std::acos(std::max(-1.0, std::min(1.0, dot(axis, e[i].nhat)))));
      phi += 1e-6;
      if (phi < 1.5707963267948966) {
        cphi = std::cos(phi);
        sphi = std::sin(phi);
      }
    }
    if (!(cphi > 0.0)) {
      axis = {1.0, 0.0, 0.0};
      cphi = 0.0;
      sphi = 1.0;
    }

    bool leaf = n <= leaf_size;
    uint32_t mid = b + n / 2;
    if (!leaf) {
#if HRT_BVH_SWEEP
      // full-sweep SAH: every split between centroid-sorted entries on each axis
      double best = HUGE_VAL;
      int best_axis = -1;
      uint32_t best_at = 0;
      std::vector<double> right_area(n);
      for (int k = 0; k < 3; ++k) {
        std::sort(e.begin() + b, e.begin() + b + n, [&](const Entry& x, const Entry& y) {
          const double cx = comp(x.centroid, k), cy = comp(y.centroid, k);
          return cx < cy || (cx == cy && x.key < y.key);
        });
        Box acc;
        for (uint32_t i = n; i-- > 1;) {
          acc.grow(e[b + i].sbox);
          right_area[i] = acc.area();
        }
        Box left;
        for (uint32_t i = 1; i < n; ++i) {
          left.grow(e[b + i - 1].sbox);
          const double cost = left.area() * i + right_area[i] * (n - i);
          if (cost < best) {
            best = cost;
            best_axis = k;
            best_at = i;
          }
        }
      }
      if (best_axis >= 0) {
        std::sort(e.begin() + b, e.begin() + b + n, [&](const Entry& x, const Entry& y) {
          const double cx = comp(x.centroid, best_axis), cy = comp(y.centroid, best_axis);
          return cx < cy || (cx == cy && x.key < y.key);
        });
        mid = b + best_at;
      }
#else
      // binned SAH over the centroid box, 16 bins per axis
      constexpr int kBins = 16;
      double best = HUGE_VAL;
      int best_axis = -1, best_split = 0;
      for (int k = 0; k < 3; ++k) {
        const double lo = comp(cbox.lo, k), hi = comp(cbox.hi, k);
        if (!(hi > lo)) continue;
        Box bins[kBins];
        uint32_t cnt[kBins] = {};
        const double scale = kBins / (hi - lo);
        for (uint32_t i = b; i < b + n; ++i) {
          int j = (int)((comp(e[i].centroid, k) - lo) * scale);
          j = std::min(kBins - 1, std::max(0, j));
          bins[j].grow(e[i].box);
          cnt[j]++;
        }
        double right_area[kBins];
        uint32_t right_cnt[kBins];
        Box acc;
        uint32_t c = 0;
        for (int j = kBins - 1; j > 0; --j) {
          acc.grow(bins[j]);
          c += cnt[j];
          right_area[j] = acc.area();
          right_cnt[j] = c;
        }
        Box left;
        uint32_t lc = 0;
        for (int j = 1; j < kBins; ++j) {
          left.grow(bins[j - 1]);
          lc += cnt[j - 1];
          if (lc == 0 || right_cnt[j] == 0) continue;
          const double cost = left.area() * lc + right_area[j] * right_cnt[j];
          if (cost < best) {
            best = cost;
            best_axis = k;
            best_split = j;
          }
        }
      }
      if (best_axis >= 0) {
        const double lo = comp(cbox.lo, best_axis), hi = comp(cbox.hi, best_axis);
        const double scale = kBins / (hi - lo);
        auto it = std::partition(e.begin() + b, e.begin() + b + n, [&](const Entry& x) {
          int j = (int)((comp(x.centroid, best_axis) - lo) * scale);
          j = std::min(kBins - 1, std::max(0, j));
          return j < best_split;
        });
        mid = (uint32_t)(it - e.begin());
      }
      if (mid <= b || mid >= b + n) mid = b + n / 2;  // coincident centroids: split the range
#endif
    }

    // mg = a + b R, plus 4e x the box's largest coordinate for the kernel's rounding of lo - mg / hi + mg
    const double coord = std::max({std::fabs(box.lo.x), std::fabs(box.lo.y), std::fabs(box.lo.z),
                                   std::fabs(box.hi.x), std::fabs(box.hi.y), std::fabs(box.hi.z)});
    const double a_m = a_tri + 4 * eps * coord;
    const double b_m = b_tri;
    out.rho_max = std::max(out.rho_max, rho);
    float* r = &out.nodes[(size_t)node * 16];
    r[0] = round_down(box.lo.x);
    r[1] = round_down(box.lo.y);
    r[2] = round_down(box.lo.z);
    r[3] = round_up(a_m * (1.0 + 1e-6));
    r[4] = round_up(box.hi.x);
    r[5] = round_up(box.hi.y);
    r[6] = round_up(box.hi.z);
    r[7] = round_up(b_m * (1.0 + 1e-6));
    r[8] = (float)axis.x;
    r[9] = (float)axis.y;
    r[10] = (float)axis.z;
    r[11] = (float)cphi;
    r[12] = (float)sphi;
    r[13] = round_up(rho + 1e-12);
    if (leaf) {
      r[14] = bits_f(out.n_prims | (n << 27));
      for (uint32_t i = b; i < b + n; ++i) emit_prim(e[i], tris);
      out.n_prims += n;
    } else {
      r[14] = bits_f(0u);
      build(b, mid - b, tris);
      // inner node: the right child's index (count bits 27..31 stay 0); the left child is node + 1
      out.nodes[(size_t)node * 16 + 14] = bits_f(out.n_nodes);
      build(mid, b + n - mid, tris);
    }
    out.nodes[(size_t)node * 16 + 15] = bits_f(out.n_nodes);  // escape: first node after the subtree
  }
};

bool finite3(const float* p) { return std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]); }

// Cube-map direction of face f (2 * major axis + negative) at tangent coordinates (u, v); the trace
// kernel's dir_cell inverts this (u, v = the two minor components over the major one).
V3 face_dir(int f, double u, double v) {
  const double s = (f & 1) ? -1.0 : 1.0;
  switch (f >> 1) {
    case 0: return {s, u, v};
    case 1: return {v, s, u};
    default: return {u, v, s};
  }
}

struct Cone {
  V3 c;
  double cr, sr;  // cos, sin of the cap radius
};

// Cap containing every direction of the cell [u0, u1] x [v0, v1] of face f (a convex spherical quad,
// so the farthest point from the centre is a corner), widened by 1e-4 rad for the kernel's rounding.
Cone cell_cone(int f, double u0, double u1, double v0, double v1) {
  V3 c = face_dir(f, 0.5 * (u0 + u1), 0.5 * (v0 + v1));
  c = c * (1.0 / norm(c));
  double r = 0.0;
  const double us[2] = {u0, u1}, vs[2] = {v0, v1};
  for (double u : us)
    for (double v : vs) {
      V3 d = face_dir(f, u, v);
      d = d * (1.0 / norm(d));
      r = std::max(r, std::acos(std::max(-1.0, std::min(1.0, dot(c, d)))));
    }
  r += 1e-4;
  return {c, std::cos(r), std::sin(r)};
}

// Is d.nhat in the grazing band (-tau - 1e-5, 2e-5) for some d in the cap?  With
// theta = angle(c, nhat): d.nhat ranges over [cos(min(pi, theta + r)), cos(max(0, theta - r))].
bool cone_hits_band(const Cone& k, V3 nhat, double tau) {
  const double x = std::max(-1.0, std::min(1.0, dot(k.c, nhat)));
  const double y = std::sqrt(std::max(0.0, 1.0 - x * x));
  const double hi = (x >= k.cr) ? 1.0 : x * k.cr + y * k.sr;
  const double lo = (x <= -k.cr) ? -1.0 : x * k.cr - y * k.sr;
  return hi > -(tau + 1e-5) && lo < 2e-5;
}

void build_band_lists(BvhHost& out) {
  std::vector<V3> nh(out.n_prims);
  for (uint32_t k = 0; k < out.n_prims; ++k) {
    const V3 n = ld(&out.prims[(size_t)k * 16 + 12]);
    nh[k] = n * (1.0 / norm(n));
  }
  const int kDirRes = (int)out.dir_res, kDirCells = 6 * kDirRes * kDirRes;
  // coarse-to-fine: a cell's candidates are its parent's entries whose band meets the cell's cap
  // (the caps nest up to their 1e-4 rad widening, which cone_hits_band's caps all carry), through
  // resolutions 8, 64, then steps of 4 (or 2, 3) up to dir_res; the fine cells test their corners.
  // Filtering keeps the candidates' order (ascending prim index).
  constexpr int kCoarse = 8;
  std::vector<int> res{kCoarse};  // the filtering levels (each divides the next and dir_res)
  if (kDirRes > 64) res.push_back(64);
  while (res.back() * 2 < kDirRes) {
    const int r = res.back();
    const int s = kDirRes % (r * 4) == 0 && r * 4 < kDirRes ? 4 : kDirRes % (r * 2) == 0 ? 2 : kDirRes % (r * 3) == 0 ? 3 : 0;
    if (s == 0) break;
    res.push_back(r * s);
  }
  out.band_off.assign(kDirCells + 1, 0);
  auto cone_of = [](int f, int r, int iu, int iv) {
    return cell_cone(f, -1.0 + 2.0 * iu / r, -1.0 + 2.0 * (iu + 1) / r, -1.0 + 2.0 * iv / r, -1.0 + 2.0 * (iv + 1) / r);
  };
  // Each coarse cell's task appends its fine cells' lists to its own buffer (cell index and length in
  // visiting order); the offsets and the global list are assembled after the tasks.
  struct TaskOut {
    std::vector<uint32_t> ents;
    std::vector<std::pair<uint32_t, uint32_t>> cells;
  };
  constexpr int kTasks = 6 * kCoarse * kCoarse;
  std::vector<TaskOut> outs(kTasks);
  // cell (iu, iv) of face f at level lv (resolution res[lv]) with its candidates: its children's
  // candidates by their caps, down to the fine cells' exact test
  std::function<void(TaskOut&, int, size_t, int, int, const std::vector<uint32_t>&)> refine =
      [&](TaskOut& o, int f, size_t lv, int iu, int iv, const std::vector<uint32_t>& cand) {
        const int s = (lv + 1 < res.size() ? res[lv + 1] : kDirRes) / res[lv];
        std::vector<uint32_t> sub;
        if (lv + 1 == res.size()) {
          // the children are fine cells: their corner directions, normalized once for the block
          const int g = s + 1;
          std::vector<V3> G((size_t)g * g);
          for (int a = 0; a < g; ++a)
            for (int b = 0; b < g; ++b) {
              const V3 d = face_dir(f, -1.0 + 2.0 * (iu * s + a) / kDirRes, -1.0 + 2.0 * (iv * s + b) / kDirRes);
              G[(size_t)a * g + b] = d * (1.0 / norm(d));
            }
          for (int su = 0; su < s; ++su) {
            for (int sv = 0; sv < s; ++sv) {
              const int ju = iu * s + su, jv = iv * s + sv;
              const V3 c[4] = {G[(size_t)su * g + sv], G[(size_t)(su + 1) * g + sv], G[(size_t)(su + 1) * g + sv + 1],
                               G[(size_t)su * g + sv + 1]};
              // d.nhat over the cell: between its corners' values, widened by the edges' bulge -- on a
              // great-circle arc of angle t between two corners, d is the chord point over its length
              // (>= cos(t / 2)), so |d.nhat| exceeds the chord's linear value by at most 1 / cos(t / 2) - 1;
              // the interior adds only +-1 when +-nhat is inside, far from the band for cells this small.
              // Then the quad test's own widening of 1e-4 + 1e-9 (the kernel's dir_cell rounding).
              double cmin = 1.0;
              for (int i = 0; i < 4; ++i) cmin = std::min(cmin, dot(c[i], c[(i + 1) & 3]));
              const double bulge = 1.0 / std::sqrt(std::max(0.5 * (1.0 + cmin), 1e-300)) - 1.0 + 1e-12;
              const double wid = bulge + 1e-4 + 1e-9;
              const size_t n0 = o.ents.size();
              for (uint32_t k : cand) {
                const V3 n = nh[k];
                const double v0 = dot(c[0], n), v1 = dot(c[1], n), v2 = dot(c[2], n), v3 = dot(c[3], n);
                const double hi = std::max(std::max(v0, v1), std::max(v2, v3)), lo = std::min(std::min(v0, v1), std::min(v2, v3));
                if (hi + wid > -(out.band_tau + 1e-5) && lo - wid < 2e-5) o.ents.push_back(k);
              }
              o.cells.emplace_back((uint32_t)(((size_t)f * kDirRes + ju) * kDirRes + jv), (uint32_t)(o.ents.size() - n0));
            }
          }
          return;
        }
        for (int su = 0; su < s; ++su) {
          for (int sv = 0; sv < s; ++sv) {
            const int ju = iu * s + su, jv = iv * s + sv;
            const Cone c = cone_of(f, res[lv + 1], ju, jv);
            sub.clear();
            for (uint32_t k : cand)
              if (cone_hits_band(c, nh[k], out.band_tau)) sub.push_back(k);
            refine(o, f, lv + 1, ju, jv, sub);
          }
        }
      };
  auto task = [&](int t) {
    const int f = t / (kCoarse * kCoarse), cu = (t / kCoarse) % kCoarse, cv = t % kCoarse;
    const Cone kc = cone_of(f, kCoarse, cu, cv);
    std::vector<uint32_t> coarse;
    for (uint32_t k = 0; k < out.n_prims; ++k)
      if (cone_hits_band(kc, nh[k], out.band_tau)) coarse.push_back(k);
    refine(outs[t], f, 0, cu, cv, coarse);
  };
  const unsigned nthreads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::atomic<int> next{0};
  auto worker = [&]() {
    for (int t; (t = next.fetch_add(1)) < kTasks;) task(t);
  };
  std::vector<std::thread> pool;
  for (unsigned i = 1; i < nthreads && out.n_prims > 64; ++i) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  for (const TaskOut& o : outs)
    for (const auto& c : o.cells) out.band_off[c.first + 1] = c.second;
  for (int c = 0; c < kDirCells; ++c) out.band_off[c + 1] += out.band_off[c];
  out.band_list.resize(out.band_off[kDirCells]);
  next = 0;  // each task's lists to their places (disjoint ranges), on the same threads
  auto copier = [&]() {
    for (int t; (t = next.fetch_add(1)) < kTasks;) {
      size_t at = 0;
      for (const auto& c : outs[t].cells) {
        std::copy(outs[t].ents.begin() + at, outs[t].ents.begin() + at + c.second, out.band_list.begin() + out.band_off[c.first]);
        at += c.second;
      }
      std::vector<uint32_t>().swap(outs[t].ents);
    }
  };
  pool.clear();
  for (unsigned i = 1; i < nthreads && out.n_prims > 64; ++i) pool.emplace_back(copier);
  copier();
  for (auto& th : pool) th.join();
  // (entries: the prim index, hrt_bvh.h) the pre-check's normals, one per prim
  out.band_nhat.assign((size_t)out.n_prims * 4, 0.0f);
  for (uint32_t k = 0; k < out.n_prims; ++k) {
    out.band_nhat[(size_t)k * 4] = (float)nh[k].x;
    out.band_nhat[(size_t)k * 4 + 1] = (float)nh[k].y;
    out.band_nhat[(size_t)k * 4 + 2] = (float)nh[k].z;
    // the plane's offset n^.a (the kernel's plane-side filter of band entries)
    const V3 a = ld(&out.prims[(size_t)k * 16]);
    out.band_nhat[(size_t)k * 4 + 3] = (float)dot(nh[k], a);
    out.band_a1 = std::max(out.band_a1, round_up(std::fabs(a.x) + std::fabs(a.y) + std::fabs(a.z)));
  }
}

// Every finite binary16 value (ascending, +0 once) with its bits: directed conversions by search.
struct Half {
  std::vector<std::pair<double, uint16_t>> v;
  Half() {
    for (uint32_t b = 0; b < 0x10000u; ++b) {
      const uint32_t e = (b >> 10) & 31u, m = b & 1023u;
      if (e == 31u || b == 0x8000u) continue;  // inf / NaN, -0
      const double mag = e ? std::ldexp(1024.0 + m, (int)e - 25) : std::ldexp((double)m, -24);
      v.emplace_back((b >> 15) ? -mag : mag, (uint16_t)b);
    }
    std::sort(v.begin(), v.end());
  }
  // dir < 0: largest value <= x; dir > 0: smallest >= x; 0: nearest (ties to the lower)
  uint16_t conv(double x, int dir) const {
    x = std::max(v.front().first, std::min(v.back().first, x));
    size_t i = (size_t)(std::lower_bound(v.begin(), v.end(), std::make_pair(x, (uint16_t)0)) - v.begin());
    if (i == v.size()) i = v.size() - 1;
    if (dir > 0) return v[i].second;                      // v[i] >= x
    if (v[i].first == x || i == 0) return v[i].second;
    if (dir < 0) return v[i - 1].second;                  // v[i - 1] < x
    return (x - v[i - 1].first <= v[i].first - x) ? v[i - 1].second : v[i].second;
  }
};

}  // namespace

bool make_wq_nodes(const BvhHost& b, std::vector<float>& out, uint32_t width, uint32_t* n_out, uint32_t* w_out) {
  out.clear();
  *n_out = 0;
  *w_out = 2;
  width = std::max(2u, std::min(width, kWqMaxWidth));
  static const Half h;
  if (b.n_nodes == 0) return true;
  auto word = [&](uint32_t k, int j) {
    uint32_t u;
    std::memcpy(&u, &b.nodes[(size_t)k * 16 + j], 4);
    return u;
  };
  auto is_leaf = [&](uint32_t k) { return (word(k, 14) >> 27) != 0; };
  auto area = [&](uint32_t k) {
    const float* r = &b.nodes[(size_t)k * 16];
    const double ex = std::max(0.0, (double)r[4] - r[0]), ey = std::max(0.0, (double)r[5] - r[1]),
                 ez = std::max(0.0, (double)r[6] - r[2]);
    return ex * ey + ey * ez + ex * ez;
  };
  // Groups: the children of a kept inner node are its binary children, the inner one of largest
  // surface area replaced by its own two children (in place, order kept) while the group has fewer
  // than `width` members.  A kept node's record is its binary node's (the same box, margins and cone);
  // the collapsed intermediate nodes are never tested.  Slots are allocated depth first.
  std::vector<uint32_t> new_of(b.n_nodes, ~0u), esc_of(b.n_nodes, 0u), info_of(b.n_nodes, 0u), order;
  order.reserve(b.n_nodes);
  new_of[0] = 0;
  esc_of[0] = 0;  // patched to the node count below
  order.push_back(0);
  uint32_t next = 1, widest = 2;
  std::vector<uint32_t> todo{0};
  while (!todo.empty()) {
    const uint32_t k = todo.back();
    todo.pop_back();
    if (is_leaf(k)) {
      info_of[k] = word(k, 14);
      continue;
    }
    std::vector<uint32_t> ch{k + 1, word(k, 14)};
    while (ch.size() < width) {
      int best = -1;
      for (size_t j = 0; j < ch.size(); ++j)
        if (!is_leaf(ch[j]) && (best < 0 || area(ch[j]) > area(ch[(size_t)best]))) best = (int)j;
      if (best < 0) break;
      const uint32_t c = ch[(size_t)best];
      ch[(size_t)best] = c + 1;
      ch.insert(ch.begin() + best + 1, word(c, 14));
    }
    const uint32_t fc = next, cnt = (uint32_t)ch.size();
    widest = std::max(widest, cnt);
    next += cnt;
    info_of[k] = fc | (cnt - 1u) << 16;
    for (uint32_t j = 0; j < cnt; ++j) {
      new_of[ch[j]] = fc + j;
      esc_of[ch[j]] = j + 1 < cnt ? fc + j + 1 : esc_of[k];  // the last child continues after the parent
      order.push_back(ch[j]);
    }
    for (uint32_t j = cnt; j-- > 0;) todo.push_back(ch[j]);  // depth first, left child on top
  }
  if (next >= 0x10000u) return false;  // 16-bit child and escape indices
  for (uint32_t k : order)
    if (esc_of[k] == 0u) esc_of[k] = next;  // the root and the right spine: end of the walk
  out.resize((size_t)next * 12);
  for (uint32_t k : order) {
    const float* r = &b.nodes[(size_t)k * 16];
    float* w = &out[(size_t)new_of[k] * 12];
    for (int j = 0; j < 8; ++j) w[j] = r[j];
    uint32_t u[4];
    u[0] = h.conv(r[8], 0) | (uint32_t)h.conv(r[9], 0) << 16;
    u[1] = h.conv(r[10], 0) | (uint32_t)h.conv(r[11], -1) << 16;
    u[2] = h.conv((double)r[12] * r[12] * 1.00001, +1) | esc_of[k] << 16;  // S >= sin^2 x 1.00001 (r[12] >= 0)
    u[3] = info_of[k];
    std::memcpy(&w[8], u, 16);
  }
  *n_out = next;
  *w_out = widest;
  return true;
}

bool build_bvh(const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes, uint32_t n_meshes,
               uint32_t leaf_size, BvhHost& out, uint32_t wq_width, float band_tau, bool bands) {
  out = BvhHost{};
  out.band_tau = band_tau;
  if (n_meshes > kBvhMaxMeshes) return false;
  uint64_t total = 0;
  for (uint32_t m = 0; m < n_meshes; ++m) total += meshes[m].len;
  if (total > kBvhMaxEntries || n_tris >= (1u << 26)) return false;
  leaf_size = std::max(1u, std::min(leaf_size, kBvhMaxLeafCount));
  std::vector<Entry> entries;
  entries.reserve(total);
  uint32_t key = 1;
  for (uint32_t m = 0; m < n_meshes; ++m) {
    out.key_base.push_back(key - meshes[m].first_index);  // key of (m, first_index + k) = key + k
    for (uint32_t k = 0; k < meshes[m].len; ++k, ++key) {
      const uint32_t i = meshes[m].first_index + k;
      if (i >= n_tris) continue;  // hrt_set_scene validated the ranges
      const hrt_triangle& t = tris[i];
      if (t.normal[0] == 0.0f && t.normal[1] == 0.0f && t.normal[2] == 0.0f) {
        out.n_never++;  // d.n is +-0 for every d: the reference's dn >= 0 rejects it (raytracing.glsl:219)
        continue;
      }
      const V3 a = ld(t.a), e1 = ld(t.edge_one), e2 = ld(t.edge_two), n = ld(t.normal);
      const V3 b = a + e1, c = a + e2;
      const double nn = norm(n), l1 = norm(e1), l2 = norm(e2);
      const double big = 1e18;
      bool regular = finite3(t.a) && finite3(t.edge_one) && finite3(t.edge_two) && finite3(t.normal) &&
                     nn >= 1e-25 && nn <= 1e30 && l1 <= big && l2 <= big;
      for (int q = 0; q < 3 && regular; ++q)
        regular = std::fabs(comp(a, q)) <= big && std::fabs(comp(b, q)) <= big && std::fabs(comp(c, q)) <= big;
      double rho = 0.0;
      if (regular) {
        rho = norm(n - cross(e1, e2)) / nn + 1e-12;
        regular = rho <= 1e-4;
      }
      if (!regular) {
        const float rec[16] = {t.a[0], t.a[1], t.a[2], bits_f(key),
                               t.edge_one[0], t.edge_one[1], t.edge_one[2], bits_f(m),
                               t.edge_two[0], t.edge_two[1], t.edge_two[2], bits_f(i),
                               t.normal[0], t.normal[1], t.normal[2], 0.0f};
        out.irregular.insert(out.irregular.end(), rec, rec + 16);
        out.n_irregular++;
        continue;
      }
      Entry en;
      en.box.grow(a);
      en.box.grow(b);
      en.box.grow(c);
      en.centroid = (a + b + c) * (1.0 / 3.0);
      en.nhat = n * (1.0 / nn);
      en.g = std::max(l1, l2) / nn;
      en.rho = rho;
      en.ext = std::max({en.box.hi.x - en.box.lo.x, en.box.hi.y - en.box.lo.y, en.box.hi.z - en.box.lo.z});
      en.key = key;
      en.mesh = m;
      en.index = i;
      entries.push_back(en);
    }
  }
  if (!entries.empty()) {
    // the SAH's boxes: each triangle's box grown by its own margin a_i + b_i R at a typical R
    Box scene;
    for (const Entry& en : entries) scene.grow(en.box);
    const double R_sah = HRT_BVH_SAH_R * norm(scene.hi - scene.lo), eps = 5.9604644775390625e-08;
    for (Entry& en : entries) {
      const double inv_tpi = 1.02 / ((double)out.band_tau - en.rho - 4e-7);
      const double m = R_sah > 0.0 ? 2.02 * en.ext * (6 * eps + (1.01 * en.rho + 3.2 * eps + 18.4 * eps * en.g * R_sah) * inv_tpi)
                                   : 0.0;
      en.sbox = en.box;
      en.sbox.lo = en.sbox.lo - V3{m, m, m};
      en.sbox.hi = en.sbox.hi + V3{m, m, m};
    }
    Builder bld{entries, leaf_size, out};
    bld.build(0, (uint32_t)entries.size(), tris);
  }
  // hierarchy quality: sum over leaves of area(leaf box) / area(root box) x leaf triangles = the
  // expected leaf triangle tests of a uniform random line through the scene, per entry
  if (out.n_nodes && out.n_prims) {
    auto area = [&](uint32_t k) {
      const float* r = &out.nodes[(size_t)k * 16];
      const double ex = std::max(0.0, (double)r[4] - r[0]), ey = std::max(0.0, (double)r[5] - r[1]),
                   ez = std::max(0.0, (double)r[6] - r[2]);
      return 2.0 * (ex * ey + ey * ez + ex * ez);
    };
    const double root = area(0);
    double tests = 0.0;
    for (uint32_t k = 0; k < out.n_nodes; ++k) {
      uint32_t info;
      std::memcpy(&info, &out.nodes[(size_t)k * 16 + 14], 4);
      if (info >> 27) tests += (info >> 27) * (root > 0.0 ? area(k) / root : 1.0);
    }
    out.sah_tri_frac = tests / out.n_prims;
    // how wide the box margins a + b R are at R = the scene's diagonal (HRT_SCENE_BVH_MARGIN_MILLI)
    const float* r0 = &out.nodes[0];
    const double R = std::sqrt((double)(r0[4] - r0[0]) * (r0[4] - r0[0]) + (double)(r0[5] - r0[1]) * (r0[5] - r0[1]) +
                               (double)(r0[6] - r0[2]) * (r0[6] - r0[2]));
    double msum = 0.0;
    for (uint32_t k = 0; k < out.n_nodes; ++k) {
      const float* r = &out.nodes[(size_t)k * 16];
      const double ext = std::max({(double)r[4] - r[0], (double)r[5] - r[1], (double)r[6] - r[2], 1e-30});
      msum += ((double)r[3] + (double)r[7] * R) / ext;
    }
    out.margin_frac = out.n_nodes ? msum / out.n_nodes : 0.0;
  }
  out.dir_res = (uint32_t)dir_res_for(out.n_prims);
  if (bands) build_bands(out);
  // t-slack of the box test for a lane at distance <= R: abs = abs_coef R, rel
  const double e = 5.9604644775390625e-08, inv_tp = 1.02 / ((double)out.band_tau - out.rho_max - 4e-7);
  out.abs_coef = round_up(2.1 * (4.2 * e + out.rho_max) * inv_tp * (1.0 + 1e-6));
  out.rel_t = round_up((2.1 * (3.2 * e + out.rho_max) * inv_tp + 4 * e) * (1.0 + 1e-6));
  out.wq_ok = make_wq_nodes(out, out.wq_nodes, wq_width, &out.wq_n_nodes, &out.wq_width);
  return true;
}

// The lists are a function of the prim records (their order and normals), tau_g and dir_res alone, and
// most of a scene's set-up time at 1024 cells per face edge (~0.5 s for island): the last two results
// are kept for the process, so contexts of one scene (a rank group in one process, or a test suite's
// many contexts) build them once.  A hit compares the whole prim image, not only its hash.  Resident
// host cost: the prim image plus the lists, ~100 MB per entry for island and ~130 MB for cave at the
// default resolution; hrt_release_caches() drops them.
struct BandCache {
  std::vector<float> prims;
  uint32_t dir_res = 0;
  float tau = 0.0f;
  std::vector<uint32_t> off, list;
  std::vector<float> nhat;
  float a1 = 0.0f;
};

namespace {
std::mutex band_cache_mu;
std::vector<std::shared_ptr<const BandCache>> band_cache;  // most recent last, at most 2
}  // namespace

uint64_t release_band_cache() {
  std::vector<std::shared_ptr<const BandCache>> gone;
  {
    std::lock_guard<std::mutex> lock(band_cache_mu);
    gone.swap(band_cache);
  }
  uint64_t bytes = 0;
  for (const auto& c : gone)
    bytes += c->prims.size() * sizeof(float) + (c->off.size() + c->list.size()) * sizeof(uint32_t) +
             c->nhat.size() * sizeof(float);
  return bytes;  // (freed as `gone` goes out of scope; a build holding an entry keeps it alive until done)
}

void build_bands(BvhHost& out) {
  std::mutex& mu = band_cache_mu;
  std::vector<std::shared_ptr<const BandCache>>& kept = band_cache;
  auto same = [&](const BandCache& c) {
    return c.dir_res == out.dir_res && c.tau == out.band_tau && c.prims.size() == out.prims.size() &&
           std::memcmp(c.prims.data(), out.prims.data(), out.prims.size() * sizeof(float)) == 0;
  };
  {
    std::lock_guard<std::mutex> lock(mu);
    for (size_t i = kept.size(); i-- > 0;) {
      if (!same(*kept[i])) continue;
      const std::shared_ptr<const BandCache> c = kept[i];
      kept.erase(kept.begin() + (long)i);
      kept.push_back(c);
      out.band_off = c->off;
      out.band_list = c->list;
      out.band_nhat = c->nhat;
      out.band_a1 = c->a1;
      return;
    }
  }
  build_band_lists(out);
  auto c = std::make_shared<BandCache>();
  c->prims = out.prims;
  c->dir_res = out.dir_res;
  c->tau = out.band_tau;
  c->off = out.band_off;
  c->list = out.band_list;
  c->nhat = out.band_nhat;
  c->a1 = out.band_a1;
  std::lock_guard<std::mutex> lock(mu);
  kept.push_back(std::move(c));
  if (kept.size() > 2) kept.erase(kept.begin());
}

}  // namespace hrt

// ---- host-only inspection (tests/test_bvh.py): build and copy out, no GPU involved ----------------
extern "C" int hrt_debug_bvh_build(const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes,
                                   uint32_t n_meshes, uint32_t leaf_size, uint32_t counts[7], float* nodes,
                                   uint64_t nodes_cap, float* prims, uint64_t prims_cap, float* irregular,
                                   uint64_t irregular_cap, uint32_t* band_off, uint64_t band_off_cap,
                                   uint32_t* band_list, uint64_t band_list_cap) {
  hrt::BvhHost b;
  const bool built = hrt::build_bvh(tris, n_tris, meshes, n_meshes, leaf_size, b);
  counts[0] = b.n_nodes;
  counts[1] = b.n_prims;
  counts[2] = b.n_irregular;
  counts[3] = b.n_never;
  counts[4] = built ? 1u : 0u;
  counts[5] = (uint32_t)b.band_list.size();
  counts[6] = b.dir_res;
  if (!built) return 0;
  auto copy = [](auto* dst, uint64_t cap, const auto& v) {
    if (dst && cap >= v.size() && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
    return !dst || cap >= v.size();
  };
  const bool ok = copy(nodes, nodes_cap, b.nodes) && copy(prims, prims_cap, b.prims) &&
                  copy(irregular, irregular_cap, b.irregular) && copy(band_off, band_off_cap, b.band_off) &&
                  copy(band_list, band_list_cap, b.band_list);
  return ok ? 1 : -1;
}

extern "C" int64_t hrt_debug_bvh_wq_nodes(const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes,
                                          uint32_t n_meshes, uint32_t leaf_size, uint32_t width, float* out,
                                          uint64_t cap) {
  hrt::BvhHost b;
  if (!hrt::build_bvh(tris, n_tris, meshes, n_meshes, leaf_size, b, width) || !b.wq_ok || b.wq_nodes.empty()) return 0;
  if (!out || cap < b.wq_nodes.size()) return -1;
  std::memcpy(out, b.wq_nodes.data(), b.wq_nodes.size() * sizeof(float));
  return (int64_t)(b.wq_nodes.size() / 12);
}
