// config_scenes.cpp -- main.cc's config scenes on the plugin surface, plus a
// small C ABI (rtsc_*) that tests and bench.py use to obtain the exact
// descriptor camera::render would hand to librt_hip.
#include "config_scenes.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <vector>

#include "../rt/gltf_loader.h"

namespace {

int W(int width, int dflt) { return width > 0 ? width : dflt; }
double A(double aspect, double dflt) { return aspect > 0 ? aspect : dflt; }

void cornell_box(int width, double aspect, config_scene* s) {  // main.cc:198-225
  hittable_list world;
  auto red = std::make_shared<lambertian>(std::make_shared<solid_color>(color{.65, .05, .05}));
  auto white = std::make_shared<lambertian>(std::make_shared<solid_color>(color{0.73, 0.73, 0.73}));
  auto green = std::make_shared<lambertian>(std::make_shared<solid_color>(color{.12, .45, .15}));
  auto light = std::make_shared<diffuse_light>(std::make_shared<solid_color>(color{15, 15, 15}));
  world.push_back(std::make_shared<quad>(point3(555, 0, 0), vec3(0, 555, 0), vec3(0, 0, 555), green));
  world.push_back(std::make_shared<quad>(point3(0, 0, 0), vec3(0, 555, 0), vec3(0, 0, 555), red));
  world.push_back(std::make_shared<quad>(point3(0, 0, 0), vec3(555, 0, 0), vec3(0, 0, 555), white));
  world.push_back(std::make_shared<quad>(point3(555, 555, 555), vec3(-555, 0, 0), vec3(0, 0, -555), white));
  world.push_back(std::make_shared<quad>(point3(0, 0, 555), vec3(555, 0, 0), vec3(0, 555, 0), white));
  world.push_back(std::make_shared<translate>(vec3(100, 0, 200), box(point3(0), point3(165, 330, 165), white)));
  world.push_back(std::make_shared<translate>(vec3(50, 0, 100), box(point3(0), point3(165, 165, 165), white)));
  auto quad_light = std::make_shared<quad>(point3(343, 554, 332), vec3(-130, 0, 0), vec3(0, 0, -105), light);
  world.push_back(quad_light);
  s->world = std::make_shared<bvh_node>(world);
  s->light = quad_light;
  s->cam.initialize_perspective(W(width, 600), A(aspect, 1.0), point3(278, 278, -800), point3(278, 278, 0), 1,
                                40.0, 40, 4);
  s->cam.background_ = solid_color::black;
}

void cornell_box_with_volume(int width, double aspect, config_scene* s) {  // main.cc:227-253
  auto world = std::make_shared<hittable_list>();
  auto red = std::make_shared<lambertian>(color(.65, .05, .05));
  auto white = std::make_shared<lambertian>(color(.73, .73, .73));
  auto green = std::make_shared<lambertian>(color(.12, .45, .15));
  auto light = std::make_shared<diffuse_light>(color(7, 7, 7));
  world->push_back(std::make_shared<quad>(point3(555, 0, 0), vec3(0, 555, 0), vec3(0, 0, 555), green));
  world->push_back(std::make_shared<quad>(point3(0, 0, 0), vec3(0, 555, 0), vec3(0, 0, 555), red));
  world->push_back(std::make_shared<quad>(point3(0, 555, 0), vec3(555, 0, 0), vec3(0, 0, 555), white));
  world->push_back(std::make_shared<quad>(point3(0, 0, 0), vec3(555, 0, 0), vec3(0, 0, 555), white));
  world->push_back(std::make_shared<quad>(point3(0, 0, 555), vec3(555, 0, 0), vec3(0, 555, 0), white));
  auto box1 = std::make_shared<translate>(
      vec3(265, 0, 285), std::make_shared<rotate_y>(box(point3(0), point3(150, 280, 150), white), 45));
  auto box2 = std::make_shared<translate>(
      vec3(130, 0, 65), std::make_shared<rotate_y>(box(point3(0), point3(140, 140, 140), white), -15));
  world->push_back(std::make_shared<volumne>(box1, 0.02, std::make_shared<solid_color>(color(0))));
  world->push_back(std::make_shared<volumne>(box2, 0.02, std::make_shared<solid_color>(color(1))));
  auto quad_light = std::make_shared<quad>(point3(113, 554, 127), vec3(330, 0, 0), vec3(0, 0, 305), light);
  world->push_back(quad_light);
  s->world = world;
  s->light = quad_light;
  s->cam.initialize_perspective(W(width, 600), A(aspect, 1.0), point3(278, 278, -800), point3(278, 278, 0), 1, 40,
                                100, 5);
  s->cam.background_ = solid_color::black;
}

// main.cc:105-153. `moving` keeps the reference's moving spheres (whose normals use
// center_ = (0,0,0), sphere.h:69); the static variant places each sphere at center1
// and still draws center2, so the random stream and the sphere list are unchanged.
void random_motion_ball(int width, double aspect, bool moving, config_scene* s) {
  hittable_list world;  // rand() from its default state, srand(1) (build_config_scene)
  auto ground = std::make_shared<lambertian>(
      std::make_shared<checker_texture>(color{1.0, 1.0, 1.0}, color{0.6, 0.6, 0.2}, 1.0));
  world.push_back(std::make_shared<sphere>(point3(0, -1000, 0), 1000, ground));
  for (int a = -11; a < 11; a++) {
    for (int b = -11; b < 11; b++) {
      double choose_mat = random_double();
      double rz = random_double();  // GCC evaluates center1's arguments right to left
      double rx = random_double();
      point3 center1(a + 0.7 * rx, 0.2, b + 0.7 * rz);
      point3 center2 = center1 + vec3(0, random_double(0, .15), 0);
      if ((center1 - point3(4, 0.2, 0)).length() <= 0.9 || choose_mat < 0.3) continue;
      std::shared_ptr<material> m;
      if (choose_mat < 0.8) {
        vec3 rhs = random_vec();  // random_vec() * random_vec(): right operand first
        vec3 lhs = random_vec();
        m = std::make_shared<lambertian>(std::make_shared<solid_color>(lhs * rhs));
      } else if (choose_mat < 0.95) {
        m = std::make_shared<metal>(std::make_shared<solid_color>(random_vec(0.5, 1)), 0.0);
      } else {
        m = std::make_shared<dielectric>(std::make_shared<solid_color>(color(1)), 1.5);
      }
      if (moving)
        world.push_back(std::make_shared<sphere>(center1, center2, 0.2, m));
      else
        world.push_back(std::make_shared<sphere>(center1, 0.2, m));
    }
  }
  auto glass = std::make_shared<dielectric>(std::make_shared<solid_color>(color(1)), 1.5);
  auto matte = std::make_shared<lambertian>(std::make_shared<solid_color>(color(0.4, 0.2, 0.1)));
  world.push_back(std::make_shared<sphere>(point3(0, 1, 0), 1.0, glass));
  world.push_back(std::make_shared<sphere>(point3(-4, 1, 0), 1.0, matte));
  world.push_back(std::make_shared<sphere>(point3(4, 1, 0), 1.0, glass));
  s->world = std::make_shared<bvh_node>(world);
  s->cam.initialize_perspective(W(width, 1280), A(aspect, 16.0 / 9.0), point3(13, 2, 3), point3(0, 0, 0), 1, 20,
                                20, 50);
  s->cam.background_ = std::make_shared<solid_color>(color(0.7, 0.8, 1.0));
}

void three_material_ball(int width, double aspect, config_scene* s) {  // main.cc:67-84
  auto world = std::make_shared<hittable_list>();
  auto ground = std::make_shared<lambertian>(
      std::make_shared<checker_texture>(color{1.0, 1.0, 1.0}, color{0.6, 0.6, 0.2}, 1.0));
  auto glass = std::make_shared<dielectric>(std::make_shared<solid_color>(color{1.0, 1.0, 1.0}), 1.5);
  auto matte = std::make_shared<lambertian>(std::make_shared<solid_color>(color(0.4, 0.2, 0.1)));
  auto metal_mat = std::make_shared<metal>(std::make_shared<solid_color>(color(0.7, 0.6, 0.5)), 0.0);
  world->push_back(std::make_shared<sphere>(point3(0, -1000, 0), 1000, ground));
  world->push_back(std::make_shared<sphere>(point3(0, 1, 0), 1.0, glass));
  world->push_back(std::make_shared<sphere>(point3(-4, 1, 0), 1.0, matte));
  world->push_back(std::make_shared<sphere>(point3(4, 1, 0), 1.0, metal_mat));
  s->world = world;
  s->cam.initialize_perspective(W(width, 1280), A(aspect, 16.0 / 9.0), point3(13, 2, 3), vec3(0, 0, 0), 1, 20.0,
                                100, 5);
  s->cam.background_ = std::make_shared<solid_color>(color(0.7, 0.8, 1.0));
}

void three_material_ball_with_defocus_blur(int width, double aspect, config_scene* s) {  // main.cc:87-103
  auto world = std::make_shared<hittable_list>();
  auto ground = std::make_shared<lambertian>(
      std::make_shared<checker_texture>(color{1.0, 1.0, 1.0}, color{0.6, 0.6, 0.2}, 1.0));
  auto glass = std::make_shared<dielectric>(std::make_shared<solid_color>(color{1.0, 1.0, 1.0}), 1.5);
  auto matte = std::make_shared<lambertian>(std::make_shared<solid_color>(color(0.4, 0.2, 0.1)));
  auto metal_mat = std::make_shared<metal>(std::make_shared<solid_color>(color(0.7, 0.6, 0.5)), 0.0);
  world->push_back(std::make_shared<sphere>(point3(0, -1000, 0), 1000, ground));
  world->push_back(std::make_shared<sphere>(point3(0, 1, 0), 1.0, glass));
  world->push_back(std::make_shared<sphere>(point3(-4, 1, 0), 1.0, matte));
  world->push_back(std::make_shared<sphere>(point3(4, 1, 0), 1.0, metal_mat));
  s->world = world;
  s->cam.initialize_lens(W(width, 1280), (float)A(aspect, 16.0 / 9.0), point3(13, 2, 3), vec3(1, 1, 1), 2.0, 15,
                         20.0, 1000, 5);
  s->cam.background_ = std::make_shared<solid_color>(color(0.7, 0.8, 1.0));
}

// main.cc:581-630: a 10 x 10 or 40 x 40 quad under an orthonormal camera, white background
void noise_quad(std::shared_ptr<texture> tex, double size, double view, int width, double aspect,
                config_scene* s) {
  auto world = std::make_shared<hittable_list>();
  world->push_back(std::make_shared<quad>(point3(0, 0, 0), vec3(size, 0, 0), vec3(0, size, 0),
                                          std::make_shared<lambertian>(tex)));
  s->world = world;
  s->cam.initialize_orthnormal(W(width, 400), A(aspect, 1), view, vec3(size / 2, size / 2, 1),
                               vec3(size / 2, size / 2, 0), 10, 5);
  s->cam.background_ = solid_color::white;
}

void perlin_texture_ball(int width, double aspect, config_scene* s) {  // main.cc:402-437
  hittable_list boxes1;
  auto ground = std::make_shared<lambertian>(color(0.48, 0.83, 0.53));
  for (int i = 0; i < 20; i++)
    for (int j = 0; j < 20; j++) {
      double w = 100.0, x0 = -1000.0 + i * w, z0 = -1000.0 + j * w, y0 = 0.0;
      double x1 = x0 + w, y1 = random_double(1, 101), z1 = z0 + w;
      boxes1.push_back(box(point3(x0, y0, z0), point3(x1, y1, z1), ground));
    }
  auto world = std::make_shared<hittable_list>();
  world->push_back(std::make_shared<bvh_node>(boxes1));
  auto light = std::make_shared<diffuse_light>(color(7, 7, 7));
  auto quad_light = std::make_shared<quad>(point3(123, 554, 147), vec3(300, 0, 0), vec3(0, 0, 265), light);
  world->push_back(quad_light);
  world->push_back(std::make_shared<sphere>(point3(260, 150, 45), 50, std::make_shared<dielectric>(1.5)));
  auto pertext = std::make_shared<perlin_texture>(8);
  world->push_back(std::make_shared<translate>(
      point3(180, 280, 400),
      std::make_shared<rotate_x>(std::make_shared<sphere>(point3(0), 80, std::make_shared<lambertian>(pertext)),
                                 -90)));
  s->cam.initialize_perspective(W(width, 600), A(aspect, 1.0), point3(478, 278, -600), point3(278, 278, 0), 1,
                                40.0, 500, 5);
  s->world = std::make_shared<bvh_node>(*world);
  // cam.render(of, bvh): the light is not importance-sampled in this scene (main.cc:436)
}

// The reference's asset directory (./assets); $RT_ASSETS overrides it.
std::string asset(const std::string& name) {
  const char* dir = std::getenv("RT_ASSETS");
  return std::string(dir && *dir ? dir : "./assets") + "/" + name;
}

void skybox_and_fisheye(int width, double aspect, config_scene* s) {  // main.cc:173-183
  auto skybox = std::make_shared<picture_texture>(std::make_shared<image>(asset("bathroom.exr").c_str()));
  auto world = std::make_shared<hittable_list>();
  world->push_back(std::make_shared<sphere>(vec3(0), 1, std::make_shared<dielectric>(solid_color::white, 1.0)));
  s->world = world;
  s->cam.initialize_fisheye(W(width, 600), A(aspect, 1), point3(1.1, 1.8, 1.1), point3(0, 0, 0), 1.0, 90, 500, 5);
  s->cam.background_ = skybox;
}

void skybox_and_motion_blur(int width, double aspect, config_scene* s) {  // main.cc:185-196
  auto skybox = std::make_shared<picture_texture>(std::make_shared<image>(asset("bathroom.exr").c_str()));
  auto world = std::make_shared<hittable_list>();
  auto earth_tex = std::make_shared<picture_texture>(std::make_shared<image>(asset("earthmap.jpg").c_str()));
  world->push_back(std::make_shared<sphere>(vec3(-0.2, 0, 0), vec3(0.2, 0, 0), 1, std::make_shared<lambertian>(earth_tex)));
  s->world = world;
  s->cam.initialize_perspective(W(width, 600), A(aspect, 1), point3(0, 0, 4), point3(0, 0, 0), 1.0, 70, 500, 5);
  s->cam.background_ = skybox;
}

// main.cc:447-485: the triangles sponza() builds from the loader's output primitives -- float
// positions only, uint16 indices only (other index types leave the primitive empty), and
// consecutive position triples when a primitive has no indices.
std::vector<std::array<vec3, 3>> gltf_triangles(std::vector<OutputPrimitives>& prims) {
  std::vector<std::array<vec3, 3>> out;
  for (auto& pr : prims) {
    std::vector<vec3> pos;
    std::vector<unsigned short> idx;
    if (pr.pos_type == DataType::kFloat) {
      for (size_t j = 0; j + 12 <= pr.positions.size(); j += 3 * sizeof(float)) {
        float x, y, z;
        std::memcpy(&x, &pr.positions[j], 4);
        std::memcpy(&y, &pr.positions[j + 4], 4);
        std::memcpy(&z, &pr.positions[j + 8], 4);
        pos.push_back(vec3(x, y, z));
      }
    }
    if (pr.use_indices && pr.indices_type == DataType::kUnsignedShort) {
      for (size_t j = 0; j + 2 <= pr.indices.size(); j += sizeof(unsigned short)) {
        unsigned short k;
        std::memcpy(&k, &pr.indices[j], 2);
        idx.push_back(k);
      }
    }
    auto at = [&](size_t k) -> const vec3& {
      if (k >= pos.size()) throw std::runtime_error("glTF: index past the positions");
      return pos[k];
    };
    if (pr.use_indices) {
      for (size_t i = 0; i + 2 < idx.size(); i += 3) out.push_back({at(idx[i]), at(idx[i + 1]), at(idx[i + 2])});
    } else {
      for (size_t i = 0; i + 2 < pos.size(); i += 3) out.push_back({pos[i], pos[i + 1], pos[i + 2]});
    }
  }
  return out;
}

// main.cc:439-498. The asset path is $RT_SPONZA_GLTF, else the reference's relative path.
// `lit` (sponza_lit, not a reference scene): the same triangles and light plus a second, unsampled
// diffuse_light quad facing down just under the stand-in's grid at y = 359 over the camera, so that C4's
// tree and kernel are compared on lit pixels (the stand-in's grids close the atrium under the
// reference's light at y = 1200, and its own frame is nearly black).
void sponza(int width, double aspect, config_scene* s, bool lit = false) {
  const char* env = std::getenv("RT_SPONZA_GLTF");
  gltf::GltfLoader model(env && *env ? env : "./assets/Sponza/glTF/Sponza.gltf");
  auto& prims = model.getOutputPrimitives();
  hittable_list world;
  for (const auto& t : gltf_triangles(prims))
    world.push_back(std::make_shared<triangle>(t[0], t[1], t[2],
                                               std::make_shared<lambertian>(std::make_shared<solid_color>(color(1.0f)))));
  auto light = std::make_shared<diffuse_light>(color(10));
  auto quad_light = std::make_shared<quad>(point3(0, 1200, 0), vec3(500, 0, 0), vec3(0, 0, 500), light);
  world.push_back(quad_light);
  if (lit)
    world.push_back(std::make_shared<quad>(point3(-400, 350, -250), vec3(800, 0, 0), vec3(0, 0, 500),
                                           std::make_shared<diffuse_light>(color(1))));
  s->world = std::make_shared<bvh_node>(world);
  s->light = quad_light;
  s->cam.initialize_perspective(W(width, 200), A(aspect, 1.0), point3(500, 320, 90), point3(0, 280, 0), 1, 45.0, 30,
                                5);
}

// main.cc:345-400: the Fox glTF (576 non-indexed float triangles) as glass triangles under a BVH,
// the bathroom.exr skybox (absent from the reference's checkout: the picture texture samples
// magenta, image.h:25,75-76), no importance-sampled light.
void glass_fox(int width, double aspect, config_scene* s) {
  gltf::GltfLoader model(asset("Fox/glTF/Fox.gltf").c_str());
  auto skybox = std::make_shared<picture_texture>(std::make_shared<image>(asset("bathroom.exr").c_str()));
  hittable_list world;
  for (const auto& t : gltf_triangles(model.getOutputPrimitives()))
    world.push_back(std::make_shared<triangle>(
        t[0], t[1], t[2], std::make_shared<dielectric>(std::make_shared<solid_color>(color(1.0f)), 1.5)));
  s->world = std::make_shared<bvh_node>(world);
  s->cam.initialize_perspective(W(width, 600), A(aspect, 1.0), point3(220, 220, 220), point3(0, 20, 0), 1, 45.0, 200,
                                5);
  s->cam.background_ = skybox;
}

}  // namespace

bool build_config_scene(const std::string& name, int width, double aspect, config_scene* out) {
  // The reference's main() builds one scene per process (main.cc:633-690), so every scene that
  // draws from rand() -- the perlin / value tables (noise.h:10-136), perlin_texture_ball's box
  // heights (main.cc:402-437), the RTOW spheres -- starts from glibc's default state, srand(1).
  // Reseeding here makes a scene independent of the scenes built before it in this process.
  std::srand(1);
  if (name == "cornell_box")
    cornell_box(width, aspect, out);
  else if (name == "cornell_box_with_volume")
    cornell_box_with_volume(width, aspect, out);
  else if (name == "rtow" || name == "rtow_motion")
    random_motion_ball(width, aspect, name == "rtow_motion", out);
  else if (name == "three_material_ball")
    three_material_ball(width, aspect, out);
  else if (name == "three_material_ball_with_defocus_blur")
    three_material_ball_with_defocus_blur(width, aspect, out);
  else if (name == "sponza")
    sponza(width, aspect, out);
  else if (name == "sponza_lit")
    sponza(width, aspect, out, true);
  else if (name == "glass_fox")
    glass_fox(width, aspect, out);
  else if (name == "skybox_and_fisheye")
    skybox_and_fisheye(width, aspect, out);
  else if (name == "skybox_and_motion_blur")
    skybox_and_motion_blur(width, aspect, out);
  else if (name == "perlin_texture_ball")
    perlin_texture_ball(width, aspect, out);
  else if (name == "test_perlin_noise")
    noise_quad(std::make_shared<perlin_texture>(1), 10, 10, width, aspect, out);
  else if (name == "test_value_noise")
    noise_quad(std::make_shared<value_texture>(40), 40, 20, width, aspect, out);
  else if (name == "test_worley_noise")
    noise_quad(std::make_shared<worley_texture>(), 40, 20, width, aspect, out);
  else if (name == "test_voronoi_noise")
    noise_quad(std::make_shared<voronoi_texture>(), 40, 20, width, aspect, out);
  else
    return false;
  return true;
}

// ---------------------------------------------------------------- C ABI for tests / bench
struct rtsc_handle {
  config_scene scene;
  scene_builder sb;
  rt_scene_desc desc{};
};

extern "C" {

// Builds a config scene and returns its descriptor and camera (owned by the handle).
void* rtsc_build(const char* name, int width, double aspect, rt_scene_desc* desc, rt_camera_desc* cam, int* spp,
                 int* max_depth, char* err, int errlen) {
  auto h = std::make_unique<rtsc_handle>();
  auto fail = [&](const std::string& m) -> void* {
    if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", m.c_str());
    return nullptr;
  };
  try {
    if (!name || !build_config_scene(name, width, aspect, &h->scene)) return fail("unknown scene");
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  try {
    int w = h->sb.add(*h->scene.world);
    int l = h->scene.light ? h->sb.add(*h->scene.light) : -1;
    int bg = h->scene.cam.background_ ? h->sb.add_texture(*h->scene.cam.background_) : -1;
    h->desc = h->sb.desc(w, l, bg);
  } catch (const unsupported_object& e) {
    return fail(e.what());
  }
  if (desc) *desc = h->desc;
  if (cam) *cam = h->scene.cam.describe();
  if (spp) *spp = h->scene.cam.samples_per_pixel_;
  if (max_depth) *max_depth = h->scene.cam.max_recur_depth_;
  return h.release();
}

void rtsc_free(void* h) { delete static_cast<rtsc_handle*>(h); }

// The triangles main.cc's sponza() builds from a glTF file (gltf_loader.h + main.cc:447-485):
// up to `cap` triangles as 9 doubles each into `xyz` (may be null); returns the total count,
// or -1 with the message in err.
long long rtsc_gltf_triangles(const char* path, double* xyz, long long cap, char* err, int errlen) {
  try {
    gltf::GltfLoader model(path ? path : "");
    auto tris = gltf_triangles(model.getOutputPrimitives());
    for (long long i = 0; i < (long long)tris.size() && i < cap && xyz; i++)
      for (int v = 0; v < 3; v++)
        for (int k = 0; k < 3; k++) xyz[9 * i + 3 * v + k] = tris[(size_t)i][v][k];
    return (long long)tris.size();
  } catch (const std::exception& e) {
    if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", e.what());
    return -1;
  }
}

// The full drop-in path: build the scene, camera::render(of, world, light) to a PPM file `repeat`
// times with the same camera (the last render's file is kept); with ndev > 0 the camera renders on
// `devices` (camera::devices_, the rt_multi_* tiling + RCCL gather).
int rtsc_render_ppm_repeat(const char* name, int width, double aspect, int spp, int max_depth, uint64_t seed,
                           int precision, const int32_t* devices, int ndev, int repeat, const char* path, char* err,
                           int errlen) {
  config_scene s;
  if (devices && ndev > 0) s.cam.devices_.assign(devices, devices + ndev);
  if (!name || !build_config_scene(name, width, aspect, &s)) {
    if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "unknown scene");
    return 1;
  }
  if (spp > 0) s.cam.samples_per_pixel_ = spp;
  if (max_depth > 0) s.cam.max_recur_depth_ = max_depth;
  s.cam.seed_ = seed;
  s.cam.precision_ = precision == RT_PREC_F64 ? RT_PREC_F64 : RT_PREC_F32;
  for (int k = 0; k < std::max(1, repeat); k++) {
    std::ofstream of(path);
    s.cam.render(of, *s.world, s.light);
    if (!s.cam.last_error_.empty()) {
      if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", s.cam.last_error_.c_str());
      return 2;
    }
  }
  return 0;
}

int rtsc_render_ppm_on(const char* name, int width, double aspect, int spp, int max_depth, uint64_t seed,
                       int precision, const int32_t* devices, int ndev, const char* path, char* err, int errlen) {
  return rtsc_render_ppm_repeat(name, width, aspect, spp, max_depth, seed, precision, devices, ndev, 1, path, err,
                                errlen);
}

int rtsc_render_ppm(const char* name, int width, double aspect, int spp, int max_depth, uint64_t seed, int precision,
                    const char* path, char* err, int errlen) {
  return rtsc_render_ppm_on(name, width, aspect, spp, max_depth, seed, precision, nullptr, 0, path, err, errlen);
}

}  // extern "C"
