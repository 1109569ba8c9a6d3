// config_scenes.h -- the reference's main.cc scenes that BASELINE.json's configs
// use, written against the plugin surface exactly as a main.cc caller would.
#pragma once
#include <array>
#include <memory>
#include <string>

#include "../rt/bvh_node.h"
#include "../rt/camera.h"
#include "../rt/hittable_list.h"
#include "../rt/quad.h"
#include "../rt/sphere.h"
#include "../rt/triangle.h"
#include "../rt/volumne.h"

struct config_scene {
  std::shared_ptr<hittable> world;
  std::shared_ptr<hittable> light;  // importance-sampled light or null
  camera cam;
};

// name: cornell_box | cornell_box_with_volume | rtow | rtow_motion | three_material_ball |
// three_material_ball_with_defocus_blur | sponza ($RT_SPONZA_GLTF or ./assets/Sponza/glTF/Sponza.gltf) |
// glass_fox ($RT_ASSETS/Fox/glTF/Fox.gltf) | the skybox and noise scenes.
// width/aspect <= 0 keep the scene's own camera. Returns false for an unknown name; throws
// std::runtime_error when a scene's asset cannot be loaded.
bool build_config_scene(const std::string& name, int width, double aspect, config_scene* out);
