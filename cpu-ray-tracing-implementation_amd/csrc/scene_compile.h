// scene_compile.h -- compile an rt_scene_desc (the reference's hittable DAG)
// into the device layout of rt_scene.h. Host-only C++; no HIP calls.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_scene.h"

namespace rtd {

struct CompiledScene {
  SceneHeader hdr{};
  std::vector<unsigned char> blob32;  // fp32 records, offsets in hdr
  std::vector<unsigned char> blob64;  // fp64 records, same offsets scaled (hdr64)
  SceneHeader hdr64{};
  int stack_need = 0;  // traversal stack entries a lane can need
  int bvh_depth = 0;
  int num_items = 0;
  int desc_quads = 0;  // quads of the descriptor (the flat program adds face copies)
  int flat_quads = 0, flat_boxes = 0;
};

// Returns RT_OK or an error with a message.
rt_status compile_scene(const rt_scene_desc* desc, CompiledScene* out, std::string* err);

}  // namespace rtd
