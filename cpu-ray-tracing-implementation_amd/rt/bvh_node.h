// bvh_node.h (reference: src/bvh_node.h:11-65). Constructed from a list like
// the reference; the device builds its own SAH BVH over the list's objects
// (the closest hit does not depend on the tree).
#pragma once
#include "hittable_list.h"

class bvh_node : public hittable_list {
 public:
  bvh_node(hittable_list list) { objects = std::move(list.objects); }
  int flatten(scene_builder& sb) const override { return flatten_as(sb, RT_OBJ_BVH); }
};
