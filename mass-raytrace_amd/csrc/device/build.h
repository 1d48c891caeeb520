// build.h — BvhNode::new (geom.rs:110-161) over many items on the GPU.
//
// The reference's tree is fixed by three things only: the item count of
// every node (the median split n/2 depends on n alone), the axis of every
// node (one fastrand::u8(0..3) draw per BvhNode::new call, in preorder) and
// the stable sort of each node's items by bbox.min[axis]. So the host
// enumerates the node ranges and draws the axes in preorder from the world's
// own scene stream (the same calls, in the same order, as World::bvh_new),
// and the device performs the sorts level by level — one stable radix sort
// of (range start, sort key) pairs per tree level — then reduces the node
// boxes bottom-up. The nodes come out numbered in preorder from the first
// free index, exactly as World::bvh_new numbers them, so the scene
// description is identical byte for byte.
#pragma once
#include <stdint.h>

#include <vector>

#include "../host/world.h"

namespace massrt {

struct DeviceBuildStats {
  double host_ms = 0, device_ms = 0;  // enumeration + axis draws; upload, sorts, boxes, download
  uint32_t levels = 0;
};

// Appends the tree over `items` to `nodes` (preorder numbering from
// nodes.size()); `rng` advances exactly as World::bvh_new's calls would.
// Throws Error on an empty list or a NaN sort key in a node of 3 or more
// items (2-item nodes compare once, as the host builder does; the reference's sort
// comparator is not a strict weak order over NaN).
void device_build_tree(int device, const std::vector<Item>& items, mrt::WyRand& rng, std::vector<mrt_node>& nodes,
                       BoundingBox& root_box, DeviceBuildStats* stats = nullptr);

}  // namespace massrt
