// rg_bvh.h — host-side builder of the 4-wide sphere BVH (rg_bvh.cpp).
//
// The BVH is an acceleration structure the reference does not have (SURVEY.md
// §8 f-4).  It only decides which spheres a ray tests exactly; the exact test,
// the closest-hit rule (smallest t, then smallest YAML index) and the ray
// counts are unchanged, so results are identical to the brute-force scan.
#pragma once
#include <cstdint>
#include <vector>

#include "rg_device.h"

struct RgBvhBuild {
    std::vector<RgBvhNode> nodes;   // nodes[0] is the root
    std::vector<uint32_t> order;    // BVH position -> index in the input sphere list
    float obound = 0.0f;            // origin bound |o_k| <= obound for which the boxes are conservative
    double margin = 0.0;            // box inflation (scene units)
    double extent = 0.0;            // S: max |coordinate| of any sphere bound
    double rbound = 0.0;            // S + 2 margin: region holding every inflated box
    int depth = 0;                  // levels of the 4-wide tree
    int leaves = 0;
    int max_stack = 0;              // worst-case traversal stack entries (3 per level)
    int lane_stack = 0;             // worst-case per-lane stack entries of the nearest-first walk:
                                    // max over root paths of sum (internal children - 1)
};

// Build over spheres (center xyz, radius) given as n x 4 doubles.  Returns false
// (and leaves `out` empty) when a BVH cannot be built conservatively: fewer
// than 2 spheres, non-finite values, or a stack bound above 64 entries.
bool rg_build_bvh(const double *spheres, int n, RgBvhBuild &out);

// Largest sphere count per leaf.
#ifndef RG_BVH_LEAF_SPHERES
#define RG_BVH_LEAF_SPHERES 4  // at most 8: a leaf link keeps (count - 1) in 3 bits
#endif
constexpr int RG_BVH_LEAF_MAX = RG_BVH_LEAF_SPHERES;
static_assert(RG_BVH_LEAF_MAX >= 1 && RG_BVH_LEAF_MAX <= 8, "leaf link format");
