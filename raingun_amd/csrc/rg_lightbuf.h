// rg_lightbuf.h — host-side builder of the shadow-ray light buffers
// (rg_lightbuf.cpp; cell lookup and descriptor: rg_lightbuf_ray.h).
//
// Like the BVH (rg_bvh.h) this is an acceleration structure the reference does
// not have: it only decides which spheres a shadow ray tests with the exact
// reference test, and it never leaves out a sphere the exact test could accept,
// so every shadow answer is the brute-force scan's.
#pragma once
#include <cstdint>
#include <vector>

#include "rg_lightbuf_ray.h"

struct RgLightBufBuild {
    RgLightBufDev dev{};              // cell_off / always0/1 relative to this light's arrays
    std::vector<uint32_t> start;      // cells + 1 words: cell c's spheres are ent[start[c], start[c + 1])
    std::vector<uint32_t> ent;        // sphere positions (in the order of the `spheres` table given)
    double mean_candidates = 0.0;     // average list length over the non-empty cells (diagnostic)
    uint32_t max_candidates = 0;
};

// One light's buffer over spheres (centre xyz, radius: n x 4 doubles, the
// kernel's sphere-table order).  kind: RG_LIGHT_DIRECTIONAL with dn =
// normalize(-direction) as the kernel uses it, or RG_LIGHT_SPHERICAL with the
// light position pos.  extent S and obound O are the BVH's (rg_bvh.h): the
// margins assume |o_k| <= O and spheres within [-S, S]^3.  Returns false (no
// buffer: the light's shadow rays keep the BVH) for non-finite input, a light
// the buffer would serve badly (lists longer than RG_LB_MAX_MEAN on average),
// or more than RG_LB_MAX_ENTRIES entries.
bool rg_build_lightbuf(const double *spheres, int n, int kind, const double dn[3], const double pos[3], double extent,
                       double obound, RgLightBufBuild &out);

#ifndef RG_LB_MAX_MEAN
#define RG_LB_MAX_MEAN 24.0  // mean spheres per non-empty cell above which a light keeps the BVH
#endif
#ifndef RG_LB_MAX_ENTRIES
#define RG_LB_MAX_ENTRIES (1u << 24)
#endif
#ifndef RG_LB_TOTAL_WORDS
#define RG_LB_TOTAL_WORDS (1u << 25)  // every buffer of a scene together (entries + cell starts): 128 MiB
#endif
#ifndef RG_LB_CUBE_G
#define RG_LB_CUBE_G 128  // spherical lights: cells per cube-face edge
#endif
#ifndef RG_LB_DIR_CELL
#define RG_LB_DIR_CELL 0.5  // directional lights: cell edge in units of the mean sphere radius
#endif
#ifndef RG_LB_DIR_MAX_G
#define RG_LB_DIR_MAX_G 1024  // directional lights: at most this many cells per grid axis
#endif
