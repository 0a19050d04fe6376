/*
 * raingun_debug.h — test/diagnostic entry points of libraingun_hip.so.
 * Not part of the reference's interface; used by tests/ to exercise every
 * kernel path on every scene.
 */
#ifndef RAINGUN_DEBUG_H
#define RAINGUN_DEBUG_H

#include "raingun.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Force the kernel path used for this scene: -1 = automatic (by body count),
 * 0 = light path (2 waves/SIMD, batched shadow rays, exact f64 tests),
 * 1 = heavy path (4 waves/SIMD, one ray per lane, f32 pre-filter + exact f64). */
rg_status rg_debug_set_path(rg_scene *scene, int32_t path);

#ifdef __cplusplus
}
#endif

#endif /* RAINGUN_DEBUG_H */
