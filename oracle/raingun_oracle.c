/*
 * raingun_oracle.c — CPU restatement of raingun's render path.
 *
 *   *** TEST INFRASTRUCTURE ONLY. ***  This file is the parity CHECKER.
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 *   load liboracle.so.  The product path (libraingun_hip.so) never links,
 *   loads or falls back to it.
 *
 * The reference (Mange/raingun) is Rust and cannot be built here (no cargo /
 * rustc in the image, crates.io unreachable), so this is a line-by-line C
 * restatement of the reference's arithmetic, written from the cited Rust and
 * pinned by the reference's own golden renders examples/test{1,2,3}.png
 * (tests/golden/, checked by tests/test_oracle_golden.py).
 *
 * Numerics rules, followed everywhere below:
 *   - geometry is f64 (lib.rs:29-30), colour is f32 (color.rs:7-11);
 *   - built with -ffp-contract=off and no fast-math: every multiply and add is
 *     rounded separately, in the reference's evaluation order;
 *   - cgmath 0.13 (Cargo.lock:97-98, not in the container) vector ops are
 *     restated as: dot = (x*x' + y*y') + z*z'; magnitude2 = dot(v,v);
 *     magnitude = sqrt(magnitude2); normalize(v) = v * (1 / magnitude(v));
 *     cross = (y*z'-z*y', z*x'-x*z', x*y'-y*x').  Pinned by test2.png (exact);
 *   - Rust `as` casts: f64->f32 round-to-nearest; f32->i32 / f32->u8 are
 *     truncating and saturating, NaN -> 0 (rs_f32_to_i32 / rs_f32_to_u8);
 *   - f32::max/min and f64::max ignore a NaN operand (fmaxf/fminf/fmax);
 *   - transcendental calls (tan, atan2, acos) go to the platform libm, as
 *     Rust's std does on Linux.
 *
 * Paths below are relative to /root/reference.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/raingun.h"

#define SHADOW_BIAS 1e-13            /* lib.rs:11 */
#define PI_F32 3.14159265358979323846f /* std::f32::consts::PI (rendering.rs:15, bodies.rs:7, lights.rs:5) */

/* ------------------------------------------------------------ vector (cgmath) */
typedef struct { double x, y, z; } v3;
typedef struct { float r, g, b; } col;

static inline v3 v3_make(double x, double y, double z) { v3 v = {x, y, z}; return v; }
static inline v3 v3_add(v3 a, v3 b) { return v3_make(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 v3_sub(v3 a, v3 b) { return v3_make(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 v3_scale(v3 a, double s) { return v3_make(a.x * s, a.y * s, a.z * s); }
static inline v3 v3_neg(v3 a) { return v3_make(-a.x, -a.y, -a.z); }
static inline double v3_dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline double v3_mag2(v3 a) { return v3_dot(a, a); }
static inline double v3_mag(v3 a) { return sqrt(v3_mag2(a)); }
static inline v3 v3_normalize(v3 a) { return v3_scale(a, 1.0 / v3_mag(a)); }
static inline v3 v3_cross(v3 a, v3 b) {
    return v3_make(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

/* ------------------------------------------------------------ colour (color.rs) */
static inline col col_make(float r, float g, float b) { col c = {r, g, b}; return c; }
static inline col col_add(col a, col b) { return col_make(a.r + b.r, a.g + b.g, a.b + b.b); } /* color.rs:62-70 */
static inline col col_mul(col a, col b) { return col_make(a.r * b.r, a.g * b.g, a.b * b.b); } /* color.rs:72-80 */
static inline col col_scale(col a, float s) { return col_make(a.r * s, a.g * s, a.b * s); }  /* color.rs:98-104 */
static inline col col_clamp(col a) {                                                          /* color.rs:39-43 */
    return col_make(fmaxf(fminf(a.r, 1.0f), 0.0f), fmaxf(fminf(a.g, 1.0f), 0.0f),
                    fmaxf(fminf(a.b, 1.0f), 0.0f));
}

/* Rust `f32 as u8` (saturating, NaN -> 0). */
uint8_t rgo_f32_to_u8(float v) {
    if (!(v > 0.0f)) return 0; /* negative, -0, NaN */
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}
/* Rust `f32 as i32` (saturating, NaN -> 0). */
int32_t rgo_f32_to_i32(float v) {
    if (v != v) return 0;
    if (v >= 2147483648.0f) return INT32_MAX;
    if (v < -2147483648.0f) return INT32_MIN;
    return (int32_t)v;
}

/* ------------------------------------------------------------ ray (ray.rs) */
typedef struct {
    v3 o, d, inv;
    int sign[3];
} ray_t;

static inline ray_t ray_new(v3 o, v3 d) { /* ray.rs:23-35 */
    ray_t r;
    r.o = o;
    r.d = d;
    r.inv = v3_make(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
    r.sign[0] = r.inv.x < 0.0 ? 1 : 0;
    r.sign[1] = r.inv.y < 0.0 ? 1 : 0;
    r.sign[2] = r.inv.z < 0.0 ? 1 : 0;
    return r;
}

/* ------------------------------------------------------------ scene access */
typedef struct {
    const rg_scene_desc *s;
    double fov_adjustment;  /* ray.rs:45, per frame */
} ctx_t;

static inline v3 p3(const double *p) { return v3_make(p[0], p[1], p[2]); }

/* ------------------------------------------------------------ bodies (bodies.rs) */
/* Returns 1 and writes *t on a hit (Option<f64>::Some). */
static int intersect(const rg_body *b, const ray_t *ray, double *t) {
    switch (b->kind) {
    case RG_BODY_SPHERE: { /* bodies.rs:76-120 */
        v3 hyp = v3_sub(p3(b->p), ray->o);
        double adj = v3_dot(hyp, ray->d);
        double opp2 = v3_dot(hyp, hyp) - (adj * adj);
        double r2 = b->p[3] * b->p[3];
        if (opp2 > r2) return 0;
        double thick = sqrt(r2 - opp2);
        double d0 = adj - thick, d1 = adj + thick;
        if (d0 < 0.0 && d1 < 0.0) return 0;
        if (d0 < 0.0) { *t = d1; return 1; }
        if (d1 < 0.0) { *t = d0; return 1; }
        *t = fmin(d0, d1); /* f64::min */
        return 1;
    }
    case RG_BODY_PLANE: { /* bodies.rs:136-149 */
        v3 n = p3(b->p + 3);
        double den = v3_dot(n, ray->d);
        if (den > 1e-6) {
            v3 v = v3_sub(p3(b->p), ray->o);
            double dist = v3_dot(v, n) / den;
            if (dist >= 0.0) { *t = dist; return 1; }
        }
        return 0;
    }
    case RG_BODY_DISK: { /* bodies.rs:173-192 */
        v3 n = p3(b->p + 3);
        double den = v3_dot(n, ray->d);
        if (den > 1e-6) {
            v3 v = v3_sub(p3(b->p), ray->o);
            double dist = v3_dot(v, n) / den;
            if (dist >= 0.0) {
                v3 hit = v3_add(ray->o, v3_scale(ray->d, dist));
                v3 w = v3_sub(hit, p3(b->p));
                double d2 = v3_dot(w, w);
                if (sqrt(d2) < b->p[6]) { *t = dist; return 1; }
            }
        }
        return 0;
    }
    case RG_BODY_AABB: { /* bodies.rs:242-282 */
        const double *lo = b->p, *hi = b->p + 3;
        const double *bx[2] = {lo, hi};
        double tmin = (bx[ray->sign[0]][0] - ray->o.x) * ray->inv.x;
        double tmax = (bx[1 - ray->sign[0]][0] - ray->o.x) * ray->inv.x;
        double tymin = (bx[ray->sign[1]][1] - ray->o.y) * ray->inv.y;
        double tymax = (bx[1 - ray->sign[1]][1] - ray->o.y) * ray->inv.y;
        if (tmin > tymax || tymin > tmax) return 0;
        if (tymin > tmin) tmin = tymin;
        if (tymax < tmax) tmax = tymax;
        double tzmin = (bx[ray->sign[2]][2] - ray->o.z) * ray->inv.z;
        double tzmax = (bx[1 - ray->sign[2]][2] - ray->o.z) * ray->inv.z;
        if (tmin > tzmax || tzmin > tmax) return 0;
        if (tzmin > tmin) tmin = tzmin;
        if (tzmax < tmax) tmax = tzmax;
        if (tmin >= 0.0) { *t = tmin; return 1; }
        if (tmax >= 0.0) { *t = tmax; return 1; }
        return 0;
    }
    }
    return 0;
}

static inline int is_close(double a, double b) { return fabs(a - b) < 1e-8; } /* bodies.rs:9-11 */

/* bodies.rs:122-124, 151-153, 194-196, 284-328.  Returns 0 on the AABB assert. */
static int surface_normal(const rg_body *b, v3 hit, v3 *n) {
    switch (b->kind) {
    case RG_BODY_SPHERE: *n = v3_normalize(v3_sub(hit, p3(b->p))); return 1;
    case RG_BODY_PLANE:
    case RG_BODY_DISK: *n = v3_neg(p3(b->p + 3)); return 1;
    case RG_BODY_AABB: {
        const double *lo = b->p, *hi = b->p + 3;
        if (is_close(hit.x, lo[0])) *n = v3_make(-1.0, 0.0, 0.0);
        else if (is_close(hit.x, hi[0])) *n = v3_make(1.0, 0.0, 0.0);
        else if (is_close(hit.y, lo[1])) *n = v3_make(0.0, -1.0, 0.0);
        else if (is_close(hit.y, hi[1])) *n = v3_make(0.0, 1.0, 0.0);
        else if (is_close(hit.z, lo[2])) *n = v3_make(0.0, 0.0, -1.0);
        else if (is_close(hit.z, hi[2])) *n = v3_make(0.0, 0.0, 1.0);
        else return 0; /* assert!(false, "Could not determine normal of point!") */
        return 1;
    }
    }
    return 0;
}

typedef struct { float x, y; } tc_t;

/* bodies.rs:126-132, 155-169, 198-212, 330-333 */
static tc_t texture_coords(const rg_body *b, v3 hit) {
    tc_t tc = {0.0f, 0.0f};
    switch (b->kind) {
    case RG_BODY_SPHERE: {
        v3 hv = v3_sub(hit, p3(b->p));
        tc.x = (1.0f + ((float)atan2(hv.z, hv.x)) / PI_F32) * 0.5f;
        tc.y = ((float)acos(hv.y / b->p[3])) / PI_F32;
        break;
    }
    case RG_BODY_PLANE:
    case RG_BODY_DISK: {
        v3 n = p3(b->p + 3);
        v3 xa = v3_cross(n, v3_make(0.0, 0.0, 1.0));
        if (v3_mag2(xa) == 0.0) xa = v3_cross(n, v3_make(0.0, 1.0, 0.0));
        v3 ya = v3_cross(n, xa);
        v3 hv = v3_sub(hit, p3(b->p));
        tc.x = (float)v3_dot(hv, xa);
        tc.y = (float)v3_dot(hv, ya);
        break;
    }
    default: break; /* AABB: (0,0) */
    }
    return tc;
}

/* ------------------------------------------------------------ material.rs */
uint32_t rgo_wrap(float val, uint32_t max) { /* material.rs:70-79 */
    int32_t smax = (int32_t)max;
    float fc = val * (float)max;
    int32_t w = rgo_f32_to_i32(fc) % smax;
    return w < 0 ? (uint32_t)(w + smax) : (uint32_t)w;
}

static col material_color(const ctx_t *c, const rg_material *m, tc_t tc) { /* material.rs:62-68, 82-89 */
    if (m->coloration == RG_COLORATION_COLOR) return col_make(m->color[0], m->color[1], m->color[2]);
    const rg_texture *t = &c->s->textures[m->texture];
    uint32_t x = rgo_wrap(tc.x + m->x_offset, t->width);
    uint32_t y = rgo_wrap(tc.y + m->y_offset, t->height);
    const uint8_t *px = t->rgba + ((size_t)y * t->width + x) * 4;
    return col_make((float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f); /* color.rs:26-30 */
}

/* ------------------------------------------------------------ lights.rs */
static inline col light_color(const rg_light *l) { return col_make(l->color[0], l->color[1], l->color[2]); }
static float light_intensity(const rg_light *l, v3 hit) { /* lights.rs:36-44 */
    if (l->kind == RG_LIGHT_DIRECTIONAL) return l->intensity;
    float r2 = (float)v3_mag2(v3_sub(p3(l->v), hit));
    return l->intensity / (4.0f * PI_F32 * r2);
}
static v3 light_direction_from(const rg_light *l, v3 p) { /* lights.rs:46-51 */
    if (l->kind == RG_LIGHT_DIRECTIONAL) return v3_normalize(v3_neg(p3(l->v)));
    return v3_normalize(v3_sub(p3(l->v), p));
}
static double light_distance(const rg_light *l, v3 p) { /* lights.rs:53-58 */
    if (l->kind == RG_LIGHT_DIRECTIONAL) return INFINITY;
    return v3_mag(v3_sub(p3(l->v), p));
}

/* ------------------------------------------------------------ render state */
typedef struct {
    rg_ray_counts counts;
    int32_t err; /* first error code hit by this pixel */
} pix_t;

/* Scene::trace (scene.rs:34-39): closest hit in list order; min_by keeps the
 * first minimum and panics (partial_cmp().unwrap()) when it compares a NaN. */
static int trace(const ctx_t *c, const ray_t *ray, double *dist, int32_t *body, pix_t *px) {
    int have = 0;
    double best = 0.0;
    int32_t bi = -1;
    for (uint32_t i = 0; i < c->s->n_bodies; ++i) {
        double t;
        if (!intersect(&c->s->bodies[i], ray, &t)) continue;
        if (!have) { have = 1; best = t; bi = (int32_t)i; continue; }
        if (best != best || t != t) { if (px && !px->err) px->err = RG_ERR_NAN_DISTANCE; continue; }
        if (best > t) { best = t; bi = (int32_t)i; }
    }
    if (have) { *dist = best; *body = bi; }
    return have;
}

static col cast_ray(const ctx_t *c, const ray_t *ray, uint32_t depth, pix_t *px);

/* rendering.rs:132-172 */
static col shade_diffuse(const ctx_t *c, const rg_body *b, v3 hit, v3 n, pix_t *px) {
    tc_t tc = texture_coords(b, hit);
    col body_color = material_color(c, &b->material, tc);
    col fin = col_make(0.0f, 0.0f, 0.0f);
    for (uint32_t li = 0; li < c->s->n_lights; ++li) {
        const rg_light *l = &c->s->lights[li];
        v3 dl = light_direction_from(l, hit);
        ray_t sr = ray_new(v3_add(hit, v3_scale(n, SHADOW_BIAS)), dl);
        double sd;
        int32_t sb;
        px->counts.shadow++;
        int hit_any = trace(c, &sr, &sd, &sb, px);
        int in_light = !hit_any || sd > light_distance(l, hit);
        float li_int = in_light ? light_intensity(l, hit) : 0.0f;
        float power = fmaxf((float)v3_dot(n, dl), 0.0f) * li_int;
        float reflected = b->material.albedo / PI_F32;
        col lc = col_scale(col_scale(light_color(l), power), reflected);
        fin = col_add(fin, col_mul(body_color, lc));
    }
    return col_clamp(fin);
}

/* rendering.rs:174-200 — including the `cos_i = cos_t.abs()` line as written (:194). */
double rgo_fresnel(double ix, double iy, double iz, double nx, double ny, double nz, float index) {
    v3 inc = v3_make(ix, iy, iz), nrm = v3_make(nx, ny, nz);
    double i_dot_n = v3_dot(inc, nrm);
    double eta_i, eta_t;
    if (i_dot_n > 0.0) { eta_i = (double)index; eta_t = 1.0; }
    else { eta_i = 1.0; eta_t = (double)index; }
    double sin_t = eta_i / eta_t * sqrt(fmax(1.0 - i_dot_n * i_dot_n, 0.0));
    if (sin_t > 1.0) return 1.0;
    double cos_t = sqrt(fmax(1.0 - sin_t * sin_t, 0.0));
    double cos_i = fabs(cos_t);
    double r_s = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    double r_p = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (r_s * r_s + r_p * r_p) / 2.0;
}

static ray_t create_reflection(v3 n, v3 inc, v3 hit) { /* ray.rs:56-60 */
    v3 o = v3_add(hit, v3_scale(n, SHADOW_BIAS));
    v3 d = v3_sub(inc, v3_scale(n, 2.0 * v3_dot(inc, n)));
    return ray_new(o, d);
}

/* ray.rs:62-94.  Returns 0 for None. */
static int create_transmission(v3 n, v3 inc, v3 hit, double bias, float index, ray_t *out) {
    v3 ref_n = n;
    double eta_t = (double)index, eta_i = 1.0;
    double i_dot_n = v3_dot(inc, n);
    if (i_dot_n < 0.0) i_dot_n = -i_dot_n;
    else { ref_n = v3_neg(n); eta_t = 1.0; eta_i = (double)index; }
    double eta = eta_i / eta_t;
    double k = 1.0 - (eta * eta) * (1.0 - i_dot_n * i_dot_n);
    if (k < 0.0) return 0;
    v3 o = v3_add(hit, v3_scale(ref_n, -bias));
    v3 d = v3_sub(v3_scale(v3_add(inc, v3_scale(ref_n, i_dot_n)), eta), v3_scale(ref_n, sqrt(k)));
    *out = ray_new(o, d);
    return 1;
}

/* rendering.rs:80-120 */
static col get_color(const ctx_t *c, const ray_t *ray, double dist, int32_t bi, uint32_t depth, pix_t *px) {
    const rg_body *b = &c->s->bodies[bi];
    v3 hit = v3_add(ray->o, v3_scale(ray->d, dist));
    v3 n;
    if (!surface_normal(b, hit, &n)) {
        if (!px->err) px->err = RG_ERR_AABB_NORMAL;
        n = v3_make(1.0, 0.0, 0.0);
    }
    const rg_material *m = &b->material;
    switch (m->surface) {
    case RG_SURFACE_DIFFUSE: return shade_diffuse(c, b, hit, n, px);
    case RG_SURFACE_REFLECTING: {
        col dc = shade_diffuse(c, b, hit, n, px);
        ray_t rr = create_reflection(n, ray->d, hit);
        float r = m->reflectivity;
        return col_add(col_scale(dc, 1.0f - r), col_scale(cast_ray(c, &rr, depth + 1, px), r));
    }
    default: { /* Refractive */
        col refr;
        float kr = (float)rgo_fresnel(ray->d.x, ray->d.y, ray->d.z, n.x, n.y, n.z, m->index);
        col surf = material_color(c, m, texture_coords(b, hit));
        if (kr < 1.0f) {
            ray_t tr;
            if (!create_transmission(n, ray->d, hit, SHADOW_BIAS, m->index, &tr)) {
                if (!px->err) px->err = RG_ERR_TRANSMISSION;
                refr = col_make(c->s->default_color[0], c->s->default_color[1], c->s->default_color[2]);
            } else {
                refr = cast_ray(c, &tr, depth + 1, px);
            }
        } else {
            refr = col_make(c->s->default_color[0], c->s->default_color[1], c->s->default_color[2]);
        }
        ray_t rr = create_reflection(n, ray->d, hit);
        col refl = cast_ray(c, &rr, depth + 1, px);
        col out = col_add(col_scale(refl, kr), col_scale(refr, 1.0f - kr));
        return col_mul(col_scale(out, m->transparency), surf);
    }
    }
}

/* rendering.rs:122-130 */
static col cast_ray(const ctx_t *c, const ray_t *ray, uint32_t depth, pix_t *px) {
    col def = col_make(c->s->default_color[0], c->s->default_color[1], c->s->default_color[2]);
    if (depth >= c->s->max_recursion_depth) return def;
    double d;
    int32_t bi;
    px->counts.secondary++;
    if (!trace(c, ray, &d, &bi, px)) return def;
    return get_color(c, ray, d, bi, depth, px);
}

/* ray.rs:37-54 */
static ray_t create_prime(const ctx_t *c, uint32_t x, uint32_t y, uint32_t w, uint32_t h) {
    double aspect = (double)w / (double)h;
    double sx = ((((double)x + 0.5) / (double)w) * 2.0 - 1.0) * aspect * c->fov_adjustment;
    double sy = (1.0 - (((double)y + 0.5) / (double)h) * 2.0) * c->fov_adjustment;
    return ray_new(v3_make(0.0, 0.0, 0.0), v3_normalize(v3_make(sx, sy, -1.0)));
}

/* rendering.rs:71-78 */
static col render_pixel(const ctx_t *c, uint32_t x, uint32_t y, uint32_t w, uint32_t h, pix_t *px) {
    ray_t r = create_prime(c, x, y, w, h);
    double d;
    int32_t bi;
    px->counts.primary++;
    if (trace(c, &r, &d, &bi, px)) return get_color(c, &r, d, bi, 0, px);
    return col_make(c->s->default_color[0], c->s->default_color[1], c->s->default_color[2]);
}

/* f64::to_radians as in the 2017 std: self * (PI / 180.0).  Then tan via libm (ray.rs:45). */
double rgo_fov_adjustment(double fov) { return tan(fov * (3.14159265358979323846 / 180.0) / 2.0); }

/* ------------------------------------------------------------ frame driver */
typedef struct {
    ctx_t ctx;
    uint32_t w, h, tile_rows, stride, offset, n_out_rows;
    uint8_t *rgba;
    float *rgb;
    volatile uint32_t next_row; /* output row counter (dynamic schedule, like Rayon's work stealing) */
    pthread_mutex_t mu;
    rg_ray_counts counts;
    int64_t err_pixel;
    int32_t err_code;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    rg_ray_counts local = {0, 0, 0};
    int64_t err_pixel = -1;
    int32_t err_code = 0;
    for (;;) {
        uint32_t orow = __atomic_fetch_add(&j->next_row, 1, __ATOMIC_RELAXED);
        if (orow >= j->n_out_rows) break;
        uint32_t tile_local = orow / j->tile_rows, r_in_tile = orow % j->tile_rows;
        uint64_t tile = (uint64_t)tile_local * j->stride + j->offset;
        uint64_t y64 = tile * j->tile_rows + r_in_tile;
        uint8_t *orgba = j->rgba + (size_t)orow * j->w * 4;
        float *orgb = j->rgb ? j->rgb + (size_t)orow * j->w * 3 : NULL;
        if (y64 >= j->h) { /* padding rows of a partial last tile */
            memset(orgba, 0, (size_t)j->w * 4);
            if (orgb) memset(orgb, 0, (size_t)j->w * 12);
            continue;
        }
        uint32_t y = (uint32_t)y64;
        for (uint32_t x = 0; x < j->w; ++x) {
            pix_t px;
            memset(&px, 0, sizeof px);
            col cc = render_pixel(&j->ctx, x, y, j->w, j->h, &px);
            local.primary += px.counts.primary;
            local.shadow += px.counts.shadow;
            local.secondary += px.counts.secondary;
            int64_t lin = (int64_t)y * j->w + x;
            if (px.err && (err_pixel < 0 || lin < err_pixel)) { err_pixel = lin; err_code = px.err; }
            orgba[4 * x + 0] = rgo_f32_to_u8(cc.r * 255.0f); /* color.rs:32-37 */
            orgba[4 * x + 1] = rgo_f32_to_u8(cc.g * 255.0f);
            orgba[4 * x + 2] = rgo_f32_to_u8(cc.b * 255.0f);
            orgba[4 * x + 3] = 255;
            if (orgb) { orgb[3 * x] = cc.r; orgb[3 * x + 1] = cc.g; orgb[3 * x + 2] = cc.b; }
        }
    }
    pthread_mutex_lock(&j->mu);
    j->counts.primary += local.primary;
    j->counts.shadow += local.shadow;
    j->counts.secondary += local.secondary;
    if (err_pixel >= 0 && (j->err_pixel < 0 || err_pixel < j->err_pixel)) {
        j->err_pixel = err_pixel;
        j->err_code = err_code;
    }
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

uint32_t rgo_tiling_rows(uint32_t h, const rg_tiling *t) {
    uint32_t tiles = (h + t->tile_rows - 1) / t->tile_rows;
    uint32_t mine = tiles > t->tile_offset ? (tiles - t->tile_offset + t->tile_stride - 1) / t->tile_stride : 0;
    return mine * t->tile_rows;
}

/* Render the tiles selected by `tiling` (rendering.rs:24-38 restated; same
 * packing as rg_render_tiles).  Returns RG_OK or the first error code by
 * pixel index; *error_pixel receives that pixel or -1. */
int32_t rgo_render(const rg_scene_desc *s, uint32_t w, uint32_t h, const rg_tiling *tiling,
                   uint8_t *rgba, float *rgb, rg_ray_counts *counts, int32_t nthreads,
                   int64_t *error_pixel) {
    if (!s || !rgba || w == 0 || h == 0) return RG_ERR_INVALID_ARGUMENT;
    if (w < h) return RG_ERR_PORTRAIT; /* ray.rs:42 */
    rg_tiling whole = {h, 1, 0};
    if (!tiling) tiling = &whole;
    if (tiling->tile_rows == 0 || tiling->tile_stride == 0 || tiling->tile_offset >= tiling->tile_stride)
        return RG_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < s->n_bodies; ++i) {
        const rg_material *m = &s->bodies[i].material;
        if (m->coloration == RG_COLORATION_TEXTURE &&
            (m->texture < 0 || (uint32_t)m->texture >= s->n_textures || !s->textures[m->texture].rgba ||
             s->textures[m->texture].width == 0 || s->textures[m->texture].height == 0))
            return RG_ERR_TEXTURE;
    }
    job_t j;
    memset(&j, 0, sizeof j);
    j.ctx.s = s;
    j.ctx.fov_adjustment = rgo_fov_adjustment(s->fov);
    j.w = w; j.h = h;
    j.tile_rows = tiling->tile_rows; j.stride = tiling->tile_stride; j.offset = tiling->tile_offset;
    j.n_out_rows = rgo_tiling_rows(h, tiling);
    j.rgba = rgba; j.rgb = rgb;
    j.err_pixel = -1;
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    /* every worker on a thread of its own with a large stack: the restatement
     * recurses like the reference (rendering.rs:122-130), one call chain per
     * ray depth, and recursion depths of 10^4 and more need ~0.5 KB per level */
    pthread_t th[256];
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, (size_t)512 << 20);
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], &attr, worker, &j);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    pthread_attr_destroy(&attr);
    pthread_mutex_destroy(&j.mu);
    if (counts) *counts = j.counts;
    if (error_pixel) *error_pixel = j.err_pixel;
    return j.err_pixel >= 0 ? j.err_code : RG_OK;
}

/* Scene::trace for a batch of rays {o.xyz, d.xyz}. */
int32_t rgo_trace(const rg_scene_desc *s, const double *rays, uint32_t n, double *dist, int32_t *body) {
    ctx_t c = {s, 0.0};
    int32_t st = RG_OK;
    for (uint32_t i = 0; i < n; ++i) {
        const double *r = rays + 6 * (size_t)i;
        ray_t ray = ray_new(v3_make(r[0], r[1], r[2]), v3_make(r[3], r[4], r[5]));
        pix_t px;
        memset(&px, 0, sizeof px);
        double d = 0.0;
        int32_t b = -1;
        if (!trace(&c, &ray, &d, &b, &px)) { d = 0.0; b = -1; }
        dist[i] = d;
        body[i] = b;
        if (px.err && st == RG_OK) st = px.err;
    }
    return st;
}
