/*
 * raingun_host.h — C ABI of the native host layer (libraingun_host.so):
 * scene loading, texture decoding and PNG output, i.e. everything the
 * reference does on the CPU around the render call.
 *
 *   reference                                          here
 *   serde_yaml::from_reader::<Scene>  (main.rs:116-118)  rgh_scene_load_file / _string
 *   Texture::image via image::open    (material.rs:34-47) rgh_image_decode[_file]
 *   ImageBuffer::save (PNG)           (render.rs:58)      rgh_png_write / rgh_png_encode
 *   the `raingun` binary              (main.rs:98-132)    raingun_amd/bin/raingun (raingun_cli.cpp)
 *
 * The loaded scene is handed to the renderer as an rg_scene_desc
 * (include/raingun.h) — the two libraries meet only through that POD struct.
 * Plain C: pointers, sizes, POD structs.  Paths are relative to /root/reference.
 */
#ifndef RAINGUN_HOST_H
#define RAINGUN_HOST_H

#include "raingun.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RGH_ABI_VERSION 1

typedef enum rgh_status {
    RGH_OK = 0,
    RGH_ERR_INVALID_ARGUMENT = -1,
    RGH_ERR_OUT_OF_MEMORY = -11,
    RGH_ERR_IO = -20,          /* File::open / image::open I/O failure (main.rs:115) */
    RGH_ERR_YAML = -21,        /* YAML syntax: "Could not load YAML" (main.rs:117) */
    RGH_ERR_SCHEMA = -22,      /* YAML does not deserialise into Scene (serde error) */
    RGH_ERR_IMAGE = -23        /* "Could not load texture file ..." (material.rs:43-46) */
} rgh_status;

/* JPEG rounding to reproduce.  RGH_JPEG_REFERENCE is the reference's decoder
 * (jpeg-decoder 0.1.11, Cargo.lock:400-406: stb_image-style integer IDCT and
 * upsampling, f32 YCbCr->RGB) and is what scene loading uses; with it the
 * CPU restatement reproduces examples/test{1,3}.png byte for byte.
 * RGH_JPEG_LIBJPEG is IJG libjpeg's ISLOW/fancy-upsampling output (PIL's). */
enum rgh_jpeg_flavor { RGH_JPEG_REFERENCE = 0, RGH_JPEG_LIBJPEG = 1 };

typedef struct rgh_scene rgh_scene;  /* a loaded scene: owns its desc arrays and textures */

int32_t rgh_abi_version(void);

/* Message for the last failing rgh_* call on this thread ("" if none). */
const char *rgh_last_error(void);

/* Load a scene the way `serde_yaml::from_reader::<Scene>` does (scene.rs:11-31:
 * camelCase keys, deny_unknown_fields, defaults fov 90 / black / depth 10;
 * externally tagged Body/Light/Coloration/Surface enums; Point3/Vector3 as
 * [x, y, z] or {x, y, z}; f32 fields rounded to f32) and decode every texture.
 * Texture paths resolve against `texture_root` (NULL: the working directory,
 * as image::open does).  Textures referenced by the same path string share
 * one rg_texture. */
int32_t rgh_scene_load_file(const char *path, const char *texture_root, rgh_scene **out);
int32_t rgh_scene_load_string(const char *yaml, size_t len, const char *texture_root, rgh_scene **out);

/* The flat description to pass to rg_scene_create; valid until rgh_scene_free. */
const rg_scene_desc *rgh_scene_desc(const rgh_scene *scene);

/* The YAML `image:` string of texture `index` (NULL if out of range). */
const char *rgh_scene_texture_path(const rgh_scene *scene, uint32_t index);

/* main.rs:119-123: lower the recursion cap to `limit` if it is smaller. */
void rgh_scene_clamp_depth(rgh_scene *scene, uint32_t limit);

void rgh_scene_free(rgh_scene *scene);

/* Decode a JPEG or PNG into malloc'd RGBA8 (free with rgh_free). */
int32_t rgh_image_decode(const uint8_t *data, size_t size, int32_t jpeg_flavor, uint32_t *width,
                         uint32_t *height, uint8_t **rgba);
int32_t rgh_image_decode_file(const char *path, int32_t jpeg_flavor, uint32_t *width, uint32_t *height,
                              uint8_t **rgba);

/* 8-bit RGBA PNG (render.rs:58).  rgh_png_encode returns a malloc'd buffer. */
int32_t rgh_png_encode(const uint8_t *rgba, uint32_t width, uint32_t height, uint8_t **png, size_t *size);
int32_t rgh_png_write(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height);

void rgh_free(void *p);

#ifdef __cplusplus
}
#endif

#endif /* RAINGUN_HOST_H */
