// scene_loader.cpp — `Scene` deserialisation (serde_yaml 0.6 over yaml-rust
// 0.3.5) into the flat rg_scene_desc of include/raingun.h, plus the
// rgh_* C ABI of include/raingun_host.h.
//
// Schema (reference paths):
//   Scene     scene.rs:11-31   camelCase, deny_unknown_fields, default
//   Body      bodies.rs:13-47  Sphere{center,radius,material} Plane{origin,normal,material}
//                              Disk{origin,normal,radius,material} AABB{bounds:[Point3;2],material}
//   Light     lights.rs:8-26   Directional{direction,color,intensity} Spherical{position,color,intensity}
//   Material  material.rs:7-12, 20-31, 49-54  coloration (Color | Texture{image,x_offset,y_offset}),
//                              albedo: f32, surface (Diffuse | Reflecting{reflectivity} |
//                              Refractive{index,transparency})
//   Color     color.rs:113-130 "#rrggbb" via u64::from_str_radix
// serde semantics kept: externally tagged enums are a bare string (unit
// variant) or a one-entry mapping; struct fields may come from a mapping or a
// sequence of exactly the right length (Point3/Vector3 "[x, y, z]"); unknown
// fields are ignored except on Scene; integers deserialise into f64/f32 by
// `as` conversion; quoted scalars are strings and never numbers.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/raingun_host.h"
#include "image_codec.h"
#include "yaml.h"

namespace rgh {
namespace {

using yaml::Node;

struct SchemaError {
    std::string msg;
};
struct ImageError {
    std::string msg;
};

[[noreturn]] void bad(const std::string &what, const std::string &msg) {
    throw SchemaError{what + ": " + msg};
}

std::string describe(const Node &n) {
    switch (n.kind) {
    case Node::Null: return "null";
    case Node::Seq: return "a sequence";
    case Node::Map: return "a mapping";
    default: break;
    }
    switch (yaml::resolve(n)) {
    case yaml::ScalarType::Null: return "null";
    case yaml::ScalarType::Bool: return "boolean `" + n.str + "`";
    case yaml::ScalarType::Integer: return "integer `" + n.str + "`";
    case yaml::ScalarType::Real: return "floating point `" + n.str + "`";
    default: return "string \"" + n.str + "\"";
    }
}

double as_f64(const Node &n, const std::string &what) {
    if (n.kind == Node::Scalar) {
        int64_t i;
        double d;
        switch (yaml::resolve(n, &i, &d)) {
        case yaml::ScalarType::Integer: return (double)i;
        case yaml::ScalarType::Real: return d;
        default: break;
        }
    }
    bad(what, "invalid type: " + describe(n) + ", expected f64");
}

float as_f32(const Node &n, const std::string &what) {
    if (n.kind == Node::Scalar) {
        int64_t i;
        double d;
        switch (yaml::resolve(n, &i, &d)) {
        case yaml::ScalarType::Integer: return (float)i;  // serde: `v as f32` from i64
        case yaml::ScalarType::Real: return (float)d;     // `v as f32` from f64
        default: break;
        }
    }
    bad(what, "invalid type: " + describe(n) + ", expected f32");
}

uint32_t as_u32(const Node &n, const std::string &what) {
    int64_t i;
    if (n.kind == Node::Scalar && yaml::resolve(n, &i) == yaml::ScalarType::Integer) {
        if (i < 0 || i > 0xFFFFFFFFll) bad(what, "invalid value: integer `" + n.str + "`, expected u32");
        return (uint32_t)i;
    }
    bad(what, "invalid type: " + describe(n) + ", expected u32");
}

const std::string &as_string(const Node &n, const std::string &what) {
    if (n.kind == Node::Scalar && yaml::resolve(n) == yaml::ScalarType::String) return n.str;
    bad(what, "invalid type: " + describe(n) + ", expected a string");
}

const Node &field(const Node &m, const char *key, const std::string &what) {
    if (m.kind != Node::Map) bad(what, "invalid type: " + describe(m) + ", expected a struct");
    const Node *v = m.get(key);
    if (!v) bad(what, std::string("missing field `") + key + "`");
    return *v;
}

// Externally tagged enum: "Name" or {Name: content}.
std::pair<std::string, const Node *> variant(const Node &n, const std::string &what) {
    if (n.kind == Node::Scalar && yaml::resolve(n) == yaml::ScalarType::String) return {n.str, nullptr};
    if (n.kind == Node::Map && n.map.size() == 1) return {n.map[0].first, &n.map[0].second};
    bad(what, "invalid type: " + describe(n) + ", expected an enum variant");
}

void vec3(const Node &n, const std::string &what, double out[3]) {
    if (n.kind == Node::Seq) {
        if (n.seq.size() != 3) bad(what, "invalid length " + std::to_string(n.seq.size()) + ", expected 3 components");
        for (int k = 0; k < 3; ++k) out[k] = as_f64(n.seq[k], what);
        return;
    }
    if (n.kind == Node::Map) {
        out[0] = as_f64(field(n, "x", what), what);
        out[1] = as_f64(field(n, "y", what), what);
        out[2] = as_f64(field(n, "z", what), what);
        return;
    }
    bad(what, "invalid type: " + describe(n) + ", expected a point/vector");
}

void color(const Node &n, const std::string &what, float out[3]) {
    if (!(n.kind == Node::Scalar && yaml::resolve(n) == yaml::ScalarType::String))
        bad(what, "invalid type: " + describe(n) + ", expected a string of a simple hex color (#000000 - #ffffff)");
    const std::string &s = n.str;
    // color.rs:117-126: len 7, '#', then u64::from_str_radix(.., 16) (an optional '+' then hex digits)
    bool ok = s.size() == 7 && s[0] == '#';
    size_t i = 1;
    if (ok && s[i] == '+') ++i;
    ok = ok && i < s.size();
    uint64_t num = 0;
    for (; ok && i < s.size(); ++i) {
        char c = s[i];
        int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
        if (d < 0) ok = false;
        else num = num * 16 + (uint64_t)d;
    }
    if (!ok) bad(what, s + " is not a valid color");
    const float d255 = 255.0f;
    out[0] = (float)((num & 0xff0000) >> 16) / d255;
    out[1] = (float)((num & 0x00ff00) >> 8) / d255;
    out[2] = (float)(num & 0x0000ff) / d255;
}

std::string join_path(const std::string &root, const std::string &p) {
    if (root.empty() || (!p.empty() && p[0] == '/')) return p;
    return root.back() == '/' ? root + p : root + "/" + p;
}

bool read_file(const std::string &path, std::vector<uint8_t> &out, std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        err = std::string(std::strerror(errno)) + " (os error " + std::to_string(errno) + ")";
        return false;
    }
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

}  // namespace

struct LoadedScene {
    rg_scene_desc desc{};
    std::vector<rg_body> bodies;
    std::vector<rg_light> lights;
    std::vector<rg_texture> textures;
    std::vector<Image> images;
    std::map<std::string, int32_t> tex_by_path;
    std::vector<std::string> tex_paths;
    std::string texture_root;

    int32_t texture(const std::string &path) {
        auto it = tex_by_path.find(path);
        if (it != tex_by_path.end()) return it->second;
        std::vector<uint8_t> bytes;
        std::string err;
        Image img;
        if (!read_file(join_path(texture_root, path), bytes, err) || !decode_image(bytes.data(), bytes.size(), img, err))
            throw ImageError{"Could not load texture file " + path + ": " + err};
        int32_t idx = (int32_t)images.size();
        images.push_back(std::move(img));
        tex_paths.push_back(path);
        tex_by_path[path] = idx;
        return idx;
    }

    void material(const Node &n, const std::string &what, rg_material &m) {
        std::memset(&m, 0, sizeof m);
        m.texture = -1;
        auto col = variant(field(n, "coloration", what), what + ".coloration");
        if (col.first == "Color") {
            if (!col.second) bad(what + ".coloration", "invalid type: unit variant, expected newtype variant");
            m.coloration = RG_COLORATION_COLOR;
            color(*col.second, what + ".coloration.Color", m.color);
        } else if (col.first == "Texture") {
            const std::string tw = what + ".coloration.Texture";
            if (!col.second) bad(what + ".coloration", "invalid type: unit variant, expected newtype variant");
            const Node &t = *col.second;
            const std::string &img = as_string(field(t, "image", tw), tw + ".image");
            m.x_offset = as_f32(field(t, "x_offset", tw), tw + ".x_offset");
            m.y_offset = as_f32(field(t, "y_offset", tw), tw + ".y_offset");
            m.coloration = RG_COLORATION_TEXTURE;
            m.texture = texture(img);
        } else {
            bad(what + ".coloration", "unknown variant `" + col.first + "`, expected `Color` or `Texture`");
        }
        m.albedo = as_f32(field(n, "albedo", what), what + ".albedo");
        auto sf = variant(field(n, "surface", what), what + ".surface");
        const std::string sw = what + ".surface";
        if (sf.first == "Diffuse") {
            if (sf.second && sf.second->kind != Node::Null) bad(sw, "Diffuse takes no fields");
            m.surface = RG_SURFACE_DIFFUSE;
        } else if (sf.first == "Reflecting") {
            if (!sf.second) bad(sw, "invalid type: unit variant, expected struct variant");
            m.surface = RG_SURFACE_REFLECTING;
            m.reflectivity = as_f32(field(*sf.second, "reflectivity", sw), what + ".reflectivity");
        } else if (sf.first == "Refractive") {
            if (!sf.second) bad(sw, "invalid type: unit variant, expected struct variant");
            m.surface = RG_SURFACE_REFRACTIVE;
            m.index = as_f32(field(*sf.second, "index", sw), what + ".index");
            m.transparency = as_f32(field(*sf.second, "transparency", sw), what + ".transparency");
        } else {
            bad(sw, "unknown variant `" + sf.first + "`, expected one of `Diffuse`, `Reflecting`, `Refractive`");
        }
    }

    void body(const Node &n, size_t i) {
        const std::string what = "bodies[" + std::to_string(i) + "]";
        auto v = variant(n, what);
        const std::string w = what + "." + v.first;
        rg_body b;
        std::memset(&b, 0, sizeof b);
        if (v.first != "Sphere" && v.first != "Plane" && v.first != "Disk" && v.first != "AABB")
            bad(what, "unknown variant `" + v.first + "`, expected one of `Sphere`, `Plane`, `Disk`, `AABB`");
        if (!v.second) bad(what, "invalid type: unit variant, expected newtype variant");
        const Node &s = *v.second;
        if (v.first == "Sphere") {
            b.kind = RG_BODY_SPHERE;
            vec3(field(s, "center", w), w + ".center", b.p);
            b.p[3] = as_f64(field(s, "radius", w), w + ".radius");
        } else if (v.first == "Plane") {
            b.kind = RG_BODY_PLANE;
            vec3(field(s, "origin", w), w + ".origin", b.p);
            vec3(field(s, "normal", w), w + ".normal", b.p + 3);
        } else if (v.first == "Disk") {
            b.kind = RG_BODY_DISK;
            vec3(field(s, "origin", w), w + ".origin", b.p);
            vec3(field(s, "normal", w), w + ".normal", b.p + 3);
            b.p[6] = as_f64(field(s, "radius", w), w + ".radius");
        } else {
            b.kind = RG_BODY_AABB;
            const Node &bd = field(s, "bounds", w);
            if (bd.kind != Node::Seq || bd.seq.size() != 2) bad(w + ".bounds", "expected two points");
            vec3(bd.seq[0], w + ".bounds[0]", b.p);
            vec3(bd.seq[1], w + ".bounds[1]", b.p + 3);
        }
        material(field(s, "material", w), w + ".material", b.material);
        bodies.push_back(b);
    }

    void light(const Node &n, size_t i) {
        const std::string what = "lights[" + std::to_string(i) + "]";
        auto v = variant(n, what);
        const std::string w = what + "." + v.first;
        rg_light l;
        std::memset(&l, 0, sizeof l);
        if (v.first != "Directional" && v.first != "Spherical")
            bad(what, "unknown variant `" + v.first + "`, expected `Directional` or `Spherical`");
        if (!v.second) bad(what, "invalid type: unit variant, expected newtype variant");
        const Node &s = *v.second;
        if (v.first == "Directional") {
            l.kind = RG_LIGHT_DIRECTIONAL;
            vec3(field(s, "direction", w), w + ".direction", l.v);
        } else {
            l.kind = RG_LIGHT_SPHERICAL;
            vec3(field(s, "position", w), w + ".position", l.v);
        }
        color(field(s, "color", w), w + ".color", l.color);
        l.intensity = as_f32(field(s, "intensity", w), w + ".intensity");
        lights.push_back(l);
    }

    void load(const Node &doc) {
        desc.fov = 90.0;
        desc.max_recursion_depth = 10;
        if (doc.kind == Node::Null) return finish();
        if (doc.kind != Node::Map) throw SchemaError{"invalid type: " + describe(doc) + ", expected struct Scene"};
        static const char *keys[] = {"fov", "defaultColor", "maxRecursionDepth", "bodies", "lights"};
        for (const auto &kv : doc.map) {
            bool known = false;
            for (const char *k : keys) known |= kv.first == k;
            if (!known)  // deny_unknown_fields (scene.rs:12)
                throw SchemaError{"unknown field `" + kv.first +
                                  "`, expected one of `fov`, `defaultColor`, `maxRecursionDepth`, `bodies`, `lights`"};
        }
        if (const Node *n = doc.get("fov")) desc.fov = as_f64(*n, "fov");
        if (const Node *n = doc.get("defaultColor")) color(*n, "defaultColor", desc.default_color);
        if (const Node *n = doc.get("maxRecursionDepth")) desc.max_recursion_depth = as_u32(*n, "maxRecursionDepth");
        if (const Node *n = doc.get("bodies")) {
            if (n->kind != Node::Seq) bad("bodies", "invalid type: " + describe(*n) + ", expected a sequence");
            for (size_t i = 0; i < n->seq.size(); ++i) body(n->seq[i], i);
        }
        if (const Node *n = doc.get("lights")) {
            if (n->kind != Node::Seq) bad("lights", "invalid type: " + describe(*n) + ", expected a sequence");
            for (size_t i = 0; i < n->seq.size(); ++i) light(n->seq[i], i);
        }
        finish();
    }

    void finish() {
        textures.resize(images.size());
        for (size_t i = 0; i < images.size(); ++i) {
            textures[i].width = images[i].width;
            textures[i].height = images[i].height;
            textures[i].rgba = images[i].rgba.data();
        }
        desc.n_bodies = (uint32_t)bodies.size();
        desc.bodies = bodies.empty() ? nullptr : bodies.data();
        desc.n_lights = (uint32_t)lights.size();
        desc.lights = lights.empty() ? nullptr : lights.data();
        desc.n_textures = (uint32_t)textures.size();
        desc.textures = textures.empty() ? nullptr : textures.data();
    }
};

}  // namespace rgh

// ---------------------------------------------------------------- C ABI
struct rgh_scene {
    rgh::LoadedScene s;
};

namespace {
thread_local std::string g_last_error;

int32_t set_error(int32_t code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int32_t load_text(const std::string &text, const char *texture_root, rgh_scene **out) {
    if (!out) return set_error(RGH_ERR_INVALID_ARGUMENT, "null output pointer");
    *out = nullptr;
    rgh::yaml::Node doc;
    std::string err;
    if (!rgh::yaml::parse(text, doc, err)) return set_error(RGH_ERR_YAML, "Could not load YAML: " + err);
    std::unique_ptr<rgh_scene> sc(new (std::nothrow) rgh_scene);
    if (!sc) return set_error(RGH_ERR_OUT_OF_MEMORY, "out of memory");
    sc->s.texture_root = texture_root ? texture_root : "";
    try {
        sc->s.load(doc);
    } catch (const rgh::SchemaError &e) {
        return set_error(RGH_ERR_SCHEMA, "Could not load YAML: " + e.msg);
    } catch (const rgh::ImageError &e) {
        return set_error(RGH_ERR_IMAGE, "Could not load YAML: " + e.msg);
    } catch (const std::bad_alloc &) {
        return set_error(RGH_ERR_OUT_OF_MEMORY, "out of memory");
    }
    g_last_error.clear();
    *out = sc.release();
    return RGH_OK;
}

uint8_t *to_malloc(const std::vector<uint8_t> &v) {
    uint8_t *p = (uint8_t *)std::malloc(v.empty() ? 1 : v.size());
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size());
    return p;
}
}  // namespace

extern "C" {

int32_t rgh_abi_version(void) { return RGH_ABI_VERSION; }

const char *rgh_last_error(void) { return g_last_error.c_str(); }

int32_t rgh_scene_load_file(const char *path, const char *texture_root, rgh_scene **out) {
    if (!path || !out) return set_error(RGH_ERR_INVALID_ARGUMENT, "null argument");
    std::vector<uint8_t> bytes;
    std::string err;
    if (!rgh::read_file(path, bytes, err)) return set_error(RGH_ERR_IO, "Could not open input file: " + err);
    return load_text(std::string(bytes.begin(), bytes.end()), texture_root, out);
}

int32_t rgh_scene_load_string(const char *yaml, size_t len, const char *texture_root, rgh_scene **out) {
    if (!yaml) return set_error(RGH_ERR_INVALID_ARGUMENT, "null argument");
    return load_text(std::string(yaml, len), texture_root, out);
}

const rg_scene_desc *rgh_scene_desc(const rgh_scene *scene) { return scene ? &scene->s.desc : nullptr; }

const char *rgh_scene_texture_path(const rgh_scene *scene, uint32_t index) {
    if (!scene || index >= scene->s.tex_paths.size()) return nullptr;
    return scene->s.tex_paths[index].c_str();
}

void rgh_scene_clamp_depth(rgh_scene *scene, uint32_t limit) {
    if (scene && limit < scene->s.desc.max_recursion_depth) scene->s.desc.max_recursion_depth = limit;
}

void rgh_scene_free(rgh_scene *scene) { delete scene; }

int32_t rgh_image_decode(const uint8_t *data, size_t size, int32_t flavor, uint32_t *width, uint32_t *height,
                         uint8_t **rgba) {
    if (!data || !width || !height || !rgba || (flavor != RGH_JPEG_REFERENCE && flavor != RGH_JPEG_LIBJPEG))
        return set_error(RGH_ERR_INVALID_ARGUMENT, "bad argument");
    rgh::Image img;
    std::string err;
    if (!rgh::decode_image(data, size, img, err, (rgh::JpegFlavor)flavor)) return set_error(RGH_ERR_IMAGE, err);
    *rgba = to_malloc(img.rgba);
    if (!*rgba) return set_error(RGH_ERR_OUT_OF_MEMORY, "out of memory");
    *width = img.width;
    *height = img.height;
    return RGH_OK;
}

int32_t rgh_image_decode_file(const char *path, int32_t flavor, uint32_t *width, uint32_t *height, uint8_t **rgba) {
    if (!path) return set_error(RGH_ERR_INVALID_ARGUMENT, "null path");
    std::vector<uint8_t> bytes;
    std::string err;
    if (!rgh::read_file(path, bytes, err)) return set_error(RGH_ERR_IO, err);
    return rgh_image_decode(bytes.data(), bytes.size(), flavor, width, height, rgba);
}

int32_t rgh_png_encode(const uint8_t *rgba, uint32_t width, uint32_t height, uint8_t **png, size_t *size) {
    if (!rgba || !png || !size || !width || !height) return set_error(RGH_ERR_INVALID_ARGUMENT, "bad argument");
    std::vector<uint8_t> v = rgh::encode_png(rgba, width, height);
    *png = to_malloc(v);
    if (!*png) return set_error(RGH_ERR_OUT_OF_MEMORY, "out of memory");
    *size = v.size();
    return RGH_OK;
}

int32_t rgh_png_write(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || !width || !height) return set_error(RGH_ERR_INVALID_ARGUMENT, "bad argument");
    std::vector<uint8_t> v = rgh::encode_png(rgba, width, height);
    FILE *f = std::fopen(path, "wb");
    if (!f) return set_error(RGH_ERR_IO, std::string("Could not encode image: ") + std::strerror(errno));
    bool ok = std::fwrite(v.data(), 1, v.size(), f) == v.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) return set_error(RGH_ERR_IO, "Could not encode image: write failed");
    return RGH_OK;
}

void rgh_free(void *p) { std::free(p); }

}  // extern "C"
