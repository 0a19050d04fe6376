// raingun_cli.cpp — the `raingun` binary (src/main.rs:98-132 + src/render.rs)
// on the native host layer (libraingun_host.so: YAML scene, textures, PNG) and
// the HIP renderer (libraingun_hip.so: rg_render_image).
//
//   raingun [-w PIXELS] [-h PIXELS] [--4k|--hd] [--draft] [-o FILE] [--gpu N] FILE
//
// Flag semantics follow construct_app / RenderOptions::from (main.rs:21-96,
// clap 2.23 overrides_with: the last of --4k/--hd wins; --draft forces
// 800x600 and caps the recursion depth at 4, main.rs:74-75, 119-123, and
// overrides --4k/--hd/--width/--height, main.rs:47-54).  Panic sites of the
// reference (`expect(...)`) print the same message and exit with status 101,
// Rust's panic status; argument errors exit with 1 like clap.  `--preview`
// (piston window) has no display on an MI355X node: it renders without one.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_host.h"

namespace {

const char *kUsage =
    "USAGE:\n    raingun [FLAGS] [OPTIONS] <FILE>\n";

const char *kHelp =
    "raingun 0.1.0\n"
    "Magnus Bergmark <magnus.bergmark@gmail.com>\n\n"
    "USAGE:\n    raingun [FLAGS] [OPTIONS] <FILE>\n\n"
    "FLAGS:\n"
    "        --4k         Renders in 4K resolution. Explicit width/height overrides.\n"
    "        --draft      Renders in 800x600 and lower quality settings.\n"
    "        --hd         Renders in 1080 (HD) resolution. Explicit width/height overrides.\n"
    "        --help       Prints help information\n"
    "        --preview    Shows render progress in a window (not available: renders without one).\n"
    "    -V, --version    Prints version information\n\n"
    "OPTIONS:\n"
    "        --gpu <N>              HIP device to render on (default 0).\n"
    "    -h, --height <PIXELS>      Height of output image.\n"
    "    -o, --output <FILENAME>    Specify filename of the rendered image.\n"
    "    -w, --width <PIXELS>       Width of output image.\n\n"
    "ARGS:\n"
    "    <FILE>    The scene definition file, in YAML format.\n";

[[noreturn]] void clap_error(const std::string &msg) {
    std::fprintf(stderr, "error: %s\n\n%s\nFor more information try --help\n", msg.c_str(), kUsage);
    std::exit(1);
}

[[noreturn]] void panic(const std::string &msg) {
    std::fflush(stdout);
    std::fprintf(stderr, "thread 'main' panicked at '%s', src/main.rs\n", msg.c_str());
    std::exit(101);
}

struct Args {
    bool draft = false, hd = false, uhd = false, preview = false;
    const char *width = nullptr, *height = nullptr, *output = nullptr, *input = nullptr;
    int gpu = 0;
};

struct RenderOptions {  // render.rs:32-46
    uint32_t width = 800, height = 600;
    bool has_depth = false;
    uint32_t max_recursion_depth = 0;
};

bool parse_u32(const char *s, uint32_t *out) {  // str::parse::<u32>
    if (!s || !*s) return false;
    const char *p = s;
    if (*p == '+') ++p;
    if (!*p) return false;
    uint64_t v = 0;
    for (; *p; ++p) {
        if (*p < '0' || *p > '9') return false;
        v = v * 10 + (uint64_t)(*p - '0');
        if (v > 0xFFFFFFFFull) return false;
    }
    *out = (uint32_t)v;
    return true;
}

Args parse_args(int argc, char **argv) {
    Args a;
    bool only_positional = false;
    auto take_value = [&](int &i, const std::string &name, const char *inline_value) -> const char * {
        if (inline_value) return inline_value;
        if (i + 1 >= argc) clap_error("The argument '" + name + "' requires a value but none was supplied");
        return argv[++i];
    };
    for (int i = 1; i < argc; ++i) {
        const char *arg = argv[i];
        if (only_positional || arg[0] != '-' || !arg[1]) {
            if (a.input) clap_error(std::string("Found argument '") + arg + "' which wasn't expected, or isn't valid in this context");
            a.input = arg;
            continue;
        }
        if (!std::strcmp(arg, "--")) { only_positional = true; continue; }
        if (arg[1] == '-') {
            std::string name(arg + 2);
            const char *val = nullptr;
            size_t eq = name.find('=');
            if (eq != std::string::npos) { val = arg + 2 + eq + 1; name = name.substr(0, eq); }
            if (name == "width") a.width = take_value(i, "--width <PIXELS>", val);
            else if (name == "height") a.height = take_value(i, "--height <PIXELS>", val);
            else if (name == "output") a.output = take_value(i, "--output <FILENAME>", val);
            else if (name == "gpu") a.gpu = std::atoi(take_value(i, "--gpu <N>", val));
            else if (val) clap_error("Found argument '" + std::string(arg) + "' which wasn't expected, or isn't valid in this context");
            else if (name == "4k") { a.uhd = true; a.hd = false; }   // overrides_with("hd")
            else if (name == "hd") { a.hd = true; a.uhd = false; }   // overrides_with("4k")
            else if (name == "draft") a.draft = true;
            else if (name == "preview") a.preview = true;
            else if (name == "help") { std::fputs(kHelp, stdout); std::exit(0); }
            else if (name == "version") { std::puts("raingun 0.1.0"); std::exit(0); }
            else clap_error("Found argument '" + std::string(arg) + "' which wasn't expected, or isn't valid in this context");
            continue;
        }
        const char c = arg[1];
        const char *inl = arg[2] ? arg + 2 : nullptr;
        if (inl && *inl == '=') ++inl;
        if (c == 'w') a.width = take_value(i, "--width <PIXELS>", inl);
        else if (c == 'h') a.height = take_value(i, "--height <PIXELS>", inl);
        else if (c == 'o') a.output = take_value(i, "--output <FILENAME>", inl);
        else if (c == 'V' && !inl) { std::puts("raingun 0.1.0"); std::exit(0); }
        else clap_error("Found argument '" + std::string(arg) + "' which wasn't expected, or isn't valid in this context");
    }
    if (!a.input) clap_error("The following required arguments were not provided:\n    <FILE>");
    return a;
}

RenderOptions options_from(const Args &a) {  // main.rs:70-96
    RenderOptions o;
    if (a.draft) {
        o.has_depth = true;
        o.max_recursion_depth = 4;
        return o;  // --draft overrides width/height (main.rs:47-54)
    }
    if (a.hd) { o.width = 1920; o.height = 1080; }
    else if (a.uhd) { o.width = 3840; o.height = 2160; }
    if (a.width && !parse_u32(a.width, &o.width)) panic("Could not parse width: ParseIntError { kind: InvalidDigit }");
    if (a.height && !parse_u32(a.height, &o.height)) panic("Could not parse height: ParseIntError { kind: InvalidDigit }");
    return o;
}

std::string format_duration(long long ms) {  // render.rs:229-244
    const long long one_minute = 1000 * 60;
    char buf[64];
    if (ms <= 800) std::snprintf(buf, sizeof buf, "%lldms", ms);
    else if (ms <= one_minute) std::snprintf(buf, sizeof buf, "%.2fs", (double)((float)ms / 1000.0f));
    else {
        long long minutes = ms / one_minute;
        std::snprintf(buf, sizeof buf, "%lldm %.2fs", minutes, (double)((float)(ms - minutes * one_minute) / 1000.0f));
    }
    return buf;
}

// PathBuf::set_extension("png"): false when there is no file name.
bool with_png_extension(const std::string &in, std::string &out) {
    std::string path = in;
    while (path.size() > 1 && path.back() == '/') path.pop_back();
    size_t slash = path.rfind('/');
    std::string dir = slash == std::string::npos ? "" : path.substr(0, slash + 1);
    std::string name = slash == std::string::npos ? path : path.substr(slash + 1);
    if (name.empty() || name == "." || name == ".." || path == "/") return false;
    size_t dot = name.rfind('.');
    std::string stem = (dot == std::string::npos || dot == 0) ? name : name.substr(0, dot);
    out = dir + stem + ".png";
    return true;
}

}  // namespace

int main(int argc, char **argv) {
    const Args args = parse_args(argc, argv);
    const RenderOptions opts = options_from(args);
    const std::string input = args.input;
    std::string output;
    if (args.output) {
        output = args.output;
    } else if (!with_png_extension(input, output)) {
        std::printf("Could not guess output filename from %s\n", input.c_str());
        return 2;
    }
    if (args.preview)
        std::fprintf(stderr, "--preview is not supported on this build (no display); rendering without preview\n");

    rgh_scene *loaded = nullptr;
    int32_t st = rgh_scene_load_file(input.c_str(), nullptr, &loaded);  // textures relative to the CWD
    if (st == RGH_ERR_IO) panic(rgh_last_error());
    if (st != RGH_OK) panic(rgh_last_error());
    if (opts.has_depth) rgh_scene_clamp_depth(loaded, opts.max_recursion_depth);  // main.rs:119-123

    rg_scene *scene = nullptr;
    st = rg_scene_create(rgh_scene_desc(loaded), args.gpu, &scene);
    if (st != RG_OK) panic(std::string("rg_scene_create: ") + rg_status_string(st));
    std::vector<uint8_t> rgba((size_t)opts.width * opts.height * 4);

    auto t0 = std::chrono::steady_clock::now();  // render.rs:54-56
    st = rg_render_image(scene, opts.width, opts.height, rgba.data(), nullptr);
    auto t1 = std::chrono::steady_clock::now();
    if (st != RG_OK) panic(rg_status_string(st));
    st = rgh_png_write(output.c_str(), rgba.data(), opts.width, opts.height);  // render.rs:58
    auto t2 = std::chrono::steady_clock::now();
    if (st != RGH_OK) panic(rgh_last_error());
    rg_scene_destroy(scene);
    rgh_scene_free(loaded);

    auto ms = [](std::chrono::steady_clock::duration d) {
        return (long long)std::chrono::duration_cast<std::chrono::milliseconds>(d).count();
    };
    std::printf("%s\t\xe2\x86\x92\t%s\t(%s render, %s write)\n", input.c_str(), output.c_str(),
                format_duration(ms(t1 - t0)).c_str(), format_duration(ms(t2 - t1)).c_str());
    return 0;
}
