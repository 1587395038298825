// san_driver.cpp — TEST INFRASTRUCTURE (SURVEY.md §5 "Host: ASan/UBSan
// builds of the C++ oracle and host").  Built with g++ -fsanitize=address,
// undefined by tests/sanitize/Makefile together with the product's host-only
// sources (csrc/scene_loader.cpp, csrc/image_io.cpp, csrc/rtc_jit_cache.hpp)
// and the f64 oracle (oracle/oracle_capi.cpp); the GPU parts of librtc are
// not in it.  Any sanitizer report aborts the run with a nonzero status.
//
//   san_driver scene FILE...          load each YAML scene, render it with the
//                                     oracle at 24x16 (2 threads), quantize,
//                                     write PNG / P3 / P6 into $SAN_TMP
//   san_driver fuzz N SEED FILE...    N byte-level mutations of each scene
//                                     (delete / insert / flip / duplicate /
//                                     truncate), each loaded (errors are fine)
//                                     and rendered at 6x4 when it loads
//   san_driver jitcache N SEED        code-object and request files written,
//                                     read back, then truncated at every length
//                                     and flipped at random bytes N times
//   san_driver images                 canvas quantization of NaN / inf / edge
//                                     values; image writes of 0x0, 1x1, 1x7,
//                                     odd widths, a missing parent directory
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rtc.h"
#include "../../include/rtc_scene.h"
#include "../../ray-tracer-challenge-rs_amd/csrc/rtc_jit_cache.hpp"

// librtc's thread-local error slot lives in rtc_host.cpp (HIP); the
// host-only sources reach it through rtc::set_error.
namespace rtc {
thread_local std::string g_err;
int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace rtc
extern "C" const char* rt_last_error(void) { return rtc::g_err.c_str(); }

extern "C" int orc_render(const rt_shape_desc*, uint32_t, const rt_material_desc*, uint32_t, const rt_pattern_desc*,
                          uint32_t, const rt_light_desc*, uint32_t, const rt_camera_desc*, uint32_t, uint32_t, uint32_t,
                          int, double*, rt_stats*);

namespace {

std::string tmpdir() {
    const char* t = std::getenv("SAN_TMP");
    return t && *t ? t : "/tmp";
}

std::string read_file(const char* path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// Load + (if it loads) render + quantize + write.  Returns the load status.
int run_scene(const std::string& text, uint32_t w, uint32_t h, bool write) {
    rt_scene* s = nullptr;
    const int rc = rt_scene_load_yaml_text(text.c_str(), &s);
    if (rc != RT_OK) return rc;
    rt_scene_view v;
    if (rt_scene_view_get(s, &v) != RT_OK) std::abort();
    rt_camera_desc cam = v.camera;
    rt_camera_resize(&cam, w, h);
    std::vector<double> img((size_t)w * h * 3);
    rt_stats st;
    if (orc_render(v.shapes, v.n_shapes, v.materials, v.n_materials, v.patterns, v.n_patterns, v.lights, v.n_lights, &cam,
                   6, 0, h, 2, img.data(), &st) == 0) {
        std::vector<uint8_t> q(img.size());
        if (rt_canvas_quantize(img.data(), img.size(), q.data()) != RT_OK) std::abort();
        if (write) {
            const std::string base = tmpdir() + "/san_scene";
            if (rt_image_write((base + ".png").c_str(), q.data(), w, h) != RT_OK ||
                rt_image_write_format((base + ".ppm").c_str(), q.data(), w, h, RT_IMAGE_PPM) != RT_OK ||
                rt_image_write_format((base + "_b.ppm").c_str(), q.data(), w, h, RT_IMAGE_PPM_BINARY) != RT_OK) {
                std::fprintf(stderr, "image write failed: %s\n", rt_last_error());
                std::exit(3);
            }
        }
    }
    rt_scene_free(s);
    return RT_OK;
}

std::string mutate(std::string t, std::mt19937_64& rng) {
    const int edits = 1 + (int)(rng() % 4);
    static const char alphabet[] = " \n\t-:[],.0123456789eE+#'\"{}&*!|>abcdefghijklmnopqrstuvwxyz";
    for (int e = 0; e < edits && !t.empty(); ++e) {
        const size_t at = rng() % t.size();
        switch (rng() % 6) {
            case 0: t.erase(at, 1 + rng() % 8); break;
            case 1: t.insert(at, 1, alphabet[rng() % (sizeof alphabet - 1)]); break;
            case 2: t[at] = alphabet[rng() % (sizeof alphabet - 1)]; break;
            case 3: t[at] = (char)(t[at] ^ (1 << (rng() % 8))); break;
            case 4: {  // duplicate a line-sized span
                const size_t n = std::min<size_t>(t.size() - at, 1 + rng() % 40);
                t.insert(at, t.substr(at, n));
                break;
            }
            default: t.resize(at); break;
        }
    }
    return t;
}

int fuzz(int n, uint64_t seed, const std::vector<std::string>& bases) {
    std::mt19937_64 rng(seed);
    int loaded = 0, total = 0;
    for (const std::string& base : bases)
        for (int i = 0; i < n; ++i, ++total) loaded += run_scene(mutate(base, rng), 6, 4, false) == RT_OK;
    std::printf("fuzz: %d of %d mutated scenes loaded\n", loaded, total);
    return 0;
}

int jitcache(int n, uint64_t seed) {
    using namespace rtc::jitfile;
    std::mt19937_64 rng(seed);
    const std::string code_path = tmpdir() + "/san_cache/sub/dir/code.co", req_path = tmpdir() + "/san_req.req";
    CodeObject co;
    co.lowered = "_ZN3rtc10trace_poolIfLb1ELb0EEEvNS_12LaunchParamsIT_EEPKNS_8ShapeRecIS2_EE";
    co.code.resize(5000);
    for (char& c : co.code) c = (char)(rng() & 0xFF);
    Request rq;
    rq.name = "rtc::trace_pool<float, true, false>";
    rq.main_src = "#define RTC_JIT 1\n__global__ void k() {}\n";
    rq.opts = {"--offload-arch=gfx950", "-O3", "-DX=1"};
    rq.headers = {{"a.hpp", "#pragma once\n"}, {"b.hpp", std::string(3000, 'x')}};
    if (!write_code(code_path, co) || !write_request(req_path, rq)) return 4;
    CodeObject back;
    Request rback;
    if (!read_code(code_path, back) || back.code != co.code || back.lowered != co.lowered) return 5;
    if (!read_request(req_path, rback) || rback.main_src != rq.main_src || rback.opts != rq.opts ||
        rback.headers != rq.headers)
        return 6;
    std::vector<char> good_code, good_req;
    read_all(code_path, good_code);
    read_all(req_path, good_req);
    const std::string damaged = tmpdir() + "/san_damaged";
    auto put = [&](const std::vector<char>& bytes) {
        FILE* f = std::fopen(damaged.c_str(), "wb");
        if (!bytes.empty()) std::fwrite(bytes.data(), 1, bytes.size(), f);
        std::fclose(f);
    };
    int accepted = 0;
    for (const std::vector<char>* good : {&good_code, &good_req}) {
        const bool is_code = good == &good_code;
        for (size_t len = 0; len < good->size(); len += (len < 200 ? 1 : 97)) {  // every truncation near the header
            put(std::vector<char>(good->begin(), good->begin() + (ptrdiff_t)len));
            CodeObject c;
            Request r;
            if (is_code ? read_code(damaged, c) : read_request(damaged, r)) return 7;  // a truncated file never loads
        }
        for (int i = 0; i < n; ++i) {
            std::vector<char> b = *good;
            const int flips = 1 + (int)(rng() % 3);
            for (int f = 0; f < flips; ++f) b[rng() % b.size()] ^= (char)(1 << (rng() % 8));
            put(b);
            CodeObject c;
            Request r;
            accepted += is_code ? read_code(damaged, c) : read_request(damaged, r);
        }
    }
    std::printf("jitcache: %d of %d flipped files still parsed\n", accepted, 2 * n);
    return 0;
}

int images() {
    const double inf = std::numeric_limits<double>::infinity(), nan = std::numeric_limits<double>::quiet_NaN();
    const double vals[] = {nan, -nan, inf, -inf, -0.0, 0.0, 0.5 / 255, 1.5 / 255, 0.999999, 1.0, 1.0000001, 1e308,
                           -1e308, std::numeric_limits<double>::denorm_min()};
    const size_t n = sizeof vals / sizeof vals[0];
    std::vector<uint8_t> q(n);
    if (rt_canvas_quantize(vals, n, q.data()) != RT_OK) return 8;
    if (q[0] != 0 || q[2] != 255 || q[3] != 0 || q[9] != 255 || q[10] != 255) return 9;
    const std::string d = tmpdir();
    for (auto wh : std::vector<std::pair<uint32_t, uint32_t>>{{0, 0}, {1, 1}, {1, 7}, {7, 1}, {5, 3}, {6, 2}, {33, 31}}) {
        std::vector<uint8_t> rgb((size_t)wh.first * wh.second * 3);
        for (size_t i = 0; i < rgb.size(); ++i) rgb[i] = (uint8_t)(i * 37);
        for (int fmt : {RT_IMAGE_PNG, RT_IMAGE_PPM, RT_IMAGE_PPM_BINARY}) {
            const std::string p = d + "/san_img/" + std::to_string(wh.first) + "x" + std::to_string(wh.second) +
                                  "_" + std::to_string(fmt) + ".img";
            const int rc = rt_image_write_format(p.c_str(), rgb.empty() ? nullptr : rgb.data(), wh.first, wh.second, fmt);
            if (fmt == RT_IMAGE_PNG && rgb.empty()) {  // a PNG has no empty image (IHDR: width, height > 0)
                if (rc != RT_ERR_INVALID) return 12;
                continue;
            }
            if (rc != RT_OK) {
                std::fprintf(stderr, "write %s: %s\n", p.c_str(), rt_last_error());
                return 10;
            }
        }
    }
    // an unwritable path fails cleanly
    uint8_t px[3] = {1, 2, 3};
    if (rt_image_write("/proc/self/no/such/dir/x.png", px, 1, 1) == RT_OK) return 11;
    std::printf("images: ok\n");
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string mode = argv[1];
    if (mode == "scene") {
        for (int i = 2; i < argc; ++i)
            if (run_scene(read_file(argv[i]), 24, 16, true) != RT_OK) {
                std::fprintf(stderr, "%s: %s\n", argv[i], rt_last_error());
                return 1;
            }
        std::printf("scene: %d loaded and rendered\n", argc - 2);
        return 0;
    }
    if (mode == "fuzz" && argc >= 5) {
        std::vector<std::string> bases;
        for (int i = 4; i < argc; ++i) bases.push_back(read_file(argv[i]));
        return fuzz(std::atoi(argv[2]), std::strtoull(argv[3], nullptr, 10), bases);
    }
    if (mode == "jitcache" && argc >= 4) return jitcache(std::atoi(argv[2]), std::strtoull(argv[3], nullptr, 10));
    if (mode == "images") return images();
    return 2;
}
