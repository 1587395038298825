// image_io.cpp — the canvas writers of the reference (canvas.rs:75-137) for
// the 8-bit frames the device produces (RT_OUT_U8: canvas.rs:117-123's
// quantization happens in the kernel's store).  Host I/O, off the timed path:
//   Canvas::to_ppm_file   canvas.rs:75-97, 107-112 -> the same P3 text, byte
//                                              for byte: header lines "P3",
//                                              "W H", "255"; then 5 pixels (15
//                                              channels) per line whatever the
//                                              row boundaries, each channel
//                                              right-aligned to width 3 and
//                                              joined by single spaces; lines
//                                              joined by '\n', no trailing
//                                              newline.  A binary P6 is an
//                                              explicit opt-in
//                                              (RT_IMAGE_PPM_BINARY).
//   Canvas::to_png_file   canvas.rs:114-137 -> RGB8 PNG, filter None on every
//                                              row, deflate at the highest
//                                              level (image's
//                                              CompressionType::Best,
//                                              FilterType::NoFilter)
//   Canvas::prepare_file  canvas.rs:99-105  -> the parent directories are
//                                              created first (create_dir_all)
//   Color::clamped + the u8 cast  canvas.rs:81, 117-123 -> rt_canvas_quantize
//                                              for f64 canvases on the host
#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/rtc_scene.h"
#include "rtc_internal.hpp"

namespace {

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

// One PNG chunk: length, type, data, CRC-32 of type + data.
void chunk(std::vector<uint8_t>& out, const char type[4], const uint8_t* data, size_t n) {
    put_be32(out, (uint32_t)n);
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    if (n) out.insert(out.end(), data, data + n);
    put_be32(out, (uint32_t)crc32(0L, out.data() + start, (uInt)(n + 4)));
}

int png_bytes(const uint8_t* rgb, uint32_t w, uint32_t h, std::vector<uint8_t>& out) {
    const size_t row = (size_t)w * 3;
    std::vector<uint8_t> raw((row + 1) * h);
    for (uint32_t y = 0; y < h; ++y) {
        raw[y * (row + 1)] = 0;  // filter type None
        std::memcpy(&raw[y * (row + 1) + 1], rgb + y * row, row);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), Z_BEST_COMPRESSION) != Z_OK)
        return rtc::set_error(RT_ERR_IO, "zlib compress2 failed");
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    out.assign(sig, sig + 8);
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, w);
    put_be32(ihdr, h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, RGB, deflate, adaptive filtering, no interlace
    chunk(out, "IHDR", ihdr.data(), ihdr.size());
    chunk(out, "IDAT", z.data(), zlen);
    chunk(out, "IEND", nullptr, 0);
    return RT_OK;
}

// Canvas::to_ppm (canvas.rs:75-97): pixels_per_line = floor(70 / 12) = 5;
// each chunk of 5 pixels (across row boundaries) is one line of 15 channels,
// every channel padded to width 3 on the left (canvas.rs:82-90) and joined by
// " "; the header's three lines and the pixel lines are joined by "\n" with
// none after the last.
void ppm_p3_bytes(const uint8_t* rgb, uint32_t w, uint32_t h, std::vector<uint8_t>& out) {
    const std::string head = "P3\n" + std::to_string(w) + " " + std::to_string(h) + "\n255";
    out.assign(head.begin(), head.end());
    const size_t n = (size_t)w * h;
    constexpr size_t kPixelsPerLine = 5;
    out.reserve(out.size() + n * 12 + n / kPixelsPerLine + 1);
    char cell[4];
    for (size_t p = 0; p < n; p += kPixelsPerLine) {
        out.push_back('\n');
        const size_t end = std::min(n, p + kPixelsPerLine);
        for (size_t c = p * 3; c < end * 3; ++c) {
            if (c != p * 3) out.push_back(' ');
            std::snprintf(cell, sizeof cell, "%3u", (unsigned)rgb[c]);
            out.insert(out.end(), cell, cell + 3);
        }
    }
}

// Canvas::prepare_file (canvas.rs:99-105): create_dir_all(parent).  Rust's
// Path::parent of a bare file name is "", for which create_dir_all is a no-op.
int make_parent_dirs(const std::string& path) {
    const size_t slash = path.find_last_of('/');
    if (slash == std::string::npos || slash == 0) return RT_OK;
    const std::string dir = path.substr(0, slash);
    for (size_t i = 1; i <= dir.size(); ++i) {
        if (i < dir.size() && dir[i] != '/') continue;
        const std::string part = dir.substr(0, i);
        if (::mkdir(part.c_str(), 0777) != 0 && errno != EEXIST)
            return rtc::set_error(RT_ERR_IO, "cannot create directory " + part + ": " + std::strerror(errno));
        struct stat st;
        if (::stat(part.c_str(), &st) != 0 || !S_ISDIR(st.st_mode))
            return rtc::set_error(RT_ERR_IO, part + " is not a directory");
    }
    return RT_OK;
}

bool ends_with(const std::string& s, const char* suffix) {
    const size_t n = std::strlen(suffix);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (std::tolower((unsigned char)s[s.size() - n + i]) != suffix[i]) return false;
    return true;
}

}  // namespace

extern "C" int rt_image_write_format(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height,
                                     int format) {
    if (!path || !*path || (!rgb && (size_t)width * height != 0) || format < RT_IMAGE_AUTO ||
        format > RT_IMAGE_PPM_BINARY)
        return rtc::set_error(RT_ERR_INVALID, "rt_image_write: bad arguments");
    if (format == RT_IMAGE_AUTO) format = ends_with(path, ".png") ? RT_IMAGE_PNG : RT_IMAGE_PPM;
    std::vector<uint8_t> bytes;
    if (format == RT_IMAGE_PNG) {
        if (!width || !height) return rtc::set_error(RT_ERR_INVALID, "rt_image_write: a PNG needs width, height > 0");
        if (int rc = png_bytes(rgb, width, height, bytes)) return rc;
    } else if (format == RT_IMAGE_PPM) {
        ppm_p3_bytes(rgb, width, height, bytes);
    } else {
        const std::string head = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
        bytes.assign(head.begin(), head.end());
        bytes.insert(bytes.end(), rgb, rgb + (size_t)width * height * 3);
    }
    if (int rc = make_parent_dirs(path)) return rc;
    FILE* f = std::fopen(path, "wb");
    if (!f) return rtc::set_error(RT_ERR_IO, std::string("cannot open ") + path);
    const bool ok = std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
    if (std::fclose(f) != 0 || !ok) return rtc::set_error(RT_ERR_IO, std::string("cannot write ") + path);
    return RT_OK;
}

extern "C" int rt_image_write(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height) {
    return rt_image_write_format(path, rgb, width, height, RT_IMAGE_AUTO);
}

// Color::clamped then (c * 255).round() as u8 (canvas.rs:81, 117-123;
// color.rs clamp to [MIN, MAX] = [0, 1]; f64::round is half away from zero;
// `as u8` saturates and maps NaN to 0).  The host twin of the kernels'
// RT_OUT_U8 store, for f64 canvases.
extern "C" int rt_canvas_quantize(const double* rgb, uint64_t n_channels, uint8_t* out) {
    if ((!rgb || !out) && n_channels) return rtc::set_error(RT_ERR_INVALID, "rt_canvas_quantize: bad arguments");
    for (uint64_t i = 0; i < n_channels; ++i) {
        const double c = rgb[i];
        const double k = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c);  // NaN falls through unchanged
        const double v = std::round(k * 255.0);
        out[i] = v >= 0.0 ? (uint8_t)v : (uint8_t)0;          // NaN compares false -> 0
    }
    return RT_OK;
}
