// image_io.cpp — the canvas writers of the reference (canvas.rs:75-137) for
// the 8-bit frames the device produces (RT_OUT_U8: canvas.rs:117-123's
// quantization happens in the kernel's store).  Host I/O, off the timed path:
//   Canvas::to_ppm        canvas.rs:75-97   -> binary P6 here (the reference
//                                              writes the P3 text form; same
//                                              pixels, 1/4 of the bytes)
//   Canvas::to_png_file   canvas.rs:114-137 -> RGB8 PNG, filter None on every
//                                              row, deflate at the highest
//                                              level (image's
//                                              CompressionType::Best,
//                                              FilterType::NoFilter)
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>
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

bool ends_with(const std::string& s, const char* suffix) {
    const size_t n = std::strlen(suffix);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (std::tolower((unsigned char)s[s.size() - n + i]) != suffix[i]) return false;
    return true;
}

}  // namespace

extern "C" int rt_image_write(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height) {
    if (!path || (!rgb && (size_t)width * height) || !width || !height)
        return rtc::set_error(RT_ERR_INVALID, "rt_image_write: bad arguments");
    std::vector<uint8_t> bytes;
    if (ends_with(path, ".png")) {
        if (int rc = png_bytes(rgb, width, height, bytes)) return rc;
    } else {
        const std::string head = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
        bytes.assign(head.begin(), head.end());
        bytes.insert(bytes.end(), rgb, rgb + (size_t)width * height * 3);
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) return rtc::set_error(RT_ERR_IO, std::string("cannot open ") + path);
    const bool ok = std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
    if (std::fclose(f) != 0 || !ok) return rtc::set_error(RT_ERR_IO, std::string("cannot write ") + path);
    return RT_OK;
}
