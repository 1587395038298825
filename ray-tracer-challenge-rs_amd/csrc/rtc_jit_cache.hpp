// rtc_jit_cache.hpp — the file formats shared by librtc (rtc_jit.cpp) and
// the per-scene compiler process (rtc_jitc.cpp): the compile request librtc
// hands the compiler, and the code-object file it gets back, which is also
// the on-disk cache entry.  Host only, header-only (no HIP, no hipRTC).
//
// Code-object file: "RTCJIT2\n" <lowered kernel name> "\n" <code bytes> " "
// <FNV-1a of the code, hex> "\n" <code object>.  Written to a temporary name
// and renamed, so concurrent processes never read a partial file; a file
// whose length or checksum does not match is ignored and rebuilt (a damaged
// code object handed to hipModuleLoadData can abort the process instead of
// failing).
//
// Request file: "RTCREQ1\n", then length-prefixed strings ("<bytes>\n" then
// the bytes): the kernel name expression, the main source, the option count
// and options, the header count and (name, text) pairs.
#pragma once

#include <atomic>
#include <cerrno>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include <sys/stat.h>
#include <unistd.h>

namespace rtc::jitfile {

inline uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

struct CodeObject {
    std::vector<char> code;
    std::string lowered;
};

struct Request {
    std::string name;      // kernel name expression (hiprtcAddNameExpression)
    std::string main_src;  // the translation unit
    std::vector<std::string> opts;
    std::vector<std::pair<std::string, std::string>> headers;  // (include name, text)
};

inline bool read_all(const std::string& path, std::vector<char>& all) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    all.clear();
    char buf[1 << 16];
    for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) all.insert(all.end(), buf, buf + n);
    std::fclose(f);
    return true;
}

inline bool make_dirs(const std::string& d) {
    for (size_t p = 1; p <= d.size(); ++p) {
        if (p < d.size() && d[p] != '/') continue;
        const std::string part = d.substr(0, p);
        if (::mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
    return true;
}

// Write `bytes` to `path` through a temporary name in the same directory.
inline bool write_atomic(const std::string& path, const std::string& bytes) {
    const size_t slash = path.find_last_of('/');
    if (slash != std::string::npos && slash > 0 && !make_dirs(path.substr(0, slash))) return false;
    static std::atomic<unsigned> seq{0};
    const std::string tmp = path + ".tmp" + std::to_string((long long)::getpid()) + "." + std::to_string(seq++);
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    bool ok = std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        return false;
    }
    return true;
}

constexpr char kCodeMagic[] = "RTCJIT2\n";
constexpr char kRequestMagic[] = "RTCREQ1\n";

inline bool read_code(const std::string& path, CodeObject& out) {
    std::vector<char> all;
    if (!read_all(path, all)) return false;
    const size_t m = sizeof kCodeMagic - 1;
    if (all.size() < m || std::memcmp(all.data(), kCodeMagic, m)) return false;
    size_t nl = m;
    while (nl < all.size() && all[nl] != '\n') ++nl;
    if (nl + 1 >= all.size() || nl == m) return false;
    size_t nl2 = nl + 1;
    while (nl2 < all.size() && all[nl2] != '\n') ++nl2;
    if (nl2 >= all.size()) return false;
    unsigned long long len = 0, sum = 0;
    const std::string meta(all.data() + nl + 1, nl2 - nl - 1);
    if (std::sscanf(meta.c_str(), "%llu %llx", &len, &sum) != 2) return false;
    if (len == 0 || all.size() - (nl2 + 1) != len || fnv(all.data() + nl2 + 1, len) != sum) return false;
    out.lowered.assign(all.data() + m, nl - m);
    out.code.assign(all.begin() + (ptrdiff_t)(nl2 + 1), all.end());
    return true;
}

inline bool write_code(const std::string& path, const CodeObject& co) {
    char meta[64];
    std::snprintf(meta, sizeof meta, "\n%llu %llx\n", (unsigned long long)co.code.size(),
                  (unsigned long long)fnv(co.code.data(), co.code.size()));
    std::string bytes(kCodeMagic);
    bytes += co.lowered;
    bytes += meta;
    bytes.append(co.code.data(), co.code.size());
    return write_atomic(path, bytes);
}

inline void put_str(std::string& out, const std::string& s) {
    out += std::to_string(s.size());
    out += '\n';
    out += s;
}

inline bool write_request(const std::string& path, const Request& rq) {
    std::string b(kRequestMagic);
    put_str(b, rq.name);
    put_str(b, rq.main_src);
    put_str(b, std::to_string(rq.opts.size()));
    for (const std::string& o : rq.opts) put_str(b, o);
    put_str(b, std::to_string(rq.headers.size()));
    for (const auto& h : rq.headers) {
        put_str(b, h.first);
        put_str(b, h.second);
    }
    return write_atomic(path, b);
}

inline bool read_request(const std::string& path, Request& rq) {
    std::vector<char> all;
    if (!read_all(path, all)) return false;
    const size_t m = sizeof kRequestMagic - 1;
    if (all.size() < m || std::memcmp(all.data(), kRequestMagic, m)) return false;
    size_t p = m;
    auto get = [&](std::string& s) {
        size_t nl = p;
        while (nl < all.size() && all[nl] != '\n') ++nl;
        if (nl >= all.size()) return false;
        const unsigned long long n = std::strtoull(std::string(all.data() + p, nl - p).c_str(), nullptr, 10);
        if (n > all.size() - nl - 1) return false;
        s.assign(all.data() + nl + 1, n);
        p = nl + 1 + n;
        return true;
    };
    std::string count;
    if (!get(rq.name) || !get(rq.main_src) || !get(count)) return false;
    rq.opts.resize(std::strtoull(count.c_str(), nullptr, 10));
    for (std::string& o : rq.opts)
        if (!get(o)) return false;
    if (!get(count)) return false;
    rq.headers.resize(std::strtoull(count.c_str(), nullptr, 10));
    for (auto& h : rq.headers)
        if (!get(h.first) || !get(h.second)) return false;
    return p == all.size();
}

}  // namespace rtc::jitfile
