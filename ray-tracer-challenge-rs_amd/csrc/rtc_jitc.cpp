// rtc_jitc.cpp — the per-scene kernel compiler process.
//
// librtc (rtc_jit.cpp) builds a world's per-scene kernel by running this
// program as a child process: `rtc_jitc REQUEST OUT`.  It reads the compile
// request (rtc_jit_cache.hpp: kernel name, source, options, headers),
// deletes it, compiles with hipRTC and writes the code object to OUT (the
// on-disk cache entry, or a temporary file), through a temporary name.  The
// compiler log goes to stderr, exit status 0 on success.
//
// Why a process: a hipRTC compile running on a thread of the render process
// raced that process's exit (heap corruption, "corrupted size vs. prev_size",
// when a Python host exited with a build in flight: comgr/LLVM state torn
// down under the compile).  A child process owns its compiler; the render
// process only waits for it, off the frame's path, and never has to join it.
// The child touches no GPU.
#include <hip/hiprtc.h>

#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "debug_knobs.hpp"
#include "rtc_jit_cache.hpp"

using namespace rtc::jitfile;

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: rtc_jitc REQUEST OUT\n");
        return 2;
    }
    Request rq;
    const bool ok = read_request(argv[1], rq);
    std::remove(argv[1]);
    if (!ok) {
        std::fprintf(stderr, "rtc_jitc: cannot read the request %s\n", argv[1]);
        return 2;
    }
    std::vector<const char*> hdr_src, hdr_name, opts;
    for (const auto& h : rq.headers) {
        hdr_name.push_back(h.first.c_str());
        hdr_src.push_back(h.second.c_str());
    }
    for (const std::string& o : rq.opts) opts.push_back(o.c_str());
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, rq.main_src.c_str(), "rtc_kernels_scene.hip", (int)hdr_src.size(), hdr_src.data(),
                            hdr_name.data()) != HIPRTC_SUCCESS) {
        std::fprintf(stderr, "hiprtcCreateProgram failed\n");
        return 1;
    }
    hiprtcAddNameExpression(prog, rq.name.c_str());
    const auto t0 = std::chrono::steady_clock::now();
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    if (r != HIPRTC_SUCCESS) {
        std::fprintf(stderr, "hiprtcCompileProgram: %s\n%s\n", hiprtcGetErrorString(r), log.c_str());
        hiprtcDestroyProgram(&prog);
        return 1;
    }
    CodeObject co;
    const char* lowered = nullptr;
    hiprtcGetLoweredName(prog, rq.name.c_str(), &lowered);
    co.lowered = lowered ? lowered : "";
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    co.code.resize(cs);
    if (cs) hiprtcGetCode(prog, co.code.data());
    hiprtcDestroyProgram(&prog);
    if (co.lowered.empty() || cs == 0) {
        std::fprintf(stderr, "hipRTC produced no kernel\n");
        return 1;
    }
    if (!write_code(argv[2], co)) {
        std::fprintf(stderr, "rtc_jitc: cannot write %s\n", argv[2]);
        return 1;
    }
    if (std::string dir; rtc::debug_knob("jit_dump", &dir)) {  // diagnostics: scene header + code object
        const std::string base = std::string(dir) + "/" +
                                 std::to_string(fnv(rq.headers.empty() ? "" : rq.headers[0].second.data(),
                                                    rq.headers.empty() ? 0 : rq.headers[0].second.size())) +
                                 (rq.name.find("pool") != std::string::npos ? "_pool" : "_direct");
        if (!rq.headers.empty()) write_atomic(base + ".hpp", rq.headers[0].second);
        write_atomic(base + ".co", std::string(co.code.data(), co.code.size()));
    }
    std::fprintf(stderr, "rtc_jitc: compiled %s in %.1f ms\n", rq.name.c_str(), ms);
    return 0;
}
