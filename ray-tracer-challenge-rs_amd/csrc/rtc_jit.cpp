// rtc_jit.cpp — per-scene builds of the f32 tracer kernels (hipRTC).
//
// The generic kernels walk the world's shape table with wave-uniform scalar
// loads: every shape of every ray costs a dependent s_load round trip, loop
// control and per-record branches.  For a large frame the
// library instead compiles, once per uploaded world, the same kernel source
// (embedded in librtc, rtc_kernels.hip) with the f32 shape table as a
// constexpr array and each kind's loop unrolled at compile time
// (rtc_kernels.hip `jit_each`): every record field becomes a constant of the
// instruction stream.  The arithmetic is the same source with the same
// operations on the same values, so frames are bit-identical to the generic
// kernel (tests/test_gpu_jit.py); only the f32 frame kernels are built this
// way (the f64 parity path, rt_color_at and small frames keep the generic
// kernels).  Builds are cached per process by table content (code objects)
// and device (loaded modules), and on disk by everything the compiler sees
// (source, scene header, options, the build's defines, hipRTC / HIP versions
// and the identity of librtc, libhiprtc and comgr), so a later process loads
// the code object instead of compiling it (RTC_JIT_CACHE: a directory, or 0
// for none; default $XDG_CACHE_HOME/rtc_jit or ~/.cache/rtc_jit).
//
// Off the frame's critical path (RT_JIT_AUTO, the default): the compile runs
// on a host thread; frames keep the generic kernel until it has landed, then
// the next frame loads the module and switches (same pixels either way).  A
// failed compile or module load keeps the generic kernel for that world; a
// build refused for occupancy or scratch keeps it for that variant only.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <dirent.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include "rtc_context.hpp"
#include "rtc_jit_sources.inc"  // kSrcKernels, kSrcInternal, kSrcRtcH (tools/embed_sources.py)

namespace rtc {
namespace {

std::string hexf(float v) {
    uint32_t b;
    std::memcpy(&b, &v, 4);
    char buf[48];
    std::snprintf(buf, sizeof buf, "__builtin_bit_cast(float, 0x%08xu)", b);
    return buf;
}

template <size_t N>
std::string floats(const float (&a)[N]) {
    std::string s = "{";
    for (size_t i = 0; i < N; ++i) s += (i ? ", " : "") + hexf(a[i]);
    return s + "}";
}

// rtc_jit_scene.hpp: the world's f32 shape table as constexpr data.
std::string scene_header(const std::vector<ShapeRec<float>>& sh, const int32_t begin[kNumKinds + 1]) {
    std::string s = "#pragma once\n#include \"rtc_internal.hpp\"\nnamespace rtc {\nnamespace jit {\n";
    s += "constexpr int kBegin[" + std::to_string(kNumKinds + 1) + "] = {";
    for (int k = 0; k <= kNumKinds; ++k) s += (k ? ", " : "") + std::to_string(begin[k]);
    s += "};\nconstexpr ShapeRec<float> kShapes[" + std::to_string(sh.size() + 1) + "] = {\n";
    for (const ShapeRec<float>& r : sh) {
        s += "    {" + floats(r.inv) + ", " + floats(r.bound) + ", " + std::to_string(r.world_index) + ", " +
             std::to_string(r.casts_shadow) + ", " + std::to_string(r.material) + ", " + std::to_string(r.flags) +
             ", " + hexf(r.ymin) + ", " + hexf(r.ymax) + ", " + floats(r.tri) + "},\n";
    }
    s += "    {}};\n}  // namespace jit\n}  // namespace rtc\n";
    return s;
}

uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

const char* kernel_name(bool pool, bool lds) {
    if (pool) return lds ? "rtc::trace_pool<float, true, false>" : "rtc::trace_pool<float, false, false>";
    return lds ? "rtc::trace_direct<float, true>" : "rtc::trace_direct<float, false>";
}

struct CodeObject {
    std::vector<char> code;
    std::string lowered;
    double compile_ms = 0;
    bool from_disk = false;
    uint64_t key = 0;  // the disk cache key (every input of the compile)
};

}  // namespace

// One per-scene kernel build: the code object of (world table, variant),
// compiled on a host thread (or in line for RT_JIT_SYNC) and shared by every
// context of the process that uploads the same world.
struct CodeBuild {
    std::atomic<int> state{0};  // 0 compiling, 1 ready, 2 failed
    CodeObject co;
    std::string log;
};

namespace {

// ------------------------------------------------------- on-disk code cache
// One file per build: "RTCJIT2\n" <lowered name> "\n" <code bytes> " "
// <FNV-1a of the code, hex> "\n" <code object>, named by a 64-bit FNV-1a of
// every input of the compile.  Written to a temporary name and renamed, so
// concurrent processes never read a partial file; a file whose length or
// checksum does not match is ignored and rebuilt (a damaged code object
// handed to hipModuleLoadData can abort the process instead of failing).
constexpr char kCacheMagic[] = "RTCJIT2\n";

std::string cache_dir() {
    const char* e = std::getenv("RTC_JIT_CACHE");
    if (e) return (!*e || !std::strcmp(e, "0")) ? std::string() : std::string(e);
    if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) return std::string(x) + "/rtc_jit";
    if (const char* h = std::getenv("HOME"); h && *h) return std::string(h) + "/.cache/rtc_jit";
    return std::string();
}

bool make_dirs(const std::string& d) {
    for (size_t p = 1; p <= d.size(); ++p) {
        if (p < d.size() && d[p] != '/') continue;
        const std::string part = d.substr(0, p);
        if (::mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
    return true;
}

std::string cache_path(const std::string& dir, uint64_t key) {
    char buf[32];
    std::snprintf(buf, sizeof buf, "/%016llx.co", (unsigned long long)key);
    return dir + buf;
}

bool cache_load(const std::string& path, CodeObject& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<char> all;
    char buf[1 << 16];
    for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) all.insert(all.end(), buf, buf + n);
    std::fclose(f);
    const size_t m = sizeof kCacheMagic - 1;
    if (all.size() < m || std::memcmp(all.data(), kCacheMagic, m)) return false;
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
    out.from_disk = true;
    return true;
}

void cache_store(const std::string& dir, const std::string& path, const CodeObject& co) {
    if (!make_dirs(dir)) return;
    static std::atomic<unsigned> seq{0};  // contexts of one process may build the same key at once
    const std::string tmp = path + ".tmp" + std::to_string((long long)::getpid()) + "." + std::to_string(seq++);
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return;
    bool ok = std::fwrite(kCacheMagic, 1, sizeof kCacheMagic - 1, f) == sizeof kCacheMagic - 1;
    ok = ok && std::fwrite(co.lowered.data(), 1, co.lowered.size(), f) == co.lowered.size();
    ok = ok && std::fprintf(f, "\n%llu %llx\n", (unsigned long long)co.code.size(),
                            (unsigned long long)fnv(co.code.data(), co.code.size())) > 0;
    ok = ok && std::fwrite(co.code.data(), 1, co.code.size(), f) == co.code.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

// Identity of a shared object: path, size and modification time.
uint64_t file_identity(const char* path, uint64_t h) {
    struct stat st;
    if (!path || ::stat(path, &st) != 0) return fnv("?", 1, h);
    h = fnv(path, std::strlen(path) + 1, h);
    const int64_t v[2] = {(int64_t)st.st_size, (int64_t)st.st_mtime};
    return fnv(v, sizeof v, h);
}

// The toolchain and library behind a build, for the disk cache key: hipRTC
// and HIP runtime versions, and the identity of librtc itself, of libhiprtc
// and of the comgr libraries next to it (the compiler proper), so a rebuilt
// librtc or an updated compiler within the same hipRTC minor version never
// loads code objects made by the old one.
uint64_t toolchain_identity() {
    static const uint64_t id = [] {
        uint64_t h = 1469598103934665603ull;
        int v[4] = {};
        hiprtcVersion(&v[0], &v[1]);
        (void)hipRuntimeGetVersion(&v[2]);
        (void)hipDriverGetVersion(&v[3]);
        h = fnv(v, sizeof v, h);
        Dl_info self{}, rtcc{};
        if (dladdr(reinterpret_cast<void*>(&toolchain_identity), &self)) h = file_identity(self.dli_fname, h);
        if (dladdr(reinterpret_cast<void*>(&hiprtcCompileProgram), &rtcc) && rtcc.dli_fname) {
            h = file_identity(rtcc.dli_fname, h);
            std::string dir(rtcc.dli_fname);
            dir = dir.substr(0, dir.find_last_of('/') + 1);
            if (DIR* d = ::opendir(dir.empty() ? "." : dir.c_str())) {
                std::vector<std::string> names;
                while (dirent* e = ::readdir(d))
                    if (std::strstr(e->d_name, "amd_comgr")) names.push_back(e->d_name);
                ::closedir(d);
                std::sort(names.begin(), names.end());
                for (const std::string& n : names) h = file_identity((dir + n).c_str(), h);
            }
        }
        return h;
    }();
    return id;
}

// Process-wide caches: builds by (table, kernel variant); loaded functions
// by (build, device).  Build threads are joined when librtc is unloaded (the
// registry is declared last, so it is destroyed first).
std::mutex g_mu;
std::condition_variable g_cv;  // a build finished
std::map<std::pair<uint64_t, int>, std::shared_ptr<CodeBuild>> g_code;
std::map<std::pair<uint64_t, int>, std::pair<hipModule_t, hipFunction_t>> g_fn;
struct BuildThreads {
    std::mutex mu;
    std::vector<std::thread> threads;
    ~BuildThreads() {
        std::lock_guard<std::mutex> lk(mu);
        for (std::thread& t : threads)
            if (t.joinable()) t.join();
    }
    void add(std::thread t) {
        std::lock_guard<std::mutex> lk(mu);
        threads.push_back(std::move(t));
    }
} g_threads;

// The static build's EXTRA flags (Makefile), passed on to hipRTC: -D/-U only.
std::vector<std::string> build_defines() {
    std::vector<std::string> out;
    const std::string all(kBuildExtra);
    for (size_t p = 0; p < all.size();) {
        size_t q = all.find_first_of(" \t\n", p);
        if (q == std::string::npos) q = all.size();
        const std::string tok = all.substr(p, q - p);
        if (tok.size() > 2 && tok[0] == '-' && (tok[1] == 'D' || tok[1] == 'U')) out.push_back(tok);
        p = q + 1;
    }
    return out;
}

int compile(const std::string& scene, const char* name, const std::string& arch, CodeObject& out, std::string& log,
            bool use_cache = true) {
    const std::string main_src = std::string("#define RTC_JIT 1\n#include \"rtc_jit_scene.hpp\"\n") + kSrcKernels;
    const char* headers[] = {scene.c_str(), kSrcInternal, kSrcRtcH};
    const char* names[] = {"rtc_jit_scene.hpp", "rtc_internal.hpp", "../../include/rtc.h"};
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, main_src.c_str(), "rtc_kernels_scene.hip", 3, headers, names) != HIPRTC_SUCCESS)
        return set_error(RT_ERR_HIP, "hiprtcCreateProgram failed");
    hiprtcAddNameExpression(prog, name);
    // The flags of the static build (Makefile): no contraction beyond the
    // source's explicit fmas, no SLP packing.  Plus no machine-level LICM:
    // with the records as constants it hoists their materialisations (and
    // values computed from them) out of the generation and tile loops, where
    // they are held across the loop and spill (reflect_refract's pool kernel:
    // 100 B/lane of scratch and 106 SGPRs with it, 8 B and 73 VGPRs without).
    // The device's own gfx target.  A build with defines of its own
    // (Makefile EXTRA: tuning macros, f32 math variants) passes all of them
    // on, so both builds run the same arithmetic and plan the same occupancy.
    const std::string arch_opt = "--offload-arch=" + arch;
    std::vector<const char*> opts = {arch_opt.c_str(),     "-O3",    "-std=c++20", "-ffp-contract=off",
                                     "-fno-slp-vectorize", "-mllvm", "-disable-machine-licm"};
    static const std::vector<std::string> defines = build_defines();
    for (const std::string& d : defines) opts.push_back(d.c_str());
    // The direct kernel fences the ray at every third shape only: the shape
    // tests in between may interleave (more ILP) and still fit 8 waves/SIMD
    // without spilling.  Same-box A/B against a fence per shape: shadow_puppets
    // -3.6 %, three_sphere 4K -2.5 %, 1080p -0.6 %; the pool kernel lost 15 %
    // on cover that way and keeps a fence per shape.
    if (!std::strstr(name, "pool")) opts.push_back("-DRTC_JIT_FENCE_EVERY=3");
    // RTC_JIT_FLAGS: extra compiler options, space-separated (A/B diagnostics)
    std::vector<std::string> extra;
    if (const char* e = std::getenv("RTC_JIT_FLAGS")) {
        std::string all(e);
        for (size_t p = 0; p < all.size();) {
            size_t q = all.find(' ', p);
            if (q == std::string::npos) q = all.size();
            if (q > p) extra.push_back(all.substr(p, q - p));
            p = q + 1;
        }
    }
    for (const std::string& x : extra) opts.push_back(x.c_str());
    // the disk cache key: every input of the compile, and the toolchain
    uint64_t key = fnv(main_src.data(), main_src.size());
    for (const char* h : headers) key = fnv(h, std::strlen(h) + 1, key);
    for (const char* o : opts) key = fnv(o, std::strlen(o) + 1, key);
    key = fnv(name, std::strlen(name) + 1, key);
    const uint64_t tool = toolchain_identity();
    key = fnv(&tool, sizeof tool, key);
    out.key = key;
    const std::string dir = cache_dir();
    const std::string path = dir.empty() || !use_cache ? std::string() : cache_path(dir, key);
    if (!path.empty()) {
        const auto c0 = std::chrono::steady_clock::now();
        if (cache_load(path, out)) {
            hiprtcDestroyProgram(&prog);
            out.compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
            return RT_OK;
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    out.compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    log.assign(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    int rc = RT_OK;
    if (r != HIPRTC_SUCCESS) {
        rc = set_error(RT_ERR_HIP, std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(r) + "\n" + log);
    } else {
        const char* lowered = nullptr;
        hiprtcGetLoweredName(prog, name, &lowered);
        out.lowered = lowered ? lowered : "";
        size_t cs = 0;
        hiprtcGetCodeSize(prog, &cs);
        out.code.resize(cs);
        hiprtcGetCode(prog, out.code.data());
        if (out.lowered.empty() || cs == 0) rc = set_error(RT_ERR_HIP, "hipRTC produced no kernel");
        else if (!path.empty()) cache_store(dir, path, out);
        if (const char* dir = std::getenv("RTC_JIT_DUMP")) {  // diagnostics: scene header + code object
            const std::string base = std::string(dir) + "/" + std::to_string(fnv(scene.data(), scene.size())) + "_" +
                                     (std::strstr(name, "pool") ? "pool" : "direct");
            if (FILE* f = std::fopen((base + ".hpp").c_str(), "w")) {
                std::fwrite(scene.data(), 1, scene.size(), f);
                std::fclose(f);
            }
            if (FILE* f = std::fopen((base + ".co").c_str(), "wb")) {
                std::fwrite(out.code.data(), 1, out.code.size(), f);
                std::fclose(f);
            }
        }
    }
    hiprtcDestroyProgram(&prog);
    return rc;
}

// Compile one build (host thread or in line) and publish it.
void run_build(std::shared_ptr<CodeBuild> b, std::string scene, std::string name, std::string arch) {
    std::string log;
    const int rc = compile(scene, name.c_str(), arch, b->co, log);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (rc) b->log = std::string(rt_last_error());
        b->state.store(rc ? 2 : 1, std::memory_order_release);
    }
    g_cv.notify_all();
}

}  // namespace

// The per-scene kernel for this context's uploaded world, or null (use the
// generic kernel this launch).  RT_JIT_SYNC compiles in line; RT_JIT_AUTO /
// RT_JIT_EAGER start the compile on a host thread at the 2nd / 1st large
// frame of an upload and return null until it has landed.
int jit_function(rt_context* ctx, bool pool, bool lds, size_t dyn_lds, int static_blocks, hipFunction_t* fn) {
    *fn = nullptr;
    if (ctx->jit_failed || ctx->jit_shapes.empty()) return RT_OK;
    const int variant = (pool ? 2 : 0) + (lds ? 1 : 0);
    if (ctx->jit_fn[variant]) {
        *fn = ctx->jit_fn[variant];
        return RT_OK;
    }
    if (ctx->jit_rejected[variant]) return RT_OK;
    std::shared_ptr<CodeBuild>& b = ctx->jit_build[variant];
    if (!b) {
        const uint64_t key = fnv(ctx->jit_begin, sizeof ctx->jit_begin,
                                 fnv(ctx->jit_shapes.data(), ctx->jit_shapes.size() * sizeof(ShapeRec<float>)));
        const bool sync = ctx->jit_mode == RT_JIT_SYNC;
        const uint32_t start_at = ctx->jit_mode == RT_JIT_AUTO ? 2 : 1;
        bool start = false;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            auto it = g_code.find({key, variant});
            if (it != g_code.end()) {
                b = it->second;  // built (or building, or failed) for another context or an earlier upload
            } else if (sync || ctx->jit_frames >= start_at) {
                b = std::make_shared<CodeBuild>();
                g_code[{key, variant}] = b;
                start = true;
            }
        }
        if (!b) return RT_OK;
        if (start) {
            ctx->jit_owner[variant] = true;
            std::string scene = scene_header(ctx->jit_shapes, ctx->jit_begin);
            if (sync) {
                run_build(b, std::move(scene), kernel_name(pool, lds), ctx->arch);
            } else {
                try {
                    g_threads.add(std::thread(run_build, b, std::move(scene), std::string(kernel_name(pool, lds)),
                                              ctx->arch));
                } catch (const std::exception& e) {  // no thread: build in line instead
                    run_build(b, scene_header(ctx->jit_shapes, ctx->jit_begin), kernel_name(pool, lds), ctx->arch);
                }
            }
        }
    }
    if (ctx->jit_mode == RT_JIT_SYNC) {  // wait for a build another context started
        std::unique_lock<std::mutex> lk(g_mu);
        g_cv.wait(lk, [&] { return b->state.load() != 0; });
    }
    const int state = b->state.load(std::memory_order_acquire);
    if (state == 0) return RT_OK;  // still compiling: the generic kernel this frame
    if (ctx->jit_owner[variant]) {
        ctx->jit_compile_ms += b->co.compile_ms;
        if (b->co.from_disk) ++ctx->jit_cache_hits;
        ctx->jit_owner[variant] = false;
    }
    if (state == 2) {
        ctx->jit_failed = true;  // keep the generic kernel for this world
        ctx->jit_log = b->log;
        return RT_OK;
    }
    std::pair<hipModule_t, hipFunction_t> mf{};
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_fn.find({(uint64_t)(uintptr_t)b.get(), ctx->device});
        if (it != g_fn.end()) mf = it->second;
    }
    if (!mf.second) {
        // a code object the device cannot load (another target, a damaged
        // build) fails like a failed compile: the generic kernel, not an error
        RT_HIP(hipSetDevice(ctx->device));
        hipError_t e = hipModuleLoadData(&mf.first, b->co.code.data());
        if (e == hipSuccess) {
            e = hipModuleGetFunction(&mf.second, mf.first, b->co.lowered.c_str());
            if (e != hipSuccess) {
                (void)hipModuleUnload(mf.first);
                mf = {};
            }
        }
        if (e != hipSuccess) {
            (void)hipGetLastError();
            ctx->jit_failed = true;
            ctx->jit_log = std::string("per-scene kernel not loaded (") + ctx->arch + "): " + hipGetErrorString(e);
            return RT_OK;
        }
        std::lock_guard<std::mutex> lk(g_mu);
        auto ins = g_fn.emplace(std::make_pair((uint64_t)(uintptr_t)b.get(), ctx->device), mf);
        if (!ins.second) {  // another context of this device loaded it meanwhile
            (void)hipModuleUnload(mf.first);
            mf = ins.first->second;
        }
    }
    // The launch is planned with the generic kernel's occupancy: use the
    // per-scene kernel only if it keeps at least as many workgroups per CU,
    // and only if it spills at most a few values (direct: none; pool:
    // 16 B/lane, e.g. cylinders: 12 B/lane, values reloaded once per tile,
    // 0.15 ms against 0.19 ms for the generic kernel).  A build with real
    // spills ran slower than the generic kernel (shadow_puppets before the
    // ray fence: 56 B/lane, +10 %).  A refusal holds for this variant only.
    int blocks = 0, scratch = 0;
    RT_HIP(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mf.second, kBlock, dyn_lds));
    RT_HIP(hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, mf.second));
    if (blocks < static_blocks || scratch > (pool ? 16 : 0)) {
        ctx->jit_rejected[variant] = true;
        ctx->jit_log = std::string("per-scene ") + (pool ? "pool" : "direct") + " kernel not used: " +
                       std::to_string(blocks) + " workgroups/CU (generic " + std::to_string(static_blocks) + "), " +
                       std::to_string(scratch) + " B/lane of scratch";
        return RT_OK;
    }
    ctx->jit_fn[variant] = mf.second;
    *fn = mf.second;
    return RT_OK;
}

// Block until this context's builds in flight have finished (rt_jit_wait).
int jit_wait(rt_context* ctx, double timeout_ms, int* pending) {
    const auto deadline = std::chrono::steady_clock::now() +
                          std::chrono::microseconds((int64_t)(timeout_ms < 0 ? 3.6e9 * 1e3 : timeout_ms * 1e3));
    auto left = [ctx] {
        int n = 0;
        for (const auto& b : ctx->jit_build) n += b && b->state.load() == 0;
        return n;
    };
    std::unique_lock<std::mutex> lk(g_mu);
    g_cv.wait_until(lk, deadline, [&] { return left() == 0; });
    if (pending) *pending = left();
    return RT_OK;
}

}  // namespace rtc
