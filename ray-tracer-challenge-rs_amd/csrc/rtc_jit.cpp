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
// kernels).
//
// The compile runs in a child process (rtc_jitc, next to librtc.so; env
// RTC_JITC overrides), never on a thread of the render process: a hipRTC
// compile on a thread raced the host's exit (rtc_jitc.cpp).  RT_JIT_AUTO
// (the default) starts it at a world's second large frame and keeps the
// generic kernel until it has landed; a thread of this process only waits
// for the child (pipe + waitpid) and is detached, so nothing ever has to be
// joined.  Builds are cached per process by table content (code objects) and
// device (loaded modules), and on disk by everything the compiler sees
// (source, scene header, options including the build's own defines, and the
// toolchain: hipRTC / HIP versions and the identity of librtc, libhiprtc and
// comgr), so a later process loads the code object instead of compiling it
// (RTC_JIT_CACHE: a directory, or 0 for none; default $XDG_CACHE_HOME/rtc_jit
// or ~/.cache/rtc_jit).  A failed compile or module load keeps the generic
// kernel for that world; a build refused for occupancy or scratch keeps it
// for that variant only.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
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
#include <fcntl.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include "debug_knobs.hpp"
#include "jit_options.hpp"
#include "rtc_context.hpp"
#include "rtc_jit_cache.hpp"
#include "rtc_jit_sources.inc"  // kSrcKernels, kSrcInternal, kSrcRtcH, kBuildExtra (tools/embed_sources.py)

extern char** environ;

namespace rtc {

// One per-scene kernel build: the code object of (world table, variant),
// compiled by a child process and shared by every context of the process
// that uploads the same world.
struct CodeBuild {
    std::atomic<int> state{0};  // 0 compiling, 1 ready, 2 failed
    jitfile::CodeObject co;
    std::string log;
    double ms = 0;              // compile (child process wall time) or disk-cache load
    bool from_disk = false;
};

namespace {

using jitfile::fnv;

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
std::string ball4(const float* a) {  // a cluster ball: 4 floats
    std::string s = "{";
    for (size_t i = 0; i < 4; ++i) s += (i ? ", " : "") + hexf(a[i]);
    return s + "}";
}

// Clusters of the world's bounded shapes for the per-scene kernels' two-level
// wave cull (rtc_kernels.hip for_all_culled): a wave that meets no lane's ray
// with a cluster's ball skips all its members' tests.  k-means on the bound
// centres (farthest-point seeds: deterministic; k from 2 to 8 by the cost
// model below), each cluster's ball enclosing its members' padded balls.
// Worlds of fewer than kClusterMinShapes bounded shapes get none
// (RTC_DEBUG=jit_clusters=0: never; =k: k clusters, for sweeps; =1: one cluster of
// every bounded shape, from two shapes on).
constexpr int kClusterMinShapes = 6;
struct Clusters {
    std::vector<std::array<float, 4>> ball;  // centre, radius^2
    std::vector<int> begin, members, unclustered;
};
Clusters make_clusters(const std::vector<ShapeRec<float>>& sh) {
    Clusters c;
    std::vector<int> bounded;
    for (int i = 0; i < (int)sh.size(); ++i) {
        const float r2 = sh[i].bound[3];
        if (std::isfinite(r2) && r2 >= 0.0f) bounded.push_back(i);
        else c.unclustered.push_back(i);
    }
    std::string knob;  // RTC_DEBUG=jit_clusters=N
    const char* e = debug_knob("jit_clusters", &knob) ? knob.c_str() : nullptr;
    const int n = (int)bounded.size();
    auto flat = [&]() {
        c.unclustered.insert(c.unclustered.end(), bounded.begin(), bounded.end());
        std::sort(c.unclustered.begin(), c.unclustered.end());
        c.ball.clear();
        c.members.clear();
        c.begin = {0};
        return c;
    };
    const int forced = e ? std::atoi(e) : 0;
    if ((n < kClusterMinShapes && !(forced >= 1 && n >= 2)) || (e && !std::strcmp(e, "0"))) return flat();
    using P3 = std::array<double, 3>;
    auto ctr = [&](int i) { return P3{sh[i].bound[0], sh[i].bound[1], sh[i].bound[2]}; };
    auto rad = [&](int i) { return std::sqrt((double)sh[i].bound[3]); };
    auto d2 = [](const P3& a, const P3& b) {
        return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
    };
    struct Cl {
        P3 cent;
        double r;
        std::vector<int> m;
    };
    auto kmeans = [&](int k) {
        std::vector<P3> cent{ctr(bounded[0])};
        while ((int)cent.size() < k) {  // farthest point from the seeds so far
            int far = bounded[0];
            double best = -1.0;
            for (int i : bounded) {
                double m = 1e300;
                for (const auto& q : cent) m = std::min(m, d2(ctr(i), q));
                if (m > best) best = m, far = i;
            }
            cent.push_back(ctr(far));
        }
        std::vector<int> lab(n, 0);
        for (int it = 0; it < 32; ++it) {
            for (int j = 0; j < n; ++j) {
                double m = 1e300;
                for (int q = 0; q < k; ++q)
                    if (const double v = d2(ctr(bounded[j]), cent[q]); v < m) m = v, lab[j] = q;
            }
            for (int q = 0; q < k; ++q) {
                P3 sum{0, 0, 0};
                int cnt = 0;
                for (int j = 0; j < n; ++j)
                    if (lab[j] == q) {
                        const P3 a = ctr(bounded[j]);
                        for (int t = 0; t < 3; ++t) sum[t] += a[t];
                        ++cnt;
                    }
                if (cnt) cent[q] = {sum[0] / cnt, sum[1] / cnt, sum[2] / cnt};
            }
        }
        std::vector<Cl> out;
        for (int q = 0; q < k; ++q) {
            Cl cl{cent[q], 0.0, {}};
            for (int j = 0; j < n; ++j)
                if (lab[j] == q) {
                    cl.m.push_back(bounded[j]);
                    cl.r = std::max(cl.r, std::sqrt(d2(ctr(bounded[j]), cent[q])) + rad(bounded[j]));
                }
            if (!cl.m.empty()) out.push_back(cl);
        }
        return out;
    };
    // k by a cost model: per ray, one ball test per cluster plus, for each
    // cluster a ray meets ((cluster radius / world radius)^2), its members at
    // twice a ball test each (a member's own cull, then its exact test for
    // some); no clusters unless that beats every shape's test by 20 %.  The
    // weight 2 picks the best measured k on the reference scenes (same-box
    // sweeps of k): reflect_refract 3, cover 5, table 6.
    P3 mid{0, 0, 0};
    for (int i : bounded)
        for (int t = 0; t < 3; ++t) mid[t] += ctr(i)[t] / n;
    double world = 0.0;
    for (int i : bounded) world = std::max(world, std::sqrt(d2(ctr(i), mid)) + rad(i));
    constexpr double kMemberWeight = 2.0;
    // k-means groups by centre only; a local search then moves single shapes
    // between clusters while that lowers the model's cost (sum over clusters of
    // members x radius^2), which k-means cannot see: a large shape pulls its
    // cluster's ball wide (RTC_DEBUG=jit_cluster_refine=0: k-means only)
    std::string rknob;  // RTC_DEBUG=jit_cluster_refine=0
    const char* rf = debug_knob("jit_cluster_refine", &rknob) ? rknob.c_str() : nullptr;
    // (quadratic per move: worlds of at most 64 bounded shapes; k-means alone
    // beyond, which stays O(n k) per iteration)
    const bool refine = !(rf && !std::strcmp(rf, "0")) && n <= 64;
    auto ball_of = [&](Cl& q) {
        q.cent = {0, 0, 0};
        for (int i : q.m)
            for (int t = 0; t < 3; ++t) q.cent[t] += ctr(i)[t] / (double)q.m.size();
        q.r = 0.0;
        for (int i : q.m) q.r = std::max(q.r, std::sqrt(d2(ctr(i), q.cent)) + rad(i));
    };
    auto term = [&](const Cl& q) { return (double)q.m.size() * q.r * q.r; };
    auto refine_clusters = [&](std::vector<Cl>& cl) {
        for (int guard = 0; guard < 256; ++guard) {
            double best_gain = 1e-9 * world * world;
            int ba = -1, bs = -1, bb = -1;
            for (int a = 0; a < (int)cl.size(); ++a) {
                if (cl[a].m.size() < 2) continue;
                for (int si = 0; si < (int)cl[a].m.size(); ++si)
                    for (int b = 0; b < (int)cl.size(); ++b) {
                        if (b == a) continue;
                        Cl na = cl[a], nb = cl[b];
                        na.m.erase(na.m.begin() + si);
                        nb.m.push_back(cl[a].m[si]);
                        ball_of(na);
                        ball_of(nb);
                        const double gain = term(cl[a]) + term(cl[b]) - term(na) - term(nb);
                        if (gain > best_gain) best_gain = gain, ba = a, bs = si, bb = b;
                    }
            }
            if (ba < 0) break;
            cl[bb].m.push_back(cl[ba].m[bs]);
            cl[ba].m.erase(cl[ba].m.begin() + bs);
            ball_of(cl[ba]);
            ball_of(cl[bb]);
        }
        for (Cl& q : cl) std::sort(q.m.begin(), q.m.end());
    };
    std::vector<Cl> best;
    double best_cost = 0.8 * kMemberWeight * n;
    for (int k = forced == 1 ? 1 : 2; k <= std::min(8, n - 1); ++k) {
        if (forced >= 1 && k != std::min(forced, n - 1)) continue;
        std::vector<Cl> cl = kmeans(k);
        if (refine) refine_clusters(cl);
        double cost = (double)cl.size();
        for (const Cl& q : cl) cost += kMemberWeight * (double)q.m.size() * std::min(1.0, (q.r / world) * (q.r / world));
        if (cost < best_cost || forced >= 1) best_cost = cost, best = std::move(cl);
    }
    if (best.empty()) return flat();
    c.begin.push_back(0);
    for (const Cl& q : best) {
        c.members.insert(c.members.end(), q.m.begin(), q.m.end());
        const double pad = 1e-4 * (q.r + std::fabs(q.cent[0]) + std::fabs(q.cent[1]) + std::fabs(q.cent[2])) + 1e-4;
        c.ball.push_back({(float)q.cent[0], (float)q.cent[1], (float)q.cent[2], (float)((q.r + pad) * (q.r + pad))});
        c.begin.push_back((int)c.members.size());
    }
    return c;
}

// rtc_jit_scene.hpp: the world's f32 shape table, its lights and whether any
// material has a pattern, as constexpr data.
std::string scene_header(const std::vector<ShapeRec<float>>& sh, const int32_t begin[kNumKinds + 1],
                         const std::vector<LightRec<float>>& lights, const std::vector<MaterialRec<float>>& mats,
                         bool patterns, uint32_t pattern_kinds, bool transparent) {
    std::string s = "#pragma once\n#include \"rtc_internal.hpp\"\nnamespace rtc {\nnamespace jit {\n";
    s += "constexpr int kBegin[" + std::to_string(kNumKinds + 1) + "] = {";
    for (int k = 0; k <= kNumKinds; ++k) s += (k ? ", " : "") + std::to_string(begin[k]);
    s += "};\nconstexpr ShapeRec<float> kShapes[" + std::to_string(sh.size() + 1) + "] = {\n";
    for (const ShapeRec<float>& r : sh) {
        s += "    {" + floats(r.inv) + ", " + floats(r.bound) + ", " + std::to_string(r.world_index) + ", " +
             std::to_string(r.casts_shadow) + ", " + std::to_string(r.material) + ", " + std::to_string(r.flags) +
             ", " + hexf(r.ymin) + ", " + hexf(r.ymax) + ", " + floats(r.tri) + "},\n";
    }
    s += "    {}};\n";
    const Clusters cl = make_clusters(sh);
    auto ints = [](const std::vector<int>& v) {
        std::string o = "{";
        for (size_t i = 0; i < v.size(); ++i) o += (i ? ", " : "") + std::to_string(v[i]);
        return o + (v.empty() ? "0}" : "}");
    };
    s += "constexpr int kNumClusters = " + std::to_string(cl.ball.size()) + ";\n";
    s += "constexpr float kClusterBall[" + std::to_string(cl.ball.size() + 1) + "][4] = {\n";
    for (const auto& b : cl.ball) s += "    " + ball4(b.data()) + ",\n";
    s += "    {}};\n";
    s += "constexpr int kClusterBegin[" + std::to_string(cl.begin.size()) + "] = " + ints(cl.begin) + ";\n";
    s += "constexpr int kClusterMembers[" + std::to_string(std::max<size_t>(1, cl.members.size())) + "] = " +
         ints(cl.members) + ";\n";
    s += "constexpr int kNumUnclustered = " + std::to_string(cl.unclustered.size()) + ";\n";
    s += "constexpr int kUnclustered[" + std::to_string(std::max<size_t>(1, cl.unclustered.size())) + "] = " +
         ints(cl.unclustered) + ";\n";
    s += "constexpr int kNumLights = " + std::to_string(lights.size()) + ";\n";
    s += "constexpr LightRec<float> kLights[" + std::to_string(lights.size() + 1) + "] = {\n";
    for (const LightRec<float>& l : lights) s += "    {" + floats(l.position) + ", " + floats(l.intensity) + "},\n";
    s += "    {}};\n";
    s += "constexpr MaterialRec<float> kMaterials[" + std::to_string(mats.size() + 1) + "] = {\n";
    for (const MaterialRec<float>& m : mats) {
        s += "    {" + floats(m.color) + ", " + hexf(m.ambient) + ", " + hexf(m.diffuse) + ", " + hexf(m.specular) + ", " +
             hexf(m.shininess) + ", " + hexf(m.reflectiveness) + ", " + hexf(m.transparency) + ", " +
             hexf(m.refractive_index) + ", " + std::to_string(m.pattern) + ", " + std::to_string(m.casts_shadow) + "},\n";
    }
    s += "    {}};\n";
    s += std::string("constexpr bool kPatterns = ") + (patterns ? "true" : "false") + ";\n";
    s += "constexpr uint32_t kPatternKinds = " + std::to_string(pattern_kinds) + "u;\n";
    s += std::string("constexpr bool kTransparent = ") + (transparent ? "true" : "false") + ";\n";
    s += "}  // namespace jit\n}  // namespace rtc\n";
    return s;
}

const char* kernel_name(bool pool, bool lds) {
    if (pool) return lds ? "rtc::trace_pool<float, true, false>" : "rtc::trace_pool<float, false, false>";
    return lds ? "rtc::trace_direct<float, true>" : "rtc::trace_direct<float, false>";
}

// Identity of a file: path, size and modification time.
uint64_t file_identity(const char* path, uint64_t h) {
    struct stat st;
    if (!path || ::stat(path, &st) != 0) return fnv("?", 1, h);
    h = fnv(path, std::strlen(path) + 1, h);
    const int64_t v[2] = {(int64_t)st.st_size, (int64_t)st.st_mtime};
    return fnv(v, sizeof v, h);
}

std::string librtc_dir() {
    Dl_info self{};
    if (!dladdr(reinterpret_cast<void*>(&scene_header), &self) || !self.dli_fname) return ".";
    std::string p(self.dli_fname);
    const size_t slash = p.find_last_of('/');
    return slash == std::string::npos ? "." : p.substr(0, slash);
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
        if (dladdr(reinterpret_cast<void*>(&scene_header), &self)) h = file_identity(self.dli_fname, h);
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

// Everything the compiler sees for one build, and the key naming it.
jitfile::Request make_request(const std::string& scene, const char* name, const std::string& arch, uint64_t* key,
                              bool no_skips, int pool_waves) {
    jitfile::Request rq;
    rq.name = name;
    rq.main_src = std::string("#define RTC_JIT 1\n#include \"rtc_jit_scene.hpp\"\n") + kSrcKernels;
    rq.headers = {{"rtc_jit_scene.hpp", scene}, {"rtc_internal.hpp", kSrcInternal}, {"../../include/rtc.h", kSrcRtcH}};
    // The flags of the static build (Makefile): no contraction beyond the
    // source's explicit fmas, no SLP packing.  Plus no machine-level LICM:
    // with the records as constants it hoists their materialisations (and
    // values computed from them) out of the generation and tile loops, where
    // they are held across the loop and spill (reflect_refract's pool kernel:
    // 100 B/lane of scratch and 106 SGPRs with it, 8 B and 73 VGPRs without).
    // The device's own gfx target.  A build with defines of its own (Makefile
    // EXTRA: tuning macros, f32 math variants) passes all of them on, so both
    // builds run the same arithmetic and plan the same occupancy.
    rq.opts = {"--offload-arch=" + arch, "-O3", "-std=c++20", "-ffp-contract=off", "-fno-slp-vectorize", "-mllvm",
               "-disable-machine-licm"};
    static const std::vector<std::string> defines = build_defines();
    rq.opts.insert(rq.opts.end(), defines.begin(), defines.end());
    // per kind: fence spacing, records as constants, the no-skips build
    const auto kind = jit_kind_defines(std::strstr(name, "pool") != nullptr, no_skips, pool_waves);
    rq.opts.insert(rq.opts.end(), kind.begin(), kind.end());
    // RTC_DEBUG=jit_flags=...: extra compiler options, space-separated (A/B diagnostics)
    if (std::string all; debug_knob("jit_flags", &all)) {
        for (size_t p = 0; p < all.size();) {
            size_t q = all.find_first_of(" ,", p);
            if (q == std::string::npos) q = all.size();
            if (q > p) rq.opts.push_back(all.substr(p, q - p));
            p = q + 1;
        }
    }
    uint64_t k = fnv(rq.main_src.data(), rq.main_src.size());
    for (const auto& h : rq.headers) k = fnv(h.second.data(), h.second.size() + 1, fnv(h.first.data(), h.first.size() + 1, k));
    for (const std::string& o : rq.opts) k = fnv(o.data(), o.size() + 1, k);
    k = fnv(rq.name.data(), rq.name.size() + 1, k);
    const uint64_t tool = toolchain_identity();
    *key = fnv(&tool, sizeof tool, k);
    return rq;
}

std::string cache_dir() {
    const char* e = std::getenv("RTC_JIT_CACHE");
    if (e) return (!*e || !std::strcmp(e, "0")) ? std::string() : std::string(e);
    if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) return std::string(x) + "/rtc_jit";
    if (const char* h = std::getenv("HOME"); h && *h) return std::string(h) + "/.cache/rtc_jit";
    return std::string();
}

std::string cache_path(const std::string& dir, uint64_t key) {
    char buf[32];
    std::snprintf(buf, sizeof buf, "/%016llx.co", (unsigned long long)key);
    return dir + buf;
}

std::string temp_path(const char* suffix) {
    static std::atomic<unsigned> seq{0};
    const char* t = std::getenv("TMPDIR");
    return std::string(t && *t ? t : "/tmp") + "/rtcjit-" + std::to_string((long long)::getpid()) + "-" +
           std::to_string(seq++) + suffix;
}

// Process-wide state, never destroyed: build waiters are detached threads
// and may still run while the process exits.
std::mutex& g_mu = *new std::mutex;
std::condition_variable& g_cv = *new std::condition_variable;  // a build finished
auto& g_code = *new std::map<std::pair<uint64_t, int>, std::shared_ptr<CodeBuild>>;   // (table, variant)
auto& g_fn = *new std::map<std::pair<uint64_t, int>, std::pair<hipModule_t, hipFunction_t>>;  // (build, device)

void finish(const std::shared_ptr<CodeBuild>& b, bool ok, std::string log) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        b->log = std::move(log);
        b->state.store(ok ? 1 : 2, std::memory_order_release);
    }
    g_cv.notify_all();
}

// Wait for the compiler process (its output through `fd` until EOF, then its
// status), load what it wrote to `out`, publish the build.
void await_child(std::shared_ptr<CodeBuild> b, pid_t pid, int fd, std::string out, bool temp_out,
                 std::chrono::steady_clock::time_point t0) {
    std::string log;
    char buf[4096];
    for (;;) {
        const ssize_t n = ::read(fd, buf, sizeof buf);
        if (n > 0) {
            if (log.size() < (1u << 20)) log.append(buf, (size_t)n);
        } else if (n < 0 && errno == EINTR) {
            continue;
        } else {
            break;
        }
    }
    ::close(fd);
    int status = 0;
    pid_t w;
    do {
        w = ::waitpid(pid, &status, 0);
    } while (w < 0 && errno == EINTR);
    // a host that reaps children itself (SIGCHLD ignored): judge by the output
    const bool exited_ok = w < 0 ? true : (WIFEXITED(status) && WEXITSTATUS(status) == 0);
    const bool ok = exited_ok && jitfile::read_code(out, b->co);
    if (temp_out) std::remove(out.c_str());
    b->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (!ok && log.empty()) log = "rtc_jitc failed (status " + std::to_string(status) + ")";
    finish(b, ok, ok ? std::string() : "per-scene build failed: " + log);
}

// Start one build: from the disk cache at once, or by a compiler process
// (waited for in line when `sync`, else by a detached thread).
void start_build(const std::shared_ptr<CodeBuild>& b, const jitfile::Request& rq, uint64_t key, bool sync) {
    const auto t0 = std::chrono::steady_clock::now();
    const std::string dir = cache_dir();
    const std::string path = dir.empty() ? std::string() : cache_path(dir, key);
    if (!path.empty() && jitfile::read_code(path, b->co)) {
        b->from_disk = true;
        b->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        finish(b, true, std::string());
        return;
    }
    const char* env_helper = std::getenv("RTC_JITC");
    const std::string helper = env_helper && *env_helper ? env_helper : librtc_dir() + "/rtc_jitc";
    if (::access(helper.c_str(), X_OK) != 0) {
        finish(b, false, "per-scene build: compiler " + helper + " not found (the generic kernel is used)");
        return;
    }
    const std::string req = temp_path(".req");
    const bool temp_out = path.empty();
    const std::string out = temp_out ? temp_path(".co") : path;
    if (!jitfile::write_request(req, rq)) {
        finish(b, false, "per-scene build: cannot write " + req);
        return;
    }
    int fds[2];
    if (::pipe2(fds, O_CLOEXEC) != 0) {
        std::remove(req.c_str());
        finish(b, false, std::string("per-scene build: pipe: ") + std::strerror(errno));
        return;
    }
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, fds[1], 1);
    posix_spawn_file_actions_adddup2(&fa, fds[1], 2);
    std::vector<char*> argv = {const_cast<char*>(helper.c_str()), const_cast<char*>(req.c_str()),
                               const_cast<char*>(out.c_str()), nullptr};
    pid_t pid = 0;
    const int e = posix_spawn(&pid, helper.c_str(), &fa, nullptr, argv.data(), environ);
    posix_spawn_file_actions_destroy(&fa);
    ::close(fds[1]);
    if (e != 0) {
        ::close(fds[0]);
        std::remove(req.c_str());
        finish(b, false, std::string("per-scene build: cannot start ") + helper + ": " + std::strerror(e));
        return;
    }
    if (sync) {
        await_child(b, pid, fds[0], out, temp_out, t0);
        return;
    }
    try {
        std::thread(await_child, b, pid, fds[0], out, temp_out, t0).detach();
    } catch (const std::exception&) {  // no thread: wait in line instead
        await_child(b, pid, fds[0], out, temp_out, t0);
    }
}

}  // namespace

// The device's gfx target ("gfx950:sramecc+:xnack-" -> "gfx950"), the
// per-scene builds' --offload-arch: read at the first build, not at context
// creation (hipGetDeviceProperties fills the whole struct).
const std::string& device_arch(rt_context* ctx) {
    if (ctx->arch.empty()) {
        hipDeviceProp_t prop;
        if (hipSetDevice(ctx->device) == hipSuccess && hipGetDeviceProperties(&prop, ctx->device) == hipSuccess) {
            const std::string a(prop.gcnArchName);
            ctx->arch = a.empty() ? std::string("gfx950") : a.substr(0, a.find(':'));
        } else {
            ctx->arch = "gfx950";
        }
    }
    return ctx->arch;
}

// The per-scene kernel for this context's uploaded world, or null (use the
// generic kernel this launch).  RT_JIT_SYNC builds in line; RT_JIT_AUTO /
// RT_JIT_EAGER start the build at the 2nd / 1st large frame of an upload and
// return null until it has landed.
// Scratch a 7-wave per-scene pool build may use (B/lane): the workgroup
// it gains outweighs up to this much spilling.  Same box, 7-wave build vs
// the 6-wave one: cover 4K (36 B/lane) 0.657 -> 0.629 ms, reflect_refract
// and table (16) -2.4 % / -3.6 %; cylinders (44) +4 % (refused).
constexpr int kPool7ScratchMax = 40;

namespace {
// One variant's build: *fn stays null while it compiles, if it failed or if
// it was refused (jit_rejected[variant]).
// start_only: make sure the build runs (in the background even in
// RT_JIT_SYNC mode) and return without waiting for it or taking it.
// scratch_max: the B/lane of scratch a pool build may use (direct: none).
int jit_variant(rt_context* ctx, int variant, bool pool, bool lds, size_t dyn_lds, int static_blocks,
                hipFunction_t* fn, bool no_skips, int pool_waves, int scratch_max, bool start_only = false) {
    *fn = nullptr;
    if (ctx->jit_fn[variant]) {
        *fn = ctx->jit_fn[variant];
        return RT_OK;
    }
    if (ctx->jit_rejected[variant]) return RT_OK;
    const bool sync = ctx->jit_mode == RT_JIT_SYNC;
    std::shared_ptr<CodeBuild>& b = ctx->jit_build[variant];
    if (!b) {
        uint64_t table = fnv(ctx->jit_begin, sizeof ctx->jit_begin,
                             fnv(ctx->jit_shapes.data(), ctx->jit_shapes.size() * sizeof(ShapeRec<float>)));
        table = fnv(ctx->jit_lights.data(), ctx->jit_lights.size() * sizeof(LightRec<float>), table);
        table = fnv(ctx->jit_materials.data(), ctx->jit_materials.size() * sizeof(MaterialRec<float>), table);
        const uint32_t traits[3] = {ctx->jit_patterns, ctx->jit_pattern_kinds, ctx->jit_transparent};
        table = fnv(traits, sizeof traits, table);
        // the device's gfx target: each build is compiled for one (make_request),
        // so devices of another target in the same process get builds of their own
        const std::string& arch = device_arch(ctx);
        table = fnv(arch.data(), arch.size() + 1, table);
        const uint32_t start_at = ctx->jit_mode == RT_JIT_AUTO ? 2 : 1;
        bool start = false;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            auto it = g_code.find({table, variant});
            if (it != g_code.end()) {
                b = it->second;  // built (or building, or failed) for another context or an earlier upload
            } else if (sync || ctx->jit_frames >= start_at) {
                b = std::make_shared<CodeBuild>();
                g_code[{table, variant}] = b;
                start = true;
            }
        }
        if (!b) return RT_OK;
        if (start) {
            ctx->jit_owner[variant] = true;
            uint64_t key = 0;
            const jitfile::Request rq =
                make_request(scene_header(ctx->jit_shapes, ctx->jit_begin, ctx->jit_lights, ctx->jit_materials,
                                          ctx->jit_patterns,
                                          ctx->jit_pattern_kinds, ctx->jit_transparent),
                             kernel_name(pool, lds), device_arch(ctx), &key, no_skips, pool_waves);
            start_build(b, rq, key, sync && !start_only);
        }
    }
    if (start_only) return RT_OK;
    if (sync) {  // a build another context started: wait for it
        std::unique_lock<std::mutex> lk(g_mu);
        g_cv.wait(lk, [&] { return b->state.load() != 0; });
    }
    const int state = b->state.load(std::memory_order_acquire);
    if (state == 0) return RT_OK;  // still compiling: the generic kernel this frame
    if (ctx->jit_owner[variant]) {
        ctx->jit_compile_ms += b->ms;
        if (b->from_disk) ++ctx->jit_cache_hits;
        ctx->jit_owner[variant] = false;
    }
    // A failed build of the optional 7-wave variant (variant >= 8) refuses
    // that variant only: jit_function falls back to the static-occupancy
    // build compiled beside it.  A failed base build keeps the generic kernel
    // for this world.
    const bool optional = variant >= 8;
    if (state == 2) {
        (optional ? ctx->jit_rejected[variant] : ctx->jit_failed) = true;
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
            (optional ? ctx->jit_rejected[variant] : ctx->jit_failed) = true;
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
    if (blocks < static_blocks || scratch > (pool ? scratch_max : 0)) {
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
}  // namespace

int jit_function(rt_context* ctx, bool pool, bool lds, size_t dyn_lds, int static_blocks, hipFunction_t* fn,
                 bool no_skips, int* pool_waves) {
    *fn = nullptr;
    if (pool_waves) *pool_waves = 0;
    if (ctx->jit_failed || ctx->jit_shapes.empty()) return RT_OK;
    const int variant = (no_skips ? 4 : 0) + (pool ? 2 : 0) + (lds ? 1 : 0);
    if (!pool) return jit_variant(ctx, variant, pool, lds, dyn_lds, static_blocks, fn, no_skips, 0, 0);
    // The pool kernel at 7 waves/SIMD (jit_options.hpp) and, compiled beside
    // it, at the static build's occupancy: a 7-wave build that spills more
    // than kPool7ScratchMax is refused and the other is taken (also while the
    // 7-wave one still compiles).  Both land in the disk cache, so a later
    // process has its kernel at the first frame either way.  The 7-wave
    // build is checked against the static plan's LDS (it passes at 6
    // workgroups/CU) and the caller re-plans the pool's LDS for 7
    // (rtc_host.cpp plan_pool_for).
    int rc = jit_variant(ctx, variant, pool, lds, dyn_lds, static_blocks, fn, no_skips, 0, 16, true);
    if (rc) return rc;
    rc = jit_variant(ctx, variant + 8, pool, lds, dyn_lds, static_blocks, fn, no_skips, 7, kPool7ScratchMax);
    if (rc || ctx->jit_failed) return rc;
    if (*fn) {
        if (pool_waves) *pool_waves = 7;
        return RT_OK;
    }
    // (0 waves: the static build's occupancy, as planned)
    return jit_variant(ctx, variant, pool, lds, dyn_lds, static_blocks, fn, no_skips, 0, 16);
}

// Block until this context's builds in flight have finished (rt_jit_wait).
int jit_wait(rt_context* ctx, double timeout_ms, int* pending) {
    const auto deadline = std::chrono::steady_clock::now() +
                          std::chrono::microseconds((int64_t)(timeout_ms < 0 ? 3.6e12 : timeout_ms * 1e3));
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
