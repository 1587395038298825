// Where a one-shot render's start-up time goes: step timings
// of a bare HIP process, optionally after loading RCCL the way librtc links
// it, and the first device-to-host copy into an untouched pageable canvas with
// several ways of faulting its pages in first.  Diagnostic only.
//   hipcc -O2 -o scripts/_init_probe scripts/init_probe.cpp -ldl -lpthread
//   scripts/_init_probe [rccl] [prefault=none|touch|huge|threads|small|register|blit]
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {
using clk = std::chrono::steady_clock;
clk::time_point g_t0, g_t;
void step(const char* name) {
    const auto now = clk::now();
    std::printf("  %-34s %8.3f ms  (%8.3f total)\n", name, std::chrono::duration<double, std::milli>(now - g_t).count(),
                std::chrono::duration<double, std::milli>(now - g_t0).count());
    g_t = now;
}
#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));     \
            return 1;                                                      \
        }                                                                  \
    } while (0)
}  // namespace

int main(int argc, char** argv) {
    bool rccl = false;
    std::string prefault = "none";
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "rccl")) rccl = true;
        if (!std::strncmp(argv[i], "prefault=", 9)) prefault = argv[i] + 9;
    }
    // blit: the runtime's copy-engine threshold raised before it starts, so the
    // canvas copy runs as a blit kernel on the compute queue instead of SDMA
    if (prefault == "blit") setenv("GPU_FORCE_BLIT_COPY_SIZE", "1048576", 1);
    std::printf("init_probe rccl=%d prefault=%s\n", rccl, prefault.c_str());
    g_t0 = g_t = clk::now();
    if (rccl) {
        if (!dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL)) std::printf("dlopen: %s\n", dlerror());
        step("dlopen librccl");
    }
    int n = 0;
    CK(hipGetDeviceCount(&n));
    step("hipGetDeviceCount (runtime start)");
    CK(hipSetDevice(0));
    step("hipSetDevice");
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    step("hipStreamCreate");
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    step("hipStreamCreate (second)");
    const size_t bytes = (size_t)1920 * 1080 * 3 * 4;
    void* d = nullptr;
    CK(hipMalloc(&d, bytes));
    step("hipMalloc 24.9 MB");
    CK(hipMemsetAsync(d, 0, 4096, s));
    CK(hipStreamSynchronize(s));
    step("hipMemsetAsync (first) + sync");
    CK(hipMemsetAsync(d, 0, bytes, s));
    CK(hipStreamSynchronize(s));
    step("hipMemsetAsync 24.9 MB + sync");
    // an untouched canvas, as numpy.zeros / a fresh Vec gives the caller
    char* h = static_cast<char*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    step("mmap canvas");
    if (prefault == "touch" || prefault == "huge") {
        if (prefault == "huge") {
            const uintptr_t a = ((uintptr_t)h + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
            const uintptr_t b = ((uintptr_t)h + bytes) & ~(uintptr_t)((2u << 20) - 1);
            if (b > a && madvise((void*)a, b - a, MADV_HUGEPAGE) != 0) std::printf("  madvise failed\n");
        }
        for (size_t i = 0; i < bytes; i += 4096) h[i] = 0;
        step(("prefault " + prefault).c_str());
    } else if (prefault == "threads") {
        const int nt = 8;
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([=] {
                const size_t lo = bytes * t / nt, hi = bytes * (t + 1) / nt;
                for (size_t i = lo & ~(size_t)4095; i < hi; i += 4096) h[i] = 0;
            });
        for (auto& x : th) x.join();
        step("prefault 8 threads");
    }
    if (prefault == "small") {  // is the first copy's cost per process or per buffer?
        static char small[4096];
        CK(hipMemcpyAsync(small, d, sizeof small, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        step("D2H 4 KB (first, pageable)");
    }
    if (prefault == "register") {
        CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
        step("hipHostRegister canvas");
    }
    CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    step("D2H 24.9 MB (first)");
    CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    step("D2H 24.9 MB (again)");
    if (prefault == "register") CK(hipHostUnregister(h));
    munmap(h, bytes);
    CK(hipFree(d));
    FILE* f = std::fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
    char buf[128] = {};
    if (f && std::fgets(buf, sizeof buf, f)) std::printf("  THP: %s", buf);
    if (f) std::fclose(f);
    return 0;
}
