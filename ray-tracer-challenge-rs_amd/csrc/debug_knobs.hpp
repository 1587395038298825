// debug_knobs.hpp — the library's A/B and diagnostic switches, all read from
// one environment variable: RTC_DEBUG="key=value,key=value,...", e.g.
//   RTC_DEBUG=cull=0,tile_order=0,split=0.5 python bench.py --ab
// Product runs set none of them.  Keys (defaults in rtc_context.hpp):
//   sched_direct=grid|static      direct-kernel tile scheduling
//   direct_oversub=T              f32 direct kernel's grid: T/10 x the resident workgroups (default 25)
//   lds_world=0                   world tables not staged in LDS
//   cull=0                        every shape uploaded unbounded (no wave cull)
//   kind_variants=0               no sphere/plane-only pool kernel
//   pool_lds_rays=N               LDS-resident LIFO slots (else sized for occupancy)
//   tile_order=0 | split=F | split_max=L | urgent=F   pool item order (rtc_host.cpp)
//   trace_init=1                  context-creation step times on stderr
//   jit_clusters=N | jit_cluster_refine=0 | jit_flags=...   per-scene builds (rtc_jit.cpp)
//   jit_dump=DIR                  per-scene header + code object per build (rtc_jitc)
// Values may not contain ','.  The variable is read at each use (contexts
// created after a change see it).
#pragma once

#include <cstdlib>
#include <cstring>
#include <string>

namespace rtc {

// The value of `key` in RTC_DEBUG, or false when absent.
inline bool debug_knob(const char* key, std::string* value) {
    const char* e = std::getenv("RTC_DEBUG");
    if (!e) return false;
    const size_t kl = std::strlen(key);
    for (const char* p = e; *p;) {
        const char* end = std::strchr(p, ',');
        if (!end) end = p + std::strlen(p);
        if ((size_t)(end - p) > kl && !std::strncmp(p, key, kl) && p[kl] == '=') {
            if (value) value->assign(p + kl + 1, end);
            return true;
        }
        p = *end ? end + 1 : end;
    }
    return false;
}

}  // namespace rtc
