// rtc_context.hpp — the per-device state behind an rt_context handle and the
// host-side internals shared by the single-device entry points
// (rtc_host.cpp) and the multi-GPU group (rtc_group.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rtc.h"
#include "flop_model.hpp"
#include "rtc_internal.hpp"

namespace rtc {

// World tables cast to R and laid out per kind (rtc_internal.hpp).
// The shape, material and pattern tables and world_slot sit in ONE
// allocation in the kernels' LDS layout ([shapes][materials][patterns]
// [world_slot], world_lds_bytes), so a workgroup stages the world into LDS
// with one contiguous copy (scene_view).
template <typename R>
struct DeviceWorld {
    void* image = nullptr;  // the allocation holding the four tables
    ShapeRec<R>* shapes = nullptr;
    MaterialRec<R>* materials = nullptr;
    PatternRec<R>* patterns = nullptr;
    LightRec<R>* lights = nullptr;
    int32_t* world_slot = nullptr;
    DevScene<R> scene{};
    // Point the tables into `image` for ns shapes, nm materials, np patterns.
    void carve(size_t ns, size_t nm, size_t np) {
        unsigned char* b = static_cast<unsigned char*>(image);
        shapes = reinterpret_cast<ShapeRec<R>*>(b);
        materials = reinterpret_cast<MaterialRec<R>*>(b + ns * sizeof(ShapeRec<R>));
        patterns = reinterpret_cast<PatternRec<R>*>(b + ns * sizeof(ShapeRec<R>) + nm * sizeof(MaterialRec<R>));
        world_slot = reinterpret_cast<int32_t*>(b + ns * sizeof(ShapeRec<R>) + nm * sizeof(MaterialRec<R>) +
                                                np * sizeof(PatternRec<R>));
    }
    void release() {
        (void)hipFree(image);
        (void)hipFree(lights);
        image = nullptr;
        shapes = nullptr;
        materials = nullptr;
        patterns = nullptr;
        world_slot = nullptr;
        lights = nullptr;
    }
};

struct CodeBuild;  // rtc_jit.cpp: one hipRTC build of a per-scene kernel, possibly in flight

}  // namespace rtc

// One device's render state.  A single-device context is one of these; a
// multi-GPU context (rtc_group.cpp) is the rank-0 member, holding the other
// devices of the process as `peers`, each member with its own communicator.
struct rt_context {
    int device = 0;
    int cu_count = 0;
    size_t lds_per_block = 64 * 1024;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    // Stream order across entry points: every launch shares the queue heads,
    // tile costs/order and pool spill.  rt_render_device runs on the caller's
    // stream, rt_render/rt_color_at on `stream`; a launch on a stream other
    // than the previous launch's first makes its stream wait on all work
    // submitted so far to that one (ev_order recorded at the switch).
    hipEvent_t ev_order = nullptr;
    hipStream_t last_stream = nullptr;
    bool launched = false;
    unsigned long long* d_tile_counter = nullptr;  // two sets of queue heads (launch: dynamic schedule)
    int head_set = 0;                              // the set the next dynamic launch uses
    unsigned long long* d_counters = nullptr;  // kNumCounters cumulative
    unsigned long long* d_gen_counts = nullptr;  // RT_FLAG_GENERATIONS: traced, shaded x kGenSlots, cumulative
    int32_t* d_error = nullptr;
    bool have_scene = false;
    rtc::DeviceWorld<float> w32;
    rtc::DeviceWorld<double> w64;
    rtc::FlopScene flops;  // per-kind shape counts for the algorithmic FLOP model
    double bright_hit = 1.0, bright_w = 0.0;  // brightness bound of the world (acc_shift_f32)
    // Defaults from A/B on MI355X (scripts/ab_sched.sh, scripts/stamps2.sh):
    // uniform-cost direct tiles -> static stride; high-variance pool tiles ->
    // per-XCD atomic queues; per-lane stores beat LDS-staged ones (the
    // staging barriers wait for store completion).
    // (RTC_DEBUG=sched_direct=grid|static; the pool kernel always takes the
    // per-XCD queues)
    uint32_t sched_direct = rtc::kSchedStatic;
    // f32 direct kernel's resident-grid multiple, in tenths (RTC_DEBUG=direct_oversub=T)
    uint32_t direct_oversub10 = 25;
    bool lds_world = true;      // RTC_DEBUG=lds_world=0 gathers shade data from global memory
    bool cull = true;  // RTC_DEBUG=cull=0 uploads every shape as unbounded (no wave cull; exactness tests)
    bool kind_variants = true;  // RTC_DEBUG=kind_variants=0: always the all-kinds kernels
    size_t occ_lds[8] = {};     // occupancy cache: {direct,pool} x {f32,f64} x {global,LDS world}
    int occ_blocks[8] = {};
    uint32_t pool_lds_rays = 0;  // RTC_DEBUG=pool_lds_rays=N: LDS-resident pool slots (0 = sized for occupancy)
    void* d_spill = nullptr;     // ray-pool overflow regions, one per resident workgroup
    // Heaviest-first tile order for repeated pool launches of the same frame
    // (order_tiles): per-tile costs of the last launch and its signature.
    bool tile_order = true;      // RTC_DEBUG=tile_order=0: raster order always
    uint32_t* d_tile_cost = nullptr;
    uint32_t* d_tile_order = nullptr;
    uint32_t order_capacity = 0;
    uint64_t order_sig = 0;
    uint64_t order_geometry = 0;  // order_sig without the camera
    bool order_valid = false;
    bool order_built = false;     // d_tile_order holds an order for order_geometry
    // First launch of a frame geometry (no recorded costs): tiles handed out
    // centre-out instead of in raster order (full frames; shards keep raster).
    uint32_t* d_cold_order = nullptr;  // centre-out order + item count, for cold_w x cold_h
    uint32_t cold_w = 0, cold_h = 0;
    // Tiles costing more than split_factor x the mean workgroup load are
    // handed out in parts (order_tiles); RTC_DEBUG=split=0 never splits.  Round-3
    // sweep (per-scene kernels, slowest of 8 shards at 4K / 1-GPU frame):
    // 1.5: cover 0.239 / 1.132 ms, table 0.244 / 1.389; 1.0: 0.217 / 1.142,
    // 0.226 / 1.369; 0.75: 0.206 / 1.128, 0.233 / 1.384; 0.5: 0.205 / 1.128,
    // 0.245 / 1.414; reflect_refract 1080p, slowest of 4: 0.146 / 0.129 /
    // 0.126 / 0.131 with whole frames unchanged (0.385-0.403).
    double split_factor = 1.0;
    // RTC_DEBUG=split_max=L: log2 of the most parts a tile is split into.  Same-box
    // sweep (profiles/ab/r03_split16_sweep.txt, r03_shard_floor.txt), slowest
    // shard ms at 2 / 3 / 4: cover 4K of 8 0.198 / 0.202 / 0.207, of 32
    // 0.130 / 0.096 / 0.115; reflect_refract 1080p of 4 0.127 / 0.128 /
    // 0.121, of 16 0.112 / 0.092 / 0.097; whole frames split nothing.
    uint32_t split_max = 3;
    // Items (tiles or parts) costing more than urgent_factor x the mean
    // workgroup load run at raised wave priority, graded 1/2/3 above 1x/2x/4x
    // that cost (RTC_DEBUG=urgent=F, 0 = none; one level for all measured no better).  Same-box sweep, kernel ms, none / flat 0.25 / flat 0.125 /
    // graded 0.125: reflect_refract 0.367 / 0.310 / 0.306 / 0.310, cylinders
    // 0.124 / 0.117 / 0.117 / 0.117, cover 4K 1.014 / 1.023 / 1.011 / 1.011,
    // table 4K, refraction, metal within 1 %; slowest of 8 shards at 4K: cover
    // 0.215 / 0.201 / 0.215 / 0.201, table 0.229 / 0.266 / 0.230 / 0.231.
    double urgent_factor = 0.125;
    int order_builds = 0;        // order_tiles runs for the current signature so far
    uint64_t scene_gen = 0;      // bumped by every rt_scene_upload
    uint32_t duplicate_shapes = 0;  // shapes value-equal to an earlier one (one identity class)
    std::vector<int32_t> world_slot;  // world index -> slot | kind << 24 of the uploaded table
    size_t spill_bytes = 0;
    unsigned long long* d_stamps = nullptr;  // RT_FLAG_STAMPS diagnostics
    uint32_t stamp_capacity = 0, stamp_count = 0;
    unsigned long long* d_item_log = nullptr;  // RT_FLAG_STAMPS pool launches: item spans
    size_t item_log_capacity = 0;  // items
    void* d_scratch = nullptr;  // host-buffer renders / color_at staging
    size_t scratch_bytes = 0;
    // Per-scene f32 kernels (rtc_jit.cpp): the f32 shape table of the last
    // upload, the kernels built for it (direct/pool x global/LDS world), and
    // RTC_JIT / rt_context_set_jit = RT_JIT_OFF | RT_JIT_SYNC | RT_JIT_AUTO
    // (default) | RT_JIT_EAGER (rtc.h).
    std::vector<rtc::ShapeRec<float>> jit_shapes;
    std::vector<rtc::LightRec<float>> jit_lights;  // per-scene builds unroll the lights as constants
    std::vector<rtc::MaterialRec<float>> jit_materials;  // ... and the direct kernel reads materials as constants
    std::vector<rtc::PatternRec<float>> jit_pattern_recs;  // (pattern kinds present)
    bool jit_patterns = true;                      // some material has a pattern (else pattern code is dropped)
    uint32_t jit_pattern_kinds = ~0u;              // pattern kinds in the world's table (bit per RT_PATTERN_*)
    bool jit_transparent = true;                   // some material is transparent (else no refraction code)
    int32_t jit_begin[rtc::kNumKinds + 1] = {};
    // variants: pool x LDS world x RT_FLAG_NO_SKIPS x (pool) 7 waves/SIMD (rtc_jit.cpp jit_function)
    static constexpr int kJitVariants = 16;
    hipFunction_t jit_fn[kJitVariants] = {};
    std::shared_ptr<rtc::CodeBuild> jit_build[kJitVariants];  // the build each variant waits for (host thread)
    bool jit_rejected[kJitVariants] = {};   // built, but refused for occupancy or scratch (that variant only)
    bool jit_owner[kJitVariants] = {};      // this context started the build: its time goes into jit_compile_ms
    uint32_t jit_frames = 0;     // large f32 frames of this upload so far (RT_JIT_AUTO starts at the 2nd)
    std::string arch;            // the device's gfx target (gcnArchName), for hipRTC; read lazily (device_arch)
    int jit_mode = 2;
    bool jit_failed = false, jit_used = false;  // jit_failed: the world's build failed (compile or load)
    double jit_compile_ms = 0;  // compile (or disk-cache load) time of this context's per-scene builds
    int jit_cache_hits = 0;     // builds loaded from the on-disk cache
    std::string jit_log;
    // rt_render: counters before/after and the error flag come back pinned,
    // on the stream, so a frame needs one host sync
    unsigned long long* h_counters = nullptr;  // 2 x kCounterShards x kNumCounters + the error flag
    // Multi-GPU group (rtc_group.cpp).  A frame is split
    // into n_ranks shards of cyclic RT_TILE_H-row blocks; this member renders
    // shard `rank` into d_strip, RCCL gathers the strips onto rank 0, which
    // de-interleaves them into the image.  Single-device contexts: comm null.
    ncclComm_t comm = nullptr;
    int n_ranks = 1, rank = 0;
    std::vector<rt_context*> peers;  // rank 0 of a one-process group: the other devices' members
    int32_t* d_status = nullptr;     // agree_status's word, allocated with the member so a rank can always join
    void* d_strip = nullptr;         // this member's shard strip
    size_t strip_bytes = 0;
    void* d_gathered = nullptr;      // rank 0: every strip, shard-major
    size_t gathered_bytes = 0;
    hipEvent_t ev_render0 = nullptr, ev_render1 = nullptr, ev_gather1 = nullptr;  // frame timing
    // Peer canvases this context created or mapped (rt_canvas_*): image
    // bytes and flag count per base pointer.
    struct Canvas {
        uint64_t bytes = 0;
        uint32_t n_flags = 0;
        bool owned = false;  // created here (hipFree) or mapped (hipIpcCloseMemHandle / peer pointer)
    };
    std::map<void*, Canvas> canvases;
    // RT_GATHER_PEER groups: the shared canvas (rank 0's allocation; mapped or
    // peer-accessed on the others) and the frame sequence number.
    int gather_mode = RT_GATHER_RCCL;
    void* group_canvas = nullptr;
    uint64_t group_canvas_bytes = 0;
    uint64_t canvas_seq = 0;
};

namespace rtc {

// rtc_host.cpp
// RTC_DEBUG=trace_init=1: per-step milliseconds of context creation, upload and
// the first renders on stderr (the one-shot breakdown).
class InitTrace {
public:
    explicit InitTrace(const char* what);
    void step(const char* name);
private:
    const char* what_;
    bool on_;
    std::chrono::steady_clock::time_point t0_, t_;
};
int create_device_context(int device, rt_context** out);
void destroy_device_context(rt_context* ctx);
int check_ready(rt_context* ctx);
int check_options(const rt_render_options* o);
int ensure_scratch(rt_context* ctx, size_t bytes);
int read_counters(rt_context* ctx, unsigned long long out[kNumCounters]);
void fill_stats(rt_context* ctx, const unsigned long long before[kNumCounters],
                const unsigned long long after[kNumCounters], float ms, rt_stats* s);
int check_pool_error(rt_context* ctx);
int order_after_last(rt_context* ctx, hipStream_t stream);  // cross-stream launch order (rtc.h)
int ensure_host_counters(rt_context* ctx);
int copy_to_host(rt_context* ctx, void* out, size_t bytes);  // d_scratch -> caller host buffer, on ctx->stream
uint32_t tile_rows_for(uint32_t height, uint32_t shards, uint32_t shard);
int validate_scene(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                   const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl);
// Flatten and upload the world tables to this device (no validation, no sync).
int build_scene(rt_context* ctx, const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl);
void scene_brightness(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                      const rt_pattern_desc* pats, uint32_t np,
                      const rt_light_desc* lights, uint32_t nl, double* bright_hit, double* bright_w);
// One frame (or shard strip) of this device into `out_device` on `stream`.
int capture_jit_table(rt_context* ctx);  // the f32 table of the uploaded world, for rtc_jit.cpp
int fetch_jit_tables(rt_context* ctx);   // build_world<float>'s host tables read back (a group's other ranks)
int launch_frame(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, uint32_t shard_index,
                 uint32_t shard_count, void* out_device, hipStream_t stream, bool image_rows = false);
// Peer canvas internals (rtc_host.cpp): flags of a canvas, and the kernels.
unsigned long long* canvas_flags(void* canvas, uint64_t image_bytes);  // n_flags ready flags, then release
int canvas_create(rt_context* ctx, uint64_t bytes, uint32_t n_flags, void** canvas);
int canvas_close(rt_context* ctx, void* canvas);
hipError_t launch_canvas_signal(unsigned long long* flag, unsigned long long seq, hipStream_t stream);
hipError_t launch_canvas_wait(const unsigned long long* flags, uint32_t n, unsigned long long seq,
                              unsigned long long timeout_ticks, int32_t* err, hipStream_t stream);
unsigned long long timeout_ticks(double timeout_ms);
// rtc_jit.cpp: the per-scene kernel of this context's world for a launch of
// `static_blocks` workgroups per CU, or null (use the generic kernel)
constexpr uint32_t kJitMinTiles = 256;  // 64K pixels
// *pool_waves: the waves/SIMD the returned pool kernel was built for (7, or
// 6 = the static build's), so the caller can plan its LDS for them.
int jit_function(rt_context* ctx, bool pool, bool lds, size_t dyn_lds, int static_blocks, hipFunction_t* fn,
                 bool no_skips = false, int* pool_waves = nullptr);
int jit_wait(rt_context* ctx, double timeout_ms, int* pending);
const std::string& device_arch(rt_context* ctx);  // rtc_jit.cpp: the device's gfx target, read once

// rtc_group.cpp: the same entry points on a multi-GPU context
int group_scene_upload(rt_context* ctx, const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats,
                       uint32_t nm, const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights,
                       uint32_t nl);
int group_render_device(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* out_device,
                        hipStream_t stream);
int group_render(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* out_host,
                 rt_stats* stats);
int group_read_counters(rt_context* ctx, rt_stats* totals);
hipError_t launch_assemble(const void* gathered, void* image, uint32_t width, uint32_t height, uint32_t shards,
                           uint32_t strip_rows, uint32_t bpp, hipStream_t stream);

#define RT_HIP(call)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return set_error(RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));       \
    } while (0)

}  // namespace rtc
