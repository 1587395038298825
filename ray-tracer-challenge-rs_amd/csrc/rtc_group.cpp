// rtc_group.cpp — multi-GPU contexts behind the C-ABI (include/rtc.h).
//
// The north star tiles one image across the GPUs of a node: "RCCL broadcast
// of the scene + gather of framebuffer strips over xGMI" (SURVEY.md §8b, §8e).
// The reference's contract is that the library owns the parallelism and the
// caller just calls render_parallel (camera.rs:97-112), so the split lives
// here, not in the caller:
//
//   rt_scene_upload   rank 0 flattens the World (rtc_host.cpp build_scene)
//                     and ncclBroadcasts a header plus the four device
//                     buffers (per precision: the table image, the lights)
//                     (f32 and f64 records) to every other GPU.
//   rt_render[_device] every member renders its shard — cyclic RT_TILE_H-row
//                     blocks (rank r takes tile rows r, r+G, ...), which
//                     spreads the cost of expensive rows (cover's reflective
//                     cubes) — into a contiguous strip; ncclGather brings the
//                     strips to rank 0 (equal counts: every strip is padded
//                     to rt_shard_rows rows); rank 0 de-interleaves them
//                     into the image (assemble_shards).
//
// Members: rank 0 of a one-process group (rt_context_create_multi) is the
// context handed to the caller and holds the other devices' members in
// `peers`; RCCL calls for all of them go in one ncclGroupStart/End.  In the
// one-process-per-GPU form (rt_context_create_rank) each process holds just
// its own member and the same code runs with one local member.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rtc.h"
#include "rtc_context.hpp"

namespace rtc {
namespace {

#define RT_NCCL(call)                                                                                      \
    do {                                                                                                   \
        ncclResult_t r_ = (call);                                                                          \
        if (r_ != ncclSuccess) return set_error(RT_ERR_COMM, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

std::vector<rt_context*> members(rt_context* ctx) {
    std::vector<rt_context*> m{ctx};
    m.insert(m.end(), ctx->peers.begin(), ctx->peers.end());
    return m;
}

// The flattened world's shape, broadcast ahead of the tables so the other
// ranks can allocate them.
struct SceneHeader {
    int32_t status;  // rank 0's validation/upload result: the others fail with it too
    uint32_t ns, nm, np, nl;
    int32_t kind_begin[kNumKinds + 1];
    int32_t any_secondary;
    uint32_t duplicates;
    double flops_per_ray;
    double bright_hit, bright_w;  // acc_shift_f32's bound
};

template <typename R>
int alloc_world(DeviceWorld<R>& w, const SceneHeader& h) {
    w.release();
    RT_HIP(hipMalloc(&w.image, std::max<size_t>(world_lds_bytes<R>(h.ns, h.nm, h.np), 16)));
    w.carve(h.ns, h.nm, h.np);
    if (h.nl) RT_HIP(hipMalloc(reinterpret_cast<void**>(&w.lights), h.nl * sizeof(LightRec<R>)));
    return RT_OK;
}

template <typename R>
void describe_world(DeviceWorld<R>& w, const SceneHeader& h) {
    w.scene.shapes = w.shapes;
    w.scene.materials = w.materials;
    w.scene.patterns = w.patterns;
    w.scene.lights = w.lights;
    w.scene.world_slot = w.world_slot;
    for (int k = 0; k <= kNumKinds; ++k) w.scene.kind_begin[k] = h.kind_begin[k];
    w.scene.n_materials = (int32_t)h.nm;
    w.scene.n_patterns = (int32_t)h.np;
    w.scene.n_lights = (int32_t)h.nl;
    w.scene.any_secondary = h.any_secondary;
}

// (device pointer, bytes) of every table of a member's world, in one order
// on every rank.
template <typename R>
void world_buffers(DeviceWorld<R>& w, const SceneHeader& h, std::vector<std::pair<void*, size_t>>& out) {
    out.push_back({w.image, world_lds_bytes<R>(h.ns, h.nm, h.np)});  // shapes, materials, patterns, world_slot
    out.push_back({w.lights, h.nl * sizeof(LightRec<R>)});
}

int ensure(void** p, size_t* have, size_t need) {
    if (*have >= need) return RT_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    RT_HIP(hipMalloc(p, need));
    *have = need;
    return RT_OK;
}

int init_member(rt_context* m, ncclComm_t comm, int n_ranks, int rank) {
    m->comm = comm;
    m->n_ranks = n_ranks;
    m->rank = rank;
    RT_HIP(hipSetDevice(m->device));
    RT_HIP(hipEventCreate(&m->ev_render0));
    RT_HIP(hipEventCreate(&m->ev_render1));
    RT_HIP(hipEventCreate(&m->ev_gather1));
    RT_HIP(hipMalloc(reinterpret_cast<void**>(&m->d_status), sizeof(int32_t)));
    return RT_OK;
}

size_t pixel_bytes(const rt_render_options* o) {
    return 3 * (o->out_format == RT_OUT_U8 ? 1 : (o->precision == RT_PRECISION_F32 ? 4 : 8));
}

// The shards of one frame: every local member renders its strip on its
// stream (rank 0's on `root_stream`), RCCL gathers the strips onto rank 0,
// rank 0 de-interleaves them into `image` (rank 0's device).  With `timed`,
// events bracket each member's render and rank 0's gather + assemble.
int render_shards_peer(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* image,
                       hipStream_t root_stream, bool timed);

int render_shards(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* image,
                  hipStream_t root_stream, bool timed) {
    if (ctx->gather_mode == RT_GATHER_PEER) return render_shards_peer(ctx, cam, o, image, root_stream, timed);
    const std::vector<rt_context*> ms = members(ctx);
    const uint32_t G = (uint32_t)ctx->n_ranks;
    const uint32_t rows = tile_rows_for(cam->height, G, 0) * RT_TILE_H;  // shard 0 has the most rows
    const size_t strip = (size_t)rows * cam->width * pixel_bytes(o);
    int rc;
    auto stream_of = [&](rt_context* m) { return m->rank == 0 ? root_stream : m->stream; };
    for (rt_context* m : ms) {
        RT_HIP(hipSetDevice(m->device));
        if (m->rank != 0 && (rc = ensure(&m->d_strip, &m->strip_bytes, strip))) return rc;
        if (m->rank == 0 && (rc = ensure(&m->d_gathered, &m->gathered_bytes, strip * G))) return rc;
    }
    // Rank 0 renders its strip straight into its slot of the gather buffer
    // (slot 0), and gathers in place: RCCL then copies only the other ranks'.
    auto strip_of = [&](rt_context* m) { return m->rank == 0 ? m->d_gathered : m->d_strip; };
    for (rt_context* m : ms) {
        hipStream_t s = stream_of(m);
        RT_HIP(hipSetDevice(m->device));
        if (timed) RT_HIP(hipEventRecord(m->ev_render0, s));
        if ((rc = launch_frame(m, cam, o, (uint32_t)m->rank, G, strip_of(m), s))) return rc;
        if (timed) RT_HIP(hipEventRecord(m->ev_render1, s));
    }
    RT_NCCL(ncclGroupStart());
    for (rt_context* m : ms)
        RT_NCCL(ncclGather(strip_of(m), m->rank == 0 ? m->d_gathered : nullptr, strip, ncclUint8, 0, m->comm,
                           stream_of(m)));
    RT_NCCL(ncclGroupEnd());
    for (rt_context* m : ms) {
        if (m->rank != 0) continue;
        RT_HIP(hipSetDevice(m->device));
        RT_HIP(launch_assemble(m->d_gathered, image, cam->width, cam->height, G, rows, (uint32_t)pixel_bytes(o),
                               root_stream));
        if (timed) RT_HIP(hipEventRecord(m->ev_gather1, root_stream));
    }
    return RT_OK;
}

// RT_GATHER_PEER: the group's canvas on rank 0, big enough for `bytes` of
// image (every rank asks for the same size: collective).  One process per
// GPU: rank 0 creates it and RCCL-broadcasts its IPC handle, the others map
// it.  One process with several GPUs: the other members write through peer
// access to rank 0's pointer.
int ensure_group_canvas(rt_context* ctx, uint64_t bytes) {
    const std::vector<rt_context*> ms = members(ctx);
    if (ctx->group_canvas && ctx->group_canvas_bytes >= bytes) return RT_OK;
    const uint32_t G = (uint32_t)ctx->n_ranks;
    const bool remote = (int)ms.size() < ctx->n_ranks;  // ranks in other processes
    int rc;
    for (rt_context* m : ms) {  // drop the old canvas (rank 0's allocation, a mapping, or a peer pointer)
        if (m->group_canvas && m->canvases.count(m->group_canvas) && (rc = canvas_close(m, m->group_canvas))) return rc;
        m->group_canvas = nullptr;
        m->group_canvas_bytes = 0;
        m->canvas_seq = 0;  // a new canvas's flags start at 0: its first frame is seq 1 on every rank
    }
    void* root = nullptr;
    for (rt_context* m : ms)
        if (m->rank == 0) {
            if ((rc = canvas_create(m, bytes, G, &root))) return rc;
            m->group_canvas = root;
            m->group_canvas_bytes = bytes;
        }
    if (remote) {  // the IPC handle from rank 0 to every rank, over RCCL
        hipIpcMemHandle_t h{};
        if (root) {
            RT_HIP(hipSetDevice(ctx->device));
            RT_HIP(hipIpcGetMemHandle(&h, root));
        }
        std::vector<void*> d_h(ms.size(), nullptr);
        for (size_t i = 0; i < ms.size(); ++i) {
            RT_HIP(hipSetDevice(ms[i]->device));
            RT_HIP(hipMalloc(&d_h[i], sizeof h));
            if (ms[i]->rank == 0) RT_HIP(hipMemcpy(d_h[i], &h, sizeof h, hipMemcpyHostToDevice));
        }
        RT_NCCL(ncclGroupStart());
        for (size_t i = 0; i < ms.size(); ++i)
            RT_NCCL(ncclBroadcast(d_h[i], d_h[i], sizeof h, ncclUint8, 0, ms[i]->comm, ms[i]->stream));
        RT_NCCL(ncclGroupEnd());
        for (size_t i = 0; i < ms.size(); ++i) {
            RT_HIP(hipSetDevice(ms[i]->device));
            RT_HIP(hipStreamSynchronize(ms[i]->stream));
            hipIpcMemHandle_t got;
            RT_HIP(hipMemcpy(&got, d_h[i], sizeof got, hipMemcpyDeviceToHost));
            (void)hipFree(d_h[i]);
            if (ms[i]->rank == 0) continue;
            void* p = nullptr;
            RT_HIP(hipIpcOpenMemHandle(&p, got, hipIpcMemLazyEnablePeerAccess));
            ms[i]->canvases[p] = {bytes, G, false};
            ms[i]->group_canvas = p;
            ms[i]->group_canvas_bytes = bytes;
        }
    } else {  // every rank in this process: peer access to rank 0's device
        for (rt_context* m : ms) {
            if (m->rank == 0) continue;
            RT_HIP(hipSetDevice(m->device));
            if (m->device != ctx->device) {
                hipError_t e = hipDeviceEnablePeerAccess(ctx->device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return set_error(RT_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();
            }
            m->group_canvas = root;
            m->group_canvas_bytes = bytes;
        }
    }
    return RT_OK;
}

// RT_GATHER_PEER frame: each member waits until rank 0 has released the
// previous frame, renders its shard at image rows into the canvas and raises
// its flag; rank 0 waits for every flag, copies the image out and releases
// the frame.  No strip, no gather, no de-interleave.
constexpr double kPeerTimeoutMs = 10000.0;
int render_shards_peer(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* image,
                       hipStream_t root_stream, bool timed) {
    const std::vector<rt_context*> ms = members(ctx);
    const uint32_t G = (uint32_t)ctx->n_ranks;
    const uint64_t bytes = (uint64_t)cam->width * cam->height * pixel_bytes(o);
    int rc;
    if ((rc = ensure_group_canvas(ctx, bytes))) return rc;
    auto stream_of = [&](rt_context* m) { return m->rank == 0 ? root_stream : m->stream; };
    for (rt_context* m : ms) {
        hipStream_t s = stream_of(m);
        RT_HIP(hipSetDevice(m->device));
        const uint64_t seq = ++m->canvas_seq;  // every rank renders the same frames: the same number
        unsigned long long* flags = canvas_flags(m->group_canvas, m->group_canvas_bytes);
        if (seq > 1) RT_HIP(launch_canvas_wait(flags + G, 1, seq - 1, timeout_ticks(kPeerTimeoutMs), m->d_error, s));
        if (timed) RT_HIP(hipEventRecord(m->ev_render0, s));
        if ((rc = launch_frame(m, cam, o, (uint32_t)m->rank, G, m->group_canvas, s, true))) return rc;
        if (timed) RT_HIP(hipEventRecord(m->ev_render1, s));
        RT_HIP(launch_canvas_signal(flags + m->rank, seq, s));
    }
    for (rt_context* m : ms) {
        if (m->rank != 0) continue;
        RT_HIP(hipSetDevice(m->device));
        unsigned long long* flags = canvas_flags(m->group_canvas, m->group_canvas_bytes);
        RT_HIP(launch_canvas_wait(flags, G, m->canvas_seq, timeout_ticks(kPeerTimeoutMs), m->d_error, root_stream));
        if (image) RT_HIP(hipMemcpyAsync(image, m->group_canvas, bytes, hipMemcpyDeviceToDevice, root_stream));
        RT_HIP(launch_canvas_signal(flags + G, m->canvas_seq, root_stream));
        if (timed) RT_HIP(hipEventRecord(m->ev_gather1, root_stream));
    }
    return RT_OK;
}

int check_group_options(rt_context* ctx, const rt_render_options* o) {
    if (o->shard_count != 1 || o->shard_index != 0)
        return set_error(RT_ERR_INVALID, "a multi-GPU context shards frames itself: shard_index/shard_count must be 0/1");
    for (rt_context* m : members(ctx))
        if (!m->have_scene) return set_error(RT_ERR_NO_SCENE, "render before rt_scene_upload");
    (void)ctx;
    return RT_OK;
}

}  // namespace

// The group's agreement on one step's outcome: every member of every rank
// contributes `local` (RT_OK or its error) to a max all-reduce of -status;
// RT_ERR_COMM when another rank failed, RT_OK when none did (a member's own
// failure is returned by its caller).
int agree_status(const std::vector<rt_context*>& ms, int local) {
    // The status words were allocated with the members (init_member), so a
    // rank always takes part in the all-reduce: a member whose word cannot be
    // written still joins (its stale word is overwritten by the max) and
    // reports its own error afterwards, instead of leaving the other ranks
    // blocked in the collective.
    const int32_t mine = local ? -local : 0;
    std::vector<int32_t> got(ms.size(), 0);
    int rc = RT_OK;
    for (size_t i = 0; i < ms.size(); ++i) {
        if (hipSetDevice(ms[i]->device) != hipSuccess ||
            hipMemcpyAsync(ms[i]->d_status, &mine, sizeof mine, hipMemcpyHostToDevice, ms[i]->stream) != hipSuccess)
            if (!rc) rc = set_error(RT_ERR_HIP, "status exchange: writing the status word");
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < ms.size() && r == ncclSuccess; ++i)
        r = ncclAllReduce(ms[i]->d_status, ms[i]->d_status, 1, ncclInt32, ncclMax, ms[i]->comm, ms[i]->stream);
    if (r == ncclSuccess) r = ncclGroupEnd();
    for (size_t i = 0; i < ms.size() && r == ncclSuccess; ++i) {
        if (hipSetDevice(ms[i]->device) != hipSuccess || hipStreamSynchronize(ms[i]->stream) != hipSuccess ||
            hipMemcpy(&got[i], ms[i]->d_status, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
            if (!rc) rc = set_error(RT_ERR_HIP, "status exchange: read back");
    }
    if (r != ncclSuccess) return set_error(RT_ERR_COMM, std::string("status exchange: ") + ncclGetErrorString(r));
    if (rc) return rc;
    for (int32_t g : got)
        if (g && !local) return set_error(RT_ERR_COMM, "another rank of the group failed (status " + std::to_string(-g) + ")");
    return RT_OK;
}

int group_scene_upload(rt_context* ctx, const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats,
                       uint32_t nm, const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights,
                       uint32_t nl) {
    const std::vector<rt_context*> ms = members(ctx);
    int rc;
    SceneHeader root_h{};
    for (rt_context* m : ms) {  // launches on caller streams may still read the old tables
        RT_HIP(hipSetDevice(m->device));
        RT_HIP(hipDeviceSynchronize());
        m->have_scene = false;
    }
    int root_rc = RT_OK;
    std::string root_err;
    if (ctx->rank == 0) {  // only rank 0's tables are used (rtc.h)
        // a failure here still takes part in the header broadcast, so the
        // other ranks return it instead of waiting in the table broadcast
        root_rc = validate_scene(shapes, ns, mats, nm, pats, np, lights, nl);
        if (!root_rc && hipSetDevice(ctx->device) != hipSuccess) root_rc = set_error(RT_ERR_HIP, "hipSetDevice");
        if (!root_rc) root_rc = build_scene(ctx, shapes, ns, mats, nm, pats, np, lights, nl);
        if (root_rc) root_err = rt_last_error();
        root_h.status = root_rc;
        root_h.ns = ns;
        root_h.nm = nm;
        root_h.np = np;
        root_h.nl = nl;
        for (int k = 0; k <= kNumKinds; ++k) root_h.kind_begin[k] = ctx->w32.scene.kind_begin[k];
        root_h.any_secondary = ctx->w32.scene.any_secondary;
        root_h.duplicates = ctx->duplicate_shapes;
        root_h.flops_per_ray = ctx->flops.per_ray;
        root_h.bright_hit = ctx->bright_hit;
        root_h.bright_w = ctx->bright_w;
    }
    // 1. the header
    std::vector<SceneHeader*> d_hdr(ms.size(), nullptr);
    std::vector<SceneHeader> hdr(ms.size(), root_h);
    for (size_t i = 0; i < ms.size(); ++i) {
        RT_HIP(hipSetDevice(ms[i]->device));
        RT_HIP(hipMalloc(reinterpret_cast<void**>(&d_hdr[i]), sizeof(SceneHeader)));
        if (ms[i]->rank == 0) RT_HIP(hipMemcpy(d_hdr[i], &root_h, sizeof(SceneHeader), hipMemcpyHostToDevice));
    }
    auto free_hdr = [&]() {
        for (size_t i = 0; i < ms.size(); ++i) {
            (void)hipSetDevice(ms[i]->device);
            (void)hipFree(d_hdr[i]);
        }
    };
    auto bcast_header = [&]() -> int {
        RT_NCCL(ncclGroupStart());
        for (size_t i = 0; i < ms.size(); ++i)
            RT_NCCL(ncclBroadcast(d_hdr[i], d_hdr[i], sizeof(SceneHeader), ncclUint8, 0, ms[i]->comm, ms[i]->stream));
        RT_NCCL(ncclGroupEnd());
        for (size_t i = 0; i < ms.size(); ++i) {
            RT_HIP(hipSetDevice(ms[i]->device));
            RT_HIP(hipStreamSynchronize(ms[i]->stream));
            RT_HIP(hipMemcpy(&hdr[i], d_hdr[i], sizeof(SceneHeader), hipMemcpyDeviceToHost));
        }
        return RT_OK;
    };
    rc = bcast_header();
    free_hdr();
    if (rc) return rc;
    if (root_rc) return set_error(root_rc, root_err);
    for (const SceneHeader& h : hdr)
        if (h.status) return set_error(h.status, "rt_scene_upload failed on rank 0");

    // 2. the tables, broadcast in place from rank 0's device buffers.  Every
    // rank first allocates its copies, then the ranks agree on the outcome
    // (one all-reduce of a status word): a rank whose allocation failed still
    // takes part, so no other rank is left waiting in the table broadcast.
    std::vector<std::vector<std::pair<void*, size_t>>> bufs(ms.size());
    int local_rc = RT_OK;
    std::string local_err;
    for (size_t i = 0; i < ms.size() && !local_rc; ++i) {
        rt_context* m = ms[i];
        if (hipSetDevice(m->device) != hipSuccess) local_rc = set_error(RT_ERR_HIP, "hipSetDevice");
        else if (m->rank != 0) {
            if ((local_rc = alloc_world(m->w32, hdr[i])) == RT_OK) local_rc = alloc_world(m->w64, hdr[i]);
        }
        if (local_rc) local_err = rt_last_error();
    }
    if ((rc = agree_status(ms, local_rc))) return rc;
    if (local_rc) return set_error(local_rc, local_err);
    for (size_t i = 0; i < ms.size(); ++i) {
        world_buffers(ms[i]->w32, hdr[i], bufs[i]);
        world_buffers(ms[i]->w64, hdr[i], bufs[i]);
    }
    RT_NCCL(ncclGroupStart());
    for (size_t i = 0; i < ms.size(); ++i)
        for (auto& b : bufs[i])
            if (b.second) RT_NCCL(ncclBroadcast(b.first, b.first, b.second, ncclUint8, 0, ms[i]->comm, ms[i]->stream));
    RT_NCCL(ncclGroupEnd());
    for (size_t i = 0; i < ms.size(); ++i) {
        rt_context* m = ms[i];
        RT_HIP(hipSetDevice(m->device));
        RT_HIP(hipStreamSynchronize(m->stream));
        if (m->rank == 0) continue;
        const SceneHeader& h = hdr[i];
        describe_world(m->w32, h);
        describe_world(m->w64, h);
        m->world_slot.assign(h.ns, 0);
        if (h.ns)
            RT_HIP(hipMemcpy(m->world_slot.data(), m->w32.world_slot, h.ns * sizeof(int32_t), hipMemcpyDeviceToHost));
        if ((rc = fetch_jit_tables(m)) || (rc = capture_jit_table(m))) return rc;
        m->flops = FlopScene{};
        m->flops.per_ray = h.flops_per_ray;
        m->flops.n_lights = h.nl;
        m->bright_hit = h.bright_hit;
        m->bright_w = h.bright_w;
        m->duplicate_shapes = h.duplicates;
        m->have_scene = true;
        ++m->scene_gen;
    }
    return RT_OK;
}

int group_render_device(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* out_device,
                        hipStream_t stream) {
    int rc = check_group_options(ctx, o);
    if (rc) return rc;
    return render_shards(ctx, cam, o, out_device, stream, false);
}

int group_render(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* out_host,
                 rt_stats* stats) {
    int rc = check_group_options(ctx, o);
    if (rc) return rc;
    if (ctx->rank == 0 && !out_host) return set_error(RT_ERR_INVALID, "null output on rank 0");
    const std::vector<rt_context*> ms = members(ctx);
    const size_t bytes = (size_t)cam->width * cam->height * pixel_bytes(o);
    if (bytes == 0) {
        if (stats) std::memset(stats, 0, sizeof(*stats));
        return RT_OK;
    }
    std::vector<std::vector<unsigned long long>> before(ms.size(), std::vector<unsigned long long>(kNumCounters));
    for (size_t i = 0; i < ms.size(); ++i) {
        RT_HIP(hipSetDevice(ms[i]->device));
        if ((rc = read_counters(ms[i], before[i].data()))) return rc;
    }
    if (ctx->rank == 0) {
        RT_HIP(hipSetDevice(ctx->device));
        if ((rc = ensure_scratch(ctx, bytes))) return rc;
    }
    if ((rc = render_shards(ctx, cam, o, ctx->rank == 0 ? ctx->d_scratch : nullptr, ctx->stream, true))) return rc;
    if (ctx->rank == 0) {  // enqueued behind the de-interleave on rank 0's stream
        RT_HIP(hipSetDevice(ctx->device));
        if ((rc = copy_to_host(ctx, out_host, bytes))) return rc;
    }
    for (rt_context* m : ms) {
        RT_HIP(hipSetDevice(m->device));
        RT_HIP(hipStreamSynchronize(m->stream));
    }
    rt_stats total{};
    float render_ms = 0.f, gather_ms = 0.f, frame_ms = 0.f;
    for (size_t i = 0; i < ms.size(); ++i) {
        rt_context* m = ms[i];
        RT_HIP(hipSetDevice(m->device));
        if ((rc = check_pool_error(m))) return rc;
        unsigned long long after[kNumCounters];
        if ((rc = read_counters(m, after))) return rc;
        float r = 0.f;
        RT_HIP(hipEventElapsedTime(&r, m->ev_render0, m->ev_render1));
        render_ms = std::max(render_ms, r);
        if (m->rank == 0) {
            RT_HIP(hipEventElapsedTime(&gather_ms, m->ev_render1, m->ev_gather1));
            RT_HIP(hipEventElapsedTime(&frame_ms, m->ev_render0, m->ev_gather1));
        }
        rt_stats s{};
        fill_stats(m, before[i].data(), after, r, &s);
        total.primary += s.primary;
        total.shadow += s.shadow;
        total.reflect += s.reflect;
        total.refract += s.refract;
        total.shaded += s.shaded;
        total.lit_patterned += s.lit_patterned;
        total.refract_evals += s.refract_evals;
        total.schlick_evals += s.schlick_evals;
        total.algorithmic_flops += s.algorithmic_flops;
    }
    if (stats) {
        *stats = total;
        stats->kernel_ms = render_ms;
        stats->gather_ms = gather_ms;
        stats->frame_ms = frame_ms;
        stats->n_shards = (uint32_t)ctx->n_ranks;
    }
    return RT_OK;
}

int group_read_counters(rt_context* ctx, rt_stats* totals) {
    rt_stats t{};
    int rc;
    for (rt_context* m : members(ctx)) {
        RT_HIP(hipSetDevice(m->device));
        RT_HIP(hipDeviceSynchronize());
        unsigned long long zero[kNumCounters] = {}, now[kNumCounters];
        if ((rc = read_counters(m, now))) return rc;
        rt_stats s{};
        fill_stats(m, zero, now, 0.f, &s);
        t.primary += s.primary;
        t.shadow += s.shadow;
        t.reflect += s.reflect;
        t.refract += s.refract;
        t.shaded += s.shaded;
        t.lit_patterned += s.lit_patterned;
        t.refract_evals += s.refract_evals;
        t.schlick_evals += s.schlick_evals;
        t.algorithmic_flops += s.algorithmic_flops;
        if ((rc = check_pool_error(m))) return rc;
    }
    t.n_shards = (uint32_t)ctx->n_ranks;
    *totals = t;
    return RT_OK;
}

}  // namespace rtc

using namespace rtc;

extern "C" {

int rt_context_create_multi(const int* devices, int n, rt_context** out) {
    if (!devices || !out || n < 1) return set_error(RT_ERR_INVALID, "rt_context_create_multi: bad arguments");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return set_error(RT_ERR_NO_DEVICE, "no HIP device available (the render path has no CPU fallback)");
    for (int i = 0; i < n; ++i) {
        if (devices[i] < 0 || devices[i] >= count) return set_error(RT_ERR_INVALID, "device ordinal out of range");
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) return set_error(RT_ERR_INVALID, "a device appears twice");
    }
    std::vector<rt_context*> ms(n, nullptr);
    auto cleanup = [&]() {
        for (rt_context* m : ms) destroy_device_context(m);
    };
    for (int i = 0; i < n; ++i)
        if (int rc = create_device_context(devices[i], &ms[i])) {
            cleanup();
            return rc;
        }
    std::vector<ncclComm_t> comms(n, nullptr);
    if (ncclResult_t r = ncclCommInitAll(comms.data(), n, devices); r != ncclSuccess) {
        cleanup();
        return set_error(RT_ERR_COMM, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    }
    for (int i = 0; i < n; ++i)
        if (int rc = init_member(ms[i], comms[i], n, i)) {
            cleanup();
            return rc;
        }
    ms[0]->peers.assign(ms.begin() + 1, ms.end());
    *out = ms[0];
    return RT_OK;
}

int rt_comm_unique_id(uint8_t id[RT_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == RT_UNIQUE_ID_BYTES, "RT_UNIQUE_ID_BYTES must match ncclUniqueId");
    if (!id) return set_error(RT_ERR_INVALID, "null id");
    ncclUniqueId u;
    if (ncclResult_t r = ncclGetUniqueId(&u); r != ncclSuccess)
        return set_error(RT_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof(u));
    return RT_OK;
}

int rt_context_create_rank(int device, int n_ranks, int rank, const uint8_t id[RT_UNIQUE_ID_BYTES],
                           rt_context** out) {
    if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return set_error(RT_ERR_INVALID, "rt_context_create_rank: bad arguments");
    *out = nullptr;
    rt_context* m = nullptr;
    if (int rc = create_device_context(device, &m)) return rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    (void)hipSetDevice(device);
    if (ncclResult_t r = ncclCommInitRank(&comm, n_ranks, u, rank); r != ncclSuccess) {
        destroy_device_context(m);
        return set_error(RT_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    if (int rc = init_member(m, comm, n_ranks, rank)) {
        destroy_device_context(m);
        return rc;
    }
    *out = m;
    return RT_OK;
}

int rt_context_set_gather(rt_context* ctx, int mode) {
    if (!ctx || (mode != RT_GATHER_RCCL && mode != RT_GATHER_PEER)) return set_error(RT_ERR_INVALID, "bad arguments");
    for (rt_context* m : members(ctx)) m->gather_mode = mode;
    return RT_OK;
}

int rt_context_group(rt_context* ctx, int* n_ranks, int* rank, int* local_devices) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    if (n_ranks) *n_ranks = ctx->n_ranks;
    if (rank) *rank = ctx->rank;
    if (local_devices) *local_devices = 1 + (int)ctx->peers.size();
    return RT_OK;
}

}  // extern "C"
