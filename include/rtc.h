/*
 * rtc.h — C-ABI of the MI355X-native render path for the Ray Tracer Challenge
 * world model of przemo199/ray-tracer-challenge-rs.
 *
 * This is the drop-in boundary.  It replaces, for one
 * frame, the reference's
 *     Camera::render           ray-tracer/src/composites/camera.rs:79-95
 *     Camera::render_parallel  ray-tracer/src/composites/camera.rs:97-112
 * and, per ray,
 *     World::color_at          ray-tracer/src/composites/world.rs:89-95
 * with a HIP wavefront tracer for gfx950.  The reference's only caller of the
 * render loop is ray-tracer-cli/src/main.rs:18-21; a GPU variant is a third
 * RenderingMode arm there (ray-tracer-cli/src/cli/rendering_mode.rs:3-7).
 *
 * Conventions (mirroring the reference's ownership rules):
 *   - every input is a plain POD array in f64, i.e. exactly the values the
 *     reference holds on the host (Matrix<4> is [[f64;4];4] row-major,
 *     primitives/matrix.rs:8);
 *   - the caller owns every host buffer; the library owns device buffers
 *     except the explicit *_device entry points, which write into a
 *     caller-owned device buffer on a caller-supplied HIP stream;
 *   - return 0 (RT_OK) on success, a negative rt_status on failure;
 *     rt_last_error() gives a thread-local message.  The reference panics
 *     instead (release profile panic=abort, Cargo.toml:16); a host wrapper
 *     mirroring it turns a negative status into a panic/exception;
 *   - one context drives one GPU and is used from one host thread at a time;
 *     its launches are ordered: rt_render / rt_color_at run on the context's
 *     own stream, rt_render_device on the caller's, and a launch on another
 *     stream than the previous launch's waits for everything submitted to
 *     that stream so far.  A stream handed to rt_render_device must stay
 *     valid until the context's next launch on a different stream (or
 *     rt_context_destroy);
 *   - there is NO CPU fallback: without a usable HIP device every entry
 *     point that computes returns RT_ERR_NO_DEVICE.
 */
#ifndef RTC_H
#define RTC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3

/* Image tile rendered by one workgroup (one wave = one 64-pixel row run, so
 * output stores are contiguous); RT_TILE_H rows are also the row-block unit
 * of shards. */
#define RT_TILE_W 64
#define RT_TILE_H 4

/* World::MAX_REFLECTION_ITERATIONS, ray-tracer/src/composites/world.rs:15 */
#define RT_DEFAULT_MAX_DEPTH 6
/* largest recursion depth the device ray pool is sized for */
#define RT_MAX_SUPPORTED_DEPTH 16

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,      /* bad argument / malformed descriptor       */
    RT_ERR_HIP = -2,          /* a HIP runtime call failed                 */
    RT_ERR_NO_DEVICE = -3,    /* no HIP device / extension not usable      */
    RT_ERR_NO_SCENE = -4,     /* render before rt_scene_upload             */
    RT_ERR_OOM = -5,          /* device allocation failed                  */
    RT_ERR_POOL = -6,         /* device ray pool overflow (never expected) */
    RT_ERR_IO = -7,           /* file / parse error (scene loader)         */
    RT_ERR_COMM = -8          /* RCCL (multi-GPU) call failed              */
} rt_status;

/* Shape kinds: ray-tracer/src/shapes.rs:1-17 */
typedef enum rt_shape_kind {
    RT_SHAPE_SPHERE = 0,   /* shapes/sphere.rs   */
    RT_SHAPE_PLANE = 1,    /* shapes/plane.rs    */
    RT_SHAPE_CUBE = 2,     /* shapes/cube.rs     */
    RT_SHAPE_CYLINDER = 3, /* shapes/cylinder.rs */
    RT_SHAPE_CONE = 4,     /* shapes/cone.rs     */
    RT_SHAPE_TRIANGLE = 5  /* shapes/triangle.rs */
} rt_shape_kind;

/* Pattern kinds: ray-tracer/src/patterns.rs:1-14 (+ test-only TestPattern,
 * patterns/pattern.rs:29-66, which the reference's own world tests use). */
typedef enum rt_pattern_kind {
    RT_PATTERN_STRIPE = 0,   /* patterns/stripe_pattern.rs   */
    RT_PATTERN_GRADIENT = 1, /* patterns/gradient_pattern.rs */
    RT_PATTERN_RING = 2,     /* patterns/ring_pattern.rs     */
    RT_PATTERN_CHECKER = 3,  /* patterns/checker_pattern.rs  */
    RT_PATTERN_COMPLEX = 4,  /* patterns/complex_pattern.rs  */
    RT_PATTERN_TEST = 5      /* patterns/pattern.rs:29-66    */
} rt_pattern_kind;

typedef enum rt_precision {
    RT_PRECISION_F32 = 0, /* the throughput path (north star: f32)          */
    RT_PRECISION_F64 = 1  /* parity path: same op order / FMA sites as ref  */
} rt_precision;

typedef enum rt_out_format {
    RT_OUT_REAL = 0, /* f32 RGB (precision f32) or f64 RGB (precision f64)  */
    RT_OUT_U8 = 1    /* u8 RGB, round(clamp(c,0,1)*255): canvas.rs:117-123  */
} rt_out_format;

/* One entry of World.shapes (world.rs:9-12).  The shape's inverse transform
 * is what Transform::transformation_inverse() returns (shapes/shape.rs:6-14);
 * the library never inverts, so host and device see the same f64 inverse. */
typedef struct rt_shape_desc {
    int32_t kind;        /* rt_shape_kind                                  */
    int32_t material;    /* index into the material table                  */
    double inverse[16];  /* row-major Matrix<4>                            */
    double minimum;      /* cylinder/cone `min` (cylinder.rs:12, cone.rs:12) */
    double maximum;      /* cylinder/cone `max`                            */
    int32_t closed;      /* cylinder/cone `closed`                         */
    int32_t reserved;
    double vertex_1[3];  /* triangle.rs:12-17 */
    double edge_1[3];
    double edge_2[3];
    double normal[3];
} rt_shape_desc;

/* composites/material.rs:9-20 */
typedef struct rt_material_desc {
    double color[3];
    double ambient;
    double diffuse;
    double specular;
    double shininess;
    double reflectiveness;
    double transparency;
    double refractive_index;
    int32_t casts_shadow;
    int32_t pattern; /* index into the pattern table, -1 = None */
} rt_material_desc;

/* One Arc<dyn Pattern> (patterns/pattern.rs:6-15). */
typedef struct rt_pattern_desc {
    int32_t kind;       /* rt_pattern_kind                                 */
    int32_t sub_a;      /* ComplexPattern pattern_a (index), else -1       */
    int32_t sub_b;      /* ComplexPattern pattern_b (index), else -1       */
    int32_t reserved;
    double color_a[3];
    double color_b[3];
    double inverse[16]; /* pattern transformation_inverse, row-major       */
} rt_pattern_desc;

/* primitives/light.rs:6-10 */
typedef struct rt_light_desc {
    double position[3];
    double intensity[3];
} rt_light_desc;

/* The private state of Camera (camera.rs:10-19) after Camera::new
 * (camera.rs:25-49) and set_transformation (camera.rs:124-127). */
typedef struct rt_camera_desc {
    uint32_t width;
    uint32_t height;
    double field_of_view;
    double half_width;
    double half_height;
    double pixel_size;
    double inverse[16]; /* camera transformation_inverse, row-major */
    double origin[3];   /* inverse * Point::ORIGIN (camera.rs:114-116)  */
} rt_camera_desc;

/* Diagnostic ablation flags (profiling only; outputs are wrong with them). */
#define RT_FLAG_NO_COUNTERS 1u /* skip the per-workgroup counter flush      */
#define RT_FLAG_NO_SHADE 2u    /* closest hit only, colour = normalised t   */
#define RT_FLAG_NO_TRACE 4u    /* camera ray only, colour = direction       */
#define RT_FLAG_STAMPS 8u      /* record per-workgroup start/end timestamps */
#define RT_FLAG_FAIL_LAUNCH 16u /* fail with RT_ERR_HIP after planning, before
                                  * the enqueue (tests the error path)      */
#define RT_FLAG_GENERATIONS 32u /* also count rays per generation (generic
                                  * kernels; rt_read_generation_counts).
                                  * Pixels and rt_stats are unchanged.      */
#define RT_FLAG_NO_SKIPS 64u    /* trace without the skips: the shadow ray's
                                  * (light behind the surface, plane side,
                                  * cube faces, blocked clusters), the cube
                                  * exit path, planes behind every ray of a
                                  * wave and the containers walk's hit-point
                                  * cull: acceleration only, so pixels and
                                  * rt_stats are unchanged (exactness tests;
                                  * per-scene kernels get a build of their
                                  * own)                                    */

typedef struct rt_render_options {
    uint32_t max_depth;    /* `remaining` of the primary ray; 6 = reference */
    uint32_t precision;    /* rt_precision                                  */
    uint32_t out_format;   /* rt_out_format                                 */
    uint32_t shard_index;  /* row-block sharding            */
    uint32_t shard_count;  /* 1 = the whole image                           */
    uint32_t flags;        /* 0; RT_FLAG_* diagnostic ablations (never in  */
                           /* a parity or benchmark result)                */
} rt_render_options;

/* Ray counts in the reference's semantics plus the terms of
 * the algorithmic-FLOP convention. */
typedef struct rt_stats {
    uint64_t primary;        /* camera rays (or rays handed to rt_color_at) */
    uint64_t shadow;         /* L per shaded hit (world.rs:46-52)           */
    uint64_t reflect;        /* spawned reflection rays (world.rs:114-128)  */
    uint64_t refract;        /* spawned refraction rays (world.rs:130-157)  */
    uint64_t shaded;         /* shaded hits (prepare_computations calls)    */
    uint64_t lit_patterned;  /* light evaluations on a patterned material   */
    uint64_t refract_evals;  /* refracted_color past the opaque/depth check */
    uint64_t schlick_evals;  /* schlicks_approximation calls                */
    double kernel_ms;        /* device time of the render launch (multi-GPU: */
                             /* the slowest shard's)                         */
    double algorithmic_flops;/* SURVEY.md §8d convention                    */
    double gather_ms;        /* multi-GPU: RCCL gather of the strips + the   */
                             /* de-interleave on rank 0 (0 on one GPU)       */
    double frame_ms;         /* device time of the whole frame               */
    uint32_t n_shards;       /* GPUs the frame was split over                */
    uint32_t reserved;
} rt_stats;

typedef struct rt_context rt_context;

int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* count);

int rt_context_create(int device_ordinal, rt_context** out);
int rt_context_destroy(rt_context* ctx);

/* Multi-GPU contexts (the north star's "image optionally
 * tiled across 8 GPUs of one node via RCCL broadcast of the scene + gather of
 * framebuffer strips over xGMI").  A group context splits every frame into
 * one shard per GPU (cyclic RT_TILE_H-row blocks, rt_shard_rows), gathers the
 * strips onto rank 0 with RCCL and de-interleaves them there;
 * rt_scene_upload flattens the world on rank 0 and RCCL-broadcasts the device
 * tables to every GPU.  The entry points keep their single-GPU meaning:
 * rt_render / rt_render_device deliver the WHOLE image on rank 0 (so
 * options.shard_index/shard_count must be 0/1), rt_color_at runs on rank 0.
 *  - one process driving several GPUs: rt_context_create_multi
 *    (ncclCommInitAll over `devices`);
 *  - one process per GPU: rank 0 makes an id with rt_comm_unique_id, the
 *    caller shares it (any channel), and every rank calls
 *    rt_context_create_rank (ncclCommInitRank).  Every rank then makes the
 *    same calls with the same camera and options (collective semantics);
 *    only rank 0's scene tables and output buffer are used — other ranks may
 *    pass NULL tables with zero counts and a NULL output.  Counters and stats
 *    are the calling process's own shards. */
#define RT_UNIQUE_ID_BYTES 128
int rt_context_create_multi(const int* devices, int n_devices, rt_context** out);
int rt_comm_unique_id(uint8_t id[RT_UNIQUE_ID_BYTES]);
int rt_context_create_rank(int device, int n_ranks, int rank, const uint8_t id[RT_UNIQUE_ID_BYTES],
                           rt_context** out);
/* Shards per frame, this context's rank, and the GPUs this process drives. */
int rt_context_group(rt_context* ctx, int* n_ranks, int* rank, int* local_devices);

/* Flatten + upload a world.  Replaces the World value that Camera::render
 * borrows (camera.rs:79).  Tables are copied; the caller may free them. */
int rt_scene_upload(rt_context* ctx,
                    const rt_shape_desc* shapes, uint32_t n_shapes,
                    const rt_material_desc* materials, uint32_t n_materials,
                    const rt_pattern_desc* patterns, uint32_t n_patterns,
                    const rt_light_desc* lights, uint32_t n_lights);

/* Rows of the strip one shard writes (RT_TILE_H-row blocks, cyclic: tile
 * row k of the image belongs to shard k % shard_count).  Every strip is
 * padded to this height (shard 0's), so gathers use equal counts. */
int rt_shard_rows(uint32_t height, uint32_t shard_count, uint32_t* rows);
/* For each image row y < height: the shard that renders it and its row in
 * that shard's strip (the map rt_assemble_shards inverts).  Host only. */
int rt_shard_row_map(uint32_t height, uint32_t shard_count, uint32_t* shard_of_row, uint32_t* strip_row_of_row);

/* Synchronous render into a caller-owned HOST buffer: Camera::render /
 * render_parallel semantics (camera.rs:79-112).  Output is row-major, y = 0
 * on top (canvas.rs:53-55); 3 channels per pixel of f32/f64/u8. With
 * shard_count > 1 the buffer holds this shard's strip (rt_shard_rows rows). */
int rt_render(rt_context* ctx, const rt_camera_desc* camera,
              const rt_render_options* options, void* out_host,
              rt_stats* stats);

/* Asynchronous render into a caller-owned DEVICE buffer on `hip_stream`
 * (a hipStream_t; NULL = HIP's default stream).  No host sync.  The caller's
 * HIP runtime must be the one librtc is bound to (one runtime per process). */
int rt_render_device(rt_context* ctx, const rt_camera_desc* camera,
                     const rt_render_options* options, void* out_device,
                     void* hip_stream);

/* Batch World::color_at (world.rs:89-95): rays[i] = {ox,oy,oz,dx,dy,dz},
 * out[i] = RGB, both f64 host arrays; `max_depth` = remaining.  In a world
 * with reflective or transparent materials (max_depth > 0) every direction
 * must be unit length within 1e-6, as the camera's are (camera.rs:66), or
 * RT_ERR_INVALID: the ray trees' fixed-point pixel sums are bounded for unit
 * directions, and with eye = -d the specular term grows as |d|^shininess. */
int rt_color_at(rt_context* ctx, const double* rays, uint64_t n_rays,
                uint32_t max_depth, uint32_t precision, double* out_rgb,
                rt_stats* stats);

/* Diagnostics: the per-workgroup {start, end} s_memrealtime stamps (100 MHz)
 * of the last launch made with RT_FLAG_STAMPS; *n = number of workgroups. */
int rt_debug_stamps(rt_context* ctx, uint64_t* out, uint32_t max_workgroups, uint32_t* n);

/* Diagnostics: per-tile durations (10 ns ticks) the last pool launch
 * recorded for heaviest-first ordering; *n = entries available (tiles of
 * the largest pool launch so far, 0 before any). */
int rt_debug_tile_costs(rt_context* ctx, uint32_t* out, uint32_t max_tiles, uint32_t* n);

/* Diagnostics: the work items of the last pool launch made with
 * RT_FLAG_STAMPS, in the order they were taken: 3 x u64 per item {item |
 * workgroup << 32, start, end} (s_memrealtime, 100 MHz; item encoding in
 * rtc_internal.hpp); *n = number of items logged. */
int rt_debug_item_log(rt_context* ctx, uint64_t* out, uint32_t max_items, uint32_t* n);

/* Known-answer harness: the device's own per-shape code for the shape at
 * world index `shape` of the uploaded world, on caller-given inputs (the
 * reference's per-shape unit tests, e.g. cone.rs:191-252, run on the GPU).
 * rt_debug_intersect: rays[i] = {ox,oy,oz,dx,dy,dz}; world_space = 0 treats
 * them as local rays (Intersect::local_intersect), 1 transforms them by the
 * shape's inverse first (Ray::intersect, ray.rs:45-49).  out[i*5] = entries
 * the reference pushes (<= RT_DEBUG_MAX_ENTRIES), out[i*5+1..] their t in push
 * order.  rt_debug_normal: points[i] = {x,y,z}; world_space = 0 gives
 * local_normal_at (not normalized), 1 gives normal_at (shape.rs:22-27);
 * out[i*3..] = the normal.  Synchronous; host buffers. */
#define RT_DEBUG_MAX_ENTRIES 4
int rt_debug_intersect(rt_context* ctx, uint32_t shape, const double* rays, uint64_t n_rays, uint32_t precision,
                       uint32_t world_space, double* out);
int rt_debug_normal(rt_context* ctx, uint32_t shape, const double* points, uint64_t n_points, uint32_t precision,
                    uint32_t world_space, double* out);

/* Per-scene kernels.  For f32 frames the library compiles (hipRTC), once
 * per uploaded world, the same tracer source with the world's shape table as
 * compile-time constants, and runs it instead of the generic kernel (same
 * pixels, bit for bit).  Modes (rt_context_set_jit; env RTC_JIT=0|1|2|3 at
 * context creation):
 *   RT_JIT_OFF    never;
 *   RT_JIT_SYNC   every f32 frame, the build compiled in line on the first
 *                 one (deterministic: tests);
 *   RT_JIT_AUTO   the default.  Frames of at least 64K pixels; the build runs
 *                 on a host thread, started by the SECOND such frame of an
 *                 uploaded world, and frames render with the generic kernel
 *                 until it is ready.  A one-shot render (Camera::render, the
 *                 CLI) never compiles; repeated renders switch once the
 *                 build lands.  A build already made in this process (or on
 *                 disk) for the same world is used from the first frame;
 *   RT_JIT_EAGER  as AUTO, but the first large frame starts the build.
 * rt_jit_status: whether the last launch ran a per-scene kernel, the compile
 * (or cache-load) milliseconds of the builds this context started, and the
 * last build error (a failed build keeps the generic kernel for that world).
 * rt_jit_wait: block until this context's builds in flight have finished
 * (at most timeout_ms; < 0 = no limit); *pending = builds still running.
 * A context destroyed with a build in flight does not wait for it: the
 * compile runs in a child process (rtc_jitc) and a DETACHED thread of this
 * process waits for it, runs librtc code when it ends, and is never joined.
 * So librtc must not be unloaded (dlclose) while rt_jit_wait reports pending
 * builds; process exit is safe (the orphaned compiler still finishes and
 * fills the disk cache).  Builds are also cached on
 * disk across processes: env RTC_JIT_CACHE = a directory, or 0 for none
 * (default $XDG_CACHE_HOME/rtc_jit, else ~/.cache/rtc_jit). */
enum { RT_JIT_OFF = 0, RT_JIT_SYNC = 1, RT_JIT_AUTO = 2, RT_JIT_EAGER = 3 };
int rt_context_set_jit(rt_context* ctx, int mode);

/* A planning hint: the caller keeps `frames` frames in flight (consecutive
 * frames alternating between that many contexts, each on a stream of its
 * own, so one frame's launch tail overlaps the next frame's start;
 * INTEGRATION.md §2).  1 (the default) plans each launch for its own
 * latency; > 1 plans the f32 direct kernel's grid for throughput (1.5x the
 * resident workgroups instead of 2.5x: round 6, three_sphere 1080p with two
 * in flight 339 -> 355-361 Gray/s, one frame alone 15.5 -> 16.1 us) and
 * splits the pool kernels' heavy tiles only above 1.5x the mean workgroup
 * load instead of 1x (a 4K shard of 8 with two in flight: cover 0.104 ->
 * 0.094 ms).  Pixels and rt_stats are unchanged.  Applies to every member of
 * a group. */
int rt_context_set_frames_in_flight(rt_context* ctx, uint32_t frames);
int rt_jit_status(rt_context* ctx, int* used_last_launch, double* compile_ms, char* log, size_t log_len);
int rt_jit_wait(rt_context* ctx, double timeout_ms, int* pending);

/* Peer canvas: a frame assembled in place instead of gathered (SURVEY.md
 * §8e; the north star's "gather of framebuffer strips over xGMI" done as the
 * shards' own stores into rank 0's image).  The owner creates a device canvas
 * (an image of `bytes` plus n_flags completion flags and one release flag)
 * and shares its IPC handle; other processes map it with rt_canvas_open.
 * rt_render_to_canvas renders shard options.shard_index of
 * options.shard_count straight into the canvas at its pixels' IMAGE rows,
 * then raises that shard's flag to `seq`; before rendering it waits (on the
 * device) until the owner has released frame seq - 1, so a shard never
 * overwrites a frame still being read.  rt_canvas_wait makes the owner's
 * stream wait until every flag has reached `seq`; rt_canvas_release marks
 * frame `seq` consumed (stream-ordered after its readers).  `seq` starts at 1
 * and grows by one per frame; the flags start at 0.  The waits are bounded:
 * after timeout_ms a wait ends and RT_ERR_POOL ("peer canvas") is reported
 * at the context's next synchronous call.  Asynchronous on `hip_stream`
 * except create / open / close, which synchronize. */
#define RT_IPC_HANDLE_BYTES 64
int rt_canvas_create(rt_context* ctx, uint64_t bytes, uint32_t n_flags, void** canvas,
                     uint8_t handle[RT_IPC_HANDLE_BYTES]);
int rt_canvas_open(rt_context* ctx, const uint8_t handle[RT_IPC_HANDLE_BYTES], uint64_t bytes, uint32_t n_flags,
                   void** canvas);
int rt_canvas_close(rt_context* ctx, void* canvas);
int rt_render_to_canvas(rt_context* ctx, const rt_camera_desc* camera, const rt_render_options* options,
                        void* canvas, uint64_t seq, double timeout_ms, void* hip_stream);
int rt_canvas_wait(rt_context* ctx, void* canvas, uint64_t seq, double timeout_ms, void* hip_stream);
int rt_canvas_release(rt_context* ctx, void* canvas, uint64_t seq, void* hip_stream);
/* The canvas image (its first `bytes`) into a host buffer, after everything
 * submitted to this context's device (synchronous). */
int rt_canvas_read(rt_context* ctx, void* canvas, void* out_host, uint64_t bytes);

/* How a multi-GPU context brings the shards to rank 0: RT_GATHER_RCCL (the
 * default) renders strips and ncclGathers + de-interleaves them;
 * RT_GATHER_PEER renders every shard into one peer canvas on rank 0 (IPC
 * handle broadcast over RCCL once; peer access within one process) and
 * copies the finished image to the caller's buffer.  Collective: every rank
 * sets the same mode. */
enum { RT_GATHER_RCCL = 0, RT_GATHER_PEER = 1 };
int rt_context_set_gather(rt_context* ctx, int mode);

/* Cumulative device counters since context creation (after a sync). */
int rt_read_counters(rt_context* ctx, rt_stats* totals);

/* Rays per generation (the wavefront's size at each bounce), cumulative
 * over this context's launches made with RT_FLAG_GENERATIONS.  Indexed by
 * `remaining` (world.rs:70-86): a primary ray is traced at max_depth and a
 * reflected or refracted child at its parent's remaining - 1
 * (world.rs:114-157), so generation g of a frame rendered at depth D is
 * entry D - g.  traced = radiance rays traced (internal_color_at calls),
 * shaded = hits shaded; each shaded hit casts one shadow ray per light
 * (world.rs:46-52).  Group contexts report the calling process's GPUs. */
typedef struct rt_generation_counts {
    uint64_t traced[RT_MAX_SUPPORTED_DEPTH + 1];
    uint64_t shaded[RT_MAX_SUPPORTED_DEPTH + 1];
} rt_generation_counts;
int rt_read_generation_counts(rt_context* ctx, rt_generation_counts* out);

/* De-interleave gathered shard strips (shard-major, each rt_shard_rows tall)
 * into one row-major image on the device, on `hip_stream`. */
int rt_assemble_shards(rt_context* ctx, const void* gathered_device,
                       uint32_t width, uint32_t height, uint32_t shard_count,
                       uint32_t bytes_per_pixel, void* image_device,
                       void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* RTC_H */
