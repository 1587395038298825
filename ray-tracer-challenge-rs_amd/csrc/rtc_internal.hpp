// rtc_internal.hpp — records shared by the host launcher (rtc_host.cpp) and
// the gfx950 kernels (rtc_kernels.hip).
//
// HBM layout of a flattened world (SURVEY.md §7 "SoA per-type shape tables"):
// the reference's Vec<Box<dyn Shape>> (world.rs:11) becomes ONE array of
// fixed-size ShapeRec sorted by kind (spheres, planes, cubes, cylinders,
// cones, triangles), with `kind_begin[k]..kind_begin[k+1]` delimiting the
// per-type loops.  Every lane of a wave walks the same records in the same
// order, so the shape loads are wave-uniform scalar (s_load) loads that hit
// the scalar cache; `world_index` restores the reference's world order for
// the stable-sort tie rule.  Materials, patterns and
// lights are small side tables.  Everything is cast once from the caller's
// f64 tables to the kernel's real type R (f32 or f64).
#pragma once

#include <cstdint>
#ifndef __HIPCC_RTC__
#include <string>
#endif

#include "../../include/rtc.h"

#if defined(__HIP__)
#define RTC_HD __host__ __device__
#else
#define RTC_HD
#endif

namespace rtc {

#ifndef __HIPCC_RTC__
int set_error(int code, const std::string& msg);  // rtc_host.cpp (thread-local)
#endif

// Row-block shards: tile row k of the image (RT_TILE_H rows)
// belongs to shard k % shards, which renders its tile rows in order into a
// contiguous strip.  One definition for the kernels' pixel mapping, the
// de-interleave kernel and the host (rt_shard_row_map, tested on CPU).
RTC_HD inline uint32_t shard_tile_rows(uint32_t height, uint32_t shards, uint32_t shard) {
    const uint32_t trows = (height + RT_TILE_H - 1) / RT_TILE_H;
    return trows > shard ? (trows - shard + shards - 1) / shards : 0;
}
// image row of row `strip_row` of shard `shard`'s strip
RTC_HD inline uint32_t shard_image_row(uint32_t strip_row, uint32_t shards, uint32_t shard) {
    return ((strip_row / RT_TILE_H) * shards + shard) * RT_TILE_H + strip_row % RT_TILE_H;
}
// shard and strip row of image row y (the inverse)
RTC_HD inline void shard_of_image_row(uint32_t y, uint32_t shards, uint32_t* shard, uint32_t* strip_row) {
    const uint32_t trow = y / RT_TILE_H;
    *shard = trow % shards;
    *strip_row = (trow / shards) * RT_TILE_H + y % RT_TILE_H;
}

constexpr int kBlock = 256;        // threads per workgroup = 4 waves of 64
constexpr int kWaves = kBlock / 64;  // waves per workgroup
// The pool kernel's shape (rtc_kernels.hip trace_pool): block-lockstep
// generations of up to kBlock rays over one tile's pixel accumulators.
constexpr int kTileSlots = 1;
constexpr uint32_t kPoolBatch = kBlock;  // rays a generation pops
constexpr int kTilePixels = RT_TILE_W * RT_TILE_H;  // one tile per workgroup pass
static_assert(kTilePixels == kBlock, "one pixel per thread per tile");
constexpr int kNumKinds = 6;
constexpr int kNumCounters = 8;    // order of rt_stats' first eight fields
constexpr int kGenSlots = RT_MAX_SUPPORTED_DEPTH + 1;  // rt_generation_counts, by `remaining`
// Event counters are sharded: workgroup b adds into shard b % kCounterShards
// (same-address global atomics from every workgroup cost ~66 us per 1080p
// frame on MI355X; sharded they are noise).  The host sums the shards.
constexpr int kCounterShards = 256;
// Tile queues: one atomic head saturates at ~88 dequeues/us on MI355X
// (MI355X_MICROARCH.md, price list row "dequeue"), i.e. ~93 us for the 8160
// tiles of a 1920x1080 frame.  Tile t lives in queue t % 8 and workgroup b
// pulls from queue b % 8 (blocks b and b+8 share an XCD under round-robin
// dispatch; placement only affects speed).
constexpr int kTileQueues = 8;
// Queue heads sit kQueueStride u64 apart (256 B): adjacent heads shared one
// cache line, so every XCD's dequeues serialized on it (~17 us per 1792
// dequeues on MI355X).
constexpr int kQueueStride = 32;
// Work items of a cost-ordered pool launch: one part of a tile split 4 to 64
// ways (order_tiles).  item = tile | part << 20 | log2(parts) << 26 |
// priority << 29; part p of a tile split 2^l ways seeds the pixels of
// threads t with t >> (8 - l) == p (waves, half-waves, wave rows, half rows
// and quarter rows of a wave's 16 x 4 block).  Cost-ordered launches need n_tiles <= 2^20
// (plan_tile_order; larger frames keep raster order).
// An item of priority p > 0 (the costliest, order_tiles) runs its waves at
// s_setprio(p).
constexpr uint32_t kItemTileMask = 0xFFFFFu;
constexpr uint32_t kItemPartShift = 20, kItemSplitShift = 26, kItemPartMask = 63u, kItemSplitMask = 7u;
constexpr uint32_t kItemPrioShift = 29;  // (bit 31 stays clear: no item equals kNoItem)
constexpr uint32_t kMaxSplitLog2 = 6;  // up to 64 items per tile (4 pixels each)
// order_tiles runs on launches 2 .. 1 + kOrderBuilds of a frame signature,
// then the order is reused (rtc_host.cpp plan_tile_order).
constexpr int kOrderBuilds = 8;
constexpr uint32_t kNoItem = 0xFFFFFFFFu;  // next_tile: the launch's items are all taken

// A work item, decoded.  Only launches that hand items out through a tile
// order (LaunchParams::tile_order set: cost-ordered or centre-out, which
// plan_tile_order allows for n_tiles <= 2^20 only) carry the packed fields;
// a raster launch's item is the plain tile index, whatever the launch's size
// (an rt_color_at batch reaches 2^24 tiles).  Decoding a raster item >= 2^20
// as packed would mask its tile and read stray part/split/priority bits.
struct WorkItem {
    uint32_t tile, part, split_log2, prio;
};
RTC_HD inline WorkItem decode_item(uint32_t item, bool packed) {
    if (!packed) return {item, 0u, 0u, 0u};
    return {item & kItemTileMask, (item >> kItemPartShift) & kItemPartMask, (item >> kItemSplitShift) & kItemSplitMask,
            (item >> kItemPrioShift) & 3u};
}
RTC_HD inline uint32_t encode_item(uint32_t tile, uint32_t part, uint32_t split_log2, uint32_t prio) {
    return tile | part << kItemPartShift | split_log2 << kItemSplitShift | prio << kItemPrioShift;
}
// Part p of a tile split 2^l ways seeds the threads t of the tile's
// workgroup with t >> (8 - l) == p (halves, wave pairs, waves, half-waves,
// wave rows); l = 0 seeds all 256.
RTC_HD inline bool item_seeds(uint32_t tid, const WorkItem& w) { return (tid >> (8u - w.split_log2)) == w.part; }

// Spilled pool entries: workgroup b of a pool launch owns records
// [b * spill_cap, (b + 1) * spill_cap) of LaunchParams::spill, 8 words each;
// slot s >= lds_cap of its LIFO is record s - lds_cap.
RTC_HD inline uint64_t spill_word(uint32_t block, uint32_t spill_cap, uint32_t slot, uint32_t lds_cap) {
    return ((uint64_t)block * spill_cap + (slot - lds_cap)) * 8u;
}

// RTC_BOUNDS_CHECK builds (debug variant, scripts/build_variant.sh): the pool
// kernel checks every computed index against its buffer before the access,
// skips a bad access and raises one of these bits of LaunchParams::error_flag
// (the host reports them as RT_ERR_POOL with the bit's name).
constexpr int32_t kErrPoolOverflow = 1;  // a child beyond the LIFO bound (no debug build needed)
constexpr int32_t kErrPoolSpin = 2;      // a pool lock's spin bound ran out (scripts/patches/pool_free_and_diag.patch only)
constexpr int32_t kErrBoundsSlot = 4;    // pool slot outside [0, cap)
constexpr int32_t kErrBoundsSpill = 8;   // spill record outside the launch's spill buffer
constexpr int32_t kErrBoundsTile = 16;   // work item's tile >= n_tiles
constexpr int32_t kErrBoundsOut = 32;    // output element outside the canvas or strip
constexpr int32_t kErrPeerTimeout = 64;  // rt_canvas_wait: a shard's flag did not arrive in time
constexpr int32_t kErrBitsAll[] = {kErrPoolOverflow, kErrPoolSpin, kErrBoundsSlot, kErrBoundsSpill,
                                   kErrBoundsTile, kErrBoundsOut, kErrPeerTimeout};
#ifndef __HIPCC_RTC__
// The kernels' error word as rt_last_error text (RT_ERR_POOL), one distinct
// phrase per bit (tests/index_math.cpp checks that every kErr* bit has one).
inline std::string device_error_text(int32_t err) {
    std::string m;
    auto add = [&](int32_t bit, const char* what) {
        if (err & bit) m += (m.empty() ? "" : "; ") + std::string(what);
    };
    add(kErrPoolOverflow, "device ray pool overflow: a child beyond the LIFO bound");
    add(kErrPoolSpin, "device ray pool: a lock's spin bound ran out (a starved wave, not an overflow)");
    add(kErrBoundsSlot, "bounds check: pool slot outside the LIFO bound");
    add(kErrBoundsSpill, "bounds check: spill region outside the spill buffer");
    add(kErrBoundsTile, "bounds check: work item tile outside the launch");
    add(kErrBoundsOut, "bounds check: output index outside the canvas");
    add(kErrPeerTimeout, "peer canvas: a shard's flag (or the owner's release) did not arrive within the timeout");
    const int32_t unknown = err & ~(kErrPoolOverflow | kErrPoolSpin | kErrBoundsSlot | kErrBoundsSpill |
                                    kErrBoundsTile | kErrBoundsOut | kErrPeerTimeout);
    if (unknown) m += (m.empty() ? "" : "; ") + std::string("device error bits ") + std::to_string(unknown);
    return m;
}
#endif

// Peer canvas (rt_canvas_create): the W x H image and, after it at this
// alignment, one u64 completion flag per shard.
constexpr uint64_t kCanvasFlagAlign = 256;
// t / d for every t < n as one multiply-high by m = ceil(2^32 / d): with
// m d = 2^32 + e, 0 <= e < d, t m / 2^32 = t/d + t e / (d 2^32), and the
// second term stays below 1/d (so below the gap to the next integer) while
// n d < 2^32.  Returns 0 where that does not hold (divide instead).  The
// tracer kernels take the tile row of tile t this way (LaunchParams::
// tiles_x_magic): one s_mul_hi_u32 instead of a ~25-instruction division.
RTC_HD inline uint32_t div_magic(uint32_t d, uint32_t n) {
    if (d < 2 || (uint64_t)n * d >= (1ull << 32)) return 0;
    return (uint32_t)(((1ull << 32) + d - 1) / d);
}
RTC_HD inline uint32_t div_by(uint32_t t, uint32_t d, uint32_t magic) {
    return magic ? (uint32_t)(((uint64_t)t * magic) >> 32) : t / d;
}

RTC_HD inline uint64_t canvas_flag_offset(uint64_t image_bytes) {
    return (image_bytes + kCanvasFlagAlign - 1) / kCanvasFlagAlign * kCanvasFlagAlign;
}
// Tile scheduling modes (the direct kernel: RTC_DEBUG=sched_direct=grid|static; the pool kernel: dynamic)
constexpr uint32_t kSchedGrid = 0;     // one workgroup per tile; the dispatcher balances
constexpr uint32_t kSchedDynamic = 1;  // resident grid, per-XCD atomic tile queues
constexpr uint32_t kSchedStatic = 2;   // resident grid, tiles b, b+G, ... (no atomics)
// World tables up to this size are staged into LDS for the per-lane gathers
// (~120 f32 shapes); larger worlds gather from global memory (L2-resident).
constexpr size_t kMaxWorldLds = 16 * 1024;

// Fixed-point pixel accumulator of the pool kernel: contributions are summed
// as int64 multiples of 2^-48 so the per-pixel sum is independent of the
// (nondeterministic) order in which waves add to it.
constexpr double kAccScale = 281474976710656.0;  // 2^48
constexpr double kAccInvScale = 1.0 / 281474976710656.0;
// The f32 pool kernel sums in int32 multiples of 2^-acc_log2 instead: half
// the LDS (3 KB of a workgroup's ~26 KB, given to the ray pool), and the
// scale is the largest that keeps the world's brightest possible pixel below
// 2^30 (acc_shift_f32), e.g. 2^-22 for reflect_refract: 2.4e-7 per
// contribution against an f32 ulp of 1.2e-7 at 1.0.
template <bool B, typename T, typename F>
struct Choose {
    using type = T;
};
template <typename T, typename F>
struct Choose<false, T, F> {
    using type = F;
};
#ifndef RTC_ACC_I64  // (A/B builds: -DRTC_ACC_I64 keeps the f32 sums in int64 too)
template <typename R>
using PoolAcc = typename Choose<sizeof(R) == 4, int32_t, long long>::type;
#else
template <typename R>
using PoolAcc = long long;
#endif
constexpr uint32_t kAccLog2Min = 8, kAccLog2Max = 28;
// A pool entry's meta word (pixel | remaining << 8: 13 bits; the pixel is the
// lane of the workgroup's tile, 0..255) as stored in the LDS part of the
// pool; spilled entries keep 32 bits in their record.
#ifndef RTC_POOL_META32  // (A/B builds: -DRTC_POOL_META32 keeps 32-bit entries)
using PoolMeta = uint16_t;
#else
using PoolMeta = uint32_t;
#endif
static_assert(RT_MAX_SUPPORTED_DEPTH < 32, "remaining must fit the pool meta's 8 high bits");

// ShapeRec::flags.  Value-equal shapes (shape_identity.hpp) form one identity
// class; its members are adjacent within their kind's run of the table, the
// last one carries kShapeClassEnd, and every member carries the class id (the
// world index of its first member), so the containers walk can toggle one
// entry per class as the reference does (intersection.rs:47).  A world with
// no value-equal shapes has one class per shape, each its own world index.
constexpr int32_t kShapeClosed = 1;    // cylinder/cone `closed`
constexpr int32_t kShapeClassEnd = 2;  // last member of its identity class
// A sphere whose transformation is a similarity (rotation, uniform scale,
// translation: rtc_host.cpp similar_sphere): tri[0..2] holds its world
// centre and tri[3] its radius^2, and the f32 kernels find its roots in world
// space (rtc_kernels.hip sphere_world).
constexpr int32_t kShapeSimilar = 4;
// A cube whose transformation has a diagonal linear part (scale and
// translation only: rtc_host.cpp axis_aligned_cube): tri[0..2] holds the
// world coordinates of its object -1 faces, tri[3..5] of its +1 faces,
// tri[6..8] the world |d| below which an axis counts as parallel (EPSILON
// over the axis's scale) and tri[9..11] the scale's signs, and the f32
// kernels run its slab test in world space (rtc_kernels.hip cube_world).
constexpr int32_t kShapeAxisAligned = 8;
constexpr int kShapeClassShift = 8;

template <typename R>
struct alignas(16) ShapeRec {
    R inv[12];     // rows 0..2 of transformation_inverse (row 3 is never read:
                   // Mul<Point>/Mul<Vector> produce 3 rows, matrix.rs:332-362)
    R bound[4];    // world bounding sphere (center, radius^2) for the wave cull; < 0 = unbounded
    // Right after inv/bound so one scalar-load burst at the top of a shape
    // iteration covers everything a sphere/plane/cube test reads (a later
    // world_index load cost a second s_waitcnt per iteration).
    int32_t world_index;
    int32_t casts_shadow;  // material.casts_shadow, hoisted for the any-hit loop
    int32_t material;
    int32_t flags;  // kShapeClosed | kShapeClassEnd | identity class << kShapeClassShift
    R ymin, ymax;  // cylinder/cone min/max (cylinder.rs:12-14)
    R tri[12];     // triangle vertex_1, edge_1, edge_2, normal (triangle.rs:12-17);
                   // a kShapeSimilar sphere: world centre, radius^2;
                   // a kShapeAxisAligned cube: its world slabs
};

template <typename R>
struct alignas(16) MaterialRec {
    R color[3];
    R ambient, diffuse, specular, shininess;
    R reflectiveness, transparency, refractive_index;
    int32_t pattern;       // -1 = None
    int32_t casts_shadow;
};

template <typename R>
struct alignas(16) PatternRec {
    R color_a[3];
    R color_b[3];
    R inv[12];
    int32_t kind;
    int32_t sub_a, sub_b;
    int32_t pad;
};

// LDS image of the world: [shapes][materials][patterns][world_slot], every
// record a multiple of 16 bytes so each section stays 16-byte aligned.
template <typename R>
constexpr size_t world_lds_bytes(size_t ns, size_t nm, size_t np) {
    return ns * sizeof(ShapeRec<R>) + nm * sizeof(MaterialRec<R>) + np * sizeof(PatternRec<R>) +
           (ns + 3) / 4 * 16;
}
static_assert(sizeof(ShapeRec<float>) % 16 == 0 && sizeof(ShapeRec<double>) % 16 == 0);
static_assert(sizeof(MaterialRec<float>) % 16 == 0 && sizeof(MaterialRec<double>) % 16 == 0);
static_assert(sizeof(PatternRec<float>) % 16 == 0 && sizeof(PatternRec<double>) % 16 == 0);

template <typename R>
struct alignas(16) LightRec {
    R position[3];
    R intensity[3];
};

template <typename R>
struct CameraRec {
    R inv[12];
    R origin[3];
    R half_width, half_height, pixel_size;
};

template <typename R>
struct DevScene {
    const ShapeRec<R>* shapes;
    const MaterialRec<R>* materials;
    const PatternRec<R>* patterns;
    const LightRec<R>* lights;
    const int32_t* world_slot;  // world order -> slot | kind << 24 (rounded up to 4 entries)
    // Per-lane gathers (the hit's shape, its material and pattern) go through
    // these: LDS copies staged at kernel start when the tables fit
    // (LaunchParams::world_lds), else the global tables above.
    const ShapeRec<R>* lshapes;
    const MaterialRec<R>* lmats;
    const PatternRec<R>* lpats;
    const int32_t* lworld_slot;
    int32_t kind_begin[kNumKinds + 1];
    int32_t n_materials, n_patterns;
    int32_t n_lights;
    int32_t any_secondary;  // some material has reflectiveness or transparency != 0
    int32_t no_skips;       // RT_FLAG_NO_SKIPS launch (the generic kernels; per-scene builds: RTC_NO_SKIPS)
};

// One launch of the tracer.
template <typename R>
struct LaunchParams {
    DevScene<R> scene;
    CameraRec<R> cam;
    const double* rays;      // color_at mode: n_rays x {o, d} (f64), else null
    uint64_t n_rays;
    void* out;               // row-major RGB of R (RT_OUT_REAL) or u8 (RT_OUT_U8)
    uint32_t out_format;
    uint32_t width, height;  // canvas
    uint32_t tiles_x;        // tiles per row
    uint32_t tile_rows;      // tile rows of THIS shard's strip
    uint32_t image_rows;     // 1: store pixels at their image rows of a whole W x H canvas (peer canvas),
                             // 0: at their strip rows (the shard's own strip)
    uint32_t shard_index, shard_count;
    uint32_t n_tiles;        // tiles_x * tile_rows (or ray chunks in color_at mode)
    uint32_t max_depth;      // `remaining` of the primary ray
    uint32_t pool_capacity;  // pool kernel: LIFO bound (rays) per workgroup
    uint32_t pool_lds_capacity;  // of which held in LDS; the rest in `spill`
    uint32_t pop_batch;      // pool kernel: rays a wave traces per iteration (<= 64)
    uint32_t acc_log2;       // f32 pool kernel: pixel sums in int32 multiples of 2^-acc_log2
    uint32_t persistent;     // kSched*: tile scheduling of this launch
    uint32_t flags;          // RT_FLAG_* diagnostic ablations
    uint32_t world_lds;      // bytes of world tables staged at the start of dynamic LDS (0 = none)
    void* spill;                 // pool overflow: grid x 8 x (pool_capacity - pool_lds_capacity) words
    uint32_t spill_blocks;       // workgroups the spill buffer holds regions for (RTC_BOUNDS_CHECK)
    uint32_t tiles_x_magic;      // div_magic(tiles_x, n_tiles): tile row = div_by(t, tiles_x, magic)
    unsigned long long* stamps;  // RT_FLAG_STAMPS: 2 x grid s_memrealtime values
    unsigned long long* item_log;  // RT_FLAG_STAMPS pool launches: [0] count, then 3 x u64 per item
    unsigned long long* tile_counter;  // kTileQueues queue heads, kQueueStride apart (zero at launch)
    unsigned long long* next_tile_counter;  // the heads of the next dynamic launch, zeroed by this one
    const uint32_t* tile_order;        // queue position -> work item (heaviest first), null = raster order
    const uint32_t* item_count;        // items in tile_order (>= n_tiles: split tiles), null = n_tiles
    uint32_t* tile_cost;               // pool kernel: per-tile duration (10 ns ticks), null = not recorded
    unsigned long long* counters;      // kCounterShards x kNumCounters cumulative u64
    unsigned long long* gen_counts;    // RT_FLAG_GENERATIONS: traced[kGenSlots], shaded[kGenSlots]; else null
    int32_t* error_flag;               // set nonzero on pool overflow
};

}  // namespace rtc
