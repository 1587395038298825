// index_math.cpp — CPU check of the pool kernel's index arithmetic
// (rtc_internal.hpp, shared with rtc_kernels.hip): work-item encoding and
// decoding, the threads a split part seeds, spill addressing and the
// row-block shard maps.  Built with g++ by tests/test_index_math.py; prints
// "ok" or the first failure.
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>

#include "../ray-tracer-challenge-rs_amd/csrc/rtc_internal.hpp"

using namespace rtc;

#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);  \
            return 1;                                                 \
        }                                                             \
    } while (0)

int main() {
    // packed items round-trip for every field value a tile order can hold
    for (uint32_t l = 0; l <= kMaxSplitLog2; ++l)
        for (uint32_t p = 0; p < (1u << l); ++p)
            for (uint32_t pr = 0; pr < 4; ++pr)
                for (uint32_t t : {0u, 1u, 4095u, 32399u, 0x7FFFFu, kItemTileMask}) {
                    const uint32_t item = encode_item(t, p, l, pr);
                    CHECK(item != kNoItem);
                    const WorkItem w = decode_item(item, true);
                    CHECK(w.tile == t && w.part == p && w.split_log2 == l && w.prio == pr);
                }
    // tile rows by multiply-high (div_magic / div_by): exhaustive over small
    // divisors, then every t near a multiple of d for large ones up to the
    // validity limit n d < 2^32, and the fallback where it does not hold
    for (uint32_t d = 1; d <= 130; ++d) {
        const uint32_t n = d * 40000u, m = div_magic(d, n);
        CHECK((d < 2) == (m == 0));
        for (uint32_t t = 0; t < n; ++t) CHECK(div_by(t, d, m) == t / d);
    }
    for (uint32_t d : {131u, 240u, 255u, 256u, 257u, 1000u, 4095u, 65535u, 65536u, 100003u}) {
        const uint32_t n = (uint32_t)(((1ull << 32) - 1) / d);  // largest n with n d < 2^32
        const uint32_t m = div_magic(d, n);
        CHECK(m != 0 && div_magic(d, n + 1) == 0);
        for (uint64_t q = 0; q * d < n; q += 1 + q / 64)
            for (int64_t k = -2; k <= 2; ++k) {
                const int64_t t = (int64_t)(q * d) + k;
                if (t >= 0 && t < (int64_t)n) CHECK(div_by((uint32_t)t, d, m) == (uint32_t)t / d);
            }
        CHECK(div_by(n - 1, d, m) == (n - 1) / d);
        CHECK(div_by(12345u, d, 0) == 12345u / d);
    }
    // raster items are plain tiles at every size (rt_color_at: up to 2^24 tiles)
    for (uint32_t t : {0u, kItemTileMask, kItemTileMask + 1u, 0x1234567u, 0xFFFFFFu, 0xFFFFFFFEu}) {
        const WorkItem w = decode_item(t, false);
        CHECK(w.tile == t && w.part == 0 && w.split_log2 == 0 && w.prio == 0);
        int seeded = 0;
        for (uint32_t tid = 0; tid < (uint32_t)kBlock; ++tid) seeded += item_seeds(tid, w);
        CHECK(seeded == kBlock);  // an unsplit item seeds the whole tile
    }
    // the parts of a split tile partition its threads into equal runs
    for (uint32_t l = 0; l <= kMaxSplitLog2; ++l) {
        std::set<uint32_t> seen;
        for (uint32_t p = 0; p < (1u << l); ++p) {
            const WorkItem w = decode_item(encode_item(7, p, l, 0), true);
            int n = 0;
            for (uint32_t tid = 0; tid < (uint32_t)kBlock; ++tid)
                if (item_seeds(tid, w)) {
                    CHECK(seen.insert(tid).second);
                    ++n;
                }
            CHECK(n == (kBlock >> l));
        }
        CHECK((int)seen.size() == kBlock);
    }
    // spill records: workgroup b's slots [lcap, cap) map to its own run of
    // records, inside grid * (cap - lcap) records
    for (uint32_t grid : {1u, 7u, 1536u})
        for (uint32_t lcap : {256u, 320u, 512u})
            for (uint32_t depth : {1u, 6u, 16u}) {
                const uint32_t cap = kBlock + depth * kBlock;
                if (cap <= lcap) continue;
                const uint32_t gcap = cap - lcap;
                const uint64_t words = (uint64_t)grid * gcap * 8;
                for (uint32_t b : {0u, grid / 2, grid - 1}) {
                    const uint64_t lo = spill_word(b, gcap, lcap, lcap), hi = spill_word(b, gcap, cap - 1, lcap);
                    CHECK(lo == (uint64_t)b * gcap * 8);
                    CHECK(hi + 8 <= words && hi + 8 == lo + (uint64_t)gcap * 8);
                }
            }
    // row-block shards: every image row has one (shard, strip row), inside
    // that shard's strip, and the map inverts
    for (uint32_t h : {1u, 7u, 1080u, 2160u, 2161u})
        for (uint32_t n : {1u, 2u, 3u, 8u}) {
            const uint32_t rows = shard_tile_rows(h, n, 0) * RT_TILE_H;
            for (uint32_t y = 0; y < h; ++y) {
                uint32_t s, r;
                shard_of_image_row(y, n, &s, &r);
                CHECK(s < n && r < shard_tile_rows(h, n, s) * RT_TILE_H && r < rows);
                CHECK(shard_image_row(r, n, s) == y);
            }
        }
    // every device error bit has its own rt_last_error phrase (VERDICT r5:
    // a spin-bound timeout once read as "pool overflow")
    {
        std::set<std::string> texts;
        int32_t all = 0;
        for (int32_t bit : kErrBitsAll) {
            CHECK(bit > 0 && (bit & (bit - 1)) == 0 && !(all & bit));  // one distinct bit each
            all |= bit;
            const std::string t = device_error_text(bit);
            CHECK(!t.empty() && t.find("device error bits") == std::string::npos);
            CHECK(texts.insert(t).second);
        }
        CHECK(device_error_text(kErrPoolOverflow | kErrPoolSpin) ==
              device_error_text(kErrPoolOverflow) + "; " + device_error_text(kErrPoolSpin));
        CHECK(device_error_text(1 << 20).find("device error bits") != std::string::npos);
        std::printf("errbits %d\n", (int)(sizeof kErrBitsAll / sizeof kErrBitsAll[0]));
    }
    std::printf("ok\n");
    return 0;
}
