"""Row-block shard math of the multi-GPU split, on CPU.

The same inline functions (rtc_internal.hpp shard_*) map a shard's strip rows
to image rows in the kernels and image rows back to strips in the
de-interleave kernel; rt_shard_row_map exposes them on the host.  Checked
here against an independent statement of the rule: tile row k (RT_TILE_H
image rows) belongs to shard k % G and is that shard's (k // G)-th tile row.
"""
import numpy as np
import pytest


@pytest.mark.parametrize("height", [1, 3, 4, 5, 136, 1080, 2160, 2161])
@pytest.mark.parametrize("shards", [1, 2, 3, 4, 7, 8])
def test_row_map_is_the_cyclic_block_rule(rtc, height, shards):
    th = rtc.RT_TILE_H
    shard, row = rtc.shard_row_map(height, shards)
    y = np.arange(height)
    k = y // th
    assert np.array_equal(shard, k % shards)
    assert np.array_equal(row, (k // shards) * th + y % th)
    strip = rtc.shard_rows(height, shards)
    assert row.max() < strip  # every strip fits the padded (shard 0) height
    # each shard's rows are exactly strip rows 0..n-1 of its strip: a bijection
    for s in range(shards):
        r = np.sort(row[shard == s])
        assert np.array_equal(r, np.arange(len(r)))
    # shard 0 has the most tile rows; strips are that tall
    counts = [int((shard == s).sum()) for s in range(shards)]
    assert strip == -(-max(counts) // th) * th if counts[0] else strip == 0


def test_config_split_is_balanced(rtc):
    """configs[3]/[4]: 3840x2160 over 8 GPUs — 540 tile rows, 67 or 68 per shard."""
    shard, _ = rtc.shard_row_map(2160, 8)
    per = np.bincount(shard, minlength=8) // rtc.RT_TILE_H
    assert per.sum() == 540 and per.max() - per.min() <= 1
    assert rtc.shard_rows(2160, 8) == 68 * rtc.RT_TILE_H
