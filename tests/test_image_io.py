"""rt_image_write (canvas.rs:75-137): the 8-bit frame as PNG (RGB8, filter
None, best deflate, as Canvas::to_png_file) or binary PPM.  Host only."""
import numpy as np
import pytest


@pytest.mark.parametrize("shape", [(1, 1), (5, 17), (64, 48)])
def test_png_round_trip(rtc, tmp_path, shape):
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(shape[0] * 100 + shape[1])
    img = rng.integers(0, 256, size=(shape[0], shape[1], 3), dtype=np.uint8)
    path = tmp_path / "frame.png"
    rtc.write_image(path, img)
    with PIL.open(path) as im:
        assert im.mode == "RGB" and im.size == (shape[1], shape[0])
        assert np.array_equal(np.asarray(im), img)
    raw = path.read_bytes()
    assert raw[:8] == b"\x89PNG\r\n\x1a\n"
    assert raw[12:16] == b"IHDR" and raw[24:29] == bytes([8, 2, 0, 0, 0])  # 8-bit RGB, no interlace


def test_png_rows_unfiltered(rtc, tmp_path):
    """Every scanline carries filter type 0 (image's FilterType::NoFilter)."""
    import zlib
    img = np.arange(4 * 6 * 3, dtype=np.uint8).reshape(4, 6, 3)
    path = tmp_path / "f.PNG"  # extension match ignores case
    rtc.write_image(path, img)
    raw = path.read_bytes()
    i = raw.index(b"IDAT")
    n = int.from_bytes(raw[i - 4:i], "big")
    rows = zlib.decompress(raw[i + 4:i + 4 + n])
    assert len(rows) == 4 * (1 + 18)
    assert all(rows[r * 19] == 0 for r in range(4))
    assert rows[1:19] == img[0].tobytes()


def test_ppm(rtc, tmp_path):
    img = np.random.default_rng(3).integers(0, 256, size=(7, 9, 3), dtype=np.uint8)
    path = tmp_path / "frame.ppm"
    rtc.write_image(path, img)
    raw = path.read_bytes()
    head = b"P6\n9 7\n255\n"
    assert raw[:len(head)] == head
    assert np.array_equal(np.frombuffer(raw[len(head):], dtype=np.uint8).reshape(7, 9, 3), img)


def test_errors(rtc, tmp_path):
    with pytest.raises(ValueError):
        rtc.write_image(tmp_path / "x.png", np.zeros((2, 2, 3), dtype=np.float32))
    with pytest.raises(rtc.RenderError):
        rtc.write_image(tmp_path / "missing_dir" / "x.png", np.zeros((2, 2, 3), dtype=np.uint8))
