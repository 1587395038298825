"""rt_image_write (canvas.rs:75-137): the 8-bit frame as PNG (RGB8, filter
None, best deflate, as Canvas::to_png_file) or the reference's P3 text
(Canvas::to_ppm_file), byte for byte; binary P6 as an opt-in.  Host only."""
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


def _reference_canvas_5x3():
    """canvas.rs:181-188: a 5x3 canvas with three pixels set (f64 colours)."""
    c = np.zeros((3, 5, 3), dtype=np.float64)
    c[0, 0] = (1.5, 0, 0)
    c[1, 2] = (0, 0.5, 0)
    c[2, 4] = (-0.5, 0, 1)
    return c


def test_ppm_header_kat(rtc, tmp_path):
    """canvas.rs:171-178: header lines "P3", "5 3", "255"."""
    path = tmp_path / "h.ppm"
    rtc.write_image(path, np.zeros((3, 5, 3), dtype=np.uint8))
    lines = path.read_bytes().decode().split("\n")
    assert lines[:3] == ["P3", "5 3", "255"]


def test_ppm_kat(rtc, tmp_path):
    """canvas.rs:180-202, byte for byte: the canvas quantized as canvas.rs:81 does
    (clamp, *255, round half away from zero: 0.5 -> 128), 15 channels per line."""
    img = rtc.canvas_quantize(_reference_canvas_5x3())
    path = tmp_path / "kat.ppm"
    rtc.write_image(path, img)
    raw = path.read_bytes()
    expected = ("P3\n5 3\n255\n"
                "255   0   0   0   0   0   0   0   0   0   0   0   0   0   0\n"
                "  0   0   0   0   0   0   0 128   0   0   0   0   0   0   0\n"
                "  0   0   0   0   0   0   0   0   0   0   0   0   0   0 255").encode()
    assert raw == expected  # no trailing newline (lines joined by "\n")


def _p3_reference(img):
    """canvas.rs:75-97 restated in Python: chunks of 5 pixels across rows."""
    h, w, _ = img.shape
    flat = img.reshape(-1, 3)
    lines = ["P3", f"{w} {h}", "255"]
    for p in range(0, len(flat), 5):
        lines.append(" ".join(f"{int(v):>3}" for v in flat[p:p + 5].reshape(-1)))
    return "\n".join(lines).encode()


@pytest.mark.parametrize("shape", [(1, 1), (7, 9), (3, 5), (2, 4), (0, 0)])
def test_ppm_lines_cross_rows(rtc, tmp_path, shape):
    """Pixels per line = floor(70 / 12) = 5 regardless of the row length (canvas.rs:76-77)."""
    img = np.random.default_rng(shape[0] * 10 + shape[1]).integers(0, 256, size=(*shape, 3), dtype=np.uint8)
    path = tmp_path / "frame.ppm"
    rtc.write_image(path, img)
    assert path.read_bytes() == _p3_reference(img)


def test_ppm_binary_opt_in(rtc, tmp_path):
    img = np.random.default_rng(3).integers(0, 256, size=(7, 9, 3), dtype=np.uint8)
    path = tmp_path / "frame.ppm"
    rtc.write_image(path, img, fmt="ppm-binary")
    raw = path.read_bytes()
    head = b"P6\n9 7\n255\n"
    assert raw[:len(head)] == head
    assert np.array_equal(np.frombuffer(raw[len(head):], dtype=np.uint8).reshape(7, 9, 3), img)


def test_canvas_quantize(rtc):
    """canvas.rs:117-123: clamp to [0, 1], *255, round half away from zero, NaN -> 0."""
    v = np.array([-1.0, 0.0, 0.5 / 255, 0.5, 1.5 / 255, 1.0, 2.0, np.nan, np.inf, -np.inf, 0.25])
    q = rtc.canvas_quantize(v)
    assert q.tolist() == [0, 0, 1, 128, 2, 255, 255, 0, 255, 0, 64]


def test_parent_dirs_created(rtc, tmp_path):
    """Canvas::prepare_file (canvas.rs:99-105): create_dir_all on the parent."""
    for name in ("a/b/c/x.png", "d/e/x.ppm"):
        path = tmp_path / name
        rtc.write_image(path, np.zeros((2, 2, 3), dtype=np.uint8))
        assert path.exists()


def test_errors(rtc, tmp_path):
    with pytest.raises(ValueError):
        rtc.write_image(tmp_path / "x.png", np.zeros((2, 2, 3), dtype=np.float32))
    (tmp_path / "file").write_text("")
    with pytest.raises(rtc.RenderError):  # a parent that is a file
        rtc.write_image(tmp_path / "file" / "x.png", np.zeros((2, 2, 3), dtype=np.uint8))
    with pytest.raises(rtc.RenderError):  # PNG of an empty canvas
        rtc.write_image(tmp_path / "e.png", np.zeros((0, 0, 3), dtype=np.uint8))


def test_u8_frame_widened_to_a_canvas_saves_the_same_bytes(rtc, oracle):
    """INTEGRATION.md 1b'': a Canvas built from the 8-bit frame as b / 255
    quantizes back to b (canvas.rs:117-123) for every byte, so its PNG equals
    the PNG of the f64 canvas the frame came from."""
    b = np.arange(256, dtype=np.float64)
    assert np.array_equal(oracle.quantize((b / 255.0).reshape(1, 256, 1)).ravel(), b.astype(np.uint8))
    # and through the library's own quantizer (rt_canvas_quantize)
    img = np.repeat((b / 255.0).reshape(1, 256, 1), 3, axis=2)
    assert np.array_equal(rtc.canvas_quantize(img)[0, :, 0], b.astype(np.uint8))
