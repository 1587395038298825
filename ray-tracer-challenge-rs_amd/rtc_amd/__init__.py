"""rtc_amd — MI355X-native render path for the Ray Tracer Challenge world model
of przemo199/ray-tracer-challenge-rs.

Python view of the C-ABI in include/rtc.h / include/rtc_scene.h (librtc.so,
built from ray-tracer-challenge-rs_amd/csrc).  It mirrors the reference's
render API:

    load_scene_description(path)   ray-tracer-cli/src/scene_loader.rs:361-367
    Camera.render / render_parallel ray-tracer/src/composites/camera.rs:79-112
                                   -> Context.render (the GPU arm)
    World.color_at                 ray-tracer/src/composites/world.rs:89-95
                                   -> Context.color_at (batched)

There is no CPU fallback: importing works without a GPU (for the scene
loader and ABI checks), but every call that renders raises RenderError with
RT_ERR_NO_DEVICE when no HIP device is usable, and the module refuses to load
at all when librtc.so is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

__all__ = [
    "RenderError", "lib_path", "abi_version", "device_count", "matrix_inverse", "camera_make",
    "camera_resize", "camera_set_transform", "load_scene", "load_scene_text", "SceneTables", "Context", "shard_rows",
    "RT_DEFAULT_MAX_DEPTH", "RT_TILE_H", "RT_TILE_W",
]

RT_ABI_VERSION = 3  # rtc.h; rt_abi_version() must agree (checked at load)
RT_TILE_W = 64
RT_TILE_H = 4
RT_DEFAULT_MAX_DEPTH = 6  # World::MAX_REFLECTION_ITERATIONS, world.rs:15
RT_MAX_SUPPORTED_DEPTH = 16

RT_OK = 0
RT_ERR_INVALID, RT_ERR_HIP, RT_ERR_NO_DEVICE, RT_ERR_NO_SCENE = -1, -2, -3, -4
RT_ERR_OOM, RT_ERR_POOL, RT_ERR_IO, RT_ERR_COMM = -5, -6, -7, -8
STATUS = {0: "RT_OK", -1: "RT_ERR_INVALID", -2: "RT_ERR_HIP", -3: "RT_ERR_NO_DEVICE", -4: "RT_ERR_NO_SCENE",
          -5: "RT_ERR_OOM", -6: "RT_ERR_POOL", -7: "RT_ERR_IO", -8: "RT_ERR_COMM"}
RT_UNIQUE_ID_BYTES = 128
RT_IPC_HANDLE_BYTES = 64
RT_GATHER_RCCL, RT_GATHER_PEER = 0, 1

SHAPE_KINDS = {"sphere": 0, "plane": 1, "cube": 2, "cylinder": 3, "cone": 4, "triangle": 5}
PATTERN_KINDS = {"stripe": 0, "gradient": 1, "ring": 2, "checker": 3, "complex": 4, "test": 5}
PRECISIONS = {"f32": 0, "f64": 1}
# rt_render_options.flags: diagnostic ablations (rtc.h); never in a parity or bench result
RT_FLAG_NO_COUNTERS, RT_FLAG_NO_SHADE, RT_FLAG_NO_TRACE, RT_FLAG_STAMPS, RT_FLAG_FAIL_LAUNCH = 1, 2, 4, 8, 16
RT_FLAG_GENERATIONS = 32  # count rays per generation (rt_read_generation_counts); pixels unchanged
RT_FLAG_NO_SKIPS = 64  # no shadow-ray skips or cube exit path (acceleration only: pixels and counters unchanged)
RT_JIT_OFF, RT_JIT_SYNC, RT_JIT_AUTO, RT_JIT_EAGER = 0, 1, 2, 3
OUT_FORMATS = {"real": 0, "u8": 1}


class RenderError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{STATUS.get(code, code)}: {message}")
        self.code = code


# ----------------------------------------------------------------- structs
class ShapeDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("inverse", C.c_double * 16),
                ("minimum", C.c_double), ("maximum", C.c_double), ("closed", C.c_int32),
                ("reserved", C.c_int32), ("vertex_1", C.c_double * 3), ("edge_1", C.c_double * 3),
                ("edge_2", C.c_double * 3), ("normal", C.c_double * 3)]


class MaterialDesc(C.Structure):
    _fields_ = [("color", C.c_double * 3), ("ambient", C.c_double), ("diffuse", C.c_double),
                ("specular", C.c_double), ("shininess", C.c_double), ("reflectiveness", C.c_double),
                ("transparency", C.c_double), ("refractive_index", C.c_double), ("casts_shadow", C.c_int32),
                ("pattern", C.c_int32)]


class PatternDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("sub_a", C.c_int32), ("sub_b", C.c_int32), ("reserved", C.c_int32),
                ("color_a", C.c_double * 3), ("color_b", C.c_double * 3), ("inverse", C.c_double * 16)]


class LightDesc(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("intensity", C.c_double * 3)]


class CameraDesc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("field_of_view", C.c_double),
                ("half_width", C.c_double), ("half_height", C.c_double), ("pixel_size", C.c_double),
                ("inverse", C.c_double * 16), ("origin", C.c_double * 3)]

    def copy(self) -> "CameraDesc":
        c = CameraDesc()
        C.pointer(c)[0] = self
        return c


class RenderOptions(C.Structure):
    _fields_ = [("max_depth", C.c_uint32), ("precision", C.c_uint32), ("out_format", C.c_uint32),
                ("shard_index", C.c_uint32), ("shard_count", C.c_uint32), ("flags", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("primary", C.c_uint64), ("shadow", C.c_uint64), ("reflect", C.c_uint64),
                ("refract", C.c_uint64), ("shaded", C.c_uint64), ("lit_patterned", C.c_uint64),
                ("refract_evals", C.c_uint64), ("schlick_evals", C.c_uint64), ("kernel_ms", C.c_double),
                ("algorithmic_flops", C.c_double), ("gather_ms", C.c_double), ("frame_ms", C.c_double),
                ("n_shards", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_}
        d["rays"] = self.primary + self.shadow + self.reflect + self.refract
        return d


class GenerationCounts(C.Structure):
    _fields_ = [("traced", C.c_uint64 * (RT_MAX_SUPPORTED_DEPTH + 1)),
                ("shaded", C.c_uint64 * (RT_MAX_SUPPORTED_DEPTH + 1))]


class SceneView(C.Structure):
    _fields_ = [("shapes", C.POINTER(ShapeDesc)), ("n_shapes", C.c_uint32),
                ("materials", C.POINTER(MaterialDesc)), ("n_materials", C.c_uint32),
                ("patterns", C.POINTER(PatternDesc)), ("n_patterns", C.c_uint32),
                ("lights", C.POINTER(LightDesc)), ("n_lights", C.c_uint32),
                ("camera", CameraDesc), ("duplicate_shapes", C.c_uint32)]


# --------------------------------------------------------------- library
_HERE = os.path.dirname(os.path.abspath(__file__))


def lib_path() -> str:
    # RTC_LIBRARY: an alternative in-tree build of the same ABI (A/B of build
    # variants, scripts/ab_builds.sh); never a different implementation.
    return os.environ.get("RTC_LIBRARY") or os.path.join(_HERE, "_lib", "librtc.so")


def _load() -> C.CDLL:
    path = lib_path()
    # torch-ROCm bundles its own HIP runtime with the same soname
    # (libamdhip64.so.7) as /opt/rocm's.  Load it first so librtc binds to the
    # SAME runtime: torch streams, events and allocations are then valid
    # handles for the C-ABI (one HIP runtime per process).
    # Kernel arguments in device memory: each wave's first s_load of its
    # arguments then hits HBM/L2 instead of crossing PCIe (measured ~2 us per
    # 1080p frame on MI355X).  Must be set before the HIP runtime starts.
    os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
    # RTC_NO_TORCH=1: a torch-free host (bench.py's one-shot child, timing
    # what a Rust caller of the C-ABI pays: the HIP runtime starts in
    # rt_context_create); librtc then binds /opt/rocm's runtime on its own.
    if os.environ.get("RTC_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(path):
        raise ImportError(f"rtc_amd: {path} is missing — build it with `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(path)
    P = C.POINTER
    sig = {
        "rt_abi_version": (C.c_int, []),
        "rt_last_error": (C.c_char_p, []),
        "rt_device_count": (C.c_int, [P(C.c_int)]),
        "rt_context_create": (C.c_int, [C.c_int, P(C.c_void_p)]),
        "rt_context_destroy": (C.c_int, [C.c_void_p]),
        "rt_scene_upload": (C.c_int, [C.c_void_p, P(ShapeDesc), C.c_uint32, P(MaterialDesc), C.c_uint32,
                                      P(PatternDesc), C.c_uint32, P(LightDesc), C.c_uint32]),
        "rt_shard_rows": (C.c_int, [C.c_uint32, C.c_uint32, P(C.c_uint32)]),
        "rt_render": (C.c_int, [C.c_void_p, P(CameraDesc), P(RenderOptions), C.c_void_p, P(Stats)]),
        "rt_render_device": (C.c_int, [C.c_void_p, P(CameraDesc), P(RenderOptions), C.c_void_p, C.c_void_p]),
        "rt_color_at": (C.c_int, [C.c_void_p, P(C.c_double), C.c_uint64, C.c_uint32, C.c_uint32, P(C.c_double),
                                  P(Stats)]),
        "rt_read_counters": (C.c_int, [C.c_void_p, P(Stats)]),
        "rt_read_generation_counts": (C.c_int, [C.c_void_p, P(GenerationCounts)]),
        "rt_debug_stamps": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_uint32, P(C.c_uint32)]),
        "rt_debug_tile_costs": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_uint32, P(C.c_uint32)]),
        "rt_debug_item_log": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_uint32, P(C.c_uint32)]),
        "rt_assemble_shards": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_void_p, C.c_void_p]),
        "rt_scene_load_yaml": (C.c_int, [C.c_char_p, P(C.c_void_p)]),
        "rt_scene_load_yaml_text": (C.c_int, [C.c_char_p, P(C.c_void_p)]),
        "rt_scene_view_get": (C.c_int, [C.c_void_p, P(SceneView)]),
        "rt_scene_free": (None, [C.c_void_p]),
        "rt_image_write": (C.c_int, [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]),
        "rt_image_write_format": (C.c_int, [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int]),
        "rt_canvas_quantize": (C.c_int, [P(C.c_double), C.c_uint64, P(C.c_uint8)]),
        "rt_camera_make": (C.c_int, [C.c_uint32, C.c_uint32, C.c_double, P(C.c_double), P(C.c_double),
                                     P(C.c_double), P(CameraDesc)]),
        "rt_camera_resize": (C.c_int, [P(CameraDesc), C.c_uint32, C.c_uint32]),
        "rt_matrix_inverse": (C.c_int, [P(C.c_double), P(C.c_double)]),
        "rt_camera_set_transform": (C.c_int, [P(CameraDesc), P(C.c_double)]),
        "rt_shard_row_map": (C.c_int, [C.c_uint32, C.c_uint32, P(C.c_uint32), P(C.c_uint32)]),
        "rt_context_create_multi": (C.c_int, [P(C.c_int), C.c_int, P(C.c_void_p)]),
        "rt_comm_unique_id": (C.c_int, [P(C.c_uint8)]),
        "rt_context_create_rank": (C.c_int, [C.c_int, C.c_int, C.c_int, P(C.c_uint8), P(C.c_void_p)]),
        "rt_context_group": (C.c_int, [C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int)]),
        "rt_context_set_jit": (C.c_int, [C.c_void_p, C.c_int]),
        "rt_context_set_frames_in_flight": (C.c_int, [C.c_void_p, C.c_uint32]),
        "rt_jit_status": (C.c_int, [C.c_void_p, P(C.c_int), P(C.c_double), C.c_char_p, C.c_size_t]),
        "rt_jit_wait": (C.c_int, [C.c_void_p, C.c_double, P(C.c_int)]),
        "rt_canvas_create": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, P(C.c_void_p), P(C.c_uint8)]),
        "rt_canvas_open": (C.c_int, [C.c_void_p, P(C.c_uint8), C.c_uint64, C.c_uint32, P(C.c_void_p)]),
        "rt_canvas_close": (C.c_int, [C.c_void_p, C.c_void_p]),
        "rt_render_to_canvas": (C.c_int, [C.c_void_p, P(CameraDesc), P(RenderOptions), C.c_void_p, C.c_uint64,
                                          C.c_double, C.c_void_p]),
        "rt_canvas_wait": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_double, C.c_void_p]),
        "rt_canvas_release": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
        "rt_canvas_read": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
        "rt_context_set_gather": (C.c_int, [C.c_void_p, C.c_int]),
        "rt_debug_intersect": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_double), C.c_uint64, C.c_uint32, C.c_uint32,
                                         P(C.c_double)]),
        "rt_debug_normal": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_double), C.c_uint64, C.c_uint32, C.c_uint32,
                                      P(C.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != RT_ABI_VERSION:
        raise ImportError(f"rtc_amd: {path} has ABI {lib.rt_abi_version()}, this module expects {RT_ABI_VERSION}")
    return lib


_lib = _load()

# Every symbol include/rtc.h and include/rtc_scene.h declare (checked by tests).
EXPORTED_SYMBOLS = (
    "rt_abi_version", "rt_last_error", "rt_device_count", "rt_context_create", "rt_context_destroy",
    "rt_scene_upload", "rt_shard_rows", "rt_render", "rt_render_device", "rt_color_at", "rt_read_counters",
    "rt_read_generation_counts",
    "rt_debug_stamps", "rt_debug_tile_costs", "rt_debug_item_log", "rt_debug_intersect", "rt_debug_normal", "rt_camera_set_transform",
    "rt_shard_row_map", "rt_context_create_multi", "rt_comm_unique_id", "rt_context_create_rank", "rt_context_group",
    "rt_context_set_jit", "rt_context_set_frames_in_flight", "rt_jit_status", "rt_jit_wait", "rt_canvas_create", "rt_canvas_open", "rt_canvas_close",
    "rt_render_to_canvas", "rt_canvas_wait", "rt_canvas_release", "rt_canvas_read", "rt_context_set_gather",
    "rt_assemble_shards", "rt_scene_load_yaml", "rt_scene_load_yaml_text", "rt_scene_view_get", "rt_scene_free",
    "rt_camera_make", "rt_camera_resize", "rt_matrix_inverse", "rt_image_write", "rt_image_write_format",
    "rt_canvas_quantize",
)


def _check(rc: int) -> None:
    if rc != RT_OK:
        raise RenderError(rc, _lib.rt_last_error().decode(errors="replace"))


def abi_version() -> int:
    return _lib.rt_abi_version()


def device_count() -> int:
    n = C.c_int(0)
    _check(_lib.rt_device_count(C.byref(n)))
    return n.value


def matrix_inverse(m) -> np.ndarray:
    """Matrix<4>::inverse (matrix.rs:247-258) on 16 row-major f64."""
    a = (C.c_double * 16)(*np.asarray(m, dtype=np.float64).reshape(16))
    out = (C.c_double * 16)()
    _check(_lib.rt_matrix_inverse(a, out))
    return np.array(out[:], dtype=np.float64).reshape(4, 4)


def camera_make(width: int, height: int, fov: float, frm, to, up) -> CameraDesc:
    """Camera::new + set_transformation(view_transform(from, to, up))."""
    cam = CameraDesc()
    v = lambda x: (C.c_double * 3)(*[float(t) for t in x])  # noqa: E731
    _check(_lib.rt_camera_make(width, height, float(fov), v(frm), v(to), v(up), C.byref(cam)))
    return cam


def camera_set_transform(cam: CameraDesc, transform) -> CameraDesc:
    """Camera::set_transformation (camera.rs:124-127) on a copy: inverse + origin."""
    c = cam.copy()
    t = (C.c_double * 16)(*np.asarray(transform, dtype=np.float64).reshape(16))
    _check(_lib.rt_camera_set_transform(C.byref(c), t))
    return c


def camera_resize(cam: CameraDesc, width: int, height: int) -> CameraDesc:
    """Camera::new for another canvas size, same fov/transform (= editing YAML width/height)."""
    c = cam.copy()
    _check(_lib.rt_camera_resize(C.byref(c), width, height))
    return c


IMAGE_FORMATS = {"auto": 0, "png": 1, "ppm": 2, "ppm-binary": 3}


def write_image(path, image: np.ndarray, fmt: str = "auto") -> None:
    """Canvas::to_png_file / to_ppm_file (canvas.rs:75-137) of an 8-bit (H, W, 3) frame
    (render(..., out_format="u8")): PNG when `path` ends in .png, the reference's P3
    text otherwise; fmt "ppm-binary" writes P6 instead (an opt-in, not the reference's)."""
    img = np.ascontiguousarray(image)
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("write_image takes a uint8 array of shape (H, W, 3)")
    _check(_lib.rt_image_write_format(os.fsencode(path), img.ctypes.data if img.size else None, img.shape[1],
                                      img.shape[0], IMAGE_FORMATS[fmt]))


def canvas_quantize(image: np.ndarray) -> np.ndarray:
    """canvas.rs:81, 117-123 on the host: round(clamp(c, 0, 1) * 255) as u8 of an f64 canvas."""
    src = np.ascontiguousarray(image, dtype=np.float64)
    out = np.zeros(src.shape, dtype=np.uint8)
    _check(_lib.rt_canvas_quantize(src.ctypes.data_as(C.POINTER(C.c_double)), src.size,
                                   out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


def shard_rows(height: int, shard_count: int) -> int:
    r = C.c_uint32(0)
    _check(_lib.rt_shard_rows(height, shard_count, C.byref(r)))
    return r.value


def shard_row_map(height: int, shard_count: int):
    """(shard, strip row) of every image row (rtc.h rt_shard_row_map; host only)."""
    shard = np.zeros(height, dtype=np.uint32)
    row = np.zeros(height, dtype=np.uint32)
    _check(_lib.rt_shard_row_map(height, shard_count, shard.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 row.ctypes.data_as(C.POINTER(C.c_uint32))))
    return shard, row


def comm_unique_id() -> bytes:
    """RCCL unique id for rt_context_create_rank (rank 0 makes it, the caller shares it)."""
    buf = (C.c_uint8 * RT_UNIQUE_ID_BYTES)()
    _check(_lib.rt_comm_unique_id(buf))
    return bytes(buf)


@dataclass
class SceneTables:
    """Flattened world: the POD tables rt_scene_upload takes, plus the camera."""
    shapes: C.Array
    materials: C.Array
    patterns: C.Array
    lights: C.Array
    camera: CameraDesc
    duplicate_shapes: int = 0

    @property
    def counts(self):
        return len(self.shapes), len(self.materials), len(self.patterns), len(self.lights)

    def args(self):
        """(shapes, n, materials, n, patterns, n, lights, n) for C calls."""
        return (self.shapes, len(self.shapes), self.materials, len(self.materials), self.patterns,
                len(self.patterns), self.lights, len(self.lights))

    def has_secondary(self) -> bool:
        return any(m.reflectiveness != 0.0 or m.transparency != 0.0 for m in self.materials)


def _tables_from_view(v: SceneView) -> SceneTables:
    def copy(ptr, n, typ):
        arr = (typ * n)()
        if n:
            C.memmove(arr, ptr, n * C.sizeof(typ))
        return arr
    return SceneTables(copy(v.shapes, v.n_shapes, ShapeDesc), copy(v.materials, v.n_materials, MaterialDesc),
                       copy(v.patterns, v.n_patterns, PatternDesc), copy(v.lights, v.n_lights, LightDesc),
                       v.camera.copy(), v.duplicate_shapes)


def _load_with(fn, arg: bytes) -> SceneTables:
    h = C.c_void_p()
    _check(fn(arg, C.byref(h)))
    try:
        v = SceneView()
        _check(_lib.rt_scene_view_get(h, C.byref(v)))
        return _tables_from_view(v)
    finally:
        _lib.rt_scene_free(h)


def load_scene(path: str) -> SceneTables:
    """load_scene_description (scene_loader.rs:361-367): YAML file -> tables + camera."""
    return _load_with(_lib.rt_scene_load_yaml, os.fsencode(path))


def load_scene_text(text: str) -> SceneTables:
    return _load_with(_lib.rt_scene_load_yaml_text, text.encode())


class Context:
    """One GPU.  Mirrors the borrow in Camera::render(&self, world: &World)."""

    def __init__(self, device: int = 0, _handle: C.c_void_p | None = None):
        h = _handle
        if h is None:
            h = C.c_void_p()
            _check(_lib.rt_context_create(device, C.byref(h)))
        self._h = h
        self.device = device
        self.scene: SceneTables | None = None

    @classmethod
    def multi(cls, devices) -> "Context":
        """One process, several GPUs (rt_context_create_multi: ncclCommInitAll).  Frames are split in
        row-block shards across the devices and gathered onto devices[0]."""
        arr = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        _check(_lib.rt_context_create_multi(arr, len(devices), C.byref(h)))
        return cls(devices[0], h)

    @classmethod
    def rank(cls, device: int, n_ranks: int, rank: int, unique_id: bytes) -> "Context":
        """One process per GPU (rt_context_create_rank: ncclCommInitRank); every rank then makes the same
        calls; rank 0's scene and output are the ones used."""
        buf = (C.c_uint8 * RT_UNIQUE_ID_BYTES).from_buffer_copy(unique_id)
        h = C.c_void_p()
        _check(_lib.rt_context_create_rank(device, n_ranks, rank, buf, C.byref(h)))
        return cls(device, h)

    def group(self):
        """(shards per frame, this context's rank, GPUs driven by this process)."""
        n, r, loc = C.c_int(), C.c_int(), C.c_int()
        _check(_lib.rt_context_group(self._h, C.byref(n), C.byref(r), C.byref(loc)))
        return n.value, r.value, loc.value

    def close(self) -> None:
        if self._h:
            _lib.rt_context_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_frames_in_flight(self, frames: int) -> None:
        """Planning hint (rtc.h rt_context_set_frames_in_flight): the caller keeps `frames` frames in
        flight on as many contexts; > 1 plans the direct kernel for throughput.  Pixels unchanged."""
        _check(_lib.rt_context_set_frames_in_flight(self._h, frames))

    def set_jit(self, mode: int) -> None:
        """Per-scene kernels (rtc.h rt_context_set_jit): 0 never, 1 every f32 frame (built in line),
        2 frames of >= 64K pixels, built on a host thread from the 2nd such frame (the default),
        3 the same from the 1st."""
        _check(_lib.rt_context_set_jit(self._h, mode))

    def jit_wait(self, timeout_ms: float = -1.0) -> int:
        """Wait for this context's per-scene builds in flight; returns how many are still running."""
        n = C.c_int(0)
        _check(_lib.rt_jit_wait(self._h, float(timeout_ms), C.byref(n)))
        return n.value

    def jit_status(self) -> dict:
        """Whether the last launch ran a per-scene kernel, compile ms so far, last build error."""
        used, ms, log = C.c_int(), C.c_double(), C.create_string_buffer(4096)
        _check(_lib.rt_jit_status(self._h, C.byref(used), C.byref(ms), log, len(log)))
        return {"used": bool(used.value), "compile_ms": ms.value, "log": log.value.decode(errors="replace")}

    def upload(self, scene: SceneTables | None) -> None:
        """rt_scene_upload; on a non-zero rank of a group, None (the scene comes from rank 0)."""
        if scene is None:
            _check(_lib.rt_scene_upload(self._h, None, 0, None, 0, None, 0, None, 0))
        else:
            _check(_lib.rt_scene_upload(self._h, *scene.args()))
        self.scene = scene

    @staticmethod
    def options(depth=RT_DEFAULT_MAX_DEPTH, precision="f32", out_format="real", shard=(0, 1),
                flags: int = 0) -> RenderOptions:
        return RenderOptions(depth, PRECISIONS[precision], OUT_FORMATS[out_format], shard[0], shard[1], flags)

    def render(self, camera: CameraDesc, depth: int = RT_DEFAULT_MAX_DEPTH, precision: str = "f32",
               out_format: str = "real", shard=(0, 1), out: np.ndarray | None = None, flags: int = 0):
        """Render one frame (or one shard's strip) into a host array (H, W, 3); returns (image, stats).
        `out` reuses a caller's array of that shape and dtype (a canvas kept across frames)."""
        opts = self.options(depth, precision, out_format, shard, flags)
        rows = camera.height if shard[1] == 1 else shard_rows(camera.height, shard[1])
        dtype = np.uint8 if out_format == "u8" else (np.float32 if precision == "f32" else np.float64)
        if out is not None:
            if out.shape != (rows, camera.width, 3) or out.dtype != dtype or not out.flags.c_contiguous:
                raise ValueError(f"out must be a C-contiguous {dtype.__name__} array of shape {(rows, camera.width, 3)}")
            img = out
        else:
            img = np.zeros((rows, camera.width, 3), dtype=dtype)
        st = Stats()
        _check(_lib.rt_render(self._h, C.byref(camera), C.byref(opts), img.ctypes.data_as(C.c_void_p),
                              C.byref(st)))
        return img, st.as_dict()

    def render_stats(self, camera: CameraDesc, depth: int = RT_DEFAULT_MAX_DEPTH, precision: str = "f32",
                     out_format: str = "real", out=None):
        """rt_render into `out` (a host array of the frame, or None on a group's non-zero ranks): stats only."""
        opts = self.options(depth, precision, out_format)
        st = Stats()
        ptr = None if out is None else out.ctypes.data_as(C.c_void_p)
        _check(_lib.rt_render(self._h, C.byref(camera), C.byref(opts), ptr, C.byref(st)))
        return st.as_dict()

    def render_device(self, camera: CameraDesc, out_ptr: int, stream_ptr: int | None = None,
                      depth: int = RT_DEFAULT_MAX_DEPTH, precision: str = "f32", out_format: str = "real",
                      shard=(0, 1), flags: int = 0) -> None:
        """Asynchronous render into a device buffer (e.g. a torch tensor's data_ptr()) on a HIP stream
        (stream_ptr None/0 = HIP's default stream, which is torch's default stream)."""
        opts = self.options(depth, precision, out_format, shard, flags)
        _check(_lib.rt_render_device(self._h, C.byref(camera), C.byref(opts), C.c_void_p(out_ptr or 0),
                                     C.c_void_p(stream_ptr or 0)))

    def color_at(self, rays, depth: int = RT_DEFAULT_MAX_DEPTH, precision: str = "f32"):
        """Batched World::color_at: rays (n, 6) = origin, direction -> colours (n, 3) f64.  In a world with
        reflective or transparent materials the directions must be unit length (rtc.h rt_color_at)."""
        r = np.ascontiguousarray(np.asarray(rays, dtype=np.float64).reshape(-1, 6))
        out = np.zeros((r.shape[0], 3), dtype=np.float64)
        st = Stats()
        _check(_lib.rt_color_at(self._h, r.ctypes.data_as(C.POINTER(C.c_double)), r.shape[0], depth,
                                PRECISIONS[precision], out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
        return out, st.as_dict()

    def debug_stamps(self) -> np.ndarray:
        """(workgroups, 2) s_memrealtime {start, end} of the last RT_FLAG_STAMPS launch (100 MHz ticks)."""
        n = C.c_uint32(0)
        _check(_lib.rt_debug_stamps(self._h, None, 0, C.byref(n)))
        out = np.zeros((n.value, 2), dtype=np.uint64)
        _check(_lib.rt_debug_stamps(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n)))
        return out

    def debug_item_log(self) -> np.ndarray:
        """Items of the last RT_FLAG_STAMPS pool launch: rows {item | wg << 32, start, end}."""
        n = C.c_uint32()
        _check(_lib.rt_debug_item_log(self._h, None, 0, C.byref(n)))
        out = np.zeros((n.value, 3), dtype=np.uint64)
        _check(_lib.rt_debug_item_log(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n)))
        return out

    def debug_tile_costs(self) -> np.ndarray:
        """Per-tile durations (10 ns ticks) recorded by the last pool launch."""
        n = C.c_uint32(0)
        _check(_lib.rt_debug_tile_costs(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=np.uint32)
        _check(_lib.rt_debug_tile_costs(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)))
        return out

    def debug_intersect(self, shape: int, rays, precision: str = "f64", world_space: bool = False):
        """The device's per-shape intersect on (n, 6) rays: list of t tuples (push order) per ray."""
        r = np.ascontiguousarray(np.asarray(rays, dtype=np.float64).reshape(-1, 6))
        out = np.zeros((r.shape[0], 5), dtype=np.float64)
        _check(_lib.rt_debug_intersect(self._h, shape, r.ctypes.data_as(C.POINTER(C.c_double)), r.shape[0],
                                       PRECISIONS[precision], int(world_space),
                                       out.ctypes.data_as(C.POINTER(C.c_double))))
        return [tuple(row[1:1 + int(row[0])]) for row in out]

    def debug_normal(self, shape: int, points, precision: str = "f64", world_space: bool = False) -> np.ndarray:
        """The device's local_normal_at (world_space=False) or normal_at on (n, 3) points."""
        p = np.ascontiguousarray(np.asarray(points, dtype=np.float64).reshape(-1, 3))
        out = np.zeros_like(p)
        _check(_lib.rt_debug_normal(self._h, shape, p.ctypes.data_as(C.POINTER(C.c_double)), p.shape[0],
                                    PRECISIONS[precision], int(world_space), out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def set_gather(self, mode: int) -> None:
        """Multi-GPU contexts: RT_GATHER_RCCL (strips + ncclGather + de-interleave) or RT_GATHER_PEER (every
        shard stores into one canvas on rank 0; rtc.h).  Collective."""
        _check(_lib.rt_context_set_gather(self._h, mode))

    # ------------------------------------------------ peer canvas (rtc.h)
    def canvas_create(self, nbytes: int, n_flags: int, ipc: bool = True):
        """(device pointer, IPC handle bytes or None) of a new canvas of `nbytes` + n_flags shard flags."""
        p = C.c_void_p()
        h = (C.c_uint8 * RT_IPC_HANDLE_BYTES)()
        _check(_lib.rt_canvas_create(self._h, nbytes, n_flags, C.byref(p), h if ipc else None))
        return p.value, (bytes(h) if ipc else None)

    def canvas_open(self, handle: bytes, nbytes: int, n_flags: int) -> int:
        """Map another process's canvas (its rt_canvas_create handle); returns the device pointer."""
        h = (C.c_uint8 * RT_IPC_HANDLE_BYTES).from_buffer_copy(handle)
        p = C.c_void_p()
        _check(_lib.rt_canvas_open(self._h, h, nbytes, n_flags, C.byref(p)))
        return p.value

    def canvas_close(self, canvas: int) -> None:
        _check(_lib.rt_canvas_close(self._h, C.c_void_p(canvas)))

    def render_to_canvas(self, camera: CameraDesc, canvas: int, seq: int, depth: int = RT_DEFAULT_MAX_DEPTH,
                         precision: str = "f32", out_format: str = "real", shard=(0, 1), stream_ptr: int | None = None,
                         timeout_ms: float = 10000.0) -> None:
        opts = self.options(depth, precision, out_format, shard)
        _check(_lib.rt_render_to_canvas(self._h, C.byref(camera), C.byref(opts), C.c_void_p(canvas), seq,
                                        float(timeout_ms), C.c_void_p(stream_ptr or 0)))

    def canvas_wait(self, canvas: int, seq: int, timeout_ms: float = 10000.0, stream_ptr: int | None = None) -> None:
        _check(_lib.rt_canvas_wait(self._h, C.c_void_p(canvas), seq, float(timeout_ms), C.c_void_p(stream_ptr or 0)))

    def canvas_release(self, canvas: int, seq: int, stream_ptr: int | None = None) -> None:
        _check(_lib.rt_canvas_release(self._h, C.c_void_p(canvas), seq, C.c_void_p(stream_ptr or 0)))

    def canvas_read(self, canvas: int, shape, dtype=np.uint8) -> np.ndarray:
        """The canvas image as a host array of `shape` (synchronous; raises on a peer-canvas timeout)."""
        out = np.zeros(shape, dtype=dtype)
        _check(_lib.rt_canvas_read(self._h, C.c_void_p(canvas), out.ctypes.data_as(C.c_void_p), out.nbytes))
        return out

    def counters(self) -> dict:
        st = Stats()
        _check(_lib.rt_read_counters(self._h, C.byref(st)))
        return st.as_dict()

    def generation_counts(self):
        """(traced, shaded) per `remaining` 0..16, cumulative over RT_FLAG_GENERATIONS launches (rtc.h)."""
        g = GenerationCounts()
        _check(_lib.rt_read_generation_counts(self._h, C.byref(g)))
        return np.array(g.traced[:], dtype=np.uint64), np.array(g.shaded[:], dtype=np.uint64)

    def render_generations(self, camera: CameraDesc, depth: int = RT_DEFAULT_MAX_DEPTH, precision: str = "f32"):
        """One diagnostic frame with RT_FLAG_GENERATIONS: (image, stats, per-generation dict).  Generation g
        (0 = camera rays) is `remaining` depth - g; shadow rays are L per shaded hit (world.rs:46-52)."""
        t0, s0 = self.generation_counts()
        opts = self.options(depth, precision, "real", (0, 1), RT_FLAG_GENERATIONS)
        dtype = np.float32 if precision == "f32" else np.float64
        img = np.zeros((camera.height, camera.width, 3), dtype=dtype)
        st = Stats()
        _check(_lib.rt_render(self._h, C.byref(camera), C.byref(opts), img.ctypes.data_as(C.c_void_p), C.byref(st)))
        t1, s1 = self.generation_counts()
        traced, shaded = (t1 - t0)[::-1][-(depth + 1):], (s1 - s0)[::-1][-(depth + 1):]
        return img, st.as_dict(), {"traced": [int(v) for v in traced], "shaded": [int(v) for v in shaded]}

    def assemble_shards(self, gathered_ptr: int, width: int, height: int, shards: int, bytes_per_pixel: int,
                        image_ptr: int, stream_ptr: int | None = None) -> None:
        _check(_lib.rt_assemble_shards(self._h, C.c_void_p(gathered_ptr), width, height, shards, bytes_per_pixel,
                                       C.c_void_p(image_ptr), C.c_void_p(stream_ptr or 0)))
