"""The per-scene kernel compiler process (csrc/rtc_jitc.cpp) on the CPU:
librtc hands it a request file (csrc/rtc_jit_cache.hpp) and loads the code
object it writes.  hipRTC cross-compiles for gfx950 without a GPU."""
import os
import subprocess

import pytest

from conftest import PKG

JITC = os.path.join(PKG, "rtc_amd", "_lib", "rtc_jitc")


def _put(s: bytes) -> bytes:
    return str(len(s)).encode() + b"\n" + s


def _request(name, src, opts, headers=()):
    b = b"RTCREQ1\n" + _put(name.encode()) + _put(src.encode()) + _put(str(len(opts)).encode())
    for o in opts:
        b += _put(o.encode())
    b += _put(str(len(headers)).encode())
    for hn, ht in headers:
        b += _put(hn.encode()) + _put(ht.encode())
    return b


def _fnv(data: bytes) -> int:
    h = 1469598103934665603
    for c in data:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


SRC = '#include "k.h"\nextern "C" __global__ void k(float* a) { a[threadIdx.x] *= kScale; }\n'


def test_compiles_a_request_into_a_code_object(tmp_path):
    req, out = tmp_path / "r.req", tmp_path / "sub" / "k.co"
    req.write_bytes(_request("k", SRC, ["--offload-arch=gfx950", "-O3"], [("k.h", "constexpr float kScale = 2.0f;\n")]))
    r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert not req.exists()  # the compiler deletes its request
    data = out.read_bytes()
    assert data.startswith(b"RTCJIT2\nk\n")
    head, _, code = data[len(b"RTCJIT2\nk\n"):].partition(b"\n")
    n, s = head.split()
    assert int(n) == len(code) and int(s, 16) == _fnv(code)
    assert code[:4] == b"\x7fELF"  # an AMDGPU code object
    assert not [p for p in os.listdir(out.parent) if ".tmp" in p]


def test_compile_error_is_reported(tmp_path):
    req, out = tmp_path / "r.req", tmp_path / "k.co"
    req.write_bytes(_request("k", SRC.replace("kScale", "kMissing"), ["--offload-arch=gfx950"],
                             [("k.h", "constexpr float kScale = 2.0f;\n")]))
    r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "kMissing" in r.stderr and not out.exists()


@pytest.mark.parametrize("content", [None, b"RTCREQ1\n5\nab", b"garbage"])
def test_bad_request(tmp_path, content):
    req = tmp_path / "r.req"
    if content is not None:
        req.write_bytes(content)
    r = subprocess.run([JITC, str(req), str(tmp_path / "k.co")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "request" in r.stderr
