"""Register budget of the f32 tracer kernels, read from the gfx950 code
object inside librtc.so (no GPU needed).

Occupancy of these kernels is set by VGPRs, and it has cliffs: the pool
kernel at 129 VGPRs ran 3 waves/SIMD instead of 4 and measured ~60% slower
(DESIGN.md §3.3a).  The build caps both kernels with amdgpu_waves_per_eu
(RTC_DIRECT_WAVES = 8, RTC_POOL_WAVES = 6).  Built with -fno-slp-vectorize the
direct kernel fits 64 VGPRs without scratch and the pool kernel spills
8 B/lane.  This test catches a build that lost the caps or started spilling
far more.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import PKG

LIB = os.path.join(PKG, "rtc_amd", "_lib", "librtc.so")
LLVM = "/opt/rocm/lib/llvm/bin"
# kernel-name prefix -> (max VGPRs, max private bytes per lane)
BUDGET = {"_ZN3rtc12trace_directIf": (64, 16), "_ZN3rtc10trace_poolIf": (80, 64)}


def kernel_metadata(tmp):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(os.path.exists(t) for t in tools):
        pytest.skip("ROCm LLVM tools not installed")
    fb, co = os.path.join(tmp, "fatbin"), os.path.join(tmp, "co.elf")
    subprocess.run([tools[0], "--dump-section", f".hip_fatbin={fb}", LIB, os.path.join(tmp, "lib.so")], check=True)
    subprocess.run([tools[1], "--unbundle", "--type=o", f"--input={fb}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True)
    notes = subprocess.run([tools[2], "--notes", co], check=True, capture_output=True, text=True).stdout
    kernels = {}
    for block in re.split(r"\n\s+- \.", notes):
        name = re.search(r"\.name:\s+(\S+)", block)
        vgpr = re.search(r"\.vgpr_count:\s+(\d+)", block)
        priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
        group = re.search(r"\.group_segment_fixed_size:\s+(\d+)", block)
        if name and vgpr and priv:
            kernels[name.group(1)] = (int(vgpr.group(1)), int(priv.group(1)), int(group.group(1)) if group else 0)
    return kernels


def test_f32_kernels_stay_within_their_occupancy_budget(tmp_path):
    if not shutil.which("nm"):
        pytest.skip("binutils missing")
    kernels = kernel_metadata(str(tmp_path))
    for prefix, (vmax, pmax) in BUDGET.items():
        found = {k: v for k, v in kernels.items() if k.startswith(prefix)}
        assert found, f"no kernel {prefix}* in {LIB}"
        for name, (vgpr, priv, group) in found.items():
            assert vgpr <= vmax, f"{name}: {vgpr} VGPRs > {vmax} (occupancy cliff)"
            assert priv <= pmax, f"{name}: {priv} B/lane of scratch > {pmax}"


def test_static_lds_fits_the_hosts_allowance(tmp_path):
    """rtc_host.cpp sizes LDS residency with kStaticLds = 512 B of static LDS
    per tracer workgroup; a kernel that declares more would be over-admitted."""
    for name, (_, _, group) in kernel_metadata(str(tmp_path)).items():
        if "trace_" in name:
            assert group <= 512, f"{name}: {group} B of static LDS > kStaticLds"
