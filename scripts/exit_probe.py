"""Diagnostic: process exit with a per-scene build in flight (RT_JIT_AUTO
starts it at the 2nd large frame).  argv[1]: 'off' (RTC_JIT=0), 'wait'
(rt_jit_wait before exit) or 'inflight' (exit while hipRTC compiles)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
mode = sys.argv[1]
if mode == "off":
    os.environ["RTC_JIT"] = "0"
import faulthandler  # noqa: E402
faulthandler.enable()
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", "cover.json"))
cam = rtc_amd.camera_resize(scene.camera, 1920, 1080)
with rtc_amd.Context(0) as ctx:
    ctx.upload(scene)
    for _ in range(3):
        ctx.render(cam, 6, precision="f32")
    if mode == "wait":
        print("pending after wait:", ctx.jit_wait(60000))
print("exiting", mode, flush=True)
