#!/usr/bin/env python3
"""Diagnostic: distribution of per-tile costs of a pool scene (f32, warm,
cost-ordered launch), optionally of one row-block shard.

Usage: tile_costs.py [scene] [WxH] [shard_index/shard_count]
"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))


def main():
    import numpy as np, torch, rtc_amd
    from rtc_amd import scene_io
    name = sys.argv[1] if len(sys.argv) > 1 else "reflect_refract"
    w, h = map(int, (sys.argv[2] if len(sys.argv) > 2 else "1920x1080").split("x"))
    si, sn = map(int, (sys.argv[3] if len(sys.argv) > 3 else "0/1").split("/"))
    sc = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
    cam = rtc_amd.camera_resize(sc.camera, w, h)
    ctx = rtc_amd.Context(0)
    ctx.upload(sc)
    rows = rtc_amd.shard_rows(h, sn)
    out = torch.empty((rows, w, 3), dtype=torch.float32, device="cuda")
    for _ in range(4):
        ctx.render_device(cam, out.data_ptr(), 0, 6, "f32", "real", (si, sn))
    torch.cuda.synchronize()
    n = ((w + 63) // 64) * (rows // 4)
    c = ctx.debug_tile_costs()[:n].astype(np.float64) * 0.01  # us
    q = [round(float(np.quantile(c, p)), 1) for p in (0, 0.5, 0.9, 0.99, 0.999, 1.0)]
    top = np.sort(c)[::-1][:8]
    print(json.dumps({"scene": name, "size": f"{w}x{h}", "shard": f"{si}/{sn}", "tiles": n,
                      "tile_us_q(0,.5,.9,.99,.999,1)": q, "top8": [round(float(v), 1) for v in top],
                      "sum_us": round(float(c.sum()), 1)}), flush=True)


if __name__ == "__main__":
    main()
