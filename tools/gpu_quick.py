"""Quick GPU sanity run: render the golden scenes on the GPU and compare with
the oracle and the fixtures (prints stats; used during development)."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import openglraytracer_amd as rt
from oracle import port, scenes

ctx = rt.Context(0)
man = json.load(open(os.path.join(ROOT, "tests/golden/manifest.json")))
for name, m in sorted(man.items()):
    if m["probe"]:
        continue
    z = np.load(os.path.join(ROOT, "tests/golden/%s.npz" % name))
    x0, y0, w, h = m["crop"]
    objs = rt.reference_objects(m["time"]) if m["scene"] == "shipped" else scenes.CONFIGS[m["scene"]][0]()
    sc = rt.Scene(ctx, objs)
    cam = rt.reference_camera(m["time"])
    view = rt.view_from_matrix(z["unproj"], list(cam.position))
    g = rt.render(ctx, sc, m["width"], m["height"], m["max_depth"], view=view, rows=(y0, y0 + h))[:, x0:x0 + w]
    d = np.abs(g[..., :3] - z["rgb"]).max(-1)
    # oracle with same pinned view
    U = np.ascontiguousarray(z["unproj"], np.float32)
    import ctypes as C
    port.lib().oracle_pin_unprojection(U.ctypes.data_as(C.c_void_p))
    o = port.render(objs, m["width"], m["height"], m["max_depth"], m["time"], rows=(y0, y0 + h))[:, x0:x0 + w]
    port.lib().oracle_pin_unprojection(None)
    do = np.abs(g - o).max(-1)
    print("%-30s vs GL: exact %.4f max %.2e | vs oracle: exact %.4f max %.2e  alpha0 %s" % (
        name, (d == 0).mean(), d.max(), (do == 0).mean(), do.max(), bool((g[..., 3] == 0).all())), flush=True)

# timing: config 2
objs = scenes.bench_objects(16)
sc = rt.Scene(ctx, objs)
import torch
out = torch.empty((1080, 1920, 4), dtype=torch.float32, device="cuda")
view = rt.make_view(None, 0.0)
for _ in range(3):
    rt.render_device(ctx, sc, out.data_ptr(), 1920, 1080, 0, view=view)
t0 = time.time(); n = 20
for _ in range(n):
    rt.render_device(ctx, sc, out.data_ptr(), 1920, 1080, 0, view=view)
dt = (time.time() - t0) / n
print("config2 wall %.3f ms/frame, kernel %.3f ms, %.1f Grays/s" % (dt * 1e3, ctx.last_kernel_ms(), 1920 * 1080 / ctx.last_kernel_ms() / 1e6))
full = out.cpu().numpy()
o = port.render(objs, 1920, 1080, 0, 0.0, rows=(0, 1080))
d = np.abs(full - o).max(-1)
print("config2 full frame vs oracle (f64 view both): exact %.5f max %.2e" % ((d == 0).mean(), d.max()))
for cfg, ns, W, H, D in [("config3", 64, 3840, 2160, 2), ("config4", 256, 7680, 4320, 4)]:
    sc = rt.Scene(ctx, scenes.bench_objects(ns))
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    rt.render_device(ctx, sc, out.data_ptr(), W, H, D, view=view)
    t0 = time.time()
    rt.render_device(ctx, sc, out.data_ptr(), W, H, D, view=view)
    print("%s kernel %.3f ms wall %.3f ms" % (cfg, ctx.last_kernel_ms(), (time.time() - t0) * 1e3), flush=True)
