"""Development timing of every benchmark config (GPU events, kernel only),
with and without culling, and a bitwise check culled == unculled == oracle
on a band. Prints one line per config."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import openglraytracer_amd as rt
from oracle import port, scenes

ctx = rt.Context(0)
view = rt.make_view(None, 0.0)
res = {}
for cfg in ["config1", "config2", "config3", "config4"]:
    build, w, h, depth = scenes.CONFIGS[cfg]
    objs = build()
    sc = rt.Scene(ctx, objs)
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    line = {}
    frames = {}
    for cull in (1, 0):
        ctx.set_culling(cull)
        reps = 20 if cfg in ("config1", "config2") else 3
        rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)
        torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)
            ms.append(ctx.last_kernel_ms())
        line["ms_cull%d" % cull] = round(float(np.median(ms)), 4)
        frames[cull] = out.clone()
    ctx.set_culling(1)
    line["cull_equal"] = bool(torch.equal(frames[0], frames[1]))
    r0 = h // 2 - 2
    o = port.render(objs, w, h, depth, 0.0, rows=(r0, r0 + 4))
    line["band_vs_oracle_exact"] = bool(np.array_equal(frames[1][r0:r0 + 4].cpu().numpy(), o))
    line["Grays_s"] = round(w * h / line["ms_cull1"] / 1e6, 3)
    print(cfg, json.dumps(line), flush=True)
    res[cfg] = line
    sc.close()
print(json.dumps(res))
