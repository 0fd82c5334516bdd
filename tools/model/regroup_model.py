"""CPU model: regrouping a work-group's secondary rays before the BVH walk (development probe).

    python tools/model/regroup_model.py [--config config4] [--tiles 128] [--seed 1]

Round 4's verdict asked whether the BVH node loop's 58 % lane utilisation
(tools/model/bvh_model.py: 22.45 node iterations per wave call for 13.84
node tests per ray) could be raised by regrouping: at walk iteration k, put
the 256 lanes' k-th rays of a work-group's four waves into LDS, sort them by
a coherence key, deal them back to the waves in chunks of 64, walk, and
return the hits to their lanes. This replays exactly that on the product's
own BVH (rt_debug_scene_blob) with walk_model's rays, grouped four wave tiles
(a work-group of the queued kernel) at a time, and reports per group and
iteration:

  waves      — wave calls of the node loop (a regrouped chunk of 64 rays is
               one wave call; a wave with no ray at iteration k makes none);
  node_iters — iterations of the node loop summed over the wave calls (the
               SIMD issue cost of the walk: every iteration costs the wave
               its instructions whatever its active lanes);
  passes     — leaf sphere-test passes summed over the wave calls;

for the kernel's grouping (each wave keeps its own lanes) and for
regroupings by: `compact` (the same order, inactive lanes squeezed out),
`octant` (ray-direction octant, then lane order), `octant_src` (octant, then
the object the ray starts on) and `morton` (octant, then a 3-D Morton code of
the origin quantised to the room). The walk (its node tests and leaf visits)
is the same per ray under every grouping; only how the rays share waves
changes. Costs the model does not price: the two LDS exchanges per
iteration (ray out, hit back: about 24 + 16 B per lane) and two barriers
that tie the four waves' iterations together.

Also reported: where secondary rays start (the room box vs a sphere).
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import bvh_model as bm  # noqa: E402
import walk_model as wm  # noqa: E402


def octant(d):
    return int(d[0] < 0) | (int(d[1] < 0) << 1) | (int(d[2] < 0) << 2)


def morton3(q):
    """10-bit-per-axis Morton code of integer coordinates q (3,)."""
    code = 0
    for bit in range(10):
        for ax in range(3):
            code |= ((int(q[ax]) >> bit) & 1) << (3 * bit + ax)
    return code


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config4")
    ap.add_argument("--tiles", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--adjacent", type=int, default=4,
                    help="tiles per run of horizontally adjacent wave tiles (4: a queued work-group's waves "
                         "start on adjacent tiles; 1: independent random tiles)")
    a = ap.parse_args()
    w, h, nsph, depth = wm.CONFIGS[a.config]
    S = wm.scene_arrays(nsph)
    B = bm.scene_bvh(nsph)
    rng = np.random.default_rng(a.seed)
    wm.links.clear()
    n_pix, pix, lev, hitl, cr, ct = wm.build_trees(S, w, h, depth, a.tiles, rng, adjacent=a.adjacent)
    ro, rd = wm.build_trees.rays
    src = wm.build_trees.src
    lo, hi = S["bmin"], S["bmax"]
    schemes = ["kernel", "compact", "octant", "octant_src", "morton", "level_octant"]
    tot = {s: dict(waves=0, node_iters=0, passes=0) for s in schemes}
    rays_total = 0
    starts = dict(box=0, sphere=0)
    groups = a.tiles // 4
    for g in range(groups):
        orders = []
        for t in range(4 * g, 4 * g + 4):
            for r in range(t * 64, (t + 1) * 64):
                od = []
                wm.lane_events(r, cr, ct, od)
                orders.append(od)
        for k in range(1, max(len(x) for x in orders)):  # secondary rays: walk iterations >= 1
            lanes = [x[k] if k < len(x) else -1 for x in orders]  # 256 node ids (-1: no ray)
            live = [n for n in lanes if n >= 0]
            if not live:
                continue
            rays_total += len(live)
            for n in live:
                starts["box" if src[n] == -1 else "sphere"] += 1

            def cost(chunks, scheme):
                for ch in chunks:
                    ch = [n for n in ch if n >= 0]
                    if not ch:
                        continue
                    rays = [(ro[n], rd[n]) for n in ch]
                    tbox = [bm.box_exit(S, ro[n], rd[n]) for n in ch]
                    it, ps, _, _ = bm.lane_walk(B, rays, tbox)
                    tot[scheme]["waves"] += 1
                    tot[scheme]["node_iters"] += it
                    tot[scheme]["passes"] += ps

            cost([lanes[i * 64:(i + 1) * 64] for i in range(4)], "kernel")
            keys = {
                "compact": lambda n: 0,
                "octant": lambda n: octant(rd[n]),
                "octant_src": lambda n: (octant(rd[n]), int(src[n])),
                "morton": lambda n: (octant(rd[n]), morton3(np.clip((ro[n] - lo) / (hi - lo) * 1023, 0, 1023))),
                "level_octant": lambda n: (int(lev[n]), octant(rd[n])),
            }
            for name, key in keys.items():
                order = sorted(range(len(live)), key=lambda i: (key(live[i]), i))
                srt = [live[i] for i in order]
                cost([srt[i:i + 64] for i in range(0, len(srt), 64)], name)
    out = {"config": a.config, "groups": groups, "secondary_rays": rays_total,
           "ray_starts": {k: round(v / max(1, rays_total), 3) for k, v in starts.items()}}
    base = tot["kernel"]["node_iters"]
    for s in schemes:
        t = tot[s]
        out[s] = {"wave_calls": t["waves"], "node_iters": t["node_iters"], "passes": t["passes"],
                  "node_iters_per_call": round(t["node_iters"] / max(1, t["waves"]), 2),
                  "node_iters_vs_kernel": round(t["node_iters"] / base, 3),
                  "passes_vs_kernel": round(t["passes"] / max(1, tot["kernel"]["passes"]), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
