"""CPU model of the secondary rays' BVH walk per 64-lane wave (development probe).

    python tools/model/bvh_model.py [--config config4] [--tiles 128] [--seed 1]

The closest hit of a secondary ray (rt_kernel.hip closest_impl, !kPrimary)
walks the scene's sphere BVH — the very nodes, boxes and ordered links the
product builds (rt_debug_scene_blob, the blob rt_scene_create uploads) —
per lane, stackless, "while-while": every lane steps through nodes until it
holds a leaf (or its walk ends), then the wave tests the spheres of all held
leaves together. A node step costs the wave an iteration whenever ANY lane
steps; a leaf pass as many sphere tests as the largest held leaf.

The rays are those of tools/model/walk_model.py (float64 restatement of the
shader's camera, hits, reflect / refract), grouped by wave and walk
iteration exactly as trace_tree runs them (iteration k = every lane's k-th
ray). Simulated walks:

  lane     — the kernel's walk (to check the model against RT_STATS:
             13.7 node tests per secondary ray, 21.3 node iterations per
             wave call, 1.43 leaf visits per ray);
  packet   — one wave-uniform walk of the same BVH in the first active
             lane's octant order: a node is entered when any lane's ray
             reaches it within its current t; a leaf's spheres are tested by
             every lane whose ray reaches the leaf;
  pair     — per-lane walk testing a node's two children in one step (both
             boxes, nearer first), so a step moves one level down or across.

Printed per wave call: iterations and sphere-test passes per scheme.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import walk_model as wm  # noqa: E402

rt = wm.rt


def scene_bvh(n_spheres):
    L = rt.lib()
    f = L.rt_debug_scene_blob
    f.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_longlong,
                  C.c_void_p]
    objs, mats, lights = rt.bench_objects(n_spheres, 0), rt.reference_materials(), rt.reference_lights()
    oa = (rt.Object * len(objs))(*objs)
    ma = (rt.Material * len(mats))(*mats)
    la = (rt.Light * len(lights))(*lights)
    meta = np.zeros(24, np.int32)
    n = f(oa, len(objs), ma, len(mats), la, len(lights), None, 0, meta.ctypes.data)
    buf = np.zeros(n, np.uint8)
    f(oa, len(objs), ma, len(mats), la, len(lights), buf.ctypes.data, n, meta.ctypes.data)
    units = buf.view(np.float32).reshape(-1, 4)
    ints = buf.view(np.int32).reshape(-1, 4)
    off_sph, off_bvh, n_bvh, off_blink, ns = meta[1], meta[7], meta[8], meta[9], meta[17]
    sph = units[off_sph:off_sph + ns].astype(np.float64)  # cx cy cz r*r
    lo = units[off_bvh:off_bvh + 2 * n_bvh:2, :3].astype(np.float64)
    hi = units[off_bvh + 1:off_bvh + 2 * n_bvh:2, :3].astype(np.float64)
    leaf = ints[off_bvh + 1:off_bvh + 2 * n_bvh:2, 3].copy()
    links = buf.view(np.uint32)[off_blink * 4:off_blink * 4 + 8 * n_bvh].reshape(n_bvh, 8)
    return dict(sph=sph, lo=lo, hi=hi, leaf=leaf, links=links, n=n_bvh)


def node_hit(B, node, o, d, tlim):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = np.where(np.abs(d) > 1e-30, 1.0 / d, np.where(d < 0, -1e30, 1e30))
    t0 = (B["lo"][node] - o) * inv
    t1 = (B["hi"][node] - o) * inv
    tn = np.max(np.minimum(t0, t1), -1)
    tf = np.min(np.maximum(t0, t1), -1)
    return (tn <= tf) & (tf >= 0) & (tn <= tlim)


def sphere_t(B, s, o, d):
    c = B["sph"][s, :3]
    oc = o - c
    b = oc @ d
    qc = oc @ oc - B["sph"][s, 3]
    disc = b * b - qc
    if disc < 0:
        return np.inf
    sq = np.sqrt(disc)
    t1, t2 = -b - sq, -b + sq
    return t1 if t1 > 0 else (t2 if t2 > 0 else np.inf)


def succ(B, node, oct_, hit):
    w = int(B["links"][node, oct_])
    n = (w & 0xFFFF) if hit else (w >> 16)
    return -1 if n == 0xFFFF else n


def lane_walk(B, rays, tbox):
    """The kernel's while-while walk for one wave call: rays = list of
    (o, d) or None per lane. Returns (node iterations, sphere passes, node
    tests, leaf visits)."""
    lanes = [i for i, r in enumerate(rays) if r is not None]
    node = {i: 0 for i in lanes}
    t = {i: tbox[i] for i in lanes}
    octs = {i: int(rays[i][1][0] < 0) | (int(rays[i][1][1] < 0) << 1) | (int(rays[i][1][2] < 0) << 2) for i in lanes}
    iters = passes = tests = visits = 0
    while any(node[i] >= 0 for i in lanes):
        held = {i: 0 for i in lanes}
        while any(node[i] >= 0 and held[i] == 0 for i in lanes):
            iters += 1
            for i in lanes:
                if node[i] >= 0 and held[i] == 0:
                    n = node[i]
                    o, d = rays[i]
                    tests += 1
                    h = bool(node_hit(B, n, o, d, t[i]))
                    if h:
                        held[i] = int(B["leaf"][n])
                    node[i] = succ(B, n, octs[i], h)
        cnt = [held[i] >> 24 for i in lanes if held[i]]
        if cnt:
            passes += max(cnt)
            for i in lanes:
                if held[i]:
                    visits += 1
                    first, count = held[i] & 0xFFFFFF, held[i] >> 24
                    o, d = rays[i]
                    for s in range(first, first + count):
                        t[i] = min(t[i], sphere_t(B, s, o, d))
    return iters, passes, tests, visits


def packet_walk(B, rays, tbox):
    lanes = [i for i, r in enumerate(rays) if r is not None]
    if not lanes:
        return 0, 0
    t = {i: tbox[i] for i in lanes}
    d0 = rays[lanes[0]][1]
    oct_ = int(d0[0] < 0) | (int(d0[1] < 0) << 1) | (int(d0[2] < 0) << 2)
    node, iters, passes = 0, 0, 0
    while node >= 0:
        iters += 1
        who = [i for i in lanes if node_hit(B, node, rays[i][0], rays[i][1], t[i])]
        if who and B["leaf"][node]:
            first, count = B["leaf"][node] & 0xFFFFFF, B["leaf"][node] >> 24
            passes += count
            for i in who:
                for s in range(first, first + count):
                    t[i] = min(t[i], sphere_t(B, s, rays[i][0], rays[i][1]))
        node = succ(B, node, oct_, bool(who))
    return iters, passes


def box_exit(S, o, d):
    with np.errstate(divide="ignore", invalid="ignore"):
        ta = (S["bmin"] - o) / d
        tb = (S["bmax"] - o) / d
    return float(np.min(np.maximum(ta, tb)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config4")
    ap.add_argument("--tiles", type=int, default=64)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    w, h, nsph, depth = wm.CONFIGS[a.config]
    S = wm.scene_arrays(nsph)
    B = scene_bvh(nsph)
    rng = np.random.default_rng(a.seed)
    wm.links.clear()
    n_pix, pix, lev, hitl, cr, ct = wm.build_trees(S, w, h, depth, a.tiles, rng)
    ro, rd = wm.build_trees.rays
    tot = dict(calls=0, rays=0, lane_iters=0, lane_passes=0, lane_tests=0, lane_visits=0, packet_iters=0,
               packet_passes=0)
    for t in range(a.tiles):
        orders = []
        for r in range(t * 64, (t + 1) * 64):
            od = []
            wm.lane_events(r, cr, ct, od)
            orders.append(od)
        for k in range(1, max(len(x) for x in orders)):  # secondary rays: walk iterations >= 1
            rays, tbox = [], []
            for x in orders:
                if k < len(x):
                    o, d = ro[x[k]], rd[x[k]]
                    rays.append((o, d))
                    tbox.append(box_exit(S, o, d))
                else:
                    rays.append(None)
                    tbox.append(0.0)
            if not any(r is not None for r in rays):
                continue
            tot["calls"] += 1
            tot["rays"] += sum(r is not None for r in rays)
            i, p, te, v = lane_walk(B, rays, tbox)
            tot["lane_iters"] += i
            tot["lane_passes"] += p
            tot["lane_tests"] += te
            tot["lane_visits"] += v
            pi, pp = packet_walk(B, rays, tbox)
            tot["packet_iters"] += pi
            tot["packet_passes"] += pp
    c, r = tot["calls"], tot["rays"]
    out = {"config": a.config, "tiles": a.tiles, "wave_calls": c, "secondary_rays": r,
           "lane": {"node_iters_per_call": round(tot["lane_iters"] / c, 2),
                    "sphere_passes_per_call": round(tot["lane_passes"] / c, 2),
                    "node_tests_per_ray": round(tot["lane_tests"] / r, 2),
                    "leaf_visits_per_ray": round(tot["lane_visits"] / r, 2),
                    "lane_utilisation": round(tot["lane_tests"] / (64 * tot["lane_iters"]), 3)},
           "packet": {"node_iters_per_call": round(tot["packet_iters"] / c, 2),
                      "sphere_passes_per_call": round(tot["packet_passes"] / c, 2)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
