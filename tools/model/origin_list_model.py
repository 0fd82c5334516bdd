"""CPU model: per-origin-sphere direction candidate lists for secondary rays (development probe).

    python tools/model/origin_list_model.py [--config config4] [--tiles 64] [--texels 16] [--seed 1]

73 % of config 4's secondary rays start on a sphere (tools/model/
regroup_model.py). For such a ray the spheres it can hit are fixed by its
origin sphere s and its direction: the rays from the ball B(c_s, r_s + 0.001)
whose directions lie in a cone (axis a, half-angle th) can reach sphere j only
if the cone from c_s meets the ball B(c_j, r_j + r_s + 0.001), i.e.
angle(a, c_j - c_s) <= th + asin((r_j + r_s + 0.001) / |c_j - c_s|) — the
shadow cube maps' geometry with the origin sphere folded into the target.
So a cube map per sphere (n x n texels per face) can list, per texel, the
candidate spheres ordered by a lower bound of their hit distance
(|c_j - c_s| - r_j - r_s - 0.001); a lane then tests candidates in order
until its closest hit so far (the room box's exit distance to start with: the
box is tested first) is below the next candidate's bound, and the BVH walk
is not needed for that ray. Its own sphere is always candidate 0 (a
refraction ray inside it exits through it).

Replays walk_model's rays, grouped per wave tile and walk iteration as
trace_tree runs them, and reports per secondary wave call:
  bvh      — the kernel today: node iterations + sphere passes (bvh_model's
             while-while walk) for every ray;
  lists    — sphere-origin lanes walk their texel's list (passes = the
             longest lane's tests), box-origin lanes the BVH as today; the
             wave pays both when it has both kinds;
and the list sizes (mean / p99 / max per texel, and as the rays meet them),
with the table's bytes at 1 B per candidate slot.
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
import shadow_model as sm  # noqa: E402


def cube_texels(n):
    """Per texel of an n x n per-face cube map (the kernel's direction_texel
    layout: the cube-map instructions' face and sc / tc coordinates, as
    rt_scene.cpp mask_cones): unit axis (6 n n, 3) and the half-angle of the
    cone that holds the texel (axis to its farthest corner)."""
    axes, halves = [], []
    g = (np.arange(n) + 0.5) / n * 2 - 1
    c = np.arange(n + 1) / n * 2 - 1
    for face in range(6):
        for row in range(n):
            for col in range(n):
                a = np.array(sm.face_dir(face, g[col], g[row]), float)
                a /= np.linalg.norm(a)
                best = 0.0
                for dr in (0, 1):
                    for dc in (0, 1):
                        q = np.array(sm.face_dir(face, c[col + dc], c[row + dr]), float)
                        q /= np.linalg.norm(q)
                        best = max(best, np.arccos(np.clip(a @ q, -1, 1)))
                axes.append(a)
                halves.append(best)
    return np.array(axes), np.array(halves)


def texel_of(d, n):
    """The kernel's direction_texel (rt_kernel.hip) in float64."""
    return sm.texel(d, n)


def build_lists(S, n, margin=1e-3):
    c, r = S["c"], S["r"]
    axes, halves = cube_texels(n)
    ns = len(c)
    lists = []  # per sphere: per texel (candidates ordered by bound, bounds)
    for s in range(ns):
        v = c - c[s]
        dist = np.linalg.norm(v, axis=1)
        rin = r + r[s] + 0.001 + margin
        near = dist <= rin
        u = np.where(near[:, None], 0.0, v / np.maximum(dist, 1e-30)[:, None])
        ang = np.where(near, np.pi, np.arcsin(np.clip(rin / np.maximum(dist, 1e-30), 0, 1)))
        bound = np.maximum(dist - r - r[s] - 0.001 - margin, 0.0)
        cosang = axes @ u.T  # (texels, spheres)
        ok = (np.arccos(np.clip(cosang, -1, 1)) <= halves[:, None] + ang[None, :] + margin) | near[None, :]
        ok[:, s] = True
        per = []
        for t in range(len(axes)):
            js = np.nonzero(ok[t])[0]
            b = np.where(js == s, -1.0, bound[js])
            o = np.argsort(b, kind="stable")
            per.append((js[o], b[o]))
        lists.append(per)
    return lists


def sphere_hit(S, j, o, d):
    oc = o - S["c"][j]
    b = oc @ d
    qc = oc @ oc - S["r"][j] ** 2
    disc = b * b - qc
    if disc < 0:
        return np.inf
    sq = np.sqrt(disc)
    t1, t2 = -b - sq, -b + sq
    return t1 if t1 > 0 else (t2 if t2 > 0 else np.inf)


def list_walk(S, per, o, d, t0, slots=None, shell=1):
    """One lane walking its texel's list from best = t0 (the box exit).
    slots=None: every candidate's bound is known (stop at the first bound >=
    best). slots=K: a fixed record of the first K candidates with the bound
    stored only every `shell` candidates (the lane may stop only there); a
    lane that reaches the record's end with candidates left over (and best
    above the next bound) must walk the BVH instead. Returns (tests, fallback)."""
    js, b = per
    best, tests = t0, 0
    n = len(js) if slots is None else min(len(js), slots)
    for i in range(n):
        if (slots is None or i % shell == 0) and b[i] >= best:
            return tests, False
        tests += 1
        best = min(best, sphere_hit(S, js[i], o, d))
    if slots is not None and len(js) > slots and b[slots] < best:
        return tests, True
    return tests, False


RECORDS = [(15, 4), (15, 1), (27, 4), (27, 9)]
# (round 6) records as the kernel walks them: (name, slots K, the candidates
# before which a stored bound is checked, bound quantum): the product's 32-B
# record (25 slots, uint16 bounds in 1/256 at candidates 8 and 16 and at the
# end) and a variant of the same 32 B with 24 slots and 8-bit bounds in 1/8
# units before every 4th candidate (4, 8, ..., 20) and at the end
KRECORDS = [("product_25_b8_16_q256", 25, (8, 16), 1.0 / 256), ("variant_24_b4_q8", 24, (4, 8, 12, 16, 20), 1.0 / 8)]


def list_walk_k(S, per, o, d, t0, slots, checks, q):
    """The kernel's record walk: the lane tests candidates 0..K-1, stopping
    before candidate i in `checks` (and at the end) when its closest hit is
    below the stored bound floor(b / q) q; past the record with candidates
    left and the end bound not reached: the BVH. Returns (tests, fallback)."""
    js, b = per
    best, tests = t0, 0
    n = min(len(js), slots)
    for i in range(n):
        if i in checks and np.floor(b[i] / q) * q > best:
            return tests, False
        tests += 1
        best = min(best, sphere_hit(S, js[i], o, d))
    if len(js) > slots and not (best < np.floor(b[slots] / q) * q):
        return tests, True
    return tests, False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config4")
    ap.add_argument("--tiles", type=int, default=64)
    ap.add_argument("--texels", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    w, h, nsph, depth = wm.CONFIGS[a.config]
    S = wm.scene_arrays(nsph)
    B = bm.scene_bvh(nsph)
    lists = build_lists(S, a.texels)
    sizes = np.array([len(p[0]) for per in lists for p in per])
    rng = np.random.default_rng(a.seed)
    wm.links.clear()
    n_pix, pix, lev, hitl, cr, ct = wm.build_trees(S, w, h, depth, a.tiles, rng, adjacent=4)
    ro, rd = wm.build_trees.rays
    src = wm.build_trees.src
    tot = dict(calls=0, rays=0, sphere_rays=0, bvh_iters=0, bvh_passes=0, mix_iters=0, mix_passes=0,
               list_passes=0, list_tests=0, met_sizes=[])
    for t in range(a.tiles):
        orders = []
        for r in range(t * 64, (t + 1) * 64):
            od = []
            wm.lane_events(r, cr, ct, od)
            orders.append(od)
        for k in range(1, max(len(x) for x in orders)):
            lanes = [x[k] for x in orders if k < len(x)]
            if not lanes:
                continue
            tot["calls"] += 1
            tot["rays"] += len(lanes)
            rays = [(ro[nd], rd[nd]) for nd in lanes]
            tb = [bm.box_exit(S, ro[nd], rd[nd]) for nd in lanes]
            it, ps, _, _ = bm.lane_walk(B, rays, tb)
            tot["bvh_iters"] += it
            tot["bvh_passes"] += ps
            tex = [texel_of(rd[nd], a.texels) if src[nd] >= 0 else -1 for nd in lanes]
            box_lanes = [i for i, nd in enumerate(lanes) if tex[i] < 0]
            sph_lanes = [i for i, nd in enumerate(lanes) if tex[i] >= 0]
            tot["sphere_rays"] += len(sph_lanes)
            if box_lanes:
                it2, ps2, _, _ = bm.lane_walk(B, [rays[i] for i in box_lanes], [tb[i] for i in box_lanes])
                tot["mix_iters"] += it2
                tot["mix_passes"] += ps2
            longest = 0
            for i in sph_lanes:
                nd = lanes[i]
                per = lists[int(src[nd])][tex[i]]
                tot["met_sizes"].append(len(per[0]))
                n_t, _ = list_walk(S, per, ro[nd], rd[nd], tb[i])
                tot["list_tests"] += n_t
                longest = max(longest, n_t)
            tot["list_passes"] += longest
            for name, K, checks, q in KRECORDS:
                r = tot.setdefault(name, dict(passes=0, iters=0, sp=0, fallback=0))
                longest, fb = 0, []
                for i in sph_lanes:
                    nd = lanes[i]
                    n_t, f = list_walk_k(S, lists[int(src[nd])][tex[i]], ro[nd], rd[nd], tb[i], K, checks, q)
                    longest = max(longest, n_t)
                    if f:
                        fb.append(i)
                r["passes"] += longest
                r["fallback"] += len(fb)
                bl = box_lanes + fb
                if bl:
                    it3, ps3, _, _ = bm.lane_walk(B, [rays[i] for i in bl], [tb[i] for i in bl])
                    r["iters"] += it3
                    r["sp"] += ps3
            # fixed records: K slots, a stored bound every `shell` candidates
            for K, sh in RECORDS:
                key = "rec%d_s%d" % (K, sh)
                r = tot.setdefault(key, dict(passes=0, iters=0, sp=0, fallback=0))
                longest, fb = 0, []
                for i in sph_lanes:
                    nd = lanes[i]
                    n_t, f = list_walk(S, lists[int(src[nd])][tex[i]], ro[nd], rd[nd], tb[i], K, sh)
                    longest = max(longest, n_t)
                    if f:
                        fb.append(i)
                r["passes"] += longest
                r["fallback"] += len(fb)
                bl = box_lanes + fb
                if bl:
                    it3, ps3, _, _ = bm.lane_walk(B, [rays[i] for i in bl], [tb[i] for i in bl])
                    r["iters"] += it3
                    r["sp"] += ps3
    c = tot["calls"]
    met = np.array(tot["met_sizes"])
    out = {"config": a.config, "tiles": a.tiles, "texels_per_face": a.texels, "wave_calls": c,
           "secondary_rays": tot["rays"], "sphere_origin_share": round(tot["sphere_rays"] / tot["rays"], 3),
           "list_sizes": {"mean": round(float(sizes.mean()), 2), "p99": int(np.percentile(sizes, 99)),
                          "max": int(sizes.max()), "met_by_rays_mean": round(float(met.mean()), 2),
                          "met_by_rays_p90": int(np.percentile(met, 90)),
                          "table_bytes_at_1B_per_slot": int(sizes.sum())},
           "per_wave_call": {
               "bvh_today": {"node_iters": round(tot["bvh_iters"] / c, 2), "sphere_passes": round(tot["bvh_passes"] / c, 2)},
               "lists": {"list_passes": round(tot["list_passes"] / c, 2),
                         "list_tests_per_sphere_ray": round(tot["list_tests"] / max(1, tot["sphere_rays"]), 2),
                         "bvh_node_iters_box_lanes": round(tot["mix_iters"] / c, 2),
                         "bvh_sphere_passes_box_lanes": round(tot["mix_passes"] / c, 2)}}}
    for K, sh in RECORDS:
        r = tot["rec%d_s%d" % (K, sh)]
        out["per_wave_call"]["record_%d_slots_bound_every_%d" % (K, sh)] = {
            "list_passes": round(r["passes"] / c, 2), "bvh_node_iters": round(r["iters"] / c, 2),
            "bvh_sphere_passes": round(r["sp"] / c, 2),
            "fallback_share_of_sphere_rays": round(r["fallback"] / max(1, tot["sphere_rays"]), 4)}
    for name, K, checks, q in KRECORDS:
        r = tot[name]
        out["per_wave_call"][name] = {
            "list_passes": round(r["passes"] / c, 2), "bvh_node_iters": round(r["iters"] / c, 2),
            "bvh_sphere_passes": round(r["sp"] / c, 2),
            "fallback_share_of_sphere_rays": round(r["fallback"] / max(1, tot["sphere_rays"]), 4)}
    bt = out["per_wave_call"]["bvh_today"]
    out["units_per_wave_call"] = {"bvh_today": round(bt["node_iters"] + bt["sphere_passes"], 2)}
    for k, v in out["per_wave_call"].items():
        if k.startswith(("record", "product", "variant")):
            out["units_per_wave_call"][k] = round(v["list_passes"] + v["bvh_node_iters"] + v["bvh_sphere_passes"], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
