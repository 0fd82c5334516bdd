"""CPU model of the wide-mask shadow queries' candidate passes per wave (development probe).

    python tools/model/shadow_model.py [--config config4] [--tiles 64] [--seed 1]

Scenes of 33-256 spheres answer a shadow query (rt_kernel.hip occluded_impl,
raytrace_compute.glsl:807-819) by walking the candidate list of the lane's
direction texel from the light (one 16-B record per live light and texel:
count + up to 15 sphere slots, rt_scene.cpp); the walk is any-hit, so a lane
leaves at its first occluder, and the wave loops as many passes as its
slowest lane needs. Ordering a texel's candidates by the sphere's angular
size from the light, largest first, lets a shadowed lane meet its occluder
earlier (the result cannot change: any-hit is order-independent).

Results (round 4): with the lists in ascending slot order, 2.34 passes per
wave call on config 4 (RT_STATS measured 2.5) and 0.95 on config 3; by
angular size 1.47 and 0.73 — built (rt_scene.cpp), measured config 4
14.73 -> 14.00 ms, config 3 0.874 -> 0.861 ms, frames unchanged
(profiles/r04d_ab_candidate_order.log). A texel-specific order (the cone
covering the texel's centre most deeply first) reaches 1.36 / 0.70: about a
further 0.7 % by the same ratio, below the 3 % bar; not built. "as_stored"
below is whatever order the product's lists now hold.

The model takes the product's own lists (rt_debug_scene_blob), the config's
rays from walk_model.py grouped per wave and walk iteration as trace_tree
runs them, casts every hit's shadow ray to each live light (when the light
is above the surface), finds each candidate's exact float64 segment hit and
counts the wave's passes for each order.
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

rt = wm.rt
NT = 64  # kGMaskTexels


def scene_lists(n_spheres):
    import ctypes as C
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
    off_sph, off_dmask, dmask_n, dmask_bytes, off_glist, ns = meta[1], meta[11], meta[12], meta[13], meta[16], meta[17]
    sph = buf.view(np.float32).reshape(-1, 4)[off_sph:off_sph + ns].astype(np.float64)
    live = [j for j, lt in enumerate(lights) if any(lt.diffuse[k] or lt.specular[k] for k in range(4))]
    lpos = [np.array(lights[j].position[:], np.float64) for j in live]
    if off_glist < 0:
        # LDS direction masks (<= 64 spheres, the depth-0/1 path): one mask
        # word per (live light, texel), dmask_n texels per face edge; the
        # kernel walks the set bits in ascending slot order. As lists:
        per = 6 * dmask_n * dmask_n
        raw = buf[off_dmask * 16:off_dmask * 16 + len(live) * per * dmask_bytes]
        words = raw.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[int(dmask_bytes)]).reshape(len(live), per)
        glist = np.zeros((len(live), per, 65), np.int32)
        for j in range(len(live)):
            for t in range(per):
                bits = [q for q in range(ns) if (int(words[j, t]) >> q) & 1]
                glist[j, t, 0] = len(bits)
                glist[j, t, 1:1 + len(bits)] = bits
        return sph, glist, lpos, int(dmask_n)
    per = 6 * NT * NT
    glist = buf[off_glist * 16:off_glist * 16 + len(live) * per * 16].reshape(len(live), per, 16)
    return sph, glist, lpos, NT


def cube_face(u):
    """The kernel's cube-map instructions (rt_kernel.hip direction_texel):
    face (+x, -x, +y, -y, +z, -z; z, then y wins a tie), sc, tc, |major|."""
    x, y, z = u
    if abs(z) >= abs(x) and abs(z) >= abs(y):
        return 4 + int(z < 0), (-x if z < 0 else x), -y, abs(z)
    if abs(y) >= abs(x):
        return 2 + int(y < 0), x, (-z if y < 0 else z), abs(y)
    return int(x < 0), (z if x < 0 else -z), -y, abs(x)


def face_dir(face, a, b):
    """Face `face`'s point (a, b) = (sc, tc) / |major| as a direction
    (rt_scene.cpp mask_cones)."""
    return [(1.0, -b, -a), (-1.0, -b, a), (a, 1.0, b), (a, -1.0, -b), (a, -b, 1.0), (-a, -b, -1.0)][face]


def texel(u, NT=NT):
    face, sc, tc, am = cube_face(u)
    if not (1e-20 < am < 1e30):
        return -1
    hh = 0.5 * NT / am
    col = min(max(int(np.floor(sc * hh + 0.5 * NT)), 0), NT - 1)
    row = min(max(int(np.floor(tc * hh + 0.5 * NT)), 0), NT - 1)
    return (face * NT + row) * NT + col


def texel_dir(t, NT=NT):
    """Unit direction of texel t's centre (the inverse of texel())."""
    face, rem = divmod(t, NT * NT)
    row, col = divmod(rem, NT)
    v = np.array(face_dir(face, (col + 0.5 - 0.5 * NT) / (0.5 * NT), (row + 0.5 - 0.5 * NT) / (0.5 * NT)))
    return v / np.linalg.norm(v)


def blocks(sph, s, start, d):
    c, rr = sph[s, :3], sph[s, 3]
    oc = start - c
    a = d @ d
    b = 2 * (d @ oc)
    cc = oc @ oc - rr
    disc = b * b - 4 * a * cc
    if disc < 0:
        return False
    sq = np.sqrt(disc)
    t1, t2 = (-b - sq) / (2 * a), (-b + sq) / (2 * a)
    t = t1 if t1 > 0 else t2
    return 0 < t < 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config4")
    ap.add_argument("--tiles", type=int, default=64)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    w, h, nsph, depth = wm.CONFIGS[a.config]
    S = wm.scene_arrays(nsph)
    sph, glist, lpos, nt = scene_lists(nsph)
    rng = np.random.default_rng(a.seed)
    wm.links.clear()
    n_pix, pix, lev, hitl, cr, ct = wm.build_trees(S, w, h, depth, a.tiles, rng)
    ro, rd = wm.build_trees.rays
    hit, p, nrm, inside, mat = wm.trace(S, ro, rd)
    tot = {"calls": 0, "queries": 0, "shadowed": 0, "passes_ascending": 0, "passes_by_size": 0, "tests_ascending": 0,
           "tests_by_size": 0, "overflow": 0, "passes_by_depth": 0, "tests_by_depth": 0}
    for t in range(a.tiles):
        orders = []
        for r in range(t * 64, (t + 1) * 64):
            od = []
            wm.lane_events(r, cr, ct, od)
            orders.append(od)
        for k in range(max(len(x) for x in orders)):
            nodes = [x[k] if k < len(x) and hitl[x[k]] else -1 for x in orders]
            for j, L in enumerate(lpos):
                lanes_a, lanes_b, lanes_c = [], [], []
                for nd in nodes:
                    if nd < 0:
                        continue
                    sdir = L - p[nd]
                    if sdir @ nrm[nd] <= 0:
                        continue
                    start = p[nd] + 0.01 * nrm[nd]
                    tx = texel(-sdir, nt)
                    rec = glist[j, tx]
                    cnt = int(rec[0])
                    if cnt == 255 and nt == NT:
                        tot["overflow"] += 1
                        continue
                    cand = [int(s) for s in rec[1:1 + cnt]]
                    size = [-(np.sqrt(sph[s, 3]) / max(np.linalg.norm(sph[s, :3] - L), 1e-9)) for s in cand]
                    by_size = [cand[i] for i in np.argsort(size, kind="stable")]
                    # the texel-specific order: the sphere whose cone (from
                    # the light) covers the texel's centre most deeply first
                    tdir = texel_dir(tx, nt)
                    depth_key = []
                    for s_ in cand:
                        v = sph[s_, :3] - L
                        dd = np.linalg.norm(v)
                        half = np.arcsin(min(1.0, (np.sqrt(sph[s_, 3]) + 0.021 + 1e-3 * dd) / dd))
                        depth_key.append(-(half - np.arccos(np.clip(v @ tdir / dd, -1, 1))))
                    by_depth = [cand[i] for i in np.argsort(depth_key, kind="stable")]
                    occ = {s for s in cand if blocks(sph, s, start, sdir)}
                    tot["queries"] += 1
                    tot["shadowed"] += bool(occ)

                    def passes(lst):
                        for i, s in enumerate(lst):
                            if s in occ:
                                return i + 1
                        return len(lst)
                    lanes_a.append(passes(cand))
                    lanes_b.append(passes(by_size))
                    lanes_c.append(passes(by_depth))
                if lanes_a:
                    tot["calls"] += 1
                    tot["passes_ascending"] += max(lanes_a)
                    tot["passes_by_size"] += max(lanes_b)
                    tot["tests_ascending"] += sum(lanes_a)
                    tot["tests_by_size"] += sum(lanes_b)
                    tot["passes_by_depth"] += max(lanes_c)
                    tot["tests_by_depth"] += sum(lanes_c)
    c, q = tot["calls"], tot["queries"]
    print(json.dumps({"config": a.config, "tiles": a.tiles, "wave_calls": c, "queries": q,
                      "shadowed_frac": round(tot["shadowed"] / q, 3), "overflow_queries": tot["overflow"],
                      "passes_per_call": {"as_stored": round(tot["passes_ascending"] / c, 3),
                                          "by_angular_size": round(tot["passes_by_size"] / c, 3),
                                          "by_texel_depth": round(tot["passes_by_depth"] / c, 3)},
                      "exact_tests_per_query": {"as_stored": round(tot["tests_ascending"] / q, 3),
                                                "by_angular_size": round(tot["tests_by_size"] / q, 3),
                                                "by_texel_depth": round(tot["tests_by_depth"] / q, 3)}}))


if __name__ == "__main__":
    main()
