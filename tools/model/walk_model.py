"""CPU model of the recursive walk's frame traffic, per 64-lane wave (development probe).

    python tools/model/walk_model.py [--config config4] [--tiles 256] [--seed 1]

The walk (rt_kernel.hip trace_tree<D>) traces ONE ray per lane per loop
iteration, every lane at its own place in its own pixel's ray tree
(raytrace_compute.glsl:848-1105: reflection subtree, then refraction
subtree, then mix(mix(phong, R, rho), T, tau)). Its per-level frames live in
scratch; a push is a 40-B frame store, a return folds the finished value into
the ancestors with one 40-B frame load per level it climbs (and a store when
it turns to a pending refraction child). In SIMT these cost the wave a round
whenever ANY lane does one, the fold loop as many rounds as the lane that
climbs furthest.

This model traces the tree of every pixel of a seeded sample of 8x8 wave
tiles of the config's frame in float64 numpy (the same scene, camera, hit
rules, reflect / refract and offsets as the shader; statistics only, not a
parity tool — it never touches oracle/), then replays each wave's walk
iteration by iteration under two frame schemes:

  exact   — the current walk: colour + pending refraction ray + flags per
            level, mixed bottom-up (bit-exact).
  linear  — forward weights: the pixel colour is accumulated as
            sum(weight * phong) down the tree, the weight of a child being its
            parent's times rho (reflection; times (1 - tau) if a refraction
            child also exists) or tau (refraction), the parent's phong
            weighted by (1 - rho)(1 - tau) over its spawned children. Only a
            node with BOTH children stores anything: its pending refraction
            ray and weight (28 B); a lane whose subtree ends pops one record
            (or finishes). Not bit-exact (a different rounding order).

Prints per scheme: wave iterations, store rounds, load rounds and bytes per
wave tile, so a calibrated cost per round (from an ablation build that keeps
no frames) predicts the time of each scheme.

Outcome (round 4): config 4 exact 29.9 frame rounds / 901 B per pixel,
linear 10.1 / 193; calibrated on the r02l no-frames ablation (-31 %), the
linear walk was predicted at about -20 %. Built (RT_PRECISION_FAST, within
4.8e-7 of every GL fixture) and measured EVEN: config 4 14.67 vs 14.69 ms,
config 3 0.873 vs 0.895 ms (profiles/r04b_ab_fast_tier_config34.log). The
frame rounds are not on the critical path; the ablation's gain came from the
different (wrong) rays it traced. The variant was removed from the product.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import openglraytracer_amd as rt  # noqa: E402  (host-side scene / camera helpers only)

CONFIGS = {"config2": (1920, 1080, 16, 0), "config3": (3840, 2160, 64, 2), "config4": (7680, 4320, 256, 4)}


def scene_arrays(n_spheres):
    objs = rt.bench_objects(n_spheres, 0)
    mats = rt.reference_materials()
    rho = np.array([m.reflectivity for m in mats])
    tau = np.array([m.transparency for m in mats])
    ior = np.array([m.refraction_index for m in mats])
    box = objs[0]
    sph = objs[1:]
    c = np.array([[o.position[0], o.position[1], o.position[2]] for o in sph], np.float64)
    r = np.array([o.radius for o in sph], np.float64)
    mat = np.array([o.material for o in sph])
    return dict(bmin=np.array(box.box_mins[:], np.float64), bmax=np.array(box.box_maxs[:], np.float64),
                bmat=box.material, c=c, r=r, mat=mat, rho=rho, tau=tau, ior=ior)


def camera_rays(w, h, xs, ys):
    v = rt.make_view(None, 0.0)
    M = np.array(v.unprojection[:], np.float64).reshape(4, 4)  # column-major: M[col][row]
    hw, hh = w // 2, h // 2
    vx = (xs - hw) / hw
    vy = (ys - hh) / hh

    def unproj(z):
        p = np.outer(vx, M[0]) + np.outer(vy, M[1]) + z * M[2] + M[3]
        return p[:, :3] / p[:, 3:4]
    d = unproj(1.0) - unproj(0.5)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(np.array(v.origin[:], np.float64), d.shape).copy()
    return o, d


def trace(S, o, d):
    """closest hit of rays (o, d): object (-1 box, >= 0 sphere, -2 none), t,
    point, normal (against the ray), inside flag, material."""
    n = len(o)
    # spheres (:583-640)
    oc = o[:, None, :] - S["c"][None, :, :]
    b = np.einsum("nk,nsk->ns", d, oc)
    qc = np.einsum("nsk,nsk->ns", oc, oc) - S["r"][None, :] ** 2
    disc = b * b - qc
    sq = np.sqrt(np.maximum(disc, 0.0))
    t1, t2 = -b - sq, -b + sq
    ts = np.where(t1 > 0, t1, np.where(t2 > 0, t2, np.inf))
    ts = np.where(disc >= 0, ts, np.inf)
    k = np.argmin(ts, axis=1)
    tsph = ts[np.arange(n), k]
    # the room box (:647-724), axis-aligned at the origin
    with np.errstate(divide="ignore", invalid="ignore"):
        ta = (S["bmin"][None] - o) / d
        tb = (S["bmax"][None] - o) / d
    tn = np.max(np.minimum(ta, tb), axis=1)
    tf = np.min(np.maximum(ta, tb), axis=1)
    tbox = np.where((tn < tf) & (tf > 0), np.where(tn < 0, tf, tn), np.inf)
    use_box = tbox < tsph
    t = np.where(use_box, tbox, tsph)
    hit = np.isfinite(t)
    p = o + d * np.where(hit, t, 0.0)[:, None]
    # normals
    ns = p - S["c"][k]
    ns /= np.linalg.norm(ns, axis=1, keepdims=True)
    inside_s = (t1[np.arange(n), k] <= 0)
    ns = np.where(inside_s[:, None], -ns, ns)
    # box: the face whose slab distance equals t, normal against the ray
    tsel = np.where(tn < 0, tf, tn)
    slab = np.where((tn < 0)[:, None], np.maximum(ta, tb), np.minimum(ta, tb))
    face = np.argmin(np.abs(slab - tsel[:, None]), axis=1)
    nb = np.zeros_like(p)
    nb[np.arange(n), face] = -np.sign(d[np.arange(n), face])
    nrm = np.where(use_box[:, None], nb, ns)
    inside = np.where(use_box, tn < 0, inside_s)
    mat = np.where(use_box, S["bmat"], S["mat"][k])
    trace.obj = np.where(hit, np.where(use_box, -1, k), -2)  # hit object: -1 the box, >= 0 a sphere, -2 none
    return hit, p, nrm, inside, mat


def refract(i, n, eta):
    dd = np.sum(n * i, axis=1)
    kk = 1.0 - eta * eta * (1.0 - dd * dd)
    r = eta[:, None] * i - (eta * dd + np.sqrt(np.maximum(kk, 0.0)))[:, None] * n
    return np.where((kk < 0)[:, None], 0.0, r)


def build_trees(S, w, h, depth, tiles, rng, adjacent=1):
    """Every pixel's ray tree, level by level. Returns per-node arrays:
    pixel, level, hit, spawned reflection / refraction child node ids.
    adjacent > 1: the tiles come in runs of that many horizontally adjacent
    wave tiles (the four waves of a queued work-group start on adjacent tiles)."""
    wtx, wty = w // 8, h // 8
    if adjacent > 1:
        runs = rng.choice(wtx // adjacent * wty, size=tiles // adjacent, replace=False)
        start = (runs // (wtx // adjacent)) * wtx + (runs % (wtx // adjacent)) * adjacent
        pick = (start[:, None] + np.arange(adjacent)[None, :]).reshape(-1)
    else:
        pick = rng.choice(wtx * wty, size=tiles, replace=False)
    lane = np.arange(64)
    xs = ((pick % wtx)[:, None] * 8 + lane % 8).reshape(-1).astype(np.float64)
    ys = ((pick // wtx)[:, None] * 8 + lane // 8).reshape(-1).astype(np.float64)
    o, d = camera_rays(w, h, xs, ys)
    n_pix = len(xs)
    pix, lev, hitl, cr, ct, ro, rd, src = [], [], [], [], [], [], [], []
    cur = dict(o=o, d=d, pix=np.arange(n_pix), parent=-np.ones(n_pix, int), kind=np.zeros(n_pix, int),
               src=np.full(n_pix, -3))
    base = 0
    for level in range(depth + 1):
        m = len(cur["o"])
        if m == 0:
            break
        hit, p, nrm, inside, mat = trace(S, cur["o"], cur["d"])
        ids = base + np.arange(m)
        pix.append(cur["pix"])
        src.append(cur["src"])
        ro.append(cur["o"])
        rd.append(cur["d"])
        lev.append(np.full(m, level))
        hitl.append(hit)
        cr.append(-np.ones(m, int))
        ct.append(-np.ones(m, int))
        # link to parents
        for kind, arr in ((0, cr), (1, ct)):
            sel = (cur["parent"] >= 0) & (cur["kind"] == kind)
            if sel.any():
                par = cur["parent"][sel]
                # parents are in earlier levels: write through the flat view later
                links.append((kind, par, ids[sel]))
        base += m
        if level == depth:
            break
        sr = hit & (S["rho"][mat] > 0)
        st = hit & (S["tau"][mat] > 0)
        dref = cur["d"] - 2.0 * np.sum(nrm * cur["d"], axis=1)[:, None] * nrm
        eta = np.where(inside, S["ior"][mat], 1.0 / S["ior"][mat])
        dtr = refract(cur["d"], nrm, eta)
        o2 = np.concatenate([(p + 0.001 * nrm)[sr], (p - 0.001 * nrm)[st]])
        d2 = np.concatenate([dref[sr], dtr[st]])
        obj = trace.obj
        cur = dict(o=o2, d=d2, pix=np.concatenate([cur["pix"][sr], cur["pix"][st]]),
                   parent=np.concatenate([ids[sr], ids[st]]),
                   kind=np.concatenate([np.zeros(sr.sum(), int), np.ones(st.sum(), int)]),
                   src=np.concatenate([obj[sr], obj[st]]))
    pix, lev, hitl = np.concatenate(pix), np.concatenate(lev), np.concatenate(hitl)
    cr, ct = np.concatenate(cr), np.concatenate(ct)
    for kind, par, child in links:
        (cr if kind == 0 else ct)[par] = child
    build_trees.rays = (np.concatenate(ro), np.concatenate(rd))
    build_trees.src = np.concatenate(src)  # the object a ray starts on (-3: camera ray, -1: the box, >= 0: sphere)
    return n_pix, pix, lev, hitl, cr, ct


links = []


def lane_events(root, cr, ct, order=None):
    """The walk of one pixel, one entry per loop iteration (one traced ray):
    (exact stores, exact loads, linear stores, linear loads); `order`
    (a list) receives the node traced at each iteration."""
    ev = []
    # exact walk: explicit stack of (node, state) as trace_tree does
    stack = []  # frames: node ids with flag: waiting for R (2) or T (4)
    node = root
    lin_pending = 0
    while True:
        if order is not None:
            order.append(node)
        kids_r, kids_t = cr[node], ct[node]
        es = el = ls = ll = 0
        if kids_r >= 0 or kids_t >= 0:
            es += 1  # push (40 B)
            if kids_r >= 0 and kids_t >= 0:
                ls += 1  # linear: the pending refraction ray (28 B)
                lin_pending += 1
            stack.append([node, 2 if kids_r >= 0 else 4])
            nxt = kids_r if kids_r >= 0 else kids_t
            ev.append((es, el, ls, ll))
            node = nxt
            continue
        # leaf: fold
        nxt = -1
        while stack and nxt < 0:
            el += 1
            fr = stack[-1]
            if fr[1] == 2 and ct[fr[0]] >= 0:
                fr[1] = 4
                es += 1
                nxt = ct[fr[0]]
            else:
                stack.pop()
        if nxt >= 0 or lin_pending:
            pass
        if nxt >= 0:
            ll += 1  # linear: pop the pending refraction ray
            lin_pending -= 1
        ev.append((es, el, ls, ll))
        if nxt < 0:
            return ev
        node = nxt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config4")
    ap.add_argument("--tiles", type=int, default=256)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    w, h, nsph, depth = CONFIGS[a.config]
    S = scene_arrays(nsph)
    rng = np.random.default_rng(a.seed)
    links.clear()
    n_pix, pix, lev, hitl, cr, ct = build_trees(S, w, h, depth, a.tiles, rng)
    roots = np.arange(n_pix)  # level-0 nodes come first, in pixel order
    tot = dict(iters=0, rays=0, ex_store_rounds=0, ex_load_rounds=0, lin_store_rounds=0, lin_load_rounds=0,
               ex_store_lanes=0, ex_load_lanes=0, lin_store_lanes=0, lin_load_lanes=0, both_children=0)
    tot["both_children"] = int(np.sum((cr >= 0) & (ct >= 0)))
    for t in range(a.tiles):
        evs = [lane_events(r, cr, ct) for r in roots[t * 64:(t + 1) * 64]]
        n_it = max(len(e) for e in evs)
        tot["iters"] += n_it
        tot["rays"] += sum(len(e) for e in evs)
        for i in range(n_it):
            row = [e[i] for e in evs if i < len(e)]
            es = [r[0] for r in row]
            el = [r[1] for r in row]
            ls = [r[2] for r in row]
            ll = [r[3] for r in row]
            tot["ex_store_rounds"] += max(es)
            tot["ex_load_rounds"] += max(el)
            tot["lin_store_rounds"] += max(ls)
            tot["lin_load_rounds"] += max(ll)
            tot["ex_store_lanes"] += sum(es)
            tot["ex_load_lanes"] += sum(el)
            tot["lin_store_lanes"] += sum(ls)
            tot["lin_load_lanes"] += sum(ll)
    per_tile = {k: round(v / a.tiles, 3) for k, v in tot.items()}
    per_tile["rays_per_pixel"] = round(tot["rays"] / (64 * a.tiles), 3)
    per_tile["lane_utilisation"] = round(tot["rays"] / (64 * tot["iters"]), 4)
    per_tile["ex_bytes_per_pixel"] = round(40 * (tot["ex_store_lanes"] + tot["ex_load_lanes"]) / (64 * a.tiles), 1)
    per_tile["lin_bytes_per_pixel"] = round(28 * (tot["lin_store_lanes"] + tot["lin_load_lanes"]) / (64 * a.tiles), 1)
    # split frames (round 6, RT_SPLIT_FRAMES): colour + flags (16 B) per push,
    # fold load and re-store; the pending refraction ray (24 B) stored only by
    # a node with both children and loaded when its refraction child starts
    # (the linear scheme's pending-ray counts)
    per_tile["split_bytes_per_pixel"] = round((16 * (tot["ex_store_lanes"] + tot["ex_load_lanes"]) +
                                               24 * (tot["lin_store_lanes"] + tot["lin_load_lanes"])) / (64 * a.tiles), 1)
    per_tile["ex_store_bytes_per_pixel"] = round(40 * tot["ex_store_lanes"] / (64 * a.tiles), 1)
    per_tile["split_store_bytes_per_pixel"] = round((16 * tot["ex_store_lanes"] + 24 * tot["lin_store_lanes"]) /
                                                    (64 * a.tiles), 1)
    print(json.dumps({"config": a.config, "tiles": a.tiles, "per_wave_tile": per_tile}))


if __name__ == "__main__":
    main()
