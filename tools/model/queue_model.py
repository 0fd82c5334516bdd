"""CPU model of the queued work distribution's tail (development probe).

    python tools/model/queue_model.py [--config config3] [--stride 1]

Deep frames (depth >= 2) run as a grid of resident work-groups whose waves
take 8x8 wave tiles from 32 queues (rt_kernel.hip render_kernel, queued):
tile t belongs to queue t % 32, global wave g to queue g % 32; a queue's
waves first take its items g / 32, then the queue's atomic head. A wave's
cost per tile is its walk's iteration count (trace_tree runs until the
lane with the most rays is done; config 3/4 are VALU-bound, so an iteration
costs about the same everywhere). This model computes every tile's
iteration count from walk_model's float64 restatement of the shader (all
tiles, or every `stride`-th tile row), then replays the queues on the
6 x 1024 resident wave slots: the makespan against perfect packing, for
the kernel's order and for longest-first (what a per-tile cost oracle could
reach). The gap is the tail a better order or work stealing could recover.
"""
import argparse
import heapq
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import walk_model as wm  # noqa: E402

KQ = 32
SLOTS = 6 * 1024  # resident waves at 6 waves per SIMD, 1024 SIMDs


def tile_iters(S, w, h, depth, tiles):
    """walk iterations (max rays over the tile's 64 lanes) of the given tiles"""
    wtx = w // 8
    lane = np.arange(64)
    xs = ((tiles % wtx)[:, None] * 8 + lane % 8).reshape(-1).astype(np.float64)
    ys = ((tiles // wtx)[:, None] * 8 + lane // 8).reshape(-1).astype(np.float64)
    o, d = wm.camera_rays(w, h, xs, ys)
    # rays per pixel: breadth-first over the levels (a missed ray ends its branch)
    count = np.ones(len(xs), np.int64)
    cur_o, cur_d, owner = o, d, np.arange(len(xs))
    for level in range(depth):
        hit, p, nrm, inside, mat = wm.trace(S, cur_o, cur_d)
        sr = hit & (S["rho"][mat] > 0)
        st = hit & (S["tau"][mat] > 0)
        dref = cur_d - 2.0 * np.sum(nrm * cur_d, axis=1)[:, None] * nrm
        eta = np.where(inside, S["ior"][mat], 1.0 / S["ior"][mat])
        dtr = wm.refract(cur_d, nrm, eta)
        cur_o = np.concatenate([(p + 0.001 * nrm)[sr], (p - 0.001 * nrm)[st]])
        cur_d = np.concatenate([dref[sr], dtr[st]])
        owner = np.concatenate([owner[sr], owner[st]])
        np.add.at(count, owner, 1)
    return count.reshape(-1, 64).max(1)


def replay(order_per_queue, cost):
    """makespan of the queued schedule: queue q's waves take its items in
    order_per_queue[q]; every wave slot is one resident wave of the grid"""
    heap = []
    waves = [[g for g in range(SLOTS) if g % KQ == q] for q in range(KQ)]
    for q in range(KQ):
        items = list(order_per_queue[q])
        # static first items, then the head (modelled as: whichever wave of
        # the queue frees first takes the next item)
        free = [(0.0, g) for g in waves[q]]
        heapq.heapify(free)
        for it in items:
            t, g = heapq.heappop(free)
            heapq.heappush(free, (t + cost[it], g))
        heap.append(max(t for t, _ in free))
    return max(heap)


def replay_pool(items, cost):
    """makespan when every wave takes the next item of one shared order (the
    queues with work stealing, at the end)"""
    free = [0.0] * SLOTS
    heapq.heapify(free)
    for it in items:
        t = heapq.heappop(free)
        heapq.heappush(free, t + cost[it])
    return max(free)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--stride", type=int, default=1, help="model every stride-th tile row (scaled)")
    ap.add_argument("--views", type=int, default=1, help="views per launch (the frame's costs repeated)")
    a = ap.parse_args()
    w, h, nsph, depth = wm.CONFIGS[a.config]
    S = wm.scene_arrays(nsph)
    wtx, wty = w // 8, h // 8
    rows = np.arange(0, wty, a.stride)
    tiles = (rows[:, None] * wtx + np.arange(wtx)).reshape(-1)
    cost = np.zeros(wtx * wty)
    for i in range(0, len(tiles), 4096):
        cost[tiles[i:i + 4096]] = tile_iters(S, w, h, depth, tiles[i:i + 4096])
    if a.stride > 1:  # fill the skipped rows with the modelled ones (same distribution)
        for r in range(wty):
            if r % a.stride:
                cost[r * wtx:(r + 1) * wtx] = cost[(r - r % a.stride) * wtx:(r - r % a.stride + 1) * wtx]
    cost = np.tile(cost, a.views)
    total = len(cost)
    ideal = cost.sum() / SLOTS
    kernel = replay([range(q, total, KQ) for q in range(KQ)], cost)
    lpt = replay([sorted(range(q, total, KQ), key=lambda t: -cost[t]) for q in range(KQ)], cost)
    steal = replay_pool(range(total), cost)
    print(json.dumps({"config": a.config, "tiles": total, "mean_iters": round(float(cost.mean()), 3),
                      "p99_iters": float(np.percentile(cost, 99)), "max_iters": float(cost.max()),
                      "makespan_over_ideal": {"kernel_order": round(kernel / ideal, 4),
                                              "longest_first_per_queue": round(lpt / ideal, 4),
                                              "one_pool (stealing)": round(steal / ideal, 4)},
                      "views": a.views,
                      "queue_totals_spread": round(float(np.std([cost[q::KQ].sum() for q in range(KQ)]) /
                                                         np.mean([cost[q::KQ].sum() for q in range(KQ)])), 5)}))


if __name__ == "__main__":
    main()
