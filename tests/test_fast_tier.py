"""The tolerance tier (RT_OPT_PRECISION = RT_PRECISION_FAST) on the MI355X.

north_star's bar is "per-channel output matches the reference GL render
within 1e-5 float tolerance". The exact tier (the default) meets it with
zero difference; the fast tier accumulates the recursion's colours forward
(rt_kernel.hip trace_tree_linear: weight x phong summed down the ray tree
instead of the nested mix() of raytrace_compute.glsl:1034-1054 on the way
back up) and must stay within it. Criterion, per channel of every pixel:

    |fast - reference| <= 1e-5 * max(1, |reference|)

(absolute 1e-5 for the reference scenes' colours, which are below 1 almost
everywhere; relative above 1, where float32 itself has a spacing of 1.2e-7
and more). The rays are the exact tier's, bit for bit, so the only
difference is the rounding of the colour sums; depth-0 renders have no
recursion and stay bit-identical. Every test prints the per-channel
statistics the criterion is judged on (mean, p99, max |d|, pixels beyond
1e-5, and the GL_RGBA8 bytes that change).
"""
import numpy as np
import pytest
import torch

import openglraytracer_amd as rt
from conftest import dev_zeros, fixture_objects, load_fixture, load_strat, manifest, row_bands, strat_manifest
from oracle import port, scenes

pytestmark = pytest.mark.gpu
MAN = manifest()
STRAT = strat_manifest()
TOL = 1e-5


@pytest.fixture(scope="module")
def fast_ctx():
    ctx = rt.Context(0)
    ctx.set_precision(rt.abi.RT_PRECISION_FAST)
    yield ctx
    ctx.close()


def tier_stats(got, ref):
    """Per-channel statistics of got vs ref (RGB), the criterion's excess,
    and the GL_RGBA8 bytes that differ (rt_pack_rgba8 of both)."""
    g = got[..., :3].astype(np.float64)
    r = ref[..., :3].astype(np.float64)
    nan = np.isnan(g) | np.isnan(r)
    assert np.array_equal(np.isnan(g), np.isnan(r)), "NaN pixels differ"
    d = np.where(nan, 0.0, np.abs(g - r))
    scale = np.maximum(1.0, np.where(nan, 0.0, np.abs(r)))
    def rgba(x):  # (the GL fixtures hold RGB only; the alpha the shader stores is 0)
        x = np.nan_to_num(x[..., :3].astype(np.float32), nan=0.0)
        return rt.pack_rgba8(np.concatenate([x, np.zeros(x.shape[:-1] + (1,), np.float32)], -1))
    rgba_g, rgba_r = rgba(got), rgba(ref)
    return {"max": float(d.max(initial=0.0)), "mean": float(d.mean()) if d.size else 0.0,
            "p99": float(np.percentile(d, 99)) if d.size else 0.0,
            "px_gt_1e5": int((d.max(-1) > TOL).sum()), "worst_ratio": float((d / (TOL * scale)).max(initial=0.0)),
            "exact_frac": float((d.max(-1) == 0).mean()) if d.size else 1.0,
            "rgba8_bytes_changed": int((rgba_g != rgba_r).sum()), "n_px": int(d.shape[0] * d.shape[1])}


def within(s):
    return s["worst_ratio"] <= 1.0


def product_render(ctx, objs, m, rows):
    """rt_render(cam = NULL, time) of rows [r0, r1) (the drop-in call)."""
    r0, r1 = rows
    sc = rt.Scene(ctx, objs)
    try:
        out = np.zeros((r1 - r0, m["width"], 4), np.float32)
        rc = rt.lib().rt_render(ctx.handle, sc.handle, None, m["time"], m["width"], m["height"], m["max_depth"],
                                r0, r1, out.ctypes.data, 0, None)
        assert rc == 0, rt.lib().rt_last_error()
    finally:
        sc.close()
    return out


@pytest.mark.parametrize("name", sorted(n for n, m in MAN.items() if m["probe"] == 0))
def test_fast_tier_every_gl_fixture_within_tolerance(fast_ctx, name):
    """Every colour fixture (configs 1-4 incl. the 4K / 8K depth-2 / depth-4
    crops, animated times, the shipped scene with its rotated boxes) through
    the product path in the fast tier, against the reference's own GL
    render; depth-0 fixtures bit-identical."""
    m = MAN[name]
    rgb, _ = load_fixture(name)
    x0, y0, w, h = m["crop"]
    objs = fixture_objects(m, rt.reference_objects)
    g = product_render(fast_ctx, objs, m, (y0, y0 + h))[:, x0:x0 + w]
    assert (g[..., 3] == 0).all()
    s = tier_stats(g, rgb)
    print(name, "depth", m["max_depth"], s)
    assert within(s), (name, s)
    if m["max_depth"] == 0:
        assert s["exact_frac"] == 1.0, (name, s)


@pytest.mark.parametrize("name", sorted(STRAT))
def test_fast_tier_stratified_deep_crops_within_tolerance(fast_ctx, name):
    """The stratified llvmpipe crops of configs 3 and 4 (edges, corners and
    the most glass-heavy regions of the 4K depth-2 and 8K depth-4 frames)."""
    m = STRAT[name]
    rgb, crops, _ = load_strat(name)
    objs = scenes.CONFIGS[m["scene"]][0]()
    bands = {rows: product_render(fast_ctx, objs, m, rows) for rows in row_bands(crops)}
    worst = None
    for k, (x0, y0, cw, ch) in enumerate(crops):
        g = bands[(int(y0), int(y0 + ch))][:, x0:x0 + cw]
        s = tier_stats(g, rgb[k])
        assert within(s), (name, k, s)
        worst = s if worst is None or s["max"] > worst["max"] else worst
    print(name, "worst crop", worst)


@pytest.mark.parametrize("cfg,bands", [("config3", [(0, 16), (1072, 1088), (2144, 2160)]),
                                       ("config4", [(0, 8), (2152, 2168), (4312, 4320)])])
def test_fast_tier_full_size_bands_against_exact_and_oracle(gpu_ctx, fast_ctx, cfg, bands):
    """Bands of the full-size config-3 / config-4 frames: fast tier vs the
    exact tier (which is bit-identical to the oracle) and vs the oracle."""
    build, w, h, depth = scenes.CONFIGS[cfg]
    objs = build()
    view = rt.make_view(None, 0.0)
    se, sf = rt.Scene(gpu_ctx, objs), rt.Scene(fast_ctx, objs)
    try:
        for rows in bands:
            e = rt.render(gpu_ctx, se, w, h, depth, view=view, rows=rows)
            f = rt.render(fast_ctx, sf, w, h, depth, view=view, rows=rows)
            s = tier_stats(f, e)
            print(cfg, rows, s)
            assert within(s), (cfg, rows, s)
            o = port.render(objs, w, h, depth, 0.0, rows=rows)
            assert np.array_equal(e, o)
    finally:
        se.close()
        sf.close()


@pytest.mark.parametrize("seed", range(24))
def test_fast_tier_random_scenes_within_tolerance(fast_ctx, seed):
    """Seeded random scenes (test_gpu_parity.random_scene: random materials
    incl. glass of random index and emissive ones, 1-4 random lights, 0-300
    spheres, rotated boxes, depth 0-5) against the oracle; depth 0 exact."""
    from test_gpu_parity import random_scene
    objs, mats, lights, t, depth, w, h = random_scene(seed)
    view = rt.make_view(None, t)
    sc = rt.Scene(fast_ctx, objs, materials=mats, lights=lights)
    try:
        g = rt.render(fast_ctx, sc, w, h, depth, view=view)
    finally:
        sc.close()
    o = port.render(objs, w, h, depth, t, materials=mats, lights=lights)
    s = tier_stats(g, o)
    print(seed, "depth", depth, s)
    assert within(s), (seed, depth, s)
    if depth == 0:
        assert np.array_equal(g, o, equal_nan=True)


def test_fast_tier_launch_shapes_agree(fast_ctx):
    """The fast tier is deterministic across launch shapes: a batch of views,
    interleaved row shards and the queued whole frame give the same bits as
    single renders (config-3 scene, depth 3)."""
    from openglraytracer_amd import frame
    objs = scenes.bench_objects(64)
    w, h, depth = 640, 360, 3
    views = [rt.make_view(None, k / 60.0) for k in range(3)]
    sc = rt.Scene(fast_ctx, objs)
    try:
        singles = [rt.render(fast_ctx, sc, w, h, depth, view=v) for v in views]
        batch = dev_zeros((3, h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch(fast_ctx, sc, batch.data_ptr(), w, h, depth, views)
        torch.cuda.synchronize()
        for k in range(3):
            assert np.array_equal(batch[k].cpu().numpy(), singles[k])
        got = np.zeros_like(singles[0])
        for s in range(3):
            buf = dev_zeros(rt.shard_rows(h, 8, 3, s) * w * 4, dtype=torch.float32, device="cuda")
            rt.render_shard(fast_ctx, sc, buf.data_ptr(), w, h, depth, 8, 3, s, view=views[0])
            torch.cuda.synchronize()
            got[frame.shard_row_ids(h, 8, 3, s)] = buf.cpu().numpy().reshape(-1, w, 4)
        assert np.array_equal(got, singles[0])
    finally:
        sc.close()


def test_precision_option_is_checked():
    ctx = rt.Context(0)
    try:
        with pytest.raises(rt.RTError) as e:
            ctx.set_precision(7)
        assert e.value.code == rt.abi.RT_ERR_INVALID
        ctx.set_precision(rt.abi.RT_PRECISION_EXACT)
    finally:
        ctx.close()
