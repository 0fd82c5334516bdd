"""GPU parity: the HIP kernel through the C-ABI against the oracle and the
reference's own renders (tests/golden). Run on the MI355X with -m gpu.

Bar (floating point, north_star tolerance 1e-5 per channel):
* with the same frame constants the kernel is BIT-EXACT against the oracle on
  every scene, and bit-exact against the reference GL render on every
  fixture — benchmark scenes and the shipped scene with its rotated,
  animated boxes (their transforms evaluated as llvmpipe evaluates them);
* full-size frames: bit-exact against the oracle on full rows / bands, plus
  size-independent properties (determinism, band == full frame, shards
  reassemble the frame, alpha 0, finite).
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

import openglraytracer_amd as rt
from conftest import dev_zeros, fixture_objects, load_fixture, manifest, parity_stats, synced_zero_
from openglraytracer_amd import frame
from oracle import port, scenes

pytestmark = pytest.mark.gpu
MAN = manifest()


def gpu_render(ctx, objs, w, h, depth, view, rows=None, **kw):
    sc = rt.Scene(ctx, objs, **kw)
    try:
        return rt.render(ctx, sc, w, h, depth, view=view, rows=rows)
    finally:
        sc.close()


def oracle_render(objs, w, h, depth, t=0.0, rows=None, unproj=None, **kw):
    if unproj is not None:
        port.lib().oracle_pin_unprojection(np.ascontiguousarray(unproj, np.float32).ctypes.data_as(C.c_void_p))
    try:
        return port.render(objs, w, h, depth, t, rows=rows, **kw)
    finally:
        port.lib().oracle_pin_unprojection(None)


@pytest.mark.parametrize("name", sorted(n for n, m in MAN.items() if m["probe"] == 0))
def test_fixture_pinned_view(gpu_ctx, name):
    m = MAN[name]
    rgb, unproj = load_fixture(name)
    x0, y0, w, h = m["crop"]
    objs = fixture_objects(m, rt.reference_objects)
    cam = rt.reference_camera(m["time"])
    view = rt.view_from_matrix(unproj, list(cam.position))
    rows = (y0, y0 + h)
    g = gpu_render(gpu_ctx, objs, m["width"], m["height"], m["max_depth"], view, rows)[:, x0:x0 + w]
    o = oracle_render(objs, m["width"], m["height"], m["max_depth"], m["time"], rows, unproj)[:, x0:x0 + w]
    assert np.array_equal(g, o), parity_stats(g, o)          # kernel == oracle, bitwise
    assert (g[..., 3] == 0).all()                             # imageStore(vec4(rgb, 0.0)), :404
    s = parity_stats(g, rgb)                                  # kernel vs the reference GL render
    assert s["exact"] == 1.0, s


@pytest.mark.parametrize("name", sorted(n for n, m in MAN.items() if m["probe"] == 0))
def test_fixture_own_view_matches_oracle(gpu_ctx, name):
    """Frame constants computed by the product (rt_make_view) — bitwise equal
    to the oracle's independent restatement."""
    m = MAN[name]
    x0, y0, w, h = m["crop"]
    objs = fixture_objects(m, rt.reference_objects)
    view = rt.make_view(None, m["time"])
    g = gpu_render(gpu_ctx, objs, m["width"], m["height"], m["max_depth"], view, (y0, y0 + h))
    o = oracle_render(objs, m["width"], m["height"], m["max_depth"], m["time"], (y0, y0 + h))
    assert np.array_equal(g, o), parity_stats(g, o)


@pytest.mark.parametrize("name", sorted(n for n, m in MAN.items() if m["probe"] == 0))
def test_product_camera_path_matches_gl(gpu_ctx, name):
    """rt_render(ctx, scene, cam = NULL, time, ...) — the C-ABI call the
    reference's draw() becomes (main.cpp:226-238) — with the product's own
    frame constants (rt_make_view: the orbit camera as the reference's GL
    evaluates it, raytrace_compute.glsl:334-392) against the reference's own
    render: bit-exact on every fixture — configs 1-4 incl. the 4K / 8K
    depth-2 / depth-4 crops, camera at t = 0 and moved, and the shipped scene
    at t = 0, 3.7 and 11.25 with its rotated, animated boxes."""
    m = MAN[name]
    rgb, _ = load_fixture(name)
    x0, y0, w, h = m["crop"]
    objs = fixture_objects(m, rt.reference_objects)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        out = np.zeros((h, m["width"], 4), np.float32)
        rc = rt.lib().rt_render(gpu_ctx.handle, sc.handle, None, m["time"], m["width"], m["height"], m["max_depth"],
                                y0, y0 + h, out.ctypes.data, 0, None)
        assert rc == 0, rt.lib().rt_last_error()
    finally:
        sc.close()
    g = out[:, x0:x0 + w]
    assert (g[..., 3] == 0).all()
    s = parity_stats(g, rgb)
    assert s["exact"] == 1.0, s


def test_config2_full_frame_bit_exact(gpu_ctx):
    objs = scenes.bench_objects(16)
    view = rt.make_view(None, 0.0)
    g = gpu_render(gpu_ctx, objs, 1920, 1080, 0, view)
    o = oracle_render(objs, 1920, 1080, 0)
    assert np.array_equal(g, o), parity_stats(g, o)


@pytest.mark.parametrize("cfg,band", [("config3", [(0, 8), (536, 544), (1076, 1084), (1620, 1628), (2152, 2160)]),
                                      ("config4", [(2156, 2164), (0, 8), (1080, 1088), (3240, 3248),
                                                   (4312, 4320)])])
def test_large_configs_bands_bit_exact(gpu_ctx, cfg, band):
    build, w, h, depth = scenes.CONFIGS[cfg]
    objs = build()
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    rt.render_device(gpu_ctx, sc, out.data_ptr(), w, h, depth, view=view)
    torch.cuda.synchronize()
    full = out.cpu().numpy()
    assert np.isfinite(full).all() and (full[..., 3] == 0).all()
    for r0, r1 in band:
        o = oracle_render(objs, w, h, depth, rows=(r0, r1))
        assert np.array_equal(full[r0:r1], o), (cfg, r0, parity_stats(full[r0:r1], o))
    # a band rendered alone equals the same rows of the full frame
    r0, r1 = band[0]
    assert np.array_equal(rt.render(gpu_ctx, sc, w, h, depth, view=view, rows=(r0, r1)), full[r0:r1])
    # deterministic
    out2 = torch.empty_like(out)
    rt.render_device(gpu_ctx, sc, out2.data_ptr(), w, h, depth, view=view)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    sc.close()


@pytest.mark.parametrize("n_shards,block", [(2, 8), (3, 16), (8, 8), (8, 1)])
def test_shards_reassemble_the_frame(gpu_ctx, n_shards, block):
    objs = scenes.bench_objects(16)
    w, h = 480, 270
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    full = rt.render(gpu_ctx, sc, w, h, 1, view=view)
    elems = frame.flat_shard_elems(1, h, w, block, n_shards)
    shards = []
    for s in range(n_shards):
        buf = dev_zeros(elems, dtype=torch.float32, device="cuda")
        rt.render_shard(gpu_ctx, sc, buf.data_ptr(), w, h, 1, block, n_shards, s, view=view)
        shards.append(buf)
    torch.cuda.synchronize()
    assembled = frame.assemble(shards, 1, h, w, block).cpu().numpy()
    assert np.array_equal(assembled[0], full)
    sc.close()


@pytest.mark.parametrize("n_shards", [1, 2, 8])
def test_batched_frames_equal_single_frames(gpu_ctx, n_shards):
    """rt_render_batch: K views in one launch == K separate renders, whole
    frames or one shard's rows of each."""
    objs = scenes.bench_objects(16)
    w, h, block = 320, 180, 8
    views = [rt.make_view(None, k / 60.0) for k in range(5)]
    sc = rt.Scene(gpu_ctx, objs)
    singles = [rt.render(gpu_ctx, sc, w, h, 1, view=v) for v in views]
    for shard in range(n_shards):
        rows = frame.shard_row_ids(h, block, n_shards, shard)
        out = dev_zeros((len(views), len(rows), w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, 1, views, block, n_shards, shard)
        got = out.cpu().numpy()
        for k in range(len(views)):
            assert np.array_equal(got[k], singles[k][rows]), (shard, k)
    sc.close()


@pytest.mark.parametrize("depth,n_views,n_shards", [(0, 64, 1), (0, 23, 3), (1, 12, 1), (3, 19, 2), (0, 256, 2)])
def test_large_batches_equal_single_frames(gpu_ctx, depth, n_views, n_shards):
    """More than 8 views in one rt_render_batch call: depth 0-1 in one launch
    with the views and their frame constants in the context's device buffer
    (render_kernel<D, false, true>), deeper frames as launches of at most 8 — each
    frame bit-identical to its own single render (whole frames or one shard's
    rows), with host frame constants and with device-derived ones, in the
    float4 and the GL_RGBA8 surface; and, repeated, the slot ring is reused
    behind its events."""
    objs = scenes.bench_objects(16 if depth < 2 else 64)
    w, h, block = 160, 90, 8
    views = [rt.make_view(None, k / 60.0) for k in range(n_views)]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        singles = [rt.render(gpu_ctx, sc, w, h, depth, view=v) for v in views]
        for consts in (True, False):
            gpu_ctx.set_host_frame_consts(consts)
            for shard in range(n_shards):
                rows = frame.shard_row_ids(h, block, n_shards, shard)
                for rep in range(2 if consts else 1):
                    out = dev_zeros((n_views, len(rows), w, 4), dtype=torch.float32, device="cuda")
                    rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, views, block, n_shards, shard)
                    got = out.cpu().numpy()
                    for k in range(n_views):
                        assert np.array_equal(got[k], singles[k][rows]), (consts, shard, rep, k)
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA8)
        texels = dev_zeros((n_views, h, w), dtype=torch.int32, device="cuda")
        rt.render_batch(gpu_ctx, sc, texels.data_ptr(), w, h, depth, views)
        got8 = texels.cpu().numpy().view(np.uint8).reshape(n_views, h, w, 4)
        for k in range(n_views):
            assert np.array_equal(got8[k], rt.pack_rgba8(singles[k])), k
    finally:
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA32F)
        gpu_ctx.set_host_frame_consts(True)
        sc.close()
    sc = rt.Scene(gpu_ctx, objs)
    try:
        with pytest.raises(rt.RTError) as e:
            rt.render_batch(gpu_ctx, sc, 0, w, h, depth, (views * (rt.abi.RT_MAX_BATCH + 1))[:rt.abi.RT_MAX_BATCH + 1])
        assert e.value.code == rt.abi.RT_ERR_INVALID
    finally:
        sc.close()


@pytest.mark.parametrize("depth,n_views,n_shards,w,h", [(2, 10, 1, 640, 360), (3, 2, 1, 640, 360),
                                                        (2, 7, 2, 640, 360), (4, 3, 1, 640, 360),
                                                        (3, 7, 3, 652, 366)])
def test_queued_view_batches_equal_single_frames(gpu_ctx, depth, n_views, n_shards, w, h):
    """Deep batches large enough for the queued distribution (more wave tiles
    than resident waves): one launch renders several views, every view's
    frame constants beside the scene in LDS, the items view-major (and
    batches beyond what one launch holds split into even launches) — each
    frame bit-identical to its own single render, with host frame constants
    (2 views of 64 spheres fit in the kernel arguments) and device-derived
    ones, whole frames and shards (ragged frames too), float4 and GL_RGBA8."""
    objs = scenes.bench_objects(64)
    block = 8
    views = [rt.make_view(None, 0.5 + k / 30.0) for k in range(n_views)]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        singles = [rt.render(gpu_ctx, sc, w, h, depth, view=v) for v in views]
        for consts in (True, False):
            gpu_ctx.set_host_frame_consts(consts)
            for shard in range(n_shards):
                rows = frame.shard_row_ids(h, block, n_shards, shard)
                out = dev_zeros((n_views, len(rows), w, 4), dtype=torch.float32, device="cuda")
                rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, views, block, n_shards, shard)
                got = out.cpu().numpy()
                for k in range(n_views):
                    assert np.array_equal(got[k], singles[k][rows]), (consts, shard, k)
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA8)
        texels = dev_zeros((n_views, h, w), dtype=torch.int32, device="cuda")
        rt.render_batch(gpu_ctx, sc, texels.data_ptr(), w, h, depth, views)
        got8 = texels.cpu().numpy().view(np.uint8).reshape(n_views, h, w, 4)
        for k in range(n_views):
            assert np.array_equal(got8[k], rt.pack_rgba8(singles[k])), k
    finally:
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA32F)
        gpu_ctx.set_host_frame_consts(True)
        sc.close()


def test_large_animated_batch_of_scenes(gpu_ctx):
    """rt_render_batch_scenes with 12 views (the device-buffer path): every
    frame its own time-animated shipped scene (per-view blobs), equal to
    single renders and to the oracle."""
    times = [0.3 * k for k in range(12)]
    w, h, depth = 64, 36, 1
    scs = [rt.Scene(gpu_ctx, rt.reference_objects(t)) for t in times]
    views = [rt.make_view(None, t) for t in times]
    try:
        out = dev_zeros((len(times), h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch_scenes(gpu_ctx, scs, out.data_ptr(), w, h, depth, views)
        got = out.cpu().numpy()
        for k, t in enumerate(times):
            assert np.array_equal(got[k], rt.render(gpu_ctx, scs[k], w, h, depth, view=views[k])), k
            assert np.array_equal(got[k], oracle_render(rt.reference_objects(t), w, h, depth, t)), k
    finally:
        for s in scs:
            s.close()


@pytest.mark.parametrize("n_views", [4, 10])
def test_batch_of_scenes_with_different_lights(gpu_ctx, n_views):
    """rt_render_batch_scenes over two scenes of one layout whose lights
    differ: the reference's (ambient-only light 0, lights 1-2 inside the room)
    and one with light 0 lit, light 2 ambient-only and light 1 outside the room
    (so it is not a room: kShapeRoom must not apply to the launch,
    rt_api.cpp render_batch_impl). Kernel-argument (4 views) and
    device-buffer (10 views) batches; every frame equal to its single render
    and the oracle."""
    w, h = 160, 90
    objs = scenes.bench_objects(16, seed=3)
    la = rt.reference_lights()
    lb = rt.reference_lights()
    lb[0].diffuse[:] = [0.6, 0.6, 0.6, 1.0]
    lb[0].specular[:] = [0.6, 0.6, 0.6, 1.0]
    lb[2].diffuse[:] = [0.0, 0.0, 0.0, 0.0]
    lb[2].specular[:] = [0.0, 0.0, 0.0, 0.0]
    lb[1].position[:] = [30.0, 7.0, 2.0]  # outside the room (x beyond 11)
    sa, sb = rt.Scene(gpu_ctx, objs, lights=la), rt.Scene(gpu_ctx, objs, lights=lb)
    try:
        scs = [sa if k % 2 == 0 else sb for k in range(n_views)]
        views = [rt.make_view(None, 0.2 * k) for k in range(n_views)]
        out = dev_zeros((n_views, h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch_scenes(gpu_ctx, scs, out.data_ptr(), w, h, 0, views)
        got = out.cpu().numpy()
        for k in range(n_views):
            single = rt.render(gpu_ctx, scs[k], w, h, 0, view=views[k])
            assert np.array_equal(got[k], single), k
            o = port.render(objs, w, h, 0, 0.2 * k, rows=(40, 42), lights=la if k % 2 == 0 else lb)
            assert np.array_equal(got[k][40:42], o), (k, parity_stats(got[k][40:42], o))
    finally:
        sa.close()
        sb.close()


def _inside_sphere_camera():
    cam = rt.Camera()
    cam.position[:] = (-3.0, 4.0, 1.2)  # inside config 1's red-glass sphere (centre (-3, 4, 1), r 2)
    cam.angles[:] = (0.3, 1.1, 0.0)
    cam.v_fov, cam.aspect, cam.near_plane, cam.far_plane = 1.5707964, 16.0 / 9.0, 0.1, 1000.0
    return cam


@pytest.mark.parametrize("case", ["bench16", "bench64", "shipped", "inside_sphere", "no_culling"])
def test_host_frame_constants_equal_device_ones(gpu_ctx, case):
    """Per-frame constants from the host (host_frame_setup, carried in the
    kernel arguments, per view of a batch when they all fit) or derived in
    every work-group (frame_setup, RT_OPT_FRAME_CONSTS = 0): the same frames,
    bit for bit — camera terms identical, footprints conservative."""
    w, h, depth, cam = 256, 144, 1, None
    if case in ("bench16", "no_culling"):
        objs, view_t = scenes.bench_objects(16), 0.4
    elif case == "bench64":
        objs, view_t, depth = scenes.bench_objects(64), 2.0, 2
    elif case == "shipped":
        objs, view_t = rt.reference_objects(1.3), 1.3
    else:
        objs, view_t, cam = scenes.config1_objects(), 0.0, _inside_sphere_camera()
    view = rt.make_view(cam, view_t)
    if case == "no_culling":
        gpu_ctx.set_culling(False)
    try:
        sc = rt.Scene(gpu_ctx, objs)
        single = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        other = rt.make_view(cam, view_t + 0.7) if cam is None else view
        other_single = rt.render(gpu_ctx, sc, w, h, depth, view=other)
        got = {}
        for host in (True, False):
            gpu_ctx.set_host_frame_consts(host)
            out = dev_zeros((2, h, w, 4), dtype=torch.float32, device="cuda")
            rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, [view, other])
            got[host] = out.cpu().numpy()
            if not host:
                dev_single = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        sc.close()
    finally:
        gpu_ctx.set_culling(True)
        gpu_ctx.set_host_frame_consts(True)
    assert np.array_equal(dev_single, single)
    for host in (True, False):
        assert np.array_equal(got[host][0], single) and np.array_equal(got[host][1], other_single), host
    if case in ("bench16", "shipped"):
        o = oracle_render(objs, w, h, depth, view_t)
        assert np.array_equal(single, o), parity_stats(single, o)


def test_async_stream_equals_sync(gpu_ctx):
    objs = scenes.bench_objects(16)
    view = rt.make_view(None, 1.0)
    sc = rt.Scene(gpu_ctx, objs)
    sync = rt.render(gpu_ctx, sc, 320, 180, 2, view=view)
    s = torch.cuda.Stream()
    out = dev_zeros((180, 320, 4), dtype=torch.float32, device="cuda")
    with torch.cuda.stream(s):
        rt.render_device(gpu_ctx, sc, out.data_ptr(), 320, 180, 2, view=view, stream=s.cuda_stream)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy(), sync)
    sc.close()


@pytest.mark.parametrize("depth", range(0, rt.RT_MAX_DEPTH + 1))
def test_every_depth_matches_oracle(gpu_ctx, depth):
    objs = rt.reference_objects(0.0)
    view = rt.make_view(None, 0.0)
    w, h = (48, 27) if depth <= 6 else (16, 9)
    g = gpu_render(gpu_ctx, objs, w, h, depth, view)
    o = oracle_render(objs, w, h, depth)
    assert np.array_equal(g, o), parity_stats(g, o)


@pytest.mark.parametrize("w,h", [(1, 1), (2, 1), (1, 2), (3, 3), (17, 5), (129, 73), (1000, 3)])
def test_odd_and_degenerate_frame_sizes(gpu_ctx, w, h):
    """W/2 and H/2 are integer halves (:377-378); a 1-pixel side divides by 0."""
    objs = rt.reference_objects(0.0)
    view = rt.make_view(None, 0.0)
    g = gpu_render(gpu_ctx, objs, w, h, 1, view)
    o = oracle_render(objs, w, h, 1)
    assert np.array_equal(g, o, equal_nan=True)


def test_empty_and_null_object_scenes_are_black(gpu_ctx):
    view = rt.make_view(None, 0.0)
    g = gpu_render(gpu_ctx, [], 64, 36, 2, view)
    assert (g == 0).all()
    null = rt.abi.Object()
    null.radius = -1.0  # null_box + null_sphere: skipped (:768-771)
    g = gpu_render(gpu_ctx, [null, null], 64, 36, 2, view)
    assert (g == 0).all()


def test_mixed_edge_scene(gpu_ctx):
    """Camera inside a sphere and inside a box, a tilted thin box, coincident
    spheres (tie -> lower index, :773), zero-radius sphere, emissive and
    negative colours, no-light and many-light scenes."""
    cam = rt.reference_camera(0.0)
    cx, cy, cz = cam.position
    objs = [scenes.sphere((cx, cy, cz), 0.5, rt.abi.RED_GLASS),
            scenes.box((-1, -1, -1), (1, 1, 1), (cx, cy, cz), (10, 20, 30), rt.abi.MIRROR),
            scenes.room_box(),
            scenes.sphere((0, 0, 0), 2.0, rt.abi.MATERIAL1), scenes.sphere((0, 0, 0), 2.0, rt.abi.MATERIAL2),
            scenes.sphere((1, 1, 1), 0.0, rt.abi.BLUE_GLASS),
            scenes.box((-5, -5, -0.01), (5, 5, 0.01), (0, 0, -2), (5, 30, 60), rt.abi.GREEN_GLASS)]
    mats = rt.reference_materials()
    mats[rt.abi.MATERIAL2].emissive[:] = (0.2, -0.1, 0.3, 0.5)
    mats[rt.abi.MIRROR].diffuse[:] = (-0.5, 0.25, 2.0, -1.0)
    lights = rt.reference_lights()
    view = rt.make_view(None, 0.0)
    for ls in ([], lights, lights * 5):
        g = gpu_render(gpu_ctx, objs, 96, 54, 3, view, materials=mats, lights=ls)
        o = oracle_render(objs, 96, 54, 3, materials=mats, lights=ls)
        assert np.array_equal(g, o, equal_nan=True), (len(ls), parity_stats(g, o))


def test_max_objects_scene(gpu_ctx):
    objs = scenes.bench_objects(rt.abi.RT_MAX_OBJECTS - 1, seed=3)
    view = rt.make_view(None, 0.0)
    g = gpu_render(gpu_ctx, objs, 64, 36, 1, view)
    o = oracle_render(objs, 64, 36, 1)
    assert np.array_equal(g, o)


def test_max_objects_queued_deep_batch(gpu_ctx):
    """The largest scene (RT_MAX_OBJECTS: the room box + 1023 spheres, the
    scene blob and its per-view records filling much of LDS) at depth 3 in a
    frame large enough for the queued distribution, as single frames and as a
    two-view batch: bands of rows against the oracle, every batched frame
    against its single render."""
    objs = scenes.bench_objects(rt.abi.RT_MAX_OBJECTS - 1, seed=5)
    w, h, depth = 768, 432, 3
    views = [rt.make_view(None, 0.0), rt.make_view(None, 1.5)]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        singles = [rt.render(gpu_ctx, sc, w, h, depth, view=v) for v in views]
        out = dev_zeros((2, h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, views)
        got = out.cpu().numpy()
        for k in range(2):
            assert np.array_equal(got[k], singles[k]), k
    finally:
        sc.close()
    for r0 in (0, 208, 424):
        o = oracle_render(objs, w, h, depth, 0.0, rows=(r0, r0 + 8))
        assert np.array_equal(singles[0][r0:r0 + 8], o), (r0, parity_stats(singles[0][r0:r0 + 8], o))


def test_animated_frames_match_oracle(gpu_ctx):
    for t in [0.5, 2.0, 7.25]:
        objs = rt.reference_objects(t)
        view = rt.make_view(None, t)
        g = gpu_render(gpu_ctx, objs, 64, 36, 2, view)
        o = oracle_render(objs, 64, 36, 2, t)
        assert np.array_equal(g, o), (t, parity_stats(g, o))


def test_errors(gpu_ctx):
    sc = rt.Scene(gpu_ctx, rt.reference_objects(0.0))
    with pytest.raises(rt.RTError) as e:
        rt.render(gpu_ctx, sc, 16, 16, rt.RT_MAX_DEPTH + 1)
    assert e.value.code == rt.abi.RT_ERR_UNSUPPORTED
    with pytest.raises(rt.RTError):
        rt.render(gpu_ctx, sc, 16, 16, 0, rows=(4, 2))
    bad = scenes.sphere((0, 0, 0), 1.0, 99)
    with pytest.raises(rt.RTError) as e:
        rt.Scene(gpu_ctx, [bad])
    assert e.value.code == rt.abi.RT_ERR_INVALID
    sc.close()


@pytest.mark.parametrize("cfg,w,h", [("config1", 128, 72), ("config2", 192, 108), ("config3", 192, 108),
                                     ("config4", 256, 144)])
def test_culling_and_bvh_change_nothing(gpu_ctx, cfg, w, h):
    """RT_OPT_CULLING (screen footprints, light cones, sphere BVH, box fast
    paths) must give bit-identical frames."""
    build, _, _, depth = scenes.CONFIGS[cfg]
    objs = build()
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        gpu_ctx.set_culling(True)
        on = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        gpu_ctx.set_culling(False)
        off = rt.render(gpu_ctx, sc, w, h, depth, view=view)
    finally:
        gpu_ctx.set_culling(True)
        sc.close()
    assert np.array_equal(on, off, equal_nan=True)
    o = oracle_render(objs, w, h, depth)
    assert np.array_equal(on, o), parity_stats(on, o)


@pytest.mark.parametrize("n_spheres,seed,depth,w,h", [(256, 0, 4, 320, 180), (64, 0, 2, 480, 270),
                                                       (64, 0, 5, 320, 180), (40, 7, 3, 256, 144),
                                                       (150, 3, 4, 320, 180), (33, 9, 9, 160, 90)])
def test_origin_lists_change_nothing(gpu_ctx, n_spheres, seed, depth, w, h):
    """RT_OPT_ORIGIN_LISTS (secondary rays leaving a sphere test its
    precomputed candidate list instead of walking the BVH, rt_internal.h
    kOListSlots) gives bit-identical frames, against the BVH walk and the
    oracle: the lists hold every sphere such a ray can hit and the closest
    hit is order-independent (raytrace_compute.glsl:738-782)."""
    objs = scenes.bench_objects(n_spheres, seed=seed)
    view = rt.make_view(None, 0.37 * seed)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        gpu_ctx.set_origin_lists(True)
        on = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        gpu_ctx.set_origin_lists(False)
        off = rt.render(gpu_ctx, sc, w, h, depth, view=view)
    finally:
        gpu_ctx.set_origin_lists(True)
        sc.close()
    assert np.array_equal(on, off, equal_nan=True), parity_stats(on, off)
    o = oracle_render(objs, w, h, depth, t=0.37 * seed)
    assert np.array_equal(on, o), parity_stats(on, o)


@pytest.mark.parametrize("n_spheres,n_boxes,seed,w,h", [(16, 1, 0, 1920, 1080), (4, 1, 2, 320, 180),
                                                         (32, 1, 5, 320, 180), (64, 1, 1, 320, 180),
                                                         (16, 3, 3, 320, 180), (48, 2, 4, 256, 144),
                                                         (16, 0, 6, 320, 180), (24, -1, 7, 320, 180)])
def test_scene_shapes_change_nothing(gpu_ctx, n_spheres, n_boxes, seed, w, h):
    """RT_OPT_SCENE_SHAPES (depth-0 renders of LDS-mask scenes run a kernel
    compiled for the scene's mask width and for a room — one translate-only
    box holding every live light, rt_internal.h kShapeRoom) gives
    bit-identical frames against the general kernel and the oracle, for 2-,
    4- and 8-byte masks, the room, several boxes, no box and one box that is
    not a room (n_boxes -1: the room replaced by a small rotated box), as
    single frames, a device-buffer batch and Monte-Carlo sums."""
    objs = scenes.bench_objects(n_spheres, seed=seed)
    if n_boxes <= 0:  # no room: no box at all, or one small rotated box the lights are outside of
        objs = objs[1:]
        if n_boxes < 0:
            objs.append(scenes.box((-1.0, -0.5, -0.5), (1.0, 0.5, 0.5), (0.0, 0.0, -6.0), (20.0, 35.0, 0.0), 3))
    for k in range(1, n_boxes):  # more boxes: small rotated cubes among the spheres
        objs.append(scenes.box((-0.5, -0.5, -0.5), (0.5, 0.5, 0.5), (2.0 * k - 3.0, -4.0, 1.5 * k),
                               (0.0, 30.0 * k, 0.0), k % 7))
    views = [rt.make_view(None, 0.25 * k + 0.1 * seed) for k in range(10)]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        out = {}
        for on in (True, False):
            gpu_ctx.set_scene_shapes(on)
            single = rt.render(gpu_ctx, sc, w, h, 0, view=views[0])
            batch = torch.empty((len(views), h, w, 4), dtype=torch.float32, device="cuda")
            rt.render_batch(gpu_ctx, sc, batch.data_ptr(), w, h, 0, views)  # > 8 views: the device-buffer kernel
            acc = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
            rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, 0, 3, 0, seed=seed, view=views[0])
            torch.cuda.synchronize()
            out[on] = (single, batch.cpu().numpy(), acc.cpu().numpy())
    finally:
        gpu_ctx.set_scene_shapes(True)
        sc.close()
    for a, b in zip(out[True], out[False]):
        assert np.array_equal(a, b, equal_nan=True), parity_stats(a, b)
    assert np.array_equal(out[True][1][0], out[True][0])
    rows = (h // 2, h // 2 + 2)
    o = port.render(objs, w, h, 0, 0.1 * seed, rows=rows)
    assert np.array_equal(out[True][0][rows[0]:rows[1]], o), parity_stats(out[True][0][rows[0]:rows[1]], o)


@pytest.mark.parametrize("n_spheres,n_boxes,seed,depth,w,h", [(64, 1, 0, 2, 480, 270), (256, 1, 1, 4, 320, 180),
                                                               (100, 2, 2, 3, 320, 180), (33, 1, 3, 9, 160, 90),
                                                               (200, 3, 4, 5, 256, 144), (64, -1, 5, 3, 320, 180)])
def test_wide_scene_shapes_change_nothing(gpu_ctx, n_spheres, n_boxes, seed, depth, w, h):
    """RT_OPT_SCENE_SHAPES for the recursive kernels (scenes whose shadow
    queries walk the wide masks' candidate lists and whose secondary rays the
    origin-sphere lists take, the room or several boxes or one box that is not
    a room, rt_internal.h kShapeWide, kShapeRoom): bit-identical frames
    against the general kernel and the oracle, single frames and a batch of
    views in one queued launch."""
    objs = scenes.bench_objects(n_spheres, seed=seed)
    if n_boxes < 0:  # the room replaced by one small rotated box the lights are outside of
        objs = objs[1:] + [scenes.box((-1.0, -0.5, -0.5), (1.0, 0.5, 0.5), (0.0, 0.0, -6.0), (20.0, 35.0, 0.0), 3)]
    for k in range(1, n_boxes):
        objs.append(scenes.box((-0.5, -0.5, -0.5), (0.5, 0.5, 0.5), (2.0 * k - 3.0, -4.0, 1.5 * k),
                               (0.0, 30.0 * k, 0.0), k % 7))
    views = [rt.make_view(None, 0.3 * k + 0.1 * seed) for k in range(3)]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        out = {}
        for on in (True, False):
            gpu_ctx.set_scene_shapes(on)
            single = rt.render(gpu_ctx, sc, w, h, depth, view=views[0])
            batch = torch.empty((len(views), h, w, 4), dtype=torch.float32, device="cuda")
            rt.render_batch(gpu_ctx, sc, batch.data_ptr(), w, h, depth, views)
            torch.cuda.synchronize()
            out[on] = (single, batch.cpu().numpy())
    finally:
        gpu_ctx.set_scene_shapes(True)
        sc.close()
    for a, b in zip(out[True], out[False]):
        assert np.array_equal(a, b, equal_nan=True), parity_stats(a, b)
    assert np.array_equal(out[True][1][0], out[True][0])
    o = oracle_render(objs, w, h, depth, t=0.1 * seed)
    assert np.array_equal(out[True][0], o), parity_stats(out[True][0], o)


def test_degenerate_spheres_do_not_break_the_bvh(gpu_ctx):
    objs = scenes.bench_objects(40, seed=5)
    objs[3].radius = float("nan")
    objs[7].position[0] = float("inf")
    objs[9].radius = 1e30
    objs[11].radius = -1.5  # radius != -1: a sphere of radius 1.5 (:759)
    view = rt.make_view(None, 0.0)
    g = gpu_render(gpu_ctx, objs, 96, 54, 3, view)
    o = oracle_render(objs, 96, 54, 3)
    assert np.array_equal(g, o, equal_nan=True), parity_stats(g, o)


def test_monte_carlo_matches_oracle(gpu_ctx):
    """Config-5 path: jittered samples accumulated in sample order, in two
    calls (samples [0, 3) then [3, 5)), bitwise equal to the oracle."""
    objs = scenes.bench_objects(16)
    w, h = 96, 54
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    acc = dev_zeros((h, w, 4), dtype=torch.float32, device="cuda")
    rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, 1, 3, 0, seed=7, view=view)
    rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, 1, 2, 3, seed=7, view=view)
    o = port.render_accumulate(objs, w, h, 1, 3, 0, seed=7)
    o = port.render_accumulate(objs, w, h, 1, 2, 3, seed=7, accum=o)
    assert np.array_equal(acc.cpu().numpy(), o)
    # without jitter every sample is the reference frame
    synced_zero_(acc)
    rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, 1, 3, 0, jitter=False, view=view)
    f = rt.render(gpu_ctx, sc, w, h, 1, view=view)
    assert np.array_equal(acc.cpu().numpy(), (f + f) + f)
    sc.close()


def test_queued_distribution_edge_scene(gpu_ctx):
    """Depth >= 2 frames with more 8x8 wave tiles than resident waves run on
    the queued (resident-grid, atomic wave-tile queue) path: the edge scene of
    test_mixed_edge_scene at 800x512 (6400 wave tiles), bands against the
    oracle, rendered repeatedly (the queue counters reset themselves)."""
    cam = rt.reference_camera(0.0)
    cx, cy, cz = cam.position
    objs = [scenes.sphere((cx, cy, cz), 0.5, rt.abi.RED_GLASS), scenes.room_box(),
            scenes.box((-1, -1, -1), (1, 1, 1), (2, 1, 0), (10, 20, 30), rt.abi.MIRROR),
            scenes.sphere((0, 0, 0), 2.0, rt.abi.MATERIAL1), scenes.sphere((0, 0, 0), 2.0, rt.abi.MATERIAL2),
            scenes.box((-5, -5, -0.01), (5, 5, 0.01), (0, 0, -2), (5, 30, 60), rt.abi.GREEN_GLASS)]
    objs += scenes.bench_objects(24, seed=9)[1:]
    w, h, depth = 800, 512, 3
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    frames = []
    for _ in range(3):
        out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_device(gpu_ctx, sc, out.data_ptr(), w, h, depth, view=view)
        torch.cuda.synchronize()
        frames.append(out.cpu().numpy())
    sc.close()
    assert all(np.array_equal(frames[0], f, equal_nan=True) for f in frames[1:])
    for r0, r1 in [(0, 6), (250, 262), (506, 512)]:
        o = oracle_render(objs, w, h, depth, rows=(r0, r1))
        assert np.array_equal(frames[0][r0:r1], o, equal_nan=True), (r0, parity_stats(frames[0][r0:r1], o))


def test_concurrent_streams_share_a_context(gpu_ctx):
    """Launches in flight on two streams of one context (queued frames use a
    counter slot per launch) give the frames a synchronous render gives."""
    objs = scenes.bench_objects(40, seed=2)
    w, h, depth = 1024, 512, 2
    view_a, view_b = rt.make_view(None, 0.0), rt.make_view(None, 0.5)
    sc = rt.Scene(gpu_ctx, objs)
    ref_a = rt.render(gpu_ctx, sc, w, h, depth, view=view_a)
    ref_b = rt.render(gpu_ctx, sc, w, h, depth, view=view_b)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(6)]
    for k, out in enumerate(outs):
        s, v = (sa, view_a) if k % 2 == 0 else (sb, view_b)
        rt.render_device(gpu_ctx, sc, out.data_ptr(), w, h, depth, view=v, stream=s.cuda_stream)
    torch.cuda.synchronize()
    for k, out in enumerate(outs):
        assert np.array_equal(out.cpu().numpy(), ref_a if k % 2 == 0 else ref_b), k
    sc.close()


def test_scene_update_animation(gpu_ctx):
    """rt_scene_update: the shipped scene animated over frames, one scene object."""
    sc = rt.Scene(gpu_ctx, rt.reference_objects(0.0))
    for t in [0.0, 1.5, 4.0]:
        objs = rt.reference_objects(t)
        sc.update(objs)
        view = rt.make_view(None, t)
        g = rt.render(gpu_ctx, sc, 64, 36, 1, view=view)
        o = oracle_render(objs, 64, 36, 1, t)
        assert np.array_equal(g, o)
    sc.update(scenes.bench_objects(64))  # larger: reallocates
    g = rt.render(gpu_ctx, sc, 64, 36, 1, view=rt.make_view(None, 0.0))
    assert np.array_equal(g, oracle_render(scenes.bench_objects(64), 64, 36, 1))
    sc.close()


def test_rgba8_surface_matches_the_gl_rgba8_render(gpu_ctx):
    """rt_render(cam = NULL) into the RGBA8 surface (RT_OUTPUT_RGBA8) — the
    shipped app's GL_RGBA8 texture, main.cpp:152-159, :223 — equals, byte for
    byte, the reference's own render stored by its GL into that format
    (tests/golden/rgba8_llvmpipe.npz: GL rounds exact halves to even)."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rgba8_llvmpipe.npz"))
    names = sorted(k[:-len("_rgba8")] for k in z.files if k.endswith("_rgba8"))
    gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA8)
    try:
        for n in names:
            w, h, depth, t, x0, y0, cw, ch = z[n + "_meta"]
            w, h, depth, x0, y0, cw, ch = (int(v) for v in (w, h, depth, x0, y0, cw, ch))
            scene = str(z[n + "_scene"])
            objs = rt.reference_objects(float(t)) if scene == "shipped" else scenes.CONFIGS[scene][0]()
            sc = rt.Scene(gpu_ctx, objs)
            try:
                out = np.zeros((ch, w, 4), np.uint8)
                rc = rt.lib().rt_render(gpu_ctx.handle, sc.handle, None, float(t), w, h, depth, y0, y0 + ch,
                                        out.ctypes.data, 0, None)
                assert rc == 0, rt.lib().rt_last_error()
            finally:
                sc.close()
            assert np.array_equal(out[:, x0:x0 + cw], z[n + "_rgba8"]), n
    finally:
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA32F)


@pytest.mark.parametrize("cfg,w,h", [("shipped", 160, 90), ("config3", 256, 144)])
def test_rgba8_surface_equals_packed_float_frame(gpu_ctx, cfg, w, h):
    """RT_OUTPUT_RGBA8 (the shipped GL_RGBA8 texture, main.cpp:152-159): the
    kernel's packed epilogue == rt_pack_rgba8 of the float frame, bytewise;
    shard / batch renders write 4 bytes per pixel too."""
    if cfg == "shipped":
        objs, depth = rt.reference_objects(0.0), 1
    else:
        build, _, _, depth = scenes.CONFIGS[cfg]
        objs = build()
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    f = rt.render(gpu_ctx, sc, w, h, depth, view=view)
    b = rt.render_rgba8(gpu_ctx, sc, w, h, depth, view=view)
    assert np.array_equal(b, rt.pack_rgba8(f))
    assert np.array_equal(rt.render_rgba8(gpu_ctx, sc, w, h, depth, view=view, rows=(7, 40)), b[7:40])
    gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA8)
    try:
        out = dev_zeros((2, h, w, 4), dtype=torch.uint8, device="cuda")
        rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, [view, view])
        got = out.cpu().numpy()
        assert np.array_equal(got[0], b) and np.array_equal(got[1], b)
        acc = dev_zeros((h, w, 4), dtype=torch.float32, device="cuda")
        with pytest.raises(rt.RTError) as e:
            rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, depth, 1, view=view)
        assert e.value.code == rt.abi.RT_ERR_UNSUPPORTED
    finally:
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA32F)
        sc.close()


@pytest.mark.parametrize("n_shards", [1, 2, 8])
def test_rgb32f_exchange_format_equals_float_frames(gpu_ctx, n_shards):
    """RT_OUTPUT_RGB32F (the multi-GPU exchange's transport form): packed
    float3 per pixel == the rgb of the float4 frame, bit for bit, for whole
    frames and for every shard's rows of a batch launch (bench.py's path);
    the exchange + assembly on 3 channels rebuilds each frame."""
    objs = scenes.bench_objects(16)
    w, h, block = 320, 180, 8
    views = [rt.make_view(None, k / 60.0) for k in range(n_shards)]
    sc = rt.Scene(gpu_ctx, objs)
    singles = [rt.render(gpu_ctx, sc, w, h, 0, view=v) for v in views]
    gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGB32F)
    try:
        one = dev_zeros((h, w, 3), dtype=torch.float32, device="cuda")
        rt.render_device(gpu_ctx, sc, one.data_ptr(), w, h, 0, view=views[0])
        torch.cuda.synchronize()
        assert np.array_equal(one.cpu().numpy(), singles[0][..., :3])
        bufs = []
        for shard in range(n_shards):
            rows = frame.shard_row_ids(h, block, n_shards, shard)
            out = dev_zeros((n_shards, len(rows), w, 3), dtype=torch.float32, device="cuda")
            rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, 0, views, block, n_shards, shard)
            got = out.cpu().numpy()
            for k in range(n_shards):
                assert np.array_equal(got[k], singles[k][rows][..., :3]), (shard, k)
            bufs.append(out.reshape(-1))
        # the all-to-all by hand: rank k receives frame k's rows of every shard
        for k in range(n_shards):
            ins = [frame.exchange_splits(h, w, block, n_shards, s, channels=3)[0] for s in range(n_shards)]
            recv = torch.cat([bufs[s][k * ins[s][k]:(k + 1) * ins[s][k]] for s in range(n_shards)])
            assert recv.numel() == sum(frame.exchange_splits(h, w, block, n_shards, k, channels=3)[1])
            fr = frame.assemble_frame(recv, h, w, block, n_shards, channels=3).cpu().numpy()
            assert np.array_equal(fr, singles[k][..., :3])
    finally:
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA32F)
        sc.close()


def test_cli_renders_a_scene_description(gpu_ctx, tmp_path):
    """rt_cli (the headless main()/draw() driver) on scenes/config1.json: its
    PPM is the RGBA8 surface of the same frame rendered through the C-ABI."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "openglraytracer_amd", "rt_cli")
    out = str(tmp_path / "f.ppm")
    r = subprocess.run([cli, "--scene", os.path.join(root, "scenes", "config1.json"), "--width", "64",
                        "--height", "48", "--depth", "1", "--ppm", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    objs, mats, lts, _ = rt.parse_scene(open(os.path.join(root, "scenes", "config1.json")).read())
    sc = rt.Scene(gpu_ctx, objs, materials=mats, lights=lts)
    f = rt.render(gpu_ctx, sc, 64, 48, 1, view=rt.make_view(None, 0.0))
    sc.close()
    data = open(out, "rb").read()
    header = b"P6\n64 48\n255\n"
    assert data.startswith(header)
    img = np.frombuffer(data[len(header):], np.uint8).reshape(48, 64, 3)
    assert np.array_equal(img, rt.pack_rgba8(f)[::-1, :, :3])  # PPM rows top-down


def test_animated_frames_in_one_launch(gpu_ctx):
    """rt_render_batch_scenes: K frames of the shipped, time-animated scene
    (raytrace_compute.glsl:277-307, the camera orbiting, main.cpp:81-86) in
    one launch, each frame its own scene — equal to K single renders and to
    the oracle; a scene of another layout is refused."""
    times = [0.0, 0.25, 1.5, 4.0]
    w, h, depth = 96, 54, 2
    scs = [rt.Scene(gpu_ctx, rt.reference_objects(t)) for t in times]
    views = [rt.make_view(None, t) for t in times]
    out = dev_zeros((len(times), h, w, 4), dtype=torch.float32, device="cuda")
    rt.render_batch_scenes(gpu_ctx, scs, out.data_ptr(), w, h, depth, views)
    got = out.cpu().numpy()
    for k, t in enumerate(times):
        assert np.array_equal(got[k], rt.render(gpu_ctx, scs[k], w, h, depth, view=views[k])), k
        assert np.array_equal(got[k], oracle_render(rt.reference_objects(t), w, h, depth, t)), k
    other = rt.Scene(gpu_ctx, scenes.bench_objects(4))
    with pytest.raises(rt.RTError) as e:
        rt.render_batch_scenes(gpu_ctx, [scs[0], other], out.data_ptr(), w, h, depth, views[:2])
    assert e.value.code == rt.abi.RT_ERR_INVALID
    for s in scs + [other]:
        s.close()


@pytest.mark.parametrize("n_spheres", [3, 16, 17, 32, 33, 64, 65, 130, 256, 257])
def test_shadow_direction_masks(gpu_ctx, n_spheres):
    """Shadow-ray direction masks (rt_internal.h, kMaskMaxSpheres): 16-bit
    masks up to 16 spheres, 32-bit up to 32, 64-bit up to 64 (staged in LDS);
    wide masks of 1-4 words read through L2 at depth >= 2 for 33-256
    (RT_GMASK_FROM, kGMaskMaxSpheres; 33-64 keep the LDS masks at depth 0);
    the per-wave cone above 256. Spheres
    cluster around the lights (one light inside a sphere, one grazing a
    surface) so that many shadow rays are blocked; culling on and off and the
    oracle must agree bit for bit, at depth 0 and through reflections."""
    rng = np.random.default_rng(n_spheres)
    lights = rt.reference_lights()
    lights[1].position[:] = (2.0, 2.0, 1.0)
    lights[2].position[:] = (-3.0, 1.0, -2.0)
    extra = rt.reference_lights()[1]
    extra.position[:] = (0.5, -4.0, 3.0)
    lights = lights + [extra]
    objs = [scenes.room_box(), scenes.sphere((2.0, 2.0, 1.0), 0.6, rt.abi.RED_GLASS),
            scenes.sphere((-3.0, 1.0, -2.75), 0.7, rt.abi.MATERIAL1)]  # light 2 ~0.05 above its top
    mats_cycle = [rt.abi.MATERIAL1, rt.abi.MATERIAL2, rt.abi.MIRROR, rt.abi.GREEN_GLASS, rt.abi.BLUE_GLASS]
    for i in range(n_spheres - 2):
        anchor = np.array(lights[1 + i % 3].position[:])
        c = anchor + rng.uniform(-4.0, 4.0, 3)
        objs.append(scenes.sphere(tuple(float(v) for v in c), float(rng.uniform(0.2, 0.9)), mats_cycle[i % 5]))
    objs = objs[:n_spheres + 1]
    view = rt.make_view(None, 0.0)
    for depth in (0, 2):
        sc = rt.Scene(gpu_ctx, objs, lights=lights)
        try:
            gpu_ctx.set_culling(True)
            on = rt.render(gpu_ctx, sc, 128, 72, depth, view=view)
            gpu_ctx.set_culling(False)
            off = rt.render(gpu_ctx, sc, 128, 72, depth, view=view)
        finally:
            gpu_ctx.set_culling(True)
            sc.close()
        assert np.array_equal(on, off, equal_nan=True), (depth, parity_stats(on, off))
        o = oracle_render(objs, 128, 72, depth, lights=lights)
        assert np.array_equal(on, o, equal_nan=True), (depth, parity_stats(on, o))


def test_config5_monte_carlo_kernel_full_frame(gpu_ctx):
    """The kernel bench.py --workload config5 times (render_kernel<0, true>:
    max_depth 0, jittered samples): the full 1920x1080 config-5 frame at 4 spp,
    split in two sample ranges like the sample-sharded multi-GPU step,
    bitwise equal to the oracle's same-order sums on bands of rows; without
    jitter every sample is the config-2 frame (main.cpp:228-238: one ray per
    pixel is the jitter-off limit)."""
    build, w, h, depth = scenes.CONFIGS["config5"]
    objs = build()
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        # plain fills on torch's default stream, no host synchronisation: the
        # NULL-stream calls are ordered after them (the r04a failure's
        # hazard, fixed in the library: include/rt.h hip_stream)
        acc = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, depth, 2, 0, seed=0, view=view)
        rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, depth, 2, 2, seed=0, view=view)
        one = torch.zeros(acc.shape, dtype=acc.dtype, device="cuda")
        rt.render_accumulate(gpu_ctx, sc, one.data_ptr(), w, h, depth, 4, 0, seed=0, view=view)
        torch.cuda.synchronize()
        split, whole = acc.cpu().numpy(), one.cpu().numpy()
        assert np.isfinite(split).all() and (split[..., 3] == 0).all()
        for r0, r1 in [(0, 4), (538, 542), (1076, 1080)]:
            o = port.render_accumulate(objs, w, h, depth, 2, 0, seed=0, rows=(r0, r1))
            o = port.render_accumulate(objs, w, h, depth, 2, 2, seed=0, rows=(r0, r1), accum=o)
            assert np.array_equal(split[r0:r1], o), (r0, parity_stats(split[r0:r1], o))
            o1 = port.render_accumulate(objs, w, h, depth, 4, 0, seed=0, rows=(r0, r1))
            assert np.array_equal(whole[r0:r1], o1), (r0, parity_stats(whole[r0:r1], o1))
        # the two orders differ only by float re-association
        assert np.allclose(split, whole, rtol=1e-6, atol=1e-6)
        one.zero_()
        rt.render_accumulate(gpu_ctx, sc, one.data_ptr(), w, h, depth, 2, 0, jitter=False, view=view)
        f = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        assert np.array_equal(one.cpu().numpy(), f + f)
    finally:
        sc.close()


def test_split_deep_batch_is_counted_and_timed_whole(gpu_ctx):
    """A deep batch larger than one queued launch holds (7 views of the
    64-sphere scene) runs as several launches: rt_batch_launches says how
    many, and rt_last_kernel_ms covers all of them, not the last one only."""
    objs = scenes.bench_objects(64)
    w, h, depth = 1280, 720, 2
    sc = rt.Scene(gpu_ctx, objs)
    try:
        cap = max(k for k in range(1, 65) if rt.batch_launches(gpu_ctx, sc, k, depth) == 1)
        assert 2 <= cap < 64
        assert rt.batch_launches(gpu_ctx, sc, cap + 1, depth) == 2
        assert rt.batch_launches(gpu_ctx, sc, 3 * cap, depth) == 3
        assert rt.batch_launches(gpu_ctx, sc, 3 * cap, 0) == 1
        views = [rt.make_view(None, k / 60.0) for k in range(3 * cap)]
        out = torch.empty((3 * cap, h, w, 4), dtype=torch.float32, device="cuda")
        gpu_ctx.set_timing(True)
        ms1, ms3 = [], []
        for _ in range(3):
            rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, views[:cap])
            ms1.append(gpu_ctx.last_kernel_ms())
            rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, views)
            ms3.append(gpu_ctx.last_kernel_ms())
        assert np.median(ms3) > 2.0 * np.median(ms1), (ms1, ms3)
    finally:
        sc.close()


def test_config5_at_its_stated_1024_spp(gpu_ctx):
    """Config 5 as BASELINE.json states it: the full 1920x1080 frame at 1024
    jittered samples per pixel, as the bench renders it at N=1 (one call of
    1024 samples) and at N=8 (eight calls of 128 samples, sample_offset 0,
    128, ..., 896, accumulating into one buffer), each bitwise equal to the
    oracle's in-order sums of the same sample ranges on two full-width 2-row
    bands. The jitter enters at the NDC step (raytrace_compute.glsl:377-392);
    sample indices 4..1023 and the 1024-term in-register sum are pinned here.
    The accumulators are plain torch.zeros on torch's default stream, not
    synchronised: a NULL-stream call is ordered after them (include/rt.h)."""
    build, w, h, depth = scenes.CONFIGS["config5"]
    spp, shards = 1024, 8
    objs = build()
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        whole = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_accumulate(gpu_ctx, sc, whole.data_ptr(), w, h, depth, spp, 0, seed=0, view=view)
        split = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        per = spp // shards
        for k in range(shards):
            rt.render_accumulate(gpu_ctx, sc, split.data_ptr(), w, h, depth, per, k * per, seed=0, view=view)
        a, b = whole.cpu().numpy(), split.cpu().numpy()
        assert np.isfinite(a).all() and (a[..., 3] == 0).all() and (b[..., 3] == 0).all()
        threads = min(16, os.cpu_count() or 1)
        for r0, r1 in [(538, 540), (1000, 1002)]:
            o = port.render_accumulate(objs, w, h, depth, spp, 0, seed=0, rows=(r0, r1), threads=threads)
            assert np.array_equal(a[r0:r1], o), (r0, parity_stats(a[r0:r1], o))
            o8 = None
            for k in range(shards):
                o8 = port.render_accumulate(objs, w, h, depth, per, k * per, seed=0, rows=(r0, r1), accum=o8,
                                            threads=threads)
            assert np.array_equal(b[r0:r1], o8), (r0, parity_stats(b[r0:r1], o8))
        # the two summation orders differ only by float re-association:
        # |error| <= (terms) * 2^-24 * sum for non-negative terms
        assert np.isfinite(b).all()
        assert np.allclose(a, b, rtol=spp * 2.0 ** -24, atol=1e-3), float(np.abs(a - b).max())
    finally:
        sc.close()


def test_null_stream_calls_follow_default_stream_work(gpu_ctx):
    """hip_stream = NULL is ordered like glDispatchCompute behind the earlier
    commands of its context (main.cpp:220-238): work queued on torch's
    default (null) stream — here tens of ms of matrix products and then a zero
    fill of the accumulator — completes before the library's accumulation
    reads the buffer, with no host synchronisation in between; a render into
    a buffer the default stream is still filling ends with the render's
    pixels, not the fill's."""
    build, w, h, depth = scenes.CONFIGS["config5"]
    objs = build()
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        acc = torch.full((h, w, 4), 7.0, dtype=torch.float32, device="cuda")
        m = torch.randn((4096, 4096), device="cuda")
        torch.cuda.synchronize()
        assert torch.cuda.current_stream().cuda_stream == 0  # torch's default stream is the null stream
        for _ in range(15):
            m = m @ m * 1e-3  # keeps the null stream busy
        acc.zero_()
        rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, depth, 2, 0, seed=0, view=view)  # NULL stream
        got = acc[538:540].cpu().numpy()
        o = port.render_accumulate(objs, w, h, depth, 2, 0, seed=0, rows=(538, 540))
        assert np.array_equal(got, o), parity_stats(got, o)
        img = torch.full((h, w, 4), 7.0, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(15):
            m = m @ m * 1e-3
        img.fill_(-1.0)
        rt.render_device(gpu_ctx, sc, img.data_ptr(), w, h, depth, view=view)  # NULL stream: synchronous
        ref = port.render(objs, w, h, depth, 0.0, rows=(538, 540))
        assert np.array_equal(img[538:540].cpu().numpy(), ref)
    finally:
        sc.close()


@pytest.mark.parametrize("fmt", [rt.abi.RT_OUTPUT_RGBA32F, rt.abi.RT_OUTPUT_RGB32F, rt.abi.RT_OUTPUT_RGBA8])
def test_render_returns_the_context_surface_format(gpu_ctx, fmt):
    """rt.render() sizes its host array from the context's surface format
    (RT_OPT_OUTPUT): float RGBA, packed float RGB or GL_RGBA8 bytes."""
    objs = scenes.bench_objects(16)
    w, h = 200, 120
    view = rt.make_view(None, 0.0)
    sc = rt.Scene(gpu_ctx, objs)
    try:
        ref = rt.render(gpu_ctx, sc, w, h, 1, view=view)
        gpu_ctx.set_output(fmt)
        got = rt.render(gpu_ctx, sc, w, h, 1, view=view, rows=(10, 90))
    finally:
        gpu_ctx.set_output(rt.abi.RT_OUTPUT_RGBA32F)
        sc.close()
    if fmt == rt.abi.RT_OUTPUT_RGBA8:
        assert got.dtype == np.uint8 and got.shape == (80, w, 4)
        assert np.array_equal(got, rt.pack_rgba8(ref[10:90]))
    elif fmt == rt.abi.RT_OUTPUT_RGB32F:
        assert got.dtype == np.float32 and got.shape == (80, w, 3)
        assert np.array_equal(got, ref[10:90, :, :3])
    else:
        assert np.array_equal(got, ref[10:90])


@pytest.mark.parametrize("fmt,block", [(rt.abi.RT_OUTPUT_RGBA32F, 8), (rt.abi.RT_OUTPUT_RGB32F, 3),
                                       (rt.abi.RT_OUTPUT_RGBA8, 8)])
def test_multi_gpu_group_equals_single_frame(fmt, block):
    """rt_render_multi (include/rt.h): the frame's interleaved row blocks on
    three contexts (peer-copy transport: the three share this box's one GPU),
    gathered to the root and de-interleaved — bit-identical to rt_render of
    the whole frame, host and device destinations, every surface format."""
    build, _, _, depth = scenes.CONFIGS["config4"]
    objs = build()
    w, h = 768, 437  # odd height: the last block is partial
    view = rt.make_view(None, 0.0)
    ctxs = [rt.Context(0) for _ in range(3)]
    scs = [rt.Scene(c, objs) for c in ctxs]
    try:
        for c in ctxs:
            c.set_output(fmt)
        whole = rt.render(ctxs[0], scs[0], w, h, depth, view=view)
        group = rt.Multi(ctxs, transport=rt.abi.RT_MULTI_COPY)
        try:
            got = group.render(scs, w, h, depth, view=view, block_rows=block)
            assert np.array_equal(got, whole)
            dt = torch.uint8 if fmt == rt.abi.RT_OUTPUT_RGBA8 else torch.float32
            dev = dev_zeros(whole.shape, dtype=dt, device="cuda")
            group.render_device(scs, dev.data_ptr(), w, h, depth, view=view, block_rows=block)
            assert np.array_equal(dev.cpu().numpy(), whole)
            k, g, a = group.last_ms()
            assert len(k) == 3 and all(v > 0 for v in k) and g >= 0 and a > 0
            # the reference orbit camera at `time` (rt_render_multi, cam = NULL)
            assert np.array_equal(group.render(scs, w, h, depth, time=0.0, block_rows=block), whole)
        finally:
            group.close()
    finally:
        for s in scs:
            s.close()
        for c in ctxs:
            c.close()


def test_multi_gpu_group_rccl_transport():
    """The RCCL transport (ncclCommInitAll over the contexts' devices, grouped
    ncclSend / ncclRecv to the root, rt_multi.hip): one context on every GPU
    of the box; bit-identical to the single-GPU frame, and the gather moved
    the shards (its time is measured). Needs two devices: on a one-GPU box
    the send / receive loop would not run, so the test is skipped there
    rather than reported as covering it."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("the RCCL transport needs at least 2 GPUs (this box has %d)" % n)
    objs = scenes.bench_objects(64)
    w, h, depth = 640, 360, 2
    view = rt.make_view(None, 0.0)
    ctxs = [rt.Context(d) for d in range(n)]
    scs = [rt.Scene(c, objs) for c in ctxs]
    try:
        whole = rt.render(ctxs[0], scs[0], w, h, depth, view=view)
        group = rt.Multi(ctxs, transport=rt.abi.RT_MULTI_RCCL)
        try:
            for block in (8, 16):
                assert np.array_equal(group.render(scs, w, h, depth, view=view, block_rows=block), whole)
                kms, gather_ms, _ = group.last_ms()
                assert gather_ms > 0.0 and all(k > 0.0 for k in kms[:n])
        finally:
            group.close()
    finally:
        for s in scs:
            s.close()
        for c in ctxs:
            c.close()


def test_multi_gpu_group_rccl_refuses_shared_device():
    """RCCL needs distinct devices: two contexts on one device are refused
    (the COPY transport serves them, test_multi_gpu_group_equals_single_frame)."""
    a, b = rt.Context(0), rt.Context(0)
    try:
        with pytest.raises(rt.RTError) as e:
            rt.Multi([a, b], transport=rt.abi.RT_MULTI_RCCL)
        assert e.value.code == rt.abi.RT_ERR_INVALID
    finally:
        a.close()
        b.close()


def test_scene_destroy_right_after_async_render_on_a_torch_stream(gpu_ctx):
    """rt_scene_destroy frees the blob in stream order on the context's
    stream behind the renders of it on other streams (an event per stream,
    rt_api.cpp note_scene_use): destroying a scene right after an
    asynchronous render on a torch stream, then creating a new scene (which
    may reuse the memory) and rendering it, leaves both frames intact."""
    objs_a, objs_b = scenes.bench_objects(64), scenes.bench_objects(64, 7)
    w, h, depth = 1920, 1080, 2
    view = rt.make_view(None, 0.0)
    want_a = gpu_render(gpu_ctx, objs_a, w, h, depth, view)
    want_b = gpu_render(gpu_ctx, objs_b, w, h, depth, view)
    s = torch.cuda.Stream()
    for _ in range(3):
        out_a = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        out_b = torch.empty_like(out_a)
        sa = rt.Scene(gpu_ctx, objs_a)
        rt.render_device(gpu_ctx, sa, out_a.data_ptr(), w, h, depth, view=view, stream=s.cuda_stream)
        sa.close()  # the render above may still be running on `s`
        sb = rt.Scene(gpu_ctx, objs_b)
        rt.render_device(gpu_ctx, sb, out_b.data_ptr(), w, h, depth, view=view, stream=s.cuda_stream)
        s.synchronize()
        sb.close()
        assert np.array_equal(out_a.cpu().numpy(), want_a)
        assert np.array_equal(out_b.cpu().numpy(), want_b)


def test_scene_update_waits_for_renders_on_other_streams(gpu_ctx):
    """rt_scene_update overwrites the blob only after the renders of it on
    any stream have finished."""
    objs_a, objs_b = scenes.bench_objects(64), scenes.bench_objects(64, 7)
    w, h, depth = 1920, 1080, 2
    view = rt.make_view(None, 0.0)
    want_a = gpu_render(gpu_ctx, objs_a, w, h, depth, view)
    s = torch.cuda.Stream()
    sc = rt.Scene(gpu_ctx, objs_a)
    try:
        out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_device(gpu_ctx, sc, out.data_ptr(), w, h, depth, view=view, stream=s.cuda_stream)
        sc.update(objs_b)
        s.synchronize()
        assert np.array_equal(out.cpu().numpy(), want_a)
    finally:
        sc.close()


def test_scene_used_on_more_than_eight_streams(gpu_ctx):
    """Past rt_scene::kMaxUseStreams (8) distinct caller streams the scene
    stops recording per-stream events and rt_scene_update / rt_scene_destroy
    fall back to a device-wide synchronisation (rt.h): renders queued on 10
    torch streams, then an update and a destroy right behind them, leave
    every frame intact."""
    objs_a, objs_b = scenes.bench_objects(64), scenes.bench_objects(64, 7)
    w, h, depth = 640, 360, 2
    view = rt.make_view(None, 0.0)
    want_a = gpu_render(gpu_ctx, objs_a, w, h, depth, view)
    want_b = gpu_render(gpu_ctx, objs_b, w, h, depth, view)
    streams = [torch.cuda.Stream() for _ in range(10)]
    sc = rt.Scene(gpu_ctx, objs_a)
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in streams]
    for o, s in zip(outs, streams):
        rt.render_device(gpu_ctx, sc, o.data_ptr(), w, h, depth, view=view, stream=s.cuda_stream)
    sc.update(objs_b)  # must wait for all ten renders of objs_a
    outs_b = [torch.empty_like(outs[0]) for _ in streams]
    for o, s in zip(outs_b, streams):
        rt.render_device(gpu_ctx, sc, o.data_ptr(), w, h, depth, view=view, stream=s.cuda_stream)
    sc.close()  # the renders of objs_b may still be running
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), want_a)
    for o in outs_b:
        assert np.array_equal(o.cpu().numpy(), want_b)


def test_concurrent_batches_on_several_streams(gpu_ctx):
    """Batches in flight together on three caller streams, none waiting for
    another: queued deep batches (their queue-counter slots, kSchedSlots) and
    depth-0 batches of more than 8 views (the device view ring, kBatchSlots),
    several rounds, so every slot is reused while other launches run — each
    frame bit-identical to its single render."""
    objs = scenes.bench_objects(64)
    w, h = 640, 360
    views = [rt.make_view(None, 0.3 + k / 40.0) for k in range(12)]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        want = {d: [rt.render(gpu_ctx, sc, w, h, d, view=v) for v in views] for d in (0, 2)}
        streams = [torch.cuda.Stream() for _ in range(3)]
        jobs = []
        for rnd in range(4):
            for i, st in enumerate(streams):
                depth = 2 if (rnd + i) % 2 == 0 else 0
                nv = 5 if depth == 2 else 12
                out = dev_zeros((nv, h, w, 4), dtype=torch.float32, device="cuda")
                rt.render_batch(gpu_ctx, sc, out.data_ptr(), w, h, depth, views[:nv], stream=st.cuda_stream)
                jobs.append((depth, nv, out))
        torch.cuda.synchronize()
        for depth, nv, out in jobs:
            got = out.cpu().numpy()
            for k in range(nv):
                assert np.array_equal(got[k], want[depth][k]), (depth, k)
    finally:
        sc.close()


STRAT = __import__("conftest").strat_manifest()


@pytest.mark.parametrize("name", sorted(STRAT))
def test_stratified_crops_product_path_matches_gl(gpu_ctx, name):
    """rt_render(cam = NULL, time) — the product path — against the
    stratified llvmpipe crops of configs 3 and 4 (a grid over the whole
    frame with its edges and corners, plus the most glass-heavy crops,
    tests/golden/make_strat_golden.py): bit-exact on every pixel; and the
    kernel equals the oracle on every full row band the crops lie in."""
    from conftest import load_strat, row_bands
    m = STRAT[name]
    rgb, crops, _ = load_strat(name)
    objs = scenes.CONFIGS[m["scene"]][0]()
    w, h, depth = m["width"], m["height"], m["max_depth"]
    sc = rt.Scene(gpu_ctx, objs)
    try:
        bands = {}
        for r0, r1 in row_bands(crops):
            out = np.zeros((r1 - r0, w, 4), np.float32)
            rc = rt.lib().rt_render(gpu_ctx.handle, sc.handle, None, m["time"], w, h, depth, r0, r1,
                                    out.ctypes.data, 0, None)
            assert rc == 0, rt.lib().rt_last_error()
            bands[(r0, r1)] = out
    finally:
        sc.close()
    for k, (x0, y0, cw, ch) in enumerate(crops):
        g = bands[(int(y0), int(y0 + ch))][:, x0:x0 + cw]
        assert (g[..., 3] == 0).all()
        s = parity_stats(g, rgb[k])
        assert s["exact"] == 1.0, (name, k, (x0, y0, cw, ch), s)
    for (r0, r1), g in bands.items():
        o = oracle_render(objs, w, h, depth, m["time"], rows=(r0, r1))
        assert np.array_equal(g, o), (name, r0, parity_stats(g, o))


# ---- randomised scenes ------------------------------------------------------
def random_scene(seed):
    """A seeded random scene: the room box or not, up to 3 extra rotated
    boxes, 0-300 spheres (LDS direction masks, wide masks with candidate
    lists and their overflow, per-wave shadow cones, the BVH), the reference
    materials plus 2 random ones (mirrors, glass of random index, emissive,
    shininess), 1-4 random lights (some dead: no diffuse / specular), the
    reference orbit camera at a random time, a ragged frame and depth 0-5."""
    rng = np.random.default_rng(1000 + seed)
    mats = rt.reference_materials()
    for _ in range(2):
        m = rt.abi.Material()
        m.ambient[:] = rng.uniform(0.0, 0.4, 4)
        m.diffuse[:] = rng.uniform(0.0, 1.0, 4)
        m.specular[:] = rng.uniform(0.0, 1.0, 4)
        m.shininess = float(rng.uniform(1.0, 120.0))
        m.emissive[:] = rng.uniform(0.0, 0.3, 4) if rng.random() < 0.3 else (0.0, 0.0, 0.0, 0.0)
        m.reflectivity = float(rng.choice([0.0, 0.3, 1.0, rng.uniform(0.0, 1.0)]))
        m.transparency = float(rng.choice([0.0, 0.5, rng.uniform(0.0, 1.0)]))
        m.refraction_index = float(rng.uniform(1.0, 2.5))
        mats.append(m)
    lights = []
    for _ in range(int(rng.integers(1, 5))):
        lt = rt.abi.Light()
        lt.position[:] = rng.uniform(-9.0, 9.0, 3)
        lt.ambient[:] = rng.uniform(0.0, 0.2, 4)
        if rng.random() < 0.25:  # dead: ambient only
            lt.diffuse[:] = (0.0, 0.0, 0.0, 0.0)
            lt.specular[:] = (0.0, 0.0, 0.0, 0.0)
        else:
            lt.diffuse[:] = rng.uniform(0.0, 1.0, 4)
            lt.specular[:] = rng.uniform(0.0, 1.0, 4)
        lights.append(lt)
    objs = [scenes.room_box()] if rng.random() < 0.8 else []
    for _ in range(int(rng.integers(0, 4))):
        objs.append(scenes.box(tuple(-rng.uniform(0.2, 2.0, 3)), tuple(rng.uniform(0.2, 2.0, 3)),
                               tuple(rng.uniform(-6.0, 6.0, 3)), tuple(rng.uniform(0.0, 360.0, 3)),
                               int(rng.integers(len(mats)))))
    n_sph = int(rng.choice([0, 5, 16, 40, 64, 100, 256, 300]))
    for _ in range(n_sph):
        objs.append(scenes.sphere(tuple(rng.uniform(-8.0, 8.0, 3)), float(rng.uniform(0.1, 1.5)),
                                  int(rng.integers(len(mats)))))
    t = float(rng.uniform(0.0, 20.0))
    depth = int(rng.integers(0, 6)) if n_sph <= 64 else int(rng.integers(0, 4))
    w, h = int(rng.integers(24, 100)), int(rng.integers(16, 70))
    return objs, mats, lights, t, depth, w, h


@pytest.mark.parametrize("seed", range(32))
def test_random_scenes_match_oracle(gpu_ctx, seed):
    """Seeded random scenes (random_scene), the product camera path at a
    random time: bit-exact against the oracle, culling on and off."""
    objs, mats, lights, t, depth, w, h = random_scene(seed)
    view = rt.make_view(None, t)
    sc = rt.Scene(gpu_ctx, objs, materials=mats, lights=lights)
    try:
        g = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        gpu_ctx.set_culling(False)
        off = rt.render(gpu_ctx, sc, w, h, depth, view=view)
    finally:
        gpu_ctx.set_culling(True)
        sc.close()
    o = oracle_render(objs, w, h, depth, t, materials=mats, lights=lights)
    desc = (seed, len(objs), len(lights), depth, w, h, round(t, 3))
    assert np.array_equal(g, o, equal_nan=True), (desc, parity_stats(g, o))
    assert np.array_equal(off, o, equal_nan=True), (desc, parity_stats(off, o))


@pytest.mark.parametrize("seed", range(8))
def test_random_scenes_batch_shards_rgba8_and_mc(gpu_ctx, seed):
    """The same random scenes through the other launch shapes: three animated
    views in one launch equal three single renders; interleaved row shards
    reassemble the frame; the GL_RGBA8 surface equals rt_pack_rgba8 of the
    float frame; two Monte-Carlo calls of 2 samples equal the oracle's
    in-order sums."""
    objs, mats, lights, t, depth, w, h = random_scene(seed)
    times = [t, t + 0.5, t + 1.25]
    views = [rt.make_view(None, x) for x in times]
    sc = rt.Scene(gpu_ctx, objs, materials=mats, lights=lights)
    try:
        singles = [rt.render(gpu_ctx, sc, w, h, depth, view=v) for v in views]
        batch = dev_zeros((3, h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch(gpu_ctx, sc, batch.data_ptr(), w, h, depth, views)
        torch.cuda.synchronize()
        for k in range(3):
            assert np.array_equal(batch[k].cpu().numpy(), singles[k], equal_nan=True), (seed, k)
        n = 3
        got = np.zeros_like(singles[0])
        for s in range(n):
            buf = dev_zeros(rt.shard_rows(h, 4, n, s) * w * 4, dtype=torch.float32, device="cuda")
            rt.render_shard(gpu_ctx, sc, buf.data_ptr(), w, h, depth, 4, n, s, view=views[0])
            torch.cuda.synchronize()
            got[frame.shard_row_ids(h, 4, n, s)] = buf.cpu().numpy().reshape(-1, w, 4)
        assert np.array_equal(got, singles[0], equal_nan=True), seed
        assert np.array_equal(rt.render_rgba8(gpu_ctx, sc, w, h, depth, view=views[0]), rt.pack_rgba8(singles[0]))
        if depth <= 2:
            acc = dev_zeros((h, w, 4), dtype=torch.float32, device="cuda")
            rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, depth, 2, 0, seed=seed, view=views[0])
            rt.render_accumulate(gpu_ctx, sc, acc.data_ptr(), w, h, depth, 2, 2, seed=seed, view=views[0])
            torch.cuda.synchronize()
            o = port.render_accumulate(objs, w, h, depth, 2, 0, seed=seed, time=times[0], materials=mats,
                                       lights=lights)
            o = port.render_accumulate(objs, w, h, depth, 2, 2, seed=seed, accum=o, time=times[0], materials=mats,
                                       lights=lights)
            assert np.array_equal(acc.cpu().numpy(), o, equal_nan=True), (seed, parity_stats(acc.cpu().numpy(), o))
    finally:
        sc.close()


def box_scene(seed):
    """A seeded scene of many oriented boxes (round 6: the slab pre-test,
    slab_may_hit): the room or not, 4-12 rotated boxes of random extents
    (thin slabs, long bars, cubes; some around the orbit camera's path, some
    holding a light), 0-8 spheres, 1-3 lights, the reference materials; the
    shipped scene's kind of work (raytrace_compute.glsl:261-321) with more of
    it."""
    rng = np.random.default_rng(5000 + seed)
    mats = rt.reference_materials()
    lights = []
    for _ in range(int(rng.integers(1, 4))):
        lt = rt.abi.Light()
        lt.position[:] = rng.uniform(-8.0, 8.0, 3)
        lt.ambient[:] = rng.uniform(0.0, 0.2, 4)
        lt.diffuse[:] = rng.uniform(0.2, 1.0, 4)
        lt.specular[:] = rng.uniform(0.2, 1.0, 4)
        lights.append(lt)
    objs = [scenes.room_box()] if rng.random() < 0.7 else []
    for _ in range(int(rng.integers(4, 13))):
        kind = rng.integers(3)
        ext = (rng.uniform(0.5, 6.0, 3) * np.array([1.0, 1.0, 0.05]) if kind == 0 else
               rng.uniform(0.1, 0.6, 3) * np.array([1.0, 1.0, 12.0]) if kind == 1 else rng.uniform(0.2, 2.5, 3))
        objs.append(scenes.box(tuple(-ext), tuple(ext * rng.uniform(0.5, 1.0, 3)), tuple(rng.uniform(-7.0, 7.0, 3)),
                               tuple(rng.uniform(0.0, 360.0, 3)), int(rng.integers(len(mats)))))
    for _ in range(int(rng.integers(0, 9))):
        objs.append(scenes.sphere(tuple(rng.uniform(-7.0, 7.0, 3)), float(rng.uniform(0.2, 1.2)),
                                  int(rng.integers(len(mats)))))
    t = float(rng.uniform(0.0, 20.0))
    return objs, mats, lights, t, int(rng.integers(0, 4)), int(rng.integers(48, 128)), int(rng.integers(32, 80))


@pytest.mark.parametrize("seed", range(16))
def test_box_scenes_match_oracle(gpu_ctx, seed):
    """Many oriented boxes: the conservative slab pre-test (approximate
    reciprocals, 2^-19 margins) in front of the exact six-division box test,
    for primary, secondary and shadow rays, leaves every pixel bit-identical
    to the oracle, with culling on (pre-test) and off (every box tested)."""
    objs, mats, lights, t, depth, w, h = box_scene(seed)
    view = rt.make_view(None, t)
    sc = rt.Scene(gpu_ctx, objs, materials=mats, lights=lights)
    try:
        g = rt.render(gpu_ctx, sc, w, h, depth, view=view)
        gpu_ctx.set_culling(False)
        off = rt.render(gpu_ctx, sc, w, h, depth, view=view)
    finally:
        gpu_ctx.set_culling(True)
        sc.close()
    o = oracle_render(objs, w, h, depth, t, materials=mats, lights=lights)
    desc = (seed, len(objs), len(lights), depth, w, h, round(t, 3))
    assert np.array_equal(g, o, equal_nan=True), (desc, parity_stats(g, o))
    assert np.array_equal(off, o, equal_nan=True), (desc, parity_stats(off, o))


def test_shipped_scene_animated_batch_full_frames(gpu_ctx):
    """The shipped workload's launch (bench.py --workload shipped): 1280x720
    frames of the reference's own animated scene, each view with its own
    scene in one rt_render_batch_scenes launch, bit-identical to the oracle
    on bands of rows of three of the frames (t = 0, 2.1, 4.25 s)."""
    times = [0.0, 2.1, 4.25]
    w, h = 1280, 720
    scs = [rt.Scene(gpu_ctx, rt.reference_objects(x)) for x in times]
    try:
        out = dev_zeros((len(times), h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch_scenes(gpu_ctx, scs, out.data_ptr(), w, h, 0, [rt.make_view(None, x) for x in times])
        torch.cuda.synchronize()
        got = out.cpu().numpy()
    finally:
        for s in scs:
            s.close()
    for k, x in enumerate(times):
        for r0, r1 in [(0, 4), (300, 308), (716, 720)]:
            o = oracle_render(rt.reference_objects(x), w, h, 0, x, rows=(r0, r1))
            assert np.array_equal(got[k, r0:r1], o), (x, r0, parity_stats(got[k, r0:r1], o))


def test_origin_lists_built_on_first_deep_render(gpu_ctx):
    """The origin-sphere lists are not built by rt_scene_create or
    rt_scene_update but by the first render that reads them (depth >= 2, a
    33-256-sphere scene), appended to the device blob (rt_api.cpp
    ensure_origin_lists): a depth-0 render first, then depth 2, then an
    update to another scene of the same size and depth 2 again, and a batch
    of two such scenes; every frame bit-identical to the oracle."""
    w, h = 192, 108
    a, b = scenes.bench_objects(100, seed=11), scenes.bench_objects(100, seed=12)
    sc = rt.Scene(gpu_ctx, a)
    sb = rt.Scene(gpu_ctx, a)
    try:
        f0 = rt.render(gpu_ctx, sc, w, h, 0, time=0.5)
        assert np.array_equal(f0, oracle_render(a, w, h, 0, 0.5))
        f2 = rt.render(gpu_ctx, sc, w, h, 2, time=0.5)
        assert np.array_equal(f2, oracle_render(a, w, h, 2, 0.5)), parity_stats(f2, oracle_render(a, w, h, 2, 0.5))
        sc.update(b)
        g2 = rt.render(gpu_ctx, sc, w, h, 2, time=1.5)
        ob = oracle_render(b, w, h, 2, 1.5)
        assert np.array_equal(g2, ob), parity_stats(g2, ob)
        sc.update(a)  # back: the lists of the new contents again
        # a batch of two scenes of one layout (the same objects), one of them
        # never rendered: its lists are built by the batch call
        views = [rt.make_view(None, 0.5), rt.make_view(None, 2.5)]
        out = dev_zeros((2, h, w, 4), dtype=torch.float32, device="cuda")
        rt.render_batch_scenes(gpu_ctx, [sc, sb], out.data_ptr(), w, h, 2, views)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert np.array_equal(got[0], f2)
        oa = oracle_render(a, w, h, 2, 2.5)
        assert np.array_equal(got[1], oa), parity_stats(got[1], oa)
    finally:
        sc.close()
        sb.close()
