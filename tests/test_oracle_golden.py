"""The oracle (C float32 restatement) against the reference itself.

Golden fixtures are llvmpipe renders of the reference's own
raytrace_compute.glsl (tests/golden/make_golden.py). Two comparisons:

* pinned frame constants: the oracle uses llvmpipe's own inverse(proj*view)
  (stored in each fixture) — isolates the per-pixel restatement;
* the oracle's own frame constants: the reference orbit camera evaluated as
  llvmpipe compiles it (rt_oracle.c gl_reference_matrices; pinned by the
  camera golden vectors, tests/golden/make_camera_golden.py).
Both are bit-exact on every fixture: the benchmark scenes and the shipped
scene, whose rotated, animated boxes carry their transforms as llvmpipe
evaluates them (rt_oracle.c gl_object_transforms; pinned by the box golden
vectors, tests/golden/make_box_golden.py).
"""
import os
import ctypes as C

import numpy as np
import pytest

from conftest import MAX_OUTLIER_FRAC, TOL, fixture_objects, load_fixture, manifest, parity_stats
from oracle import port

MAN = manifest()
COLOUR = sorted(n for n, m in MAN.items() if m["probe"] == 0)
ALL = sorted(MAN)


def oracle_fixture(name, pinned):
    m = MAN[name]
    rgb, unproj = load_fixture(name)
    x0, y0, w, h = m["crop"]
    objs = fixture_objects(m, port.reference_objects)
    if pinned:
        port.lib().oracle_pin_unprojection(unproj.ctypes.data_as(C.c_void_p))
    try:
        out = port.render(objs, m["width"], m["height"], m["max_depth"], m["time"], rows=(y0, y0 + h),
                          probe=m["probe"])[:, x0:x0 + w]
    finally:
        port.lib().oracle_pin_unprojection(None)
    return out, rgb


@pytest.mark.parametrize("name", ALL)
def test_pinned_within_tolerance(name):
    out, rgb = oracle_fixture(name, pinned=True)
    s = parity_stats(out, rgb)
    assert s["frac_gt_1e5"] <= MAX_OUTLIER_FRAC and s["max"] <= 1e-4, s
    assert s["mean"] <= 1e-6, s


@pytest.mark.parametrize("name", ALL)
def test_pinned_bit_exact(name):
    out, rgb = oracle_fixture(name, pinned=True)
    s = parity_stats(out, rgb)
    assert s["exact"] == 1.0, s


@pytest.mark.parametrize("name", COLOUR)
def test_own_frame_constants(name):
    """The oracle's own camera (no pinned matrix) against the reference's
    render: bit-exact on every fixture (configs 1-4, camera at t = 0 and
    moved; the shipped scene at t = 0, 3.7, 11.25)."""
    out, rgb = oracle_fixture(name, pinned=False)
    s = parity_stats(out, rgb)
    assert s["exact"] == 1.0, s


def test_probe_ray_direction_independent():
    out, rgb = oracle_fixture("probe_dir_t0_128", pinned=False)
    assert np.array_equal(out[..., :3], rgb)


def test_camera_matches_llvmpipe_golden_vectors():
    """oracle_camera_matrices(NULL, t): inverse(proj*view) bit for bit and
    view_mat equal (up to the sign of zero entries, which nothing consumes)
    to llvmpipe's at 600 camera times (tests/golden/camera_llvmpipe.npz)."""
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "camera_llvmpipe.npz"))
    out = np.zeros(48, np.float32)
    for i, t in enumerate(z["time"]):
        port.lib().oracle_camera_matrices(None, C.c_float(t), out.ctypes.data_as(C.c_void_p))
        assert np.array_equal(out[:16].view(np.uint32), z["unproj"][i].view(np.uint32)), float(t)
        assert np.array_equal(out[16:32], z["view"][i]), float(t)


def test_box_transforms_match_llvmpipe_golden_vectors():
    """oracle_object_transforms (an independent C restatement): the shipped
    scene's box transforms bit for bit against llvmpipe's at 32 times
    (tests/golden/box_llvmpipe.npz): rows 0-2, the entries the shader
    consumes, bit for bit; row 3 by value (two dead entries are -0.0 there)."""
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "box_llvmpipe.npz"))
    out = np.zeros(41, np.float32)
    used = np.array([r < 3 for c in range(4) for r in range(4)])
    for i, t in enumerate(z["time"]):
        objs = port.reference_objects(float(t))
        for k in range(4):
            port.lib().oracle_object_transforms(C.byref(objs[k]), out.ctypes.data_as(C.c_void_p))
            for name, mine in (("l2w", out[:16]), ("w2l", out[16:32]), ("nrm", out[32:41])):
                ref = z[name][i, k]
                bitwise = used if name != "nrm" else np.ones(9, bool)
                assert np.array_equal(mine[bitwise].view(np.uint32), ref[bitwise].view(np.uint32)), (float(t), k, name)
                assert np.array_equal(mine, ref), (float(t), k, name)


def test_probe_hit_object_and_shadow_mask_match():
    out, rgb = oracle_fixture("probe_hit_t0_128", pinned=True)
    assert np.array_equal(out[..., 0], rgb[..., 0])  # object index
    assert np.array_equal(out[..., 2], rgb[..., 2])  # shadow mask (:816)


def test_known_answers_shipped_scene():
    """SURVEY.md §8(c) known answers (shipped scene, t=0, 256x256, depth 0)."""
    rgb, _ = load_fixture("shipped_t0_d0_256")
    kat = {(0, 0): (0.6670141, 1.4770919, 0.6400700), (128, 128): (0.4878497, 0.3011093, 0.3011093),
           (255, 255): (0.5528139, 0.2689192, 0.2689192)}
    out = port.render(port.reference_objects(0.0), 256, 256, 0, 0.0)
    for (x, y), v in kat.items():
        assert np.allclose(rgb[y, x], v, atol=1e-6)
        assert np.allclose(out[y, x, :3], v, atol=TOL)


def test_stack_machine_red_guard_unreachable_below_depth_10():
    """The runaway guard (:1077-1101) needs > 10000 steps; a traced ray takes
    6, so depth <= 9 (<= 1023 rays) cannot trigger it: a depth-9 render of a
    scene of perfect mirrors and glass has no pure-red pixel."""
    from openglraytracer_amd.abi import Object
    from oracle import scenes
    objs = scenes.bench_objects(8)
    out = port.render(objs, 16, 9, 9, 0.0)
    red = (out[..., 0] == 1.0) & (out[..., 1] == 0.0) & (out[..., 2] == 0.0)
    assert not red.any()
    assert Object  # layout import sanity


def test_oracle_rejects_bad_arguments():
    with pytest.raises(ValueError):
        port.render(port.reference_objects(0.0), 0, 10)


STRAT = __import__("conftest").strat_manifest()


@pytest.mark.parametrize("name", sorted(STRAT))
def test_stratified_crops_bit_exact(name):
    """The oracle with its own frame constants against the stratified
    llvmpipe crops of configs 3 and 4 (tests/golden/make_strat_golden.py:
    a grid over the whole frame, edges and corners included, plus the most
    glass-heavy crops; depth-2 / depth-4 recursion, raytrace_compute.glsl:
    848-1105): bit-exact on every pixel."""
    from conftest import load_strat, row_bands
    from oracle import scenes
    m = STRAT[name]
    rgb, crops, _ = load_strat(name)
    objs = scenes.CONFIGS[m["scene"]][0]()
    bands = {b: port.render(objs, m["width"], m["height"], m["max_depth"], m["time"], rows=b) for b in row_bands(crops)}
    for k, (x0, y0, w, h) in enumerate(crops):
        got = bands[(int(y0), int(y0 + h))][:, x0:x0 + w]
        s = parity_stats(got, rgb[k])
        assert s["exact"] == 1.0, (name, k, (x0, y0, w, h), s)
