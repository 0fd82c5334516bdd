import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_fixture(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return z["rgb"], z["unproj"].astype(np.float32)


def fixture_objects(meta, reference_objects):
    """Objects of a fixture: the shipped scene at its time, or a bench config."""
    from oracle import scenes
    if meta["scene"] == "shipped":
        return reference_objects(meta["time"])
    return scenes.CONFIGS[meta["scene"]][0]()


def parity_stats(a, b):
    """Per-pixel max-over-channel |a-b| statistics (RGB)."""
    d = np.abs(a[..., :3].astype(np.float64) - b[..., :3].astype(np.float64))
    pm = d.max(-1)
    return {"exact": float((pm == 0).mean()), "max": float(pm.max()), "mean": float(d.mean()),
            "p99": float(np.percentile(pm, 99)), "frac_gt_1e5": float((pm > 1e-5).mean()),
            "flips": int((pm > 1e-3).sum()), "n": int(pm.size)}


# The parity tolerances (north_star: per-channel 1e-5; BASELINE.md criterion
# for independently computed frame constants).
TOL = 1e-5
MAX_OUTLIER_FRAC = 1e-4  # <= 0.01% pixels beyond TOL ("discrete flips")


@pytest.fixture(scope="session")
def gpu_ctx():
    import openglraytracer_amd as rt
    ctx = rt.Context(0)
    yield ctx
    ctx.close()


def dev_zeros(*shape, dtype=None, device="cuda"):
    """A zero-filled device tensor whose fill has completed. Since round 5 a
    NULL-stream call is ordered after torch's default stream by the library
    itself (its context stream is a blocking HIP stream, include/rt.h), so
    this only matters for fills queued on other torch streams; the
    Monte-Carlo tests use plain torch.zeros on purpose."""
    import torch
    t = torch.zeros(*shape, dtype=dtype, device=device)
    torch.cuda.synchronize()
    return t


def synced_zero_(t):
    """t.zero_() completed before the next library call (see dev_zeros)."""
    import torch
    t.zero_()
    torch.cuda.synchronize()
    return t


def strat_manifest():
    """Stratified crop sets of the deep configs (tests/golden/make_strat_golden.py)."""
    with open(os.path.join(GOLDEN, "strat_manifest.json")) as f:
        return json.load(f)


def load_strat(name):
    """(rgb (n, h, w, 3), crops (n, 4) of (x0, y0, w, h), unproj (4, 4))."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return z["rgb"], z["crops"], z["unproj"].astype(np.float32)


def row_bands(crops):
    """The distinct row ranges (y0, y0 + h) of a crop set."""
    return sorted({(int(c[1]), int(c[1] + c[3])) for c in crops})
