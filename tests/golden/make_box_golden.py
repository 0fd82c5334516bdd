"""Golden vectors of the reference's box transforms, from the reference itself.

intersect_box_object (raytrace_compute.glsl:647-724) evaluates, per ray and
box object, local_to_world = calc_transform_matrix(o.position, o.angles)
(:650, :529-532), world_to_local = inverse(local_to_world) (:652) and the
normal matrix transpose(inverse(mat3(local_to_world))) (:718). The llvmpipe
harness (oracle/glref, probe 7) renders, for the shipped scene at `time`,
element [x % 4][y % 4] of the three matrices of object x / 4 — computed by the
reference's own functions on objects[k] with a run-time index, as in the
shader's object loop (:749-771).

Writes tests/golden/box_llvmpipe.npz: float32 `time` (N,), `l2w` (N, 5, 16),
`w2l` (N, 5, 16) (column-major, m[col][row] at col * 4 + row) and `nrm`
(N, 5, 9) (column-major 3x3). rt_object_transforms and the oracle must
reproduce every entry of the box objects (0-3) bit for bit
(tests/test_host.py, tests/test_oracle_golden.py).

    python tests/golden/make_box_golden.py      # needs oracle/_ref (make -C oracle ref)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import glref  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "box_llvmpipe.npz")
# the fixture times, negative and large times, and a seeded spread
TIMES = [0.0, 3.7, 11.25, -100.0, 1.0e4, 0.016666668, 137.5] + \
    [float(np.float32(t)) for t in np.random.default_rng(7).uniform(-50.0, 500.0, 25)]


def main():
    times, l2w, w2l, nrm = [], [], [], []
    for t in TIMES:
        out, _ = glref.render(None, 20, 4, max_depth=0, time=t, probe=7)  # out[y, x, channel]
        L = np.zeros((5, 4, 4), np.float32)
        W = np.zeros((5, 4, 4), np.float32)
        N = np.zeros((5, 3, 3), np.float32)
        for k in range(5):
            for c in range(4):
                for r in range(4):
                    L[k, c, r] = out[r, 4 * k + c, 0]
                    W[k, c, r] = out[r, 4 * k + c, 1]
                    if c < 3 and r < 3:
                        N[k, c, r] = out[r, 4 * k + c, 2]
        times.append(np.float32(t))
        l2w.append(L.reshape(5, 16))
        w2l.append(W.reshape(5, 16))
        nrm.append(N.reshape(5, 9))
    np.savez_compressed(OUT, time=np.array(times, np.float32), l2w=np.stack(l2w), w2l=np.stack(w2l),
                        nrm=np.stack(nrm), renderer=np.array(glref.renderer()))
    print("wrote %s: %d times x 5 objects (%s)" % (OUT, len(times), glref.renderer()))


if __name__ == "__main__":
    main()
