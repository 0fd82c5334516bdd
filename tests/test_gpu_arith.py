"""The short arithmetic forms the kernel relies on, re-checked on the GPU.

rt_kernel.hip replaces hipcc's IEEE division / square-root expansions by
shorter sequences that are only valid because of how gfx950's v_rcp_f32 and
v_sqrt_f32 behave ("Arithmetic, bit-exact by construction"):
the refined reciprocal is the correctly rounded 1/b for every significand,
so inversesqrt needs no quotient step and one correction gives the correctly
rounded quotient. tools/probes/arith_probe (built by build()) checks them
against the IEEE operations: every significand of [1, 4) exhaustively, and
random quotient pairs."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "probes", "arith_probe")


@pytest.mark.gpu
def test_short_division_and_square_root_forms_are_exact():
    assert os.path.exists(PROBE), "build() first (make -C openglraytracer_amd/csrc)"
    out = subprocess.run([PROBE, "quick"], capture_output=True, text=True, timeout=120, check=True).stdout
    line = re.search(r"\[1,4\)\s+n=(\d+)\s+raw_sqrt=\d+ sqrt_short=(\d+) raw_rcp=(\d+) rcp_refined=(\d+) "
                     r"invsqrt_short=(\d+)", out)
    assert line, out
    n, sqrt_short, raw_rcp, rcp_refined, invsqrt = map(int, line.groups())
    assert n == 1 << 24
    assert raw_rcp > 0  # the raw reciprocal is not exact: the refinement step is needed
    assert (sqrt_short, rcp_refined, invsqrt) == (0, 0, 0), out
    div = re.search(r"division emax=30 samples=(\d+) one_correction_bad=(\d+) two_corrections_bad=(\d+)", out)
    assert div, out
    samples, one, two = map(int, div.groups())
    assert samples >= 60_000_000 and one == 0 and two == 0, out
