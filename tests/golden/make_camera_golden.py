"""Golden vectors of the reference's camera, from the reference itself (dev container).

The reference computes its orbiting camera per invocation
(raytrace_compute.glsl:334-392): view_mat = calc_view_matrix(c) (:538-545),
proj_mat = calc_projection_matrix(c) (:411-426), inverse(proj_mat * view_mat)
(:383), camera position c.position (:343-344). This script builds a probe
compute shader AT RUN TIME from the reference's own function text
(calc_projection_matrix, translation_matrix, rotation_matrix_x/y/z,
rotation_matrix, calc_transform_matrix, calc_view_matrix, copied out of
/root/reference/OpenGLRaytracer/raytrace_compute.glsl into the shader string,
never into the repository) plus a main() that repeats main()'s camera lines
(:336-367) for time = T0 + i * 0.7310585 on invocation row i, and runs it on
Mesa llvmpipe (oracle/glref, the harness the golden frames come from).

Writes tests/golden/camera_llvmpipe.npz: float32 `time` (N,), `view` (N, 16),
`pv` (N, 16), `unproj` (N, 16) (column-major, m[col][row] at col*4+row) and
`position` (N, 3). rt_make_view(NULL, time) and the oracle must reproduce
every entry bit for bit (tests/test_host.py, tests/test_oracle_golden.py).

    python tests/golden/make_camera_golden.py      # needs oracle/_ref (make -C oracle ref)
"""
import ctypes as C
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import glref  # noqa: E402

REFERENCE = "/root/reference/OpenGLRaytracer/raytrace_compute.glsl"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "camera_llvmpipe.npz")
FUNCTIONS = ["mat4 calc_projection_matrix(Camera c)", "mat4 translation_matrix(vec3 t)",
             "mat4 rotation_matrix_x(float deg)", "mat4 rotation_matrix_y(float deg)",
             "mat4 rotation_matrix_z(float deg)", "mat4 rotation_matrix(vec3 r)",
             "mat4 calc_transform_matrix(vec3 position, vec3 angles)", "mat4 calc_view_matrix(Camera c)"]
# (T0, rows): negative, zero, animated and large times
RUNS = [(0.0, 200), (-100.0, 100), (0.016666668, 100), (137.5, 100), (1.0e4, 100)]
N_OUT = 51  # view 16, pv 16, unproj 16, position 3

MAIN = r"""
struct Camera { vec3 position; vec3 angles; float v_fov; float aspect; float near; float far; };
%s
void main()
{
    int i = int(gl_GlobalInvocationID.y);
    int e = int(gl_GlobalInvocationID.x);
    float t = time + float(i) * 0.7310585;
    Camera c;
    float radius = 10.0;
    float speed = t * time_scale + 0.5;
    c.position = vec3(radius * cos(speed), radius * sin(speed), 0);
    float pitch = 0.0;
    float yaw = 0.0;
    float roll = 0.0;
    yaw = mod(1.0 * speed * (180.0/3.1416), 360.0) + 90.0;
    c.angles = vec3(pitch,yaw,roll);
    c.near = 0.1;
    c.far = 1000;
    c.aspect = 16.0/9.0;
    c.v_fov = 90.0;
    mat4 proj_mat = calc_projection_matrix(c);
    mat4 view_mat = calc_view_matrix(c);
    mat4 inverse_proj_mat = inverse(proj_mat * view_mat);
    mat4 pv = proj_mat * view_mat;
    int k = e %% 16;
    float v = 0.0;
    if (e < 16) v = view_mat[k / 4][k %% 4];
    else if (e < 32) v = pv[k / 4][k %% 4];
    else if (e < 48) v = inverse_proj_mat[k / 4][k %% 4];
    else v = c.position[e - 48];
    imageStore(output_texture, ivec2(e, i), vec4(v, 0.0, 0.0, 0.0));
}
"""
HEADER = """#version 430
uniform float time;
writeonly uniform image2D output_texture;
layout (local_size_x = 1, local_size_y = 1) in;
const float PI = 3.14159265358;
const float DEG_TO_RAD = PI / 180.0;
float time_scale = 0.4;
"""


def reference_functions():
    src = open(REFERENCE).read()
    out = []
    for sig in FUNCTIONS:
        m = re.search(re.escape(sig) + r"\s*\n\{", src)
        if not m:
            raise SystemExit("function not found in the reference: " + sig)
        out.append(src[m.start():src.index("\n}", m.start()) + 2])
    return "\n".join(out)


def main():
    lib = glref.lib()
    lib.glref_run_source.argtypes = [C.c_char_p, C.c_float, C.c_int, C.c_int, C.c_void_p]
    prog = HEADER + MAIN % reference_functions()
    times, rows = [], []
    for t0, n in RUNS:
        out = np.zeros((n, N_OUT, 4), np.float32)
        if lib.glref_run_source(prog.encode(), C.c_float(t0), N_OUT, n, out.ctypes.data) != 0:
            raise SystemExit("glref: " + lib.glref_last_error().decode())
        rows.append(out[..., 0])
        # the shader's time: t0 + float(i) * 0.7310585 in float32
        times.append(np.float32(t0) + np.arange(n, dtype=np.float32) * np.float32(0.7310585))
    data = np.concatenate(rows)
    np.savez_compressed(OUT, time=np.concatenate(times).astype(np.float32), view=data[:, 0:16], pv=data[:, 16:32],
                        unproj=data[:, 32:48], position=data[:, 48:51], renderer=np.array(glref.renderer()))
    print("wrote %s: %d camera samples (%s)" % (OUT, data.shape[0], glref.renderer()))


if __name__ == "__main__":
    main()
