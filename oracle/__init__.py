"""Oracle package — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker. The product (openglraytracer_amd/) never imports it.

  oracle.port    ctypes front-end of the C float32 restatement (rt_oracle.c)
  oracle.glref   ctypes front-end of the llvmpipe harness that runs the
                 reference's own GLSL (glref/glref.c; needs oracle/_ref)
  oracle.scenes  the benchmark scenes restated in Python
"""
