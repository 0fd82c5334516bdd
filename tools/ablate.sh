#!/bin/bash
# Timing-only ablation builds of the kernel (outputs are wrong by design):
# builds variants into build/ablate/<name>/ and times config 2 with each.
set -euo pipefail
cd "$(dirname "$0")/.."
for v in full:"" noshadow:"-DRT_ABLATE_SHADOW" nophong:"-DRT_ABLATE_PHONG" notrace:"-DRT_ABLATE_TRACE"; do
  name=${v%%:*}; flag=${v#*:}
  out=tools/_ablate/$name; mkdir -p $out/obj
  make -s -C openglraytracer_amd/csrc OBJDIR=$(pwd)/$out/obj OUT=$(pwd)/$out/libopenglraytracer_amd.so CLI=/dev/null \
       FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flag" $(pwd)/$out/libopenglraytracer_amd.so
done
