#!/bin/bash
# Timing-only builds of the kernel into _ab/<name>/ (delete _ab/ after use: it travels with every gpurun call):
#   tools/ablate.sh            ablation variants (outputs wrong by design)
#   tools/ablate.sh rev REV    the library as of git revision REV (A/B timing
#                              against the working tree in one GPU call)
#   tools/ablate.sh flags NAME "-DX ..."   the working tree with extra flags
set -euo pipefail
cd "$(dirname "$0")/.."
build() {  # name srcdir extra-flags
  local out=_ab/$1; mkdir -p $out/obj
  make -s -C "$2" OBJDIR=$(pwd)/$out/obj OUT=$(pwd)/$out/libopenglraytracer_amd.so CLI=/dev/null \
       FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize $3" $(pwd)/$out/libopenglraytracer_amd.so
}
if [ "${1:-}" = rev ]; then
  rev=${2:?revision}; src=_ab/rev_src
  rm -rf $src _ab/rev; mkdir -p $src/pkg/csrc $src/include
  for f in $(git ls-tree --name-only $rev openglraytracer_amd/csrc/); do git show $rev:$f > $src/pkg/csrc/$(basename $f); done
  git show $rev:include/rt.h > $src/include/rt.h
  build rev $src/pkg/csrc ""
  exit 0
fi
if [ "${1:-}" = flags ]; then
  build ${2:?name} openglraytracer_amd/csrc "${3:-}"
  exit 0
fi
# (built in parallel, 4 at a time: each is ~1 min of hipcc)
n=0
for v in full:"" cycles:"-DRT_CYCLES" stats:"-DRT_STATS" noshadow:"-DRT_ABLATE_SHADOW" nophong:"-DRT_ABLATE_PHONG" notrace:"-DRT_ABLATE_TRACE" \
         noraygen:"-DRT_ABLATE_RAYGEN" noframes:"-DRT_ABLATE_FRAMES"; do
  build ${v%%:*} openglraytracer_amd/csrc "${v#*:}" &
  n=$((n + 1)); [ $((n % 4)) -eq 0 ] && wait
done
wait
