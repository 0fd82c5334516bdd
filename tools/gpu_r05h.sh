# Round-5 GPU session: origin-list texel resolution (8 / 16 / 32 per face edge).
set -uo pipefail
out=gpurun_out/r05h; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run ab 600 python tools/ab.py config3,config3x7,config4 main olist8 olist32
echo done
