#!/bin/bash
# Quick A/B library: recompile only the named sources with extra DEFS, link with the main build's
# other objects.  usage: tools/build_variant.sh <name> "<defs>" src1.hip [src2.hip ...]
set -e
name=$1; defs=$2; shift 2
HERE=$(cd "$(dirname "$0")/.." && pwd)
CS=$HERE/sir-gcn_amd/csrc
B=$HERE/sir-gcn_amd/build
VO=$B/v_$name
mkdir -p $VO
objs=""
for o in $B/*.o; do
  base=$(basename $o .o)
  skip=0
  for s in "$@"; do [ "$(basename $s .hip)" = "$base" ] && skip=1; done
  [ $skip = 1 ] || objs="$objs $o"
done
for s in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function \
    -I$HERE/include -I$CS $defs $([ "$s" = sirconv_gemm_w.hip ] && echo -fno-slp-vectorize) -x hip -c $CS/$s -o $VO/$(basename $s .hip).o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $HERE/sir-gcn_amd/lib/libsirconv_$name.so $objs $VO/*.o
echo built lib/libsirconv_$name.so
