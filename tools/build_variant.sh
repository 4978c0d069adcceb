#!/bin/bash
# Fast A/B variant library: reuse the main build's objects except the ones compiled from the listed
# sources (the only files the DEFS can change), then link libsirconv_<name>.so.
#   tools/build_variant.sh <name> "<DEFS>" sirconv_gemm.hip [more sources]
set -e
name=$1; defs=$2; shift 2
C=$(dirname "$0")/../sir-gcn_amd/csrc
B=$C/../build
mkdir -p $B/$name
for o in $B/*.o; do
  base=$(basename $o .o)
  skip=0
  for s in "$@"; do [ "$base" = "$(basename $s .hip)" ] && skip=1; done
  [ $skip -eq 1 ] || cp -p $o $B/$name/
done
for s in "$@"; do rm -f $B/$name/$(basename $s .hip).o; done
make -s -C $C VARIANT=$name DEFS="$defs" -j8
