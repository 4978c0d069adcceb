#!/bin/bash
# Host-side ASan/UBSan build of the C ABI's argument validation (tools/abi_sanitize.cpp), CPU only.
# sirconv_abi.cpp and the driver are instrumented (host code: -fno-gpu-sanitize keeps the gfx950
# device code as is); the kernel translation units are the normally built objects.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-$ROOT/sir-gcn_amd/build/asan}"
mkdir -p "$OUT"
make -s -C "$ROOT/sir-gcn_amd/csrc" -j8 >/dev/null
HIPCC=/opt/rocm/bin/hipcc
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -fno-gpu-sanitize"
INC="-I$ROOT/include -I$ROOT/sir-gcn_amd/csrc"
$HIPCC -O1 -g -std=c++17 --offload-arch=gfx950 $SAN $INC -x hip -c "$ROOT/sir-gcn_amd/csrc/sirconv_abi.cpp" -o "$OUT/sirconv_abi_asan.o"
$HIPCC -O1 -g -std=c++17 $SAN $INC -c "$ROOT/tools/abi_sanitize.cpp" -o "$OUT/abi_sanitize.o"
OBJS=$(ls "$ROOT"/sir-gcn_amd/build/*.o | grep -v sirconv_abi.o)
$HIPCC --offload-arch=gfx950 $SAN -o "$OUT/abi_sanitize" "$OUT/abi_sanitize.o" "$OUT/sirconv_abi_asan.o" $OBJS
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 "$OUT/abi_sanitize"
