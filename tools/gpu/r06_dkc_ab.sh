#!/bin/bash
# A/B of the chunked dK pass (mask_item_src_chunk, SIR_DK_CHUNK) against the shipped build, S2 sum,
# fp32 and bf16, interleaved in one process (tools/edge_ab.py checks bit-equality)
set -o pipefail
O=gpurun_out/dkc
mkdir -p $O
L=sir-gcn_amd/lib
for d in f32 bf16; do
  SIRGCN_LIB=$L/libsirconv_dkc4.so timeout -k 10 300 python3 -u tools/edge_ab.py --graph S2 --dtype $d --rounds 7 \
    --libs base=$L/libsirconv.so dkc4=$L/libsirconv_dkc4.so dkc8=$L/libsirconv_dkc8.so > $O/ab_$d.txt 2>&1 || exit $?
  cat $O/ab_$d.txt
done
