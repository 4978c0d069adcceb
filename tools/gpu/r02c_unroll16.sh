# 16-bit storage rows in flight per wave after the writelane / index-prefetch changes: forward 6 / 3 (base 4), dK 6 / 10 (base 8)
set -o pipefail
mkdir -p gpurun_out/u16
O=gpurun_out/u16
L=sir-gcn_amd/lib
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sum --dtype bf16 --libs base=$L/libsirconv.so fh6=$L/libsirconv_fh6.so fh3=$L/libsirconv_fh3.so sh6=$L/libsirconv_sh6.so sh10=$L/libsirconv_sh10.so > $O/ab.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab.txt; exit $r
