// Phase clocks of the LDS-tiled small GEMM (k_gemm_lt) at config 5's shapes: build with
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DSIR_LT_TRACE -I include \
//         -I sir-gcn_amd/csrc tools/dbg/lt_trace.hip -o tools/dbg/lt_trace
// and run on the GPU box: ./tools/dbg/lt_trace <M> <K> <N> <trans>  (SIR_LT_NT picks the arrangement)
#include "../../sir-gcn_amd/csrc/sirconv_gemm.hip"
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const int64_t M = argc > 1 ? atoll(argv[1]) : 1582;
    const int K = argc > 2 ? atoi(argv[2]) : 300, N = argc > 3 ? atoi(argv[3]) : 300, trans = argc > 4 ? atoi(argv[4]) : 0;
    std::vector<float> hA(M * K), hW((size_t)K * N);
    for (size_t i = 0; i < hA.size(); ++i) hA[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    for (size_t i = 0; i < hW.size(); ++i) hW[i] = (float)((i * 40503u) % 1000) / 1000.f - 0.5f;
    float *A, *W, *C;
    uint64_t* tr;
    const size_t nblk = 65536;
    CK(hipMalloc(&A, hA.size() * 4)); CK(hipMalloc(&W, hW.size() * 4)); CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMalloc(&tr, nblk * 24 * 8));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(sir::g_lt_trace), &tr, sizeof(tr)));
    for (int rep = 0; rep < 20; ++rep) {
        CK(hipMemset(tr, 0, nblk * 24 * 8));
        CK(sir::run_gemm_nt_direct(A, K, M, K, W, trans ? N : K, trans, N, nullptr, C, N, 0, sir::Drop{}));
        CK(hipDeviceSynchronize());
    }
    std::vector<uint64_t> h(nblk * 24);
    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    int nb = 0;
    while (nb < (int)nblk && h[nb * 24 + 21] != 0) ++nb;
    double issue = 0, first = 0, epi = 0, tot = 0, comp[8] = {}, wait[8] = {}, s1_issue = 0, s1_read = 0;
    uint64_t t0 = ~0ull, t1 = 0;
    std::vector<double> totals;
    for (int b = 0; b < nb; ++b) {
        const uint64_t* r = &h[b * 24];
        issue += r[2] - r[1];
        first += r[4] - r[2];
        for (int s = 0; s < 8; ++s) {
            if (r[5 + 2 * s] == 0) continue;
            comp[s] += r[5 + 2 * s] - r[4 + 2 * s];
            if (s > 0 && r[4 + 2 * s]) wait[s] += r[4 + 2 * s] - r[5 + 2 * (s - 1)];
        }
        epi += r[20] - r[3];
        s1_issue += r[22] - r[6];
        s1_read += r[23] - r[22];
        tot += r[20] - r[1];
        totals.push_back((double)(r[20] - r[1]));
        t0 = std::min(t0, r[0]); t1 = std::max(t1, r[21]);
    }
    std::sort(totals.begin(), totals.end());
    printf("M=%ld K=%d N=%d trans=%d blocks=%d  (s_memtime cycles, mean per block)\n", (long)M, K, N, trans, nb);
    printf("  prologue issue %.0f  first wait %.0f  epilogue %.0f  total %.0f (p50 %.0f max %.0f)\n", issue / nb,
           first / nb, epi / nb, tot / nb, totals[nb / 2], totals[nb - 1]);
    printf("  step 1 split: issue %.0f  LDS reads %.0f  rest (split + MFMA issue) %.0f\n", s1_issue / nb, s1_read / nb,
           comp[1] / nb - s1_issue / nb - s1_read / nb);
    for (int s = 0; s < 8; ++s) printf("  step %d: wait %.0f compute %.0f\n", s, wait[s] / nb, comp[s] / nb);
    printf("  grid span (realtime 100 MHz): %.2f us\n", (t1 - t0) * 1e-2);
    return 0;
}
