// GraphNorm kernel timing at config 5's batch (64 molecules x ~25 nodes, F = 300): HIP events over
// 200 back-to-back launches.  hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//   -I sir-gcn_amd/csrc tools/dbg/gn_probe.hip -o tools/dbg/gn_probe ; ./tools/dbg/gn_probe [B] [rows] [F]
#include "../../sir-gcn_amd/csrc/sirconv_graphnorm.hip"
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 64, R = argc > 2 ? atoi(argv[2]) : 25, F = argc > 3 ? atoi(argv[3]) : 300;
    const int64_t V = (int64_t)B * R;
    std::vector<int64_t> off(B + 1);
    for (int b = 0; b <= B; ++b) off[b] = (int64_t)b * R;
    std::vector<float> hx(V * F);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
    int64_t* doff; float *X, *Y, *dY, *dX, *w, *bias, *ms, *mean, *sd, *p0, *p1, *p2;
    CK(hipMalloc(&doff, (B + 1) * 8)); CK(hipMalloc(&X, V * F * 4)); CK(hipMalloc(&Y, V * F * 4));
    CK(hipMalloc(&dY, V * F * 4)); CK(hipMalloc(&dX, V * F * 4));
    for (float** p : {&w, &bias, &ms}) CK(hipMalloc(p, F * 4));
    for (float** p : {&mean, &sd, &p0, &p1, &p2}) CK(hipMalloc(p, (size_t)B * F * 4));
    CK(hipMemcpy(doff, off.data(), (B + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(X, hx.data(), V * F * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dY, hx.data(), V * F * 4, hipMemcpyHostToDevice));
    CK(hipMemset(w, 0, F * 4)); CK(hipMemset(bias, 0, F * 4)); CK(hipMemset(ms, 0, F * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int dir = 0; dir < 2; ++dir) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 200; ++i) {
                if (dir == 0) CK(sir::run_graph_norm_fwd(doff, B, F, X, F, w, bias, ms, 1e-5f, Y, F, mean, sd, 0));
                else CK(sir::run_graph_norm_bwd(doff, B, F, X, F, dY, F, w, ms, mean, sd, dX, F, p0, p1, p2, 0));
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms_ = 0;
            CK(hipEventElapsedTime(&ms_, e0, e1));
            if (rep) printf("B=%d rows=%d F=%d %s: %.2f us per launch\n", B, R, F, dir ? "bwd" : "fwd", ms_ * 1000 / 200);
        }
    }
    return 0;
}
