// Host-side AddressSanitizer / UndefinedBehaviorSanitizer run of the C ABI's argument validation
// (SURVEY §5 "ASan/UBSan build of the C-ABI shim").  Built by tools/build_abi_asan.sh with
// sirconv_abi.cpp instrumented (host code only: -fno-gpu-sanitize) and linked against the normally
// built kernel objects; needs no GPU: every call below must be rejected (or be a no-op on empty
// work) before anything is launched.  Exit status 0 = every expectation held and the sanitizers
// reported nothing.
#include <cstdio>
#include <cstring>
#include <vector>

#include "sirconv.h"

static int failures = 0;

static void expect(const char* what, int got, int want, const char* needle = nullptr) {
    const char* msg = sir_last_error();
    const bool ok = got == want && (needle == nullptr || std::strstr(msg, needle) != nullptr);
    if (!ok) {
        std::printf("FAIL %-52s rc=%d (want %d) msg='%s'\n", what, got, want, msg);
        ++failures;
    }
}

int main() {
    if (sir_abi_version() != SIR_ABI_VERSION) {
        std::printf("FAIL abi version\n");
        return 1;
    }
    // host buffers only stand in for device pointers: no call below may dereference them
    std::vector<int32_t> buf(64, 0);
    int32_t* p = buf.data();
    float* f = reinterpret_cast<float*>(buf.data());
    void* v = buf.data();

    // edge passes
    expect("fwd: unknown dtype", sir_edge_agg_fwd(nullptr, nullptr, nullptr, 0, nullptr, 0, 256, 7, nullptr, 256,
                                                  nullptr, 256, nullptr, nullptr, 0, 2, 0.2f, nullptr, 256, nullptr,
                                                  nullptr, nullptr), SIR_EINVAL, "dtype");
    expect("fwd: bad agg", sir_edge_agg_fwd(nullptr, nullptr, nullptr, 0, nullptr, 0, 256, 0, nullptr, 256, nullptr, 256,
                                            nullptr, nullptr, 9, 2, 0.2f, nullptr, 256, nullptr, nullptr, nullptr),
           SIR_EINVAL, "agg");
    expect("fwd: H too large", sir_edge_agg_fwd(p, p, p, 1, nullptr, 0, 4096, 0, v, 4096, v, 4096, nullptr, nullptr, 0, 2,
                                                0.2f, v, 4096, nullptr, nullptr, nullptr), SIR_EINVAL, "H must be");
    expect("fwd: SYM without norms", sir_edge_agg_fwd(p, p, p, 1, nullptr, 0, 16, 0, v, 16, v, 16, nullptr, nullptr, 2, 2,
                                                      0.2f, v, 16, nullptr, nullptr, nullptr), SIR_EINVAL, "SYM");
    expect("fwd: ld < H", sir_edge_agg_fwd(p, p, p, 1, nullptr, 0, 16, 0, v, 8, v, 16, nullptr, nullptr, 0, 2, 0.2f, v, 16,
                                           nullptr, nullptr, nullptr), SIR_EINVAL, "leading");
    expect("fwd: split rows w/o partial", sir_edge_agg_fwd(p, p, p, 1, p, 1, 16, 0, v, 16, v, 16, nullptr, nullptr, 0, 2,
                                                           0.2f, v, 16, nullptr, nullptr, nullptr), SIR_EINVAL, "partial");
    expect("fwd: mask with GELU", sir_edge_agg_fwd(p, p, p, 1, nullptr, 0, 256, 0, v, 256, v, 256, nullptr, nullptr, 0, 3,
                                                   0.f, v, 256, reinterpret_cast<uint64_t*>(v), nullptr, nullptr),
           SIR_EUNSUPPORTED, "sign mask");
    for (int dt = 0; dt < 3; ++dt)
        expect("fwd: empty work is a no-op", sir_edge_agg_fwd(nullptr, nullptr, nullptr, 0, nullptr, 0, 256, dt, nullptr,
                                                               256, nullptr, 256, nullptr, nullptr, 0, 2, 0.2f, nullptr,
                                                               256, nullptr, nullptr, nullptr), SIR_OK);
    expect("dst: NULL G", sir_edge_agg_bwd_dst(p, p, p, 1, nullptr, 0, 64, 0, v, 64, v, 64, nullptr, nullptr, 64, nullptr,
                                               nullptr, 0, 2, 0.2f, v, 64, nullptr, 64, nullptr, nullptr, nullptr), SIR_EINVAL, "G must");
    expect("src: mask without perm", sir_edge_agg_bwd_src(p, p, nullptr, p, 1, nullptr, 0, 256, 0, nullptr, 256, nullptr,
                                                          256, reinterpret_cast<uint64_t*>(v), v, 256, nullptr, nullptr,
                                                          0, 2, 0.2f, v, 256, nullptr, nullptr, nullptr), SIR_EINVAL, "perm");
    expect("bwd (one launch): MEAN refused", sir_edge_agg_bwd(p, p, p, 1, nullptr, 0, p, p, p, p, 1, nullptr, 0, 256, 0,
                                                               reinterpret_cast<uint64_t*>(v), v, 256, nullptr, nullptr, 1,
                                                               2, 0.2f, v, 256, v, 256, nullptr, nullptr, nullptr, nullptr),
           SIR_EUNSUPPORTED, "MEAN");
    expect("bwd (one launch): needs mask", sir_edge_agg_bwd(p, p, p, 1, nullptr, 0, p, p, p, p, 1, nullptr, 0, 256, 0,
                                                             nullptr, v, 256, nullptr, nullptr, 0, 2, 0.2f, v, 256, v, 256,
                                                             nullptr, nullptr, nullptr, nullptr), SIR_EINVAL, "mask");
    expect("mask words", (int)sir_mask_words(300, SIR_ACT_LEAKY_RELU), 8);
    expect("mask words (GELU)", (int)sir_mask_words(256, SIR_ACT_GELU), 0);
    // generic path, GraphNorm, plan build
    expect("gather_add: F range", sir_edge_gather_add(p, p, p, 1, 0, f, 1, f, 1, f, 1, nullptr), SIR_EINVAL, "F must");
    expect("segment_sum: norm pairing", sir_segment_sum(p, p, nullptr, p, 1, nullptr, 0, 8, f, 8, f, nullptr, 0, f, 8,
                                                        nullptr, nullptr), SIR_EINVAL, "pairing");
    expect("segment_max: splits w/o ws", sir_segment_max(p, 1, p, 1, 8, f, 8, f, 8, p, 8, nullptr, nullptr, nullptr),
           SIR_EINVAL, "split");
    expect("graph_norm: bad F", sir_graph_norm_fwd(nullptr, 1, 0, f, 1, f, nullptr, nullptr, 1e-5f, f, 1, f, f, nullptr),
           SIR_EINVAL, "shape");
    expect("csr_build: chunk 0", sir_csr_build(nullptr, nullptr, 0, 4, 4, 0, p, p, nullptr, p, p, nullptr, v, 64, nullptr),
           SIR_EINVAL, "chunk");
    expect("csr_build: E >= 2^31", sir_csr_build(nullptr, nullptr, (int64_t)1 << 31, 4, 4, 256, p, p, nullptr, p, p,
                                                 nullptr, v, 64, nullptr), SIR_EINVAL, "2^31");
    expect("csr_build_workspace: negative", (int)sir_csr_build_workspace(-1, 4), -1);
    // GEMMs
    expect("gemm_nt: K % 4", sir_gemm_nt(f, 6, 1, 6, v, 8, nullptr, f, 8, nullptr, nullptr), SIR_EINVAL, "multiples");
    expect("gemm_nt: lda overflow", sir_gemm_nt(f, (int64_t)1 << 21, 1, 16, v, 16, nullptr, f, 16, nullptr, nullptr), SIR_EINVAL,
           "lda too large");
    expect("gemm_tn: ldb overflow", sir_gemm_tn(f, 16, f, (int64_t)1 << 21, 1, 16, 16, f, 16, nullptr, v, 1 << 20,
                                                nullptr), SIR_EINVAL, "too large");
    expect("gemm_pack: N range", sir_gemm_pack(f, 4, 0, 4, 0, v, nullptr), SIR_EINVAL, "N and K");
    expect("gemm_pack_bytes: range", (int)sir_gemm_pack_bytes(70000, 4), 0);
    // fused per-edge dense layer
    expect("mlp_fwd: act2 GELU", sir_edge_mlp_fwd(p, p, p, 1, nullptr, 0, 64, 64, f, 64, f, 64, nullptr, nullptr, 0, 1,
                                                  0.f, SIR_ACT_GELU, v, nullptr, f, 64, nullptr, 64, nullptr, nullptr,
                                                  nullptr), SIR_EUNSUPPORTED, "act2");
    expect("mlp_fwd: MAX needs arg", sir_edge_mlp_fwd(p, p, p, 1, nullptr, 0, 64, 64, f, 64, f, 64, nullptr, nullptr,
                                                      SIR_AGG_MAX, 1, 0.f, 0, v, nullptr, f, 64, nullptr, 64, nullptr,
                                                      nullptr, nullptr), SIR_EINVAL, "arg");
    expect("mlp_bwd_dst: H > 256", sir_edge_mlp_bwd_dst(p, p, p, 1, nullptr, 0, 260, 64, f, 260, f, 260, f, 64, nullptr,
                                                        nullptr, 0, 1, 0.f, 1, v, f, nullptr, f, 260, nullptr, nullptr,
                                                        f, nullptr), SIR_EUNSUPPORTED, "H");
    expect("mlp_bwd_parts: range", (int)sir_edge_mlp_bwd_parts(100, 64, 300), 0);
    expect("mlp_bwd_src: MAX refused", sir_edge_mlp_bwd_src(p, p, p, 1, nullptr, 0, 64, 64, f, 64, f, 64, f, 64, nullptr,
                                                            nullptr, SIR_AGG_MAX, 1, 0.f, 1, v, f, nullptr, f, 64,
                                                            nullptr, nullptr), SIR_EINVAL, "agg");
    expect("mlp_pack_bytes: range", (int)sir_edge_mlp_pack_bytes(1024, 64), 0);
    expect("max_bwd_dst: H > 256", sir_edge_max_bwd_dst(p, p, p, 1, nullptr, 0, 300, 64, f, 300, f, 300, f, 64, p, 64, 1,
                                                        0.f, f, f, 300, nullptr, f, nullptr), SIR_EUNSUPPORTED, "H");
    expect("max_bwd_src: NULL perm", sir_edge_max_bwd_src(p, p, nullptr, p, 1, nullptr, 0, 64, 64, f, 64, f, 64, f, 64,
                                                          p, 64, 1, 0.f, f, f, 64, nullptr, nullptr), SIR_EINVAL, "perm");
    std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
