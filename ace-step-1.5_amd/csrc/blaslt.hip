// blaslt.hip — hipBLASLt as an opt-in, per-projection alternative to the hand-written GEMMs
// for the DiT's N ≤ 4096 projections (ACEHIP_BLASLT, A/B; read per call).
//
// Measured in isolation (tools/ab_gemm.py, cold weights, one process, r03n4): hipBLASLt's
// plain-store kernels beat ours on QKV (84.3 vs 97.0 µs), down (118.6 vs 146.4 with our
// residual epilogue) and O (43.4 vs 51.1), and lose on SwiGLU (300.3 vs 265.5).  hipBLASLt
// has no head-post epilogue, so its QKV path is the projection into a staging buffer + the
// standalone head_post kernel; the gated residual X += gate ⊙ (A·Wᵀ) maps onto its
// D = α ⊙ (A·Wᵀ) + β·C with a per-row α vector (rows of the column-major D = output channels)
// and β = 1, C = D = X — one fp32 rounding instead of the reference's bf16 product then bf16
// sum, so that path is within tolerance of the oracle, not bit-faithful to its rounding.
//
// Row-major C[M][N] = A[M][K]·W[N][K]ᵀ is the column-major D[N][M] = op_T(W as K×N)·(A as K×M).
#include <hipblaslt/hipblaslt.h>

#include <array>
#include <map>
#include <mutex>

#include "kernels.h"

namespace acehip {
namespace {

struct LtPlan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    bool ok = false;
};

struct LtCtx {
    hipblasLtHandle_t h = nullptr;
    void *ws = nullptr;
    size_t ws_bytes = 0;
    bool failed = false;
    std::map<std::array<int64_t, 7>, LtPlan> plans;
};

std::mutex g_lt_mu;
std::map<int, LtCtx> g_lt;
constexpr size_t LT_WS = (size_t)64 << 20;

#define LT_OK(x) ((x) == HIPBLAS_STATUS_SUCCESS)

bool make_plan(LtCtx &c, LtPlan &p, int M, int N, int K, int64_t lda, int64_t ldw, int64_t ldc, bool avec) {
    const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    if (!LT_OK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F))) return false;
    if (!LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta))) ||
        !LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb))))
        return false;
    if (avec) {
        const int32_t pm = HIPBLASLT_POINTER_MODE_ALPHA_DEVICE_VECTOR_BETA_HOST;
        if (!LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_POINTER_MODE, &pm, sizeof(pm))))
            return false;
    }
    if (!LT_OK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, ldw)) ||
        !LT_OK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, lda)) ||
        !LT_OK(hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, N, M, ldc)))
        return false;
    hipblasLtMatmulPreference_t pref = nullptr;
    if (!LT_OK(hipblasLtMatmulPreferenceCreate(&pref))) return false;
    const uint64_t wsb = c.ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    const bool got = LT_OK(hipblasLtMatmulAlgoGetHeuristic(c.h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n));
    hipblasLtMatmulPreferenceDestroy(pref);
    if (!got || n < 1 || res[0].workspaceSize > c.ws_bytes) return false;
    p.algo = res[0].algo;
    return true;
}

}  // namespace

// ACEHIP_BLASLT bit mask: 1 = QKV projection (+ standalone head_post), 2 = gated-residual
// projections (self-O, down), 4 = plain-residual projection (cross-O).  Default 2: 240 s song
// (tools/ab_env_song.py, one process, profiles/r03n5_blaslt_song_ab.txt) DiT 492.6 ms hand-
// written, 494.4 with 1 (the standalone head_post eats the QKV gain), 481.8 with 2, 493.4 with 4.
int blaslt_mask() {
    const char *e = getenv("ACEHIP_BLASLT");
    return e ? atoi(e) : 2;
}

// C = α ⊙ (A·Wᵀ) + β·C (α: per-column device vector alpha_vec[N], or 1 when null).  Returns 0
// when launched, 1 when hipBLASLt cannot take the call (no plan, first use inside a stream
// capture) — the caller then runs its own kernel — and < 0 on a launch error.
int blaslt_gemm(const bf16_t *A, int64_t lda, const bf16_t *W, int64_t ldw, bf16_t *C, int64_t ldc, int M, int N,
                int K, const float *alpha_vec, float beta, hipStream_t s) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_lt_mu);
    LtCtx &c = g_lt[dev];
    if (c.failed) return 1;
    if (!c.h) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 1;
        if (!LT_OK(hipblasLtCreate(&c.h)) || hipMalloc(&c.ws, LT_WS) != hipSuccess) {
            c.failed = true;
            return 1;
        }
        c.ws_bytes = LT_WS;
    }
    const std::array<int64_t, 7> key{M, N, K, lda, ldw, ldc, alpha_vec ? 1 : 0};
    auto it = c.plans.find(key);
    if (it == c.plans.end()) {
        LtPlan p;
        p.ok = make_plan(c, p, M, N, K, lda, ldw, ldc, alpha_vec != nullptr);
        it = c.plans.emplace(key, p).first;
    }
    const LtPlan &p = it->second;
    if (!p.ok) return 1;
    const float one = 1.0f;
    const void *alpha = alpha_vec ? (const void *)alpha_vec : (const void *)&one;
    if (!LT_OK(hipblasLtMatmul(c.h, p.desc, alpha, W, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo, c.ws,
                               c.ws_bytes, s)))
        return fail(-1, "hipblasLtMatmul failed");
    return 0;
}

}  // namespace acehip
