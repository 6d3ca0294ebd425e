// gemm.hip — bf16 MFMA GEMM for the DiT projections: C[M,N] = A[M,K]·W[N,K]^T.
//
// Every dense contraction of the DiT (QKV, O, cross Q/O, SwiGLU gate/up and
// down, proj_in, proj_out, condition_embedder, cross K/V) goes through here
// with a fused epilogue (bias / AdaLN-Zero gated residual / plain residual /
// SwiGLU) so the reference's separate elementwise kernels never touch HBM
// (reference base:499-533).
//
// Structure (templated on tile BM×BN, waves WM×WN, LDS ring depth STAGES):
//   * both operands are K-contiguous ([rows][K]); each K-tile of 64 is staged
//     global→LDS by global_load_lds_dwordx4 into an STAGES-deep ring, the
//     [A tile; W tile] image lane-linear with the XOR swizzle applied on the
//     SOURCE address (chunk' = chunk ^ ((row>>1)&7)) so the ds_read_b128
//     fragment reads are bank-conflict free;
//   * STAGES−1 K-tiles are kept in flight ACROSS the barrier: a counted
//     s_waitcnt vmcnt(N) (never 0 in the steady state) + a raw s_barrier —
//     __syncthreads() would drain the LDS-DMA queue every tile (the ~900 TF
//     ceiling of the 2-barrier structure, cdna_hip_programming.md §5);
//   * v_mfma_f32_16x16x32_bf16 computes the transposed tile (W as the A
//     operand) so each lane owns 4 consecutive output columns of one row
//     (8-byte epilogue stores; the SwiGLU pairs gate/up in registers);
//   * block ids are remapped XCD-aware, then grouped along M so co-resident
//     blocks share the weight panel in L2.
#include "kernels.h"

namespace acehip {
namespace {

constexpr int BK = 64;
constexpr int GROUP_M = 8;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// own LDS-DMAs retired down to N outstanding + own LDS reads retired, then a
// raw barrier (no implicit vmcnt(0)) and a compiler fence so no LDS access
// moves across it
template <int N>
__device__ __forceinline__ void ring_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int BM, int BN, int WM, int WN, int STAGES, int EPI>
__global__ __launch_bounds__(WM *WN * 64, 1) void gemm_kernel(GemmArgs a) {
    constexpr int NW = WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;          // wave tile
    constexpr int SM = TM / 16, SN = TN / 16;          // 16×16 sub-tiles per wave
    constexpr int ROWS = BM + BN;                      // rows of one stage image (128 B each)
    constexpr int STAGE = ROWS * 128;
    constexpr int NINS = ROWS / 8;                     // glds instructions per stage
    constexpr int PER_WAVE = NINS / NW;
    static_assert(NINS % NW == 0, "staging must split evenly over waves");
    static_assert(EPI != EPI_SWIGLU || TN == 64, "SwiGLU pairs 32+32 columns per wave");
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int tilesM = (a.M + BM - 1) / BM, tilesN = a.N / BN;
    const int nwg = tilesM * tilesN;
    const int wg = xcd_remap(blockIdx.x, nwg);
    const int per_group = GROUP_M * tilesN;
    const int gid = wg / per_group, first_m = gid * GROUP_M;
    const int gsz = min(tilesM - first_m, GROUP_M);
    const int tm = first_m + (wg % per_group) % gsz;
    const int tn = (wg % per_group) / gsz;
    const int m0 = tm * BM, n0 = tn * BN;

    // staging sources: wave issues image rows [8q, 8q+8) for q = wave + NW·i
    const bf16_t *src[PER_WAVE];
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
        const int q = wave + NW * i;
        const int r = q * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        if (r < BM) src[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8;
        else src[i] = a.W + (int64_t)(n0 + r - BM) * a.ldw + c * 8;
    }
    auto stage = [&](int buf, int k0) {
        char *b = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) glds16(src[i] + k0, b + (wave + NW * i) * 1024);
    };

    f32x4 acc[SM][SN];
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = a.K / BK;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) stage(s, s * BK);
    const int fr = lane & 15, fc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt landed (its own wave's DMAs), leaving STAGES-2 newer tiles in flight
        // every wave's DMA for tile kt landed; tile kt-1 fully read (WAR for the refill below)
        if (kt + STAGES - 2 < nk) ring_barrier<(STAGES - 2) * PER_WAVE>();
        else ring_barrier<0>();
        if (kt + STAGES - 1 < nk) stage((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);
        const char *b = lds + (kt % STAGES) * STAGE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xf[SM], wf[SN];
#pragma unroll
            for (int i = 0; i < SM; ++i) xf[i] = *(const bf16x8 *)(b + swz(wm * TM + i * 16 + fr, ks * 4 + fc));
#pragma unroll
            for (int j = 0; j < SN; ++j) wf[j] = *(const bf16x8 *)(b + swz(BM + wn * TN + j * 16 + fr, ks * 4 + fc));
#pragma unroll
            for (int i = 0; i < SM; ++i)
#pragma unroll
                for (int j = 0; j < SN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
        }
    }

    // epilogue: lane owns row m, columns n..n+3 of each 16x16 sub-tile
#pragma unroll
    for (int i = 0; i < SM; ++i) {
        const int m = m0 + wm * TM + i * 16 + fr;
        if (m >= a.M) continue;
        if constexpr (EPI == EPI_SWIGLU) {
            // packed rows: within each 64-row wave panel, rows [0,32) gate, [32,64) up
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int nout = ((n0 + wn * 64) >> 1) + j * 16 + fc * 4;
                float o[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float g = rbf(acc[i][j][r]);
                    const float u = rbf(acc[i][j + 2][r]);
                    o[r] = rbf(silu_f(g)) * u;
                }
                *(uint2 *)(a.C + (int64_t)m * a.ldc + nout) = pack4(o);
            }
        } else {
            const int b = (EPI == EPI_GATED_RES) ? m / a.rows_per_batch : 0;
#pragma unroll
            for (int j = 0; j < SN; ++j) {
                const int n = n0 + wn * TN + j * 16 + fc * 4;
                float o[4];
                if constexpr (EPI == EPI_STORE) {
                    float bb[4] = {0.f, 0.f, 0.f, 0.f};
                    if (a.bias) unpack4(*(const uint2 *)(a.bias + n), bb);
#pragma unroll
                    for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r] + bb[r];
                } else {
                    float rr[4];
                    unpack4(*(const uint2 *)(a.res + (int64_t)m * a.ldr + n), rr);
                    if constexpr (EPI == EPI_GATED_RES) {
                        float gg[4];
                        unpack4(*(const uint2 *)(a.gate + (int64_t)b * a.gate_bstride + n), gg);
#pragma unroll
                        for (int r = 0; r < 4; ++r) o[r] = rr[r] + rbf(rbf(acc[i][j][r]) * gg[r]);
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) o[r] = rr[r] + rbf(acc[i][j][r]);
                    }
                }
                *(uint2 *)(a.C + (int64_t)m * a.ldc + n) = pack4(o);
            }
        }
    }
}

template <int BM, int BN, int WM, int WN, int STAGES>
int launch(const GemmArgs &a, hipStream_t s) {
    if (a.N % BN) return fail(-1, "gemm: N not a multiple of the tile");
    const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
    constexpr int NT = WM * WN * 64;
    switch (a.epi) {
        case EPI_STORE: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_STORE><<<tiles, NT, 0, s>>>(a); break;
        case EPI_GATED_RES: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_GATED_RES><<<tiles, NT, 0, s>>>(a); break;
        case EPI_RES: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_RES><<<tiles, NT, 0, s>>>(a); break;
        case EPI_SWIGLU: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_SWIGLU><<<tiles, NT, 0, s>>>(a); break;
        default: return fail(-1, "gemm: bad epilogue");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace

int gemm_variant(const GemmArgs &a, int variant, hipStream_t s) {
    switch (variant) {
        case 0: return launch<128, 128, 2, 2, 2>(a, s);   // 4 waves, 2-stage (2 blocks/CU)
        case 1: return launch<256, 128, 4, 2, 3>(a, s);   // 8 waves, 3-stage ring (144 KiB)
        case 2: return launch<128, 128, 2, 2, 3>(a, s);   // 4 waves, 3-stage ring (96 KiB)
        case 3: return launch<128, 256, 2, 4, 3>(a, s);   // 8 waves, wide N, 3-stage (144 KiB)
        case 4: return launch<256, 128, 4, 2, 2>(a, s);   // 8 waves, 2-stage (96 KiB)
        case 5: return launch<256, 256, 2, 4, 2>(a, s);   // 8 waves, 128x64 wave tile (128 KiB)
        case 6: return launch<192, 256, 2, 4, 2>(a, s);   // 8 waves, 96x64 wave tile (112 KiB)
        default: return fail(-1, "gemm: bad variant");
    }
}

static int g_variant_override = -1;
void gemm_set_variant(int v) { g_variant_override = v; }

int gemm(const GemmArgs &a, hipStream_t s) {
    if (a.M <= 0) return 0;
    if (a.N % 128 || a.K % BK || a.K <= 0)
        return fail(-1, "gemm: N%128 / K%64 violated (M=" + std::to_string(a.M) + " N=" +
                            std::to_string(a.N) + " K=" + std::to_string(a.K) + ")");
    if ((a.lda | a.ldw | a.ldc) % 8) return fail(-1, "gemm: leading dims must be multiples of 8");
    if (a.epi == EPI_GATED_RES && (!a.gate || a.rows_per_batch <= 0)) return fail(-1, "gemm: gate");
    if ((a.epi == EPI_GATED_RES || a.epi == EPI_RES) && !a.res) return fail(-1, "gemm: res");
    int v = g_variant_override;
    // measured on MI355X (tools/bench_gemm.py, uniform random operands): the
    // 256x128 2-stage tile wins on the wide SwiGLU GEMM (N = 12288), the
    // 128x128 2-stage tile (2 blocks/CU) on every N <= 4096 shape
    if (v < 0) v = a.N >= 8192 ? 4 : 0;
    if ((v == 3 || v == 5 || v == 6) && a.N % 256) v = 0;
    return gemm_variant(a, v, s);
}

}  // namespace acehip
