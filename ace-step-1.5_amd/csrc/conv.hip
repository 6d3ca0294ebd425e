// conv.hip — Oobleck VAE convolutions as implicit GEMMs on MFMA.
//
// Activations are channels-last [L][C] bf16 (NLC), so every convolution of
// the Oobleck decoder/encoder (reference spec acestep/models/mlx/
// vae_model.py:24-230; diffusers AutoencoderOobleck) is one GEMM
//   out[m·c_stride + c_off + phase][n] = Σ_tap Σ_ci in[m·a_stride + tap·dil + a_off][ci]·W[n][tap·Cin+ci]
// with zero padding outside [0, L_in):
//   * Conv1d k=7 dilation d (residual units):  taps 7, a_off −3d
//   * Conv1d k=1:                              taps 1
//   * ConvTranspose1d k=2s stride s pad s/2:   s phases r (gridDim.y); output rows
//     m·s + r − s/2, each the GEMM of the 2 overlapping input rows [m−1 | m]
//   * strided Conv1d k=2s (encoder):           taps 2s, a_stride s, a_off −s/2
// Snake1d (x + 1/(e^β+1e-9)·sin(e^α·x)², vae_model.py:38-55) is applied ONCE,
// in the epilogue of the conv that produces its input ("out_s"), instead of
// in every consumer tile (a k=7 conv would recompute it 7× per N-tile); the
// bias and the residual skip (OobleckResidualUnit, vae_model.py:77-87) are
// fused in the same epilogue.  The residual may alias the raw output (each
// element is read and written by the same lane).
//
// Tile 128×128×64, 4 waves (2×2) of v_mfma_f32_16x16x32_bf16; both operands
// are staged one tile ahead — W by global_load_lds into a double buffer, the
// A (im2col) tile through registers (its global loads are in flight during
// the MFMAs of the current tile), XOR-swizzled for conflict-free ds_read_b128.
#include "kernels.h"
#include "conv.h"
#include <algorithm>
#include <type_traits>

namespace acehip {
namespace {

constexpr int BM = 128, BN = 128, BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// A-row source for im2col staging: row m, tap → in[m·a_stride + tap·dil + a_off][ci0 + 8c]
// (a zero page outside [0, L_in) — glds cannot write zeros, it copies them)
__device__ __forceinline__ const bf16_t *a_src(const ConvArgs &a, int64_t m, int tap, int ci0, int c) {
    const int64_t pos = m * a.a_stride + (int64_t)tap * a.dil + a.a_off;
    if (m >= a.M || pos < 0 || pos >= a.L_in) return a.zero + c * 8;
    return a.in + pos * a.Cin + ci0 + c * 8;
}

// snake1 over 8 channels with 16-B parameter loads (sa / sib fp32 per channel)
__device__ __forceinline__ void snake8(const float (&x)[8], const float *sa, const float *sib, float (&y)[8]) {
    const float4 a0 = *(const float4 *)sa, a1 = *(const float4 *)(sa + 4);
    const float4 b0 = *(const float4 *)sib, b1 = *(const float4 *)(sib + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    snake_n<8>(x, av, bv, y);
}

// Both operands by global_load_lds into a 2-stage ring: [A im2col rows | W rows],
// 128-B rows, XOR-swizzled on the source address (as gemm.hip).
struct ConvTile {
    static constexpr int BM = 128, BN = 128, ROWS = BM + BN, STAGE = ROWS * 128;
};

template <bool RES, bool RAW, bool SN>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvArgs a) {
    constexpr int BM = ConvTile::BM, BN = ConvTile::BN, STAGE = ConvTile::STAGE;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tilesN = a.N / BN;
    const int64_t tilesM = (a.M + BM - 1) / BM;
    const int64_t wg = xcd_remap(blockIdx.x, (int)(tilesM * tilesN));
    const int64_t tm = wg / tilesN;
    const int tn = (int)(wg % tilesN);     // N-fastest: neighbouring blocks share the A panel
    const int64_t m0 = tm * BM;
    const int n0 = tn * BN;
    const int phase = blockIdx.y;
    const bf16_t *Wp = a.W + (int64_t)phase * a.w_pstride;
    const int K = a.taps * a.Cin;

    // staging: 32 glds per stage (16 A + 16 W) → 8 per wave; instruction q covers rows 8q..8q+7
    int rowq[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) rowq[i] = (wave + 4 * i) * 8 + (lane >> 3);
    auto stage = [&](int buf, int k0) {
        char *b = lds + buf * STAGE;
        const int tap = k0 / a.Cin, ci0 = k0 % a.Cin;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = rowq[i];
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const bf16_t *src = r < BM ? a_src(a, m0 + r, tap, ci0, c)
                                       : Wp + (int64_t)(n0 + r - BM) * K + k0 + c * 8;
            glds16(src, b + (wave + 4 * i) * 1024);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    stage(0, 0);
    const int fr = lane & 15, fc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * BK);
        const char *b = lds + (kt & 1) * STAGE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xf[4], wf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xf[i] = *(const bf16x8 *)(b + swz(wm * 64 + i * 16 + fr, ks * 4 + fc));
                wf[i] = *(const bf16x8 *)(b + swz(BM + wn * 64 + i * 16 + fr, ks * 4 + fc));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
        }
    }

    // epilogue: sub-tiles paired by a lane exchange (pair8) → 8 contiguous channels per lane,
    // 16-B loads / stores (the store tail is issue-bound); partners (lane ^ 16) share the row
    const bool odd = fc & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t m = m0 + wm * 64 + i * 16 + fr;
        const int64_t row = m * a.c_stride + a.c_off + phase;
        if (m >= a.M || row < 0 || row >= a.L_out) continue;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            float o[8];
            pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
            const int n = n0 + wn * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8;
            if (a.bias) {
                float bb[8];
                unpack8(*(const uint4 *)(a.bias + n), bb);
                add_n<8>(o, bb);
            }
            rbf_n<8>(o);                                                     // conv output (bf16)
            if constexpr (RES) {
                float rr[8];
                unpack8(*(const uint4 *)(a.res + row * a.N + n), rr);
                add_n<8>(o, rr);
                rbf_n<8>(o);
            }
            if constexpr (RAW) *(uint4 *)(a.out + row * a.N + n) = pack8(o);
            if constexpr (SN) {
                float sn[8];
                snake8(o, a.sa + n, a.sib + n, sn);
                *(uint4 *)(a.out_s + row * a.N + n) = pack8(sn);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Persistent implicit-GEMM conv for the ConvTranspose phases, the k = 1 convs at C ≥ 256
// and the encoder's strided convs.  conv_gemm_kernel stages one K-tile ahead on a 2-slot
// ring, waits vmcnt(0) every K-tile and starts every tile with the operand latency
// exposed; with 4–32 K-tiles per tile those launches ran at ≈ 40 % of the HBM roof.
// Here one block per CU (8 waves, 64×32 wave tiles) walks a contiguous range of work
// items (M-tile, N-tile, phase; phase fastest, then N, so consecutive items share the A
// panel in L2 — phases as the slowest index sent every ConvTranspose input through HBM
// once per phase)
// and the K-tiles of consecutive items form ONE stream through an NS-stage ring
// (NS = 4, or 3 with a residual): NS − 1 stages are in flight, so the next item's
// operands land during the current item's epilogue.
// All loads are LDS-DMA by inline asm with explicit counted waits (hipcc, seeing no
// vector loads in the loop, inserts no waits of its own — with the builtin DMA it placed
// vmcnt(0) at every loop merge): the operand stages, the item's residual tile (issued at
// its first K-step into a swizzled 32 KiB image) and, once per block, the bias / Snake
// parameters of all N columns.  vmcnt per wave at K-step g (stage g issued at g − NS + 1):
// younger are the ≤ NS − 2 newer stages, the residual pieces if the item began at a step
// after stage g was issued, and the previous epilogue's stores if they followed it
// (partial tiles, whose store count varies, are left out: a safe over-wait).
namespace cp {
constexpr int BM = 128, BN = 128, STAGE = (BM + BN) * 128, NW = 8;
constexpr int PW = (BM + BN) / 8 / NW;                    // operand pieces per wave per stage
constexpr int RW = BM * 256 / 1024 / NW;                  // residual pieces per wave per item
constexpr int WM = 2, WN = 4, TM = BM / WM, TN = BN / WN, SM = TM / 16, SN = TN / 16;   // 64×32
constexpr int MAXN = 1024;                                // parameter image: N ≤ 1024 columns
constexpr int PAR = MAXN * 10;                            // bias bf16 | sa f32 | sib f32
}  // namespace cp

__device__ __forceinline__ void cp_dma_v(const void *src, uint32_t lds_addr) {   // 64-bit per-lane address
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds_addr), "v"(src)
                 : "memory");
}
__device__ __forceinline__ const void *cp_uniform(const void *p) {   // pointer known wave-uniform → SGPRs
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const void *)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void cp_dma_s(const void *base, uint32_t voff, uint32_t lds_addr) {   // saddr form
    base = cp_uniform(base);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr), "v"(voff), "s"(base)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void cp_wait() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

template <bool RES, bool RAW, bool SN>
__global__ __launch_bounds__(512, 1) void convp_kernel(ConvArgs a, int64_t nitems, int phases) {
    constexpr int CBM = cp::BM, CBN = cp::BN, STG = cp::STAGE, PW = cp::PW, RW = RES ? cp::RW : 0;
    constexpr int NS = RES ? 3 : 4;
    constexpr int SM = cp::SM, SNT = cp::SN, TM = cp::TM, TN = cp::TN;
    constexpr int KST = ((RAW ? 1 : 0) + (SN ? 1 : 0)) * SM;   // epilogue stores per wave per item
    constexpr int RESB = RES ? CBM * 256 : 0;
    __shared__ __attribute__((aligned(16))) char lds[cp::PAR + NS * STG + RESB];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / cp::WN, wn = wave % cp::WN;
    const int fr = lane & 15, fc = lane >> 4;
    const bool odd = fc & 1;
    const int64_t i0 = nitems * blockIdx.x / gridDim.x, i1 = nitems * (blockIdx.x + 1) / gridDim.x;
    if (i0 >= i1) return;
    const int K = a.taps * a.Cin, nk = K / BK;
    const int64_t G = (i1 - i0) * nk;
    const int tilesN = a.N / CBN;
    // parameters of all N columns → LDS (plain loads, retired before the first DMA)
    bf16_t *pbias = (bf16_t *)lds;
    float *psa = (float *)(lds + cp::MAXN * 2), *psib = psa + cp::MAXN;
    for (int c = tid; c < a.N; c += 512) {
        pbias[c] = a.bias ? a.bias[c] : (bf16_t)0;
        if constexpr (SN) { psa[c] = a.sa[c]; psib[c] = a.sib[c]; }
    }
    __builtin_amdgcn_s_waitcnt(0x0070);
    const uint32_t l0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)lds;
    const uint32_t lst = l0 + cp::PAR, lres = lst + NS * STG;
    const char *stb = lds + cp::PAR, *resb = stb + NS * STG;

    // staging cursor (block-uniform): item (phase, m0, n0) and K-tile of the next stage
    int s_kt = 0, s_phase, s_n0;
    int64_t s_m0;
    {
        s_phase = (int)(i0 % phases);
        const int64_t w = i0 / phases;
        s_m0 = (w / tilesN) * CBM;
        s_n0 = (int)(w % tilesN) * CBN;
    }
    int s_slot = 0;            // ring slot of the next stage (rotating: no 64-bit modulo per step)
    // the lane's W row offset inside a piece (8 rows of 128 B, source-swizzled chunk)
    const int r8 = lane >> 3;
    auto stage = [&] {
        const int k0 = s_kt * BK, tap = k0 / a.Cin, ci0 = k0 - tap * a.Cin;
        const uint32_t dst = lst + (uint32_t)s_slot * STG;
#pragma unroll
        for (int i = 0; i < PW / 2; ++i) {                  // A: im2col rows (zero page outside)
            const int q = wave + cp::NW * i, r = q * 8 + r8;
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            cp_dma_v(a_src(a, s_m0 + r, tap, ci0, c), dst + q * 1024);
        }
        const char *wb = (const char *)(a.W + (int64_t)s_phase * a.w_pstride + (int64_t)s_n0 * K + k0);
#pragma unroll
        for (int i = PW / 2; i < PW; ++i) {                 // W rows
            const int q = wave + cp::NW * i, r = q * 8 + r8 - CBM;
            const int c = (lane & 7) ^ (((r + CBM) >> 1) & 7);
            cp_dma_s(wb, (uint32_t)(r * K + c * 8) * 2, dst + q * 1024);
        }
        if (++s_slot == NS) s_slot = 0;
        if (++s_kt == nk) {
            s_kt = 0;
            if (++s_phase == phases) {
                s_phase = 0;
                s_n0 += CBN;
                if (s_n0 == a.N) { s_n0 = 0; s_m0 += CBM; }
            }
        }
    };
    // the item's residual tile: 4 rows × 256 B per piece, chunk c of row r stored at c ^ (r & 15)
    auto stage_res = [&](int64_t m0, int n0, int phase) {
#pragma unroll
        for (int i = 0; i < RW; ++i) {
            const int q = wave + cp::NW * i, r = q * 4 + (lane >> 4);
            const int c = (lane & 15) ^ (r & 15);
            const int64_t m = min(m0 + r, a.M - 1);
            const int64_t row = min(max(m * a.c_stride + a.c_off + phase, (int64_t)0), a.L_out - 1);
            cp_dma_v(a.res + row * a.N + n0 + c * 8, lres + q * 1024);
        }
    };

    f32x4 acc[SM][SNT];
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int s = 0; s < NS - 1; ++s)
        if (s < G) stage();
    // compute cursor
    int kt = 0, phase = 0, n0 = 0;
    int64_t m0 = 0;
    {
        phase = (int)(i0 % phases);
        const int64_t w = i0 / phases;
        m0 = (w / tilesN) * CBM;
        n0 = (int)(w % tilesN) * CBN;
    }
    bool prev_st = false;      // previous epilogue issued exactly KST stores per wave
    int slot = 0;
    for (int64_t g = 0; g < G; ++g) {
        const int64_t left = G - 1 - g;   // K-steps after this one
        const int newer = left < NS - 2 ? (int)left : NS - 2;
        // residual pieces (issued at this item's first step, before that step's refill) are
        // younger than stage g when g ≥ item start + 1 and stage g was issued at or before it
        const bool rs = RES && kt >= 1 && kt <= NS - 2;
        const bool st = prev_st && kt <= NS - 2;
        const int extra = (rs ? RW : 0) + (st ? KST : 0);
#define CP_W(E)                                                    \
    do {                                                           \
        if (newer == 2) cp_wait<2 * PW + (E)>();                   \
        else if (newer == 1) cp_wait<PW + (E)>();                  \
        else cp_wait<(E)>();                                       \
    } while (0)
        if (extra == RW + KST) CP_W(RW + KST);
        else if (extra == KST) CP_W(KST);
        else if (extra == RW) CP_W(RW);
        else CP_W(0);
#undef CP_W
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (RES && kt == 0) stage_res(m0, n0, phase);
        if (g + NS - 1 < G) stage();
        const char *b = stb + slot * STG;
        if (++slot == NS) slot = 0;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xf[SM], wf[SNT];
#pragma unroll
            for (int i = 0; i < SM; ++i) xf[i] = *(const bf16x8 *)(b + swz(wm * TM + i * 16 + fr, ks * 4 + fc));
#pragma unroll
            for (int j = 0; j < SNT; ++j) wf[j] = *(const bf16x8 *)(b + swz(CBM + wn * TN + j * 16 + fr, ks * 4 + fc));
#pragma unroll
            for (int i = 0; i < SM; ++i)
#pragma unroll
                for (int j = 0; j < SNT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
        }
        if (++kt < nk) continue;
        // epilogue: the residual image retired (younger: the ≤ NS − 1 stages issued after
        // stage g, all after it), then visible to every wave
        if (RES) {
            const int en = left < NS - 1 ? (int)left : NS - 1;
            if (en == 2) cp_wait<2 * PW>();
            else if (en == 1) cp_wait<PW>();
            else cp_wait<0>();
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        const int n = n0 + wn * TN + (odd ? 16 : 0) + (fc >> 1) * 8;
        float bb[8];
        unpack8(*(const uint4 *)(pbias + n), bb);
#pragma unroll
        for (int i = 0; i < SM; ++i) {
            float o[8];
            pair8(acc[i][0], acc[i][1], odd, o);
            acc[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
            acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int rl = wm * TM + i * 16 + fr;
            const int64_t m = m0 + rl;
            const int64_t row = m * a.c_stride + a.c_off + phase;
            add_n<8>(o, bb);
            rbf_n<8>(o);
            if constexpr (RES) {
                float rr[8];
                const int cl = (n - n0) >> 3;           // 16-B chunk of the item's 128 columns
                unpack8(*(const uint4 *)(resb + rl * 256 + ((cl ^ (rl & 15)) << 4)), rr);
                add_n<8>(o, rr);
                rbf_n<8>(o);
            }
            float sn[8];
            if constexpr (SN) {
                snake_n<8>(o, psa + n, psib + n, sn);
            }
            if (m < a.M && row >= 0 && row < a.L_out) {
                if constexpr (RAW) *(uint4 *)(a.out + row * a.N + n) = pack8(o);
                if constexpr (SN) *(uint4 *)(a.out_s + row * a.N + n) = pack8(sn);
            }
        }
        prev_st = m0 + CBM <= a.M && m0 * a.c_stride + a.c_off + phase >= 0 &&
                  (m0 + CBM - 1) * a.c_stride + a.c_off + phase < a.L_out;
        kt = 0;
        if (++phase == phases) {
            phase = 0;
            n0 += CBN;
            if (n0 == a.N) { n0 = 0; m0 += CBM; }
        }
    }
}

// Fused Oobleck residual unit at C = 128 (vae_model.py:62-87):
//   y_s = snake2(conv7_dil(x_s) + b1)            (kept in LDS, never in HBM)
//   x'  = x + (W2·y_s + b2);  x'_s = snake_next(x')
// One 128-position tile per block: the k=7 GEMM (K = 896) through the
// 2-stage glds ring, its epilogue writes y_s into the swizzled LDS image of
// the k=1 GEMM's A operand, W2 (128×128) is staged alongside, then the k=1
// GEMM (K = 128) and the residual / next-Snake epilogue.
template <bool RAW>
__global__ __launch_bounds__(256, 2) void resunit128_kernel(ResUnitArgs u) {
    constexpr int BM = 128, STAGE = ConvTile::STAGE;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
    const ConvArgs &a = u.c1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t tilesM = (a.M + BM - 1) / BM;
    const int64_t m0 = (int64_t)xcd_remap(blockIdx.x, (int)tilesM) * BM;
    const int K = a.taps * 128;
    int rowq[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) rowq[i] = (wave + 4 * i) * 8 + (lane >> 3);
    auto stage = [&](int buf, int k0) {
        char *b = lds + buf * STAGE;
        const int tap = k0 >> 7, ci0 = k0 & 127;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = rowq[i];
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const bf16_t *src = r < BM ? a_src(a, m0 + r, tap, ci0, c) : a.W + (int64_t)(r - BM) * K + k0 + c * 8;
            glds16(src, b + (wave + 4 * i) * 1024);
        }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
    stage(0, 0);
    const int fr = lane & 15, fc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * BK);
        const char *b = lds + (kt & 1) * STAGE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xf[4], wf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xf[i] = *(const bf16x8 *)(b + swz(wm * 64 + i * 16 + fr, ks * 4 + fc));
                wf[i] = *(const bf16x8 *)(b + swz(BM + wn * 64 + i * 16 + fr, ks * 4 + fc));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
        }
    }
    // all waves done reading the ring; reuse it: [y_s k 0..63 | y_s k 64..127 | W2 k 0..63 | W2 k 64..127]
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char *ys = lds;                 // 2 × 16 KiB
    char *w2 = lds + 2 * 16384;     // 2 × 16 KiB
    // W2 [128][128] → 2 k-halves of [128 rows][64]: 32 glds, 8 per wave
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int qq = wave + 4 * i;        // 0..31: half = qq >> 4, rows 8(qq&15)..+7
        const int h = qq >> 4, r = (qq & 15) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        glds16(u.W2 + (int64_t)r * 128 + h * 64 + c * 8, w2 + h * 16384 + (qq & 15) * 1024);
    }
    // epilogue 1: y_s = snake2(bf16(acc + b1)) → LDS (A image of the k=1 GEMM)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = wn * 64 + j * 16 + fc * 4;
            float bb[4];
            unpack4(*(const uint2 *)(a.bias + n), bb);
            const float4 sa = *(const float4 *)(a.sa + n);
            const float4 sb = *(const float4 *)(a.sib + n);
            const float sav[4] = {sa.x, sa.y, sa.z, sa.w}, sbv[4] = {sb.x, sb.y, sb.z, sb.w};
            float o[4];
            float t[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            add_n<4>(t, bb);
            rbf_n<4>(t);
            snake_n<4>(t, sav, sbv, o);
            const int h = n >> 6, cc = (n & 63) >> 3;
            *(uint2 *)(ys + h * 16384 + swz(row, cc) + (n & 7) * 2) = pack4(o);
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // k=1 GEMM: K = 128 = 2 halves × 2 k-steps
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xf[4], wf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xf[i] = *(const bf16x8 *)(ys + h * 16384 + swz(wm * 64 + i * 16 + fr, ks * 4 + fc));
                wf[i] = *(const bf16x8 *)(w2 + h * 16384 + swz(wn * 64 + i * 16 + fr, ks * 4 + fc));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
        }
    // epilogue 2: x' = x + bf16(acc + b2); raw (optional) + snake_next
    const bool odd = fc & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t m = m0 + wm * 64 + i * 16 + fr;
        if (m >= a.M) continue;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            float o[8], bb[8], rr[8];
            pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
            const int n = wn * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8;
            unpack8(*(const uint4 *)(u.b2 + n), bb);
            unpack8(*(const uint4 *)(u.x + m * 128 + n), rr);
            add_n<8>(o, bb);
            rbf_n<8>(o);
            add_n<8>(o, rr);
            rbf_n<8>(o);
            if constexpr (RAW) *(uint4 *)(u.x + m * 128 + n) = pack8(o);
            float sn[8];
            snake8(o, u.sa_next + n, u.sib_next + n, sn);
            *(uint4 *)(u.out_s + m * 128 + n) = pack8(sn);
        }
    }
}

// ---------------------------------------------------------------------------
// k=7 dilated stride-1 convolution with the INPUT WINDOW staged once per channel
// chunk instead of an im2col tile per tap (conv_gemm_kernel fetches every input row
// 7× through L2 and waits vmcnt(0) on a one-tile ring every K-tile).
// Tile 256 positions × 128 output channels, 8 waves (4 M × 2 N, 64×64 wave tiles).
// K loop: kt = cc·7 + tap over 64-channel chunks cc; per K-tile the A fragments
// come from the window image of chunk cc (row = position − m0 + 3·dil + tap·dil −
// 3·dil), the W tile (128 rows × 64 k) from a 3-slot ring.  One barrier per K-tile:
//   top of kt   own DMAs of W(kt) (and, older, window(cc)) retired — counted vmcnt,
//               newer W(kt+1) / window(cc+1) stay in flight — then the barrier
//   after it    stage W(kt+2) into slot (kt+2)%3 (tile kt−1's, read before the
//               barrier), and at tap 0 window(cc+1) into the other window buffer
//               (chunk cc−1's, last read at K-tile kt−1).
// Window image: 128-B rows (64 channels), physical chunk = chunk ^ (row & 7), which
// keeps every ds_read_b128 lane group conflict-free for ANY row offset (the tap
// shift tap·dil misaligns the fragment rows; tools/conv_swizzle check, r02).
// FUSED (C = 128): the residual unit — y_s = snake2(conv7 + b1) into LDS, then the
// k=1 GEMM with W2 and x' = x + (W2·y_s + b2), snaked for the next unit.
// Two geometries: BM = 256 / 8 waves / 3 W slots (128 KiB LDS, one block per CU) and
// BM = 128 / 4 waves / 2 W slots (80 KiB: two blocks per CU, whose epilogues and main
// loops interleave — the epilogue VALU (bias, bf16 rounding, Snake) is ≈ the MFMA time)
template <int BM_>
struct Conv7 {
    static constexpr int BM = BM_, BN = 128, NW = BM / 32;
    static constexpr int WSLOTS = BM == 256 ? 3 : 2;
    static constexpr int WROWS = BM == 256 ? 320 : 192;      // window rows ≥ BM + 6·9
    static constexpr int WIN = WROWS * 128;                  // one window buffer (64 channels)
    static constexpr int WT = BN * 128;                      // 16 KiB per W tile
    static constexpr int LDS = 2 * WIN + WSLOTS * WT;        // 128 / 80 KiB
    static constexpr int PWIN = WROWS / 8 / NW;              // window pieces per wave (5 / 6)
    static constexpr int PW = BN / 8 / NW;                   // W pieces per wave (2 / 4)
    static_assert(PWIN * 8 * NW == WROWS && PW * 8 * NW == BN, "pieces split evenly over the waves");
};
#ifndef CONV7_BM
#define CONV7_BM 128
#endif
__device__ __forceinline__ int sw7(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <int BM_, bool FUSED, bool RAW>
__global__ __launch_bounds__(BM_ * 2, BM_ == 256 ? 1 : 2) void conv7_kernel(ConvArgs a, ResUnitArgs u) {
    using C7 = Conv7<BM_>;
    constexpr int BM = C7::BM, BN = C7::BN;
    __shared__ __attribute__((aligned(16))) char lds[C7::LDS];
    char *win = lds, *wring = lds + 2 * C7::WIN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tilesN = a.N / BN;
    const int64_t tilesM = (a.M + BM - 1) / BM;
    const int64_t wg = xcd_remap(blockIdx.x, (int)(tilesM * tilesN));
    const int64_t m0 = (wg / tilesN) * BM;
    const int n0 = (int)(wg % tilesN) * BN;
    const int dil = a.dil, Cin = a.Cin, K = 7 * Cin;
    const int nch = Cin / 64, nk = 7 * nch;

    auto stage_win = [&](int buf, int cc) {
#pragma unroll
        for (int i = 0; i < C7::PWIN; ++i) {
            const int q = wave + C7::NW * i, row = q * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (row & 7);
            const int64_t pos = m0 - 3 * dil + row;
            const bf16_t *src = (row < BM + 6 * dil && pos >= 0 && pos < a.L_in)
                                    ? a.in + pos * Cin + cc * 64 + c * 8 : a.zero + c * 8;
            glds16(src, win + buf * C7::WIN + q * 1024);
        }
    };
    auto stage_w = [&](int slot, int kt) {
        const int cc = kt / 7, tap = kt - cc * 7;
#pragma unroll
        for (int i = 0; i < C7::PW; ++i) {
            const int q = wave + C7::NW * i, row = q * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (row & 7);
            glds16(a.W + (int64_t)(n0 + row) * K + tap * Cin + cc * 64 + c * 8, wring + slot * C7::WT + q * 1024);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fc = lane >> 4;
    const bool odd = fc & 1;
    // residual-unit tail operands (x, b2) loaded up front: they land during the main
    // loop (older than every DMA, so the loop's counted waits are unaffected)
    uint4 xv[4][2], b2v[2];
    if constexpr (FUSED) {
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            const int n = wn * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8;
            b2v[jp] = *(const uint4 *)(u.b2 + n);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t m = min(m0 + wm * 64 + i * 16 + fr, a.M - 1);
                xv[i][jp] = *(const uint4 *)(u.x + m * 128 + n);
            }
        }
    }
    stage_win(0, 0);
    stage_w(0, 0);
    if (C7::WSLOTS == 3 && nk > 1) stage_w(1, 1);
    for (int kt = 0; kt < nk; ++kt) {
        const int cc = kt / 7, tap = kt - cc * 7;
        // own DMAs newer than W(kt): W(kt+1) (issued at kt−1) and a window refill issued at
        // kt−1 or kt−2 (at a tap 0, right after that iteration's W refill)
        // (3 W slots: W(kt+1) is newer, issued at kt−1; 2 slots: W(kt+1) is staged after
        // this wait, and only a window refill at kt−1 is newer)
        const bool w1 = C7::WSLOTS == 3 && kt + 1 < nk;
        const bool wn1 = (kt >= 1 && (kt - 1) % 7 == 0 && (kt - 1) / 7 + 1 < nch) ||
                         (C7::WSLOTS == 3 && kt >= 2 && (kt - 2) % 7 == 0 && (kt - 2) / 7 + 1 < nch);
        if (w1 && wn1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(C7::PW + C7::PWIN) : "memory");
        else if (w1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(C7::PW) : "memory");
        else if (wn1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(C7::PWIN) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + C7::WSLOTS - 1 < nk)
            stage_w((kt + C7::WSLOTS - 1) % C7::WSLOTS, kt + C7::WSLOTS - 1);
        if (tap == 0 && cc + 1 < nch) stage_win((cc + 1) & 1, cc + 1);
        const char *wb = win + (cc & 1) * C7::WIN, *tb = wring + (kt % C7::WSLOTS) * C7::WT;
        const int rb = wm * 64 + tap * dil + fr;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xf[4], wf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xf[i] = *(const bf16x8 *)(wb + sw7(rb + i * 16, ks * 4 + fc));
                wf[i] = *(const bf16x8 *)(tb + sw7(wn * 64 + i * 16 + fr, ks * 4 + fc));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
        }
    }

    if constexpr (!FUSED) {
        // conv output → bf16 (+bias) → Snake → out_s (the next conv's input)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t m = m0 + wm * 64 + i * 16 + fr;
            if (m >= a.M) continue;
#pragma unroll
            for (int jp = 0; jp < 2; ++jp) {
                float o[8];
                pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
                const int n = n0 + wn * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8;
                if (a.bias) {
                    float bb[8];
                    unpack8(*(const uint4 *)(a.bias + n), bb);
                    add_n<8>(o, bb);
                }
                rbf_n<8>(o);
                float sn[8];
                snake8(o, a.sa + n, a.sib + n, sn);
                *(uint4 *)(a.out_s + m * a.N + n) = pack8(sn);
            }
        }
    } else {
        // residual unit tail (C = 128): every wave done with the window / ring
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        constexpr int YH = BM * 128;    // y_s image: 2 k-halves × [BM rows][128 B]
        char *ys = lds;
        char *w2 = lds + 2 * YH;        // W2: 2 k-halves × [128 rows][128 B] = 32 KiB
        static_assert(2 * YH + 32768 <= C7::LDS, "residual-unit tail must fit the LDS");
        // W2 [128][128] → 2 k-halves: 32 glds
#pragma unroll
        for (int i = 0; i < 32 / C7::NW; ++i) {
            const int qq = wave + C7::NW * i;  // 0..31: half = qq >> 4, rows 8(qq&15)..+7
            const int h = qq >> 4, r = (qq & 15) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (r & 7);
            glds16(u.W2 + (int64_t)r * 128 + h * 64 + c * 8, w2 + h * 16384 + (qq & 15) * 1024);
        }
        // epilogue 1: y_s = snake2(bf16(acc + b1)) → LDS (A image of the k=1 GEMM)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = wm * 64 + i * 16 + fr;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = wn * 64 + j * 16 + fc * 4;
                float bb[4];
                unpack4(*(const uint2 *)(a.bias + n), bb);
                const float4 sa = *(const float4 *)(a.sa + n);
                const float4 sb = *(const float4 *)(a.sib + n);
                const float sav[4] = {sa.x, sa.y, sa.z, sa.w}, sbv[4] = {sb.x, sb.y, sb.z, sb.w};
                float o[4];
                float t[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                add_n<4>(t, bb);
                rbf_n<4>(t);
                snake_n<4>(t, sav, sbv, o);
                const int h = n >> 6, cc = (n & 63) >> 3;
                *(uint2 *)(ys + h * YH + sw7(row, cc) + (n & 7) * 2) = pack4(o);
                acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // k=1 GEMM: K = 128 = 2 halves × 2 k-steps
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 xf[4], wf[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    xf[i] = *(const bf16x8 *)(ys + h * YH + sw7(wm * 64 + i * 16 + fr, ks * 4 + fc));
                    wf[i] = *(const bf16x8 *)(w2 + h * 16384 + sw7(wn * 64 + i * 16 + fr, ks * 4 + fc));
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
            }
        // epilogue 2: x' = x + bf16(acc + b2); raw (optional) + snake_next
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t m = m0 + wm * 64 + i * 16 + fr;
            if (m >= a.M) continue;
#pragma unroll
            for (int jp = 0; jp < 2; ++jp) {
                float o[8], bb[8], rr[8];
                pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
                const int n = wn * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8;
                unpack8(b2v[jp], bb);
                unpack8(xv[i][jp], rr);
                add_n<8>(o, bb);
                rbf_n<8>(o);
                add_n<8>(o, rr);
                rbf_n<8>(o);
                if constexpr (RAW) *(uint4 *)(u.x + m * 128 + n) = pack8(o);
                float sn[8];
                snake8(o, u.sa_next + n, u.sib_next + n, sn);
                *(uint4 *)(u.out_s + m * 128 + n) = pack8(sn);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Persistent, software-pipelined Oobleck residual unit at C = 128 (vae_model.py:62-87):
//   y_s = snake2(conv7_dil(x_s) + b1);  x' = x + (W2·y_s + b2);  out_s = snake_next(x')
// conv7_kernel<FUSED> runs one tile per block; its per-tile tail (W2 staging, epilogue
// parameter loads, the y_s LDS round trip, two barriers, the k=1 GEMM, the stores) measured
// more than half of the kernel (r02: decode −11 ms with the tail skipped).  Here every block
// walks a contiguous range of 128-row tiles:
//  * each wave owns 32 rows × all 128 channels, so y_s never leaves registers: the k=7
//    accumulators (lane: row fr, channels 16j + 4fc + r) ARE the B operand of the k=1 MFMA
//    once W2's columns are permuted within each 32-block (permute_k1_kernel);
//  * the W stream has 16 K-tiles per row tile — 14 k=7 (tap, 64-channel chunk) tiles, then
//    W2's two 64-column halves — through a 2-slot ring that waves 0-2 refill one K-tile
//    ahead (wrapping into the next tile's W(0)), so W2 arrives like any W tile;
//  * wave 3 alone stages the input windows (x_s rows m0−3d … m0+127+3d: 182 rows × 64
//    channels per chunk, chunk c in buffer c) a tile ahead: chunk 0 of tile t+1 behind
//    K-tiles 7–12 (buffer 0 is free after K-tile 6), chunk 1 after the epilogue and behind
//    K-tiles 0–3.  vmcnt is per wave: the W waves' one-K-tile waits never include a window
//    piece, and wave 3 waits only where a chunk is consumed (K-tiles 0 and 7);
//  * the epilogue parameters (b1, b2, both Snakes) sit in LDS; x (the residual) is loaded
//    two K-tiles before its use.
// LDS: 2 560 (parameters) + 2 × 23 296 (windows) + 2 × 16 KiB (W ring) = 80 KiB: two blocks
// per CU, whose K-loops and epilogues interleave.
namespace ru {
constexpr int BM = 128, WROWS = 182, WINB = WROWS * 128, WT = 128 * 128, PAR = 2560;
constexpr int LDS = 2 * WINB + 2 * WT + PAR;
constexpr int NPW = (WROWS + 7) / 8;   // 23 window pieces (8 rows) per chunk; the last is 6 rows
static_assert(LDS <= 81920, "two blocks per CU");
}  // namespace ru

// The kernel's LDS-DMA is inline asm (global_load_lds, saddr form: SGPR
// base + one 32-bit VGPR lane offset) with explicit counted waits:
//  * the builtin LDS-DMA forms either build a 64-bit VGPR address per piece (46 window + 16 W
//    pieces per tile: hoisted and spilled, and every spill reload waits vmcnt(0)) or, for
//    the buffer form, make the compiler wait vmcnt(0) before every LDS read;
//  * the compiler, not seeing these loads, inserts no vmcnt waits for them (the x loads,
//    which fill registers, stay compiler-visible).
// M0 (the LDS destination) is set in the same asm; nothing else in this kernel uses M0.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ru_dma(const char *base, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr), "v"(voff), "s"(base)
                 : "memory");
}

// window pieces [P0, P1) (8 rows each) of 64-channel chunk cc for the tile at m0, from input
// row m0 − 3d + 8·P0 (≥ −27, and ≤ L_in + 181 at the end: the input carries zero rows in
// front and zeroed / addressable rows behind, ResUnitArgs::in_zero_pad); lanes of rows
// ≥ WROWS are masked off.  buf: LDS address; voff: (lane>>3)·256 + swizzled chunk + cc·128.
template <int P0, int P1>
__device__ __forceinline__ void ru_win(const ConvArgs &a, uint32_t buf, int64_t m0, uint32_t voff, int lane) {
    const char *base = (const char *)(a.in + (m0 - 3 * a.dil + P0 * 8) * 128);
#pragma unroll
    for (int q = P0; q < P1; ++q) {
        if (q * 8 + 8 <= ru::WROWS || (lane >> 3) < ru::WROWS - q * 8)
            ru_dma(base, buf + q * 1024, voff + (q - P0) * 2048);
    }
}

// W K-tile kt (0-13: W1 tap kt%7 of chunk kt/7; 14, 15: W2 column half kt−14) into the ring
// slot at LDS address `slot`: 16 pieces of 8 rows, piece q by wave q % 3; voff1 / voff2: lane
// offsets in the 1792-B W1 rows and the 256-B W2 rows
__device__ __forceinline__ void ru_w(const ResUnitArgs &u, uint32_t slot, int kt, int wave, uint32_t voff1,
                                     uint32_t voff2) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int q = wave + 3 * i;
        if (q < 16) {
            if (kt < 14) {
                const int cc = kt >= 7 ? 1 : 0, tap = kt - 7 * cc;
                ru_dma((const char *)u.c1.W + q * 8 * 1792 + tap * 256 + cc * 128, slot + q * 1024, voff1);
            } else {
                ru_dma((const char *)u.W2p + q * 8 * 256 + (kt - 14) * 128, slot + q * 1024, voff2);
            }
        }
    }
}

template <bool RAW>
__global__ __launch_bounds__(256, 2) void ru7_kernel(ResUnitArgs u, int64_t ntiles) {
    constexpr int RBM = ru::BM, WINB = ru::WINB, WT = ru::WT, NPW = ru::NPW;
    __shared__ __attribute__((aligned(16))) char lds[ru::LDS];
    const ConvArgs &a = u.c1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool dma = wave == 3;
    const int fr = lane & 15, fc = lane >> 4;
    const bool odd = fc & 1;
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    if (t0 >= t1) return;
    // parameters first: their per-lane reads then fold into the 16-bit ds offset field
    // parameters first: their per-lane reads then fold into the 16-bit ds offset field
    char *par = lds, *win = lds + ru::PAR, *wr = win + 2 * WINB;
    const uint32_t win3 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)lds + ru::PAR;
    const uint32_t wr3 = win3 + 2 * WINB;                                 // LDS-DMA destinations
    float *psa2 = (float *)par, *psib2 = psa2 + 128, *psan = psa2 + 256, *psibn = psa2 + 384;
    bf16_t *pb1 = (bf16_t *)(par + 2048), *pb2 = (bf16_t *)(par + 2304);
    if (tid < 128) {
        psa2[tid] = a.sa[tid]; psib2[tid] = a.sib[tid];
        psan[tid] = u.sa_next[tid]; psibn[tid] = u.sib_next[tid];
        pb1[tid] = a.bias[tid]; pb2[tid] = u.b2[tid];
    }
    __builtin_amdgcn_s_waitcnt(0x0070);          // parameter loads retired before the first DMA
    // DMA lane offsets: row lane>>3 of a piece, 16-B chunk swizzled by row & 7 (= lane>>3)
    const int l3 = lane >> 3, lc = ((lane & 7) ^ l3) * 16;
    const uint32_t vw0 = l3 * 256 + lc, vw1 = vw0 + 128;          // window chunk 0 / 1
    const uint32_t vk1 = l3 * 1792 + lc, vk2 = l3 * 256 + lc;       // W1 / W2 rows
    if (dma) {
        ru_win<0, NPW>(a, win3, t0 * RBM, vw0, lane);
        ru_win<0, 8>(a, win3 + WINB, t0 * RBM, vw1, lane);
    } else {
        ru_w(u, wr3, 0, wave, vk1, vk2);
    }
    // W fragment lane offsets: rows 16j + fr, 16-B chunk 4ks + fc (swizzled like the DMA)
    const int wl[2] = {fr * 128 + ((fc ^ (fr & 7)) << 4), fr * 128 + (((4 + fc) ^ (fr & 7)) << 4)};

    f32x4 acc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int64_t t = t0; t < t1; ++t) {
        const int64_t m0 = t * RBM;
        const bool more = t + 1 < t1;
        u32x4 xv[2][4];
        bf16x8 yf[2][4];
        auto ktile = [&](const int kt, auto SLOTC) {
            constexpr int SLOT = decltype(SLOTC)::value;
            // W waves: W(kt) (issued at kt−1) retired; younger only x (issued at 14 after W(15)).
            // Wave 3: chunk 0 (K-tile 0; younger: chunk 1's first 8 pieces) or chunk 1 (K-tile 7).
            if (!dma) {
                if (kt == 15) __builtin_amdgcn_s_waitcnt(0x0078);       // vmcnt(8) lgkmcnt(0)
                else __builtin_amdgcn_s_waitcnt(0x0070);
            } else {
                if (kt == 0) __builtin_amdgcn_s_waitcnt(0x0078);
                else if (kt == 7) __builtin_amdgcn_s_waitcnt(0x0070);
                else __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0) only
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (!dma) {
                if (kt < 15 || more) ru_w(u, wr3 + (SLOT ^ 1) * WT, kt == 15 ? 0 : kt + 1, wave, vk1, vk2);
            } else if (kt == 0) {
                ru_win<8, 12>(a, win3 + WINB, m0, vw1, lane);
            } else if (kt == 1) {
                ru_win<12, 16>(a, win3 + WINB, m0, vw1, lane);
            } else if (kt == 2) {
                ru_win<16, 20>(a, win3 + WINB, m0, vw1, lane);
            } else if (kt == 3) {
                ru_win<20, NPW>(a, win3 + WINB, m0, vw1, lane);
            } else if (more) {
                if (kt == 7) ru_win<0, 4>(a, win3, m0 + RBM, vw0, lane);
                else if (kt == 8) ru_win<4, 8>(a, win3, m0 + RBM, vw0, lane);
                else if (kt == 9) ru_win<8, 12>(a, win3, m0 + RBM, vw0, lane);
                else if (kt == 10) ru_win<12, 16>(a, win3, m0 + RBM, vw0, lane);
                else if (kt == 11) ru_win<16, 20>(a, win3, m0 + RBM, vw0, lane);
                else if (kt == 12) ru_win<20, NPW>(a, win3, m0 + RBM, vw0, lane);
            }
            if (kt == 14) {
                // x (residual) rows of this wave: 8 loads, waited before epilogue 2
                const char *xb = (const char *)(u.x + m0 * 128);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jp = 0; jp < 4; ++jp) {
                        const int r = (int)min((int64_t)(32 * wave + 16 * i + fr), a.M - 1 - m0);
                        const uint32_t off = (uint32_t)(r * 128 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8) * 2;
                        xv[i][jp] = *(const u32x4 *)(xb + off);
                    }
            }
            const char *tb = wr + SLOT * WT;
            if (kt < 14) {
                const int cc = kt >= 7 ? 1 : 0, tap = kt - 7 * cc;
                int dl = a.dil;
                asm volatile("" : "+s"(dl));    // per-tap address math stays here (not hoisted out of the tile loop)
                const int rb = 32 * wave + fr + tap * dl;
                const char *wb = win + cc * WINB + rb * 128;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int xo = ((4 * ks + fc) ^ (rb & 7)) << 4;
                    bf16x8 xf[2], wf[8];
                    xf[0] = *(const bf16x8 *)(wb + xo);
                    xf[1] = *(const bf16x8 *)(wb + 2048 + xo);
#pragma unroll
                    for (int j = 0; j < 8; ++j) wf[j] = *(const bf16x8 *)(tb + j * 2048 + wl[ks]);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
                }
            } else {
                constexpr int h = SLOT;       // K-tiles 14 / 15 sit in slots 0 / 1
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    bf16x8 wf[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) wf[j] = *(const bf16x8 *)(tb + j * 2048 + wl[ks]);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], yf[i][2 * h + ks], acc[i][j],
                                                                                0, 0, 0);
                }
            }
            if (kt == 13) {
                // epilogue 1: y_s = snake2(bf16(acc + b1)) → the k=1 B fragments (k-step s =
                // channel tiles 2s, 2s+1: lane group fc holds channels 32s + 4fc + {0-3, 16-19})
                uint2 yv[2][8];
                int pl = 4 * fc;
                asm volatile("" : "+v"(pl));
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int n = 16 * j + pl;
                    float b[4];
                    unpack4(*(const uint2 *)(pb1 + n), b);
                    const float4 sa = *(const float4 *)(psa2 + n), sb = *(const float4 *)(psib2 + n);
                    const float sav[4] = {sa.x, sa.y, sa.z, sa.w}, sbv[4] = {sb.x, sb.y, sb.z, sb.w};
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        float o[4];
                        float t[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                        add_n<4>(t, b);
                        rbf_n<4>(t);
                        snake_n<4>(t, sav, sbv, o);
                        yv[i][j] = pack4(o);
                        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    }
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int s = 0; s < 4; ++s)
                        yf[i][s] = __builtin_bit_cast(bf16x8, make_uint4(yv[i][2 * s].x, yv[i][2 * s].y,
                                                                         yv[i][2 * s + 1].x, yv[i][2 * s + 1].y));
            }
        };
        // K-tiles 0-11 in a loop; 12-15 peeled so that x and the y_s fragments are not
        // loop-carried (they would pin 64 VGPRs through the whole K loop)
#pragma unroll 1
        for (int kt = 0; kt < 12; kt += 2) {
            ktile(kt, std::integral_constant<int, 0>{});
            ktile(kt + 1, std::integral_constant<int, 1>{});
        }
        ktile(12, std::integral_constant<int, 0>{});
        ktile(13, std::integral_constant<int, 1>{});
        ktile(14, std::integral_constant<int, 0>{});
        ktile(15, std::integral_constant<int, 1>{});
        // epilogue 2: x' = x + bf16(acc + b2) (raw, optional) and snake_next(x') → out_s.
        // (x is a compiler-visible load: an asm load's destination registers may be copied by
        // the register allocator before an asm wait retires them; the compiler's own wait
        // here is vmcnt(0), which also retires the W waves' W(0) pieces of the next tile)
        int64_t me = m0;
        asm volatile("" : "+s"(me));
        int pl2 = (odd ? 16 : 0) + (fc >> 1) * 8;
        asm volatile("" : "+v"(pl2));
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
            const int n = 32 * jp + pl2;
            float bb[8];
            unpack8(*(const uint4 *)(pb2 + n), bb);
            const float4 a0 = *(const float4 *)(psan + n), a1 = *(const float4 *)(psan + n + 4);
            const float4 s0 = *(const float4 *)(psibn + n), s1 = *(const float4 *)(psibn + n + 4);
            const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float o[8], rr[8], sn[8];
                pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
                acc[i][2 * jp] = f32x4{0.f, 0.f, 0.f, 0.f};
                acc[i][2 * jp + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
                unpack8(make_uint4(xv[i][jp].x, xv[i][jp].y, xv[i][jp].z, xv[i][jp].w), rr);
                add_n<8>(o, bb);
                rbf_n<8>(o);
                add_n<8>(o, rr);
                rbf_n<8>(o);
                snake_n<8>(o, av, sv, sn);
                const int64_t m = me + 32 * wave + 16 * i + fr;
                if (m < a.M) {
                    if constexpr (RAW) *(uint4 *)(u.x + m * 128 + n) = pack8(o);
                    *(uint4 *)(u.out_s + m * 128 + n) = pack8(sn);
                }
            }
        }
        // chunk 1 of the next tile: buffer 1 was last read at K-tile 13
        if (dma && more) ru_win<0, 8>(a, win3 + WINB, m0 + RBM, vw1, lane);
    }
}

// ---------------------------------------------------------------------------
// The same residual unit on 256-row tiles, one block per CU (ru8_kernel).  ru7_kernel streams
// the whole 256 KiB W1 | W2 stream through LDS once per 128 rows, one K-tile ahead, and its MFMA
// waves issue those LDS-DMA pieces themselves: per tile the W refill alone measured 2.7 of the
// ≈ 6 ms of a 11.52 M-row unit (r02), MFMA-busy 33 %.  Here:
//  * four MFMA waves own 64 rows × 128 channels each (4 row fragments: 128 accumulators), so the
//    W stream is paid once per 256 rows, and W(kt) is consumed by 4 × 64 MFMAs per wave;
//  * two helper waves issue every LDS-DMA piece (window chunks and W K-tiles) — the MFMA waves
//    carry none in their stream (the GEMM's half-chip tile measured the same lever);
//  * W runs through a 3-slot ring two K-tiles ahead (W(kt+2) issued behind barrier kt into the
//    slot of K-tile kt−1): a piece has two K-tile intervals (≈ 1 µs) to land.
// Helper step kt (behind barrier kt) issues its window pieces first, then W: the chunk-1 window
// of THIS tile (pieces 14-38, steps 0-3 — not for the block's first tile, whose windows the
// prologue stages whole), the chunk-0 window of the NEXT tile (steps 7-12: buffer 0 was last
// read at K-tile 6) and the first part of its chunk 1 (steps 14-15: buffer 1 last read at 13),
// then W(kt+2) (steps 14-15: W(0), W(1) of the next tile).  Before barrier kt a helper waits
// until at most the pieces of its step kt−1 are in flight: W(kt) and every window piece issued
// before it have landed (vmcnt retires in order), and every chunk a K-tile reads was issued
// before the W that K-tile's barrier waits for.
// LDS: 2 560 (parameters) + 2 × 39 680 (windows: 310 rows × 64 channels) + 3 × 16 KiB = 128 KiB.
template <int V>
using IC7 = std::integral_constant<int, V>;
template <int I0, int I1, typename F>
__device__ __forceinline__ void sfor(F &&f) {     // compile-time unrolled loop (f gets an integral_constant)
    if constexpr (I0 < I1) {
        f(std::integral_constant<int, I0>{});
        sfor<I0 + 1, I1>(f);
    }
}
namespace ru8 {
// W ring distance: W(kt + D) is issued behind barrier kt into the slot of K-tile kt − 1 (D + 1
// slots).  Measured (tools/ab_vae.py, one process, bit-identical): D = 3 (4 slots) 39.93 vs 39.90
// ms per decode; D = 3 with the MFMA waves reading K-tile kt+1's k-step-0 fragments during
// K-tile kt 40.61 (`profiles/r04ru8d_ab.log`) — W latency is not what bounds this kernel
constexpr int D = 2;
constexpr int BM = 256, WROWS = 310, WINB = WROWS * 128, WT = 128 * 128, PAR = 2560, NSLOT = D + 1;
constexpr int LDS = PAR + 2 * WINB + NSLOT * WT;
constexpr int NPW = (WROWS + 7) / 8;   // 39 window pieces (8 rows) per chunk; the last is 6 rows
static_assert(LDS <= 160 * 1024, "LDS");
static_assert(BM + 54 <= WROWS, "halo of dilation 9");
static_assert(WROWS - 3 <= kResWindowBackRows, "the activation back pad covers the last tile's window");
// (chunk 0 of the next tile, steps 7-12, is issued before W(0'), step 16 − D; chunk 1's pieces of
// steps 0-3 before W(7), step 7 − D — so waiting for a K-tile's W also covers its window chunk)
static_assert(16 - D > 12 && 7 - D > 3, "window pieces ordered before the W that guards them");
// window piece ranges per helper step: chunk 0 of the next tile over steps 7-12; chunk 1 of the
// next tile over steps 14-15 (pieces 0-13) and of the current one over steps 0-3 (14-38)
__host__ __device__ constexpr int c0_lo(int s) { return s == 0 ? 0 : s == 1 ? 7 : s == 2 ? 14 : s == 3 ? 20 : s == 4 ? 26 : 33; }
__host__ __device__ constexpr int c0_hi(int s) { return s == 5 ? NPW : c0_lo(s + 1); }
__host__ __device__ constexpr int c1a_lo(int s) { return s == 0 ? 0 : 7; }
__host__ __device__ constexpr int c1a_hi(int s) { return s == 0 ? 7 : 14; }
__host__ __device__ constexpr int c1b_lo(int s) { return s == 0 ? 14 : s == 1 ? 20 : s == 2 ? 26 : 33; }
__host__ __device__ constexpr int c1b_hi(int s) { return s == 3 ? NPW : c1b_lo(s + 1); }
// pieces q in [a, b) with q % 2 == h (helper h's share)
__host__ __device__ constexpr int share(int a, int b, int h) { return (b - h + 1) / 2 - (a - h + 1) / 2; }
// DMA instructions helper h issues in step s (window pieces + 8 W pieces), for a tile that is
// (not) the block's first and has (no) successor
__host__ __device__ constexpr int step_count(int s, int h, bool first, bool more) {
    int n = 0;
    if (s <= 3 && !first) n += share(c1b_lo(s), c1b_hi(s), h);
    if (s >= 7 && s <= 12 && more) n += share(c0_lo(s - 7), c0_hi(s - 7), h);
    if (s >= 14 && more) n += share(c1a_lo(s - 14), c1a_hi(s - 14), h);
    if (s + D <= 15 || more) n += 8;
    return n;
}
// pieces helper h may leave in flight before barrier kt: everything issued after W(kt) (issued in
// step kt − D, a step of the previous tile when negative, or by the first tile's prologue:
// chunk 0, W(0), chunk 1, W(1) … W(D − 1))
__host__ __device__ constexpr int allowed(int kt, int h, bool first, bool more) {
    const int need = kt;
    int n = 0;
    if (first && need < D) {
        n = (D - 1 - need) * 8 + (need == 0 ? share(0, NPW, h) : 0);
        for (int s = 0; s < kt; ++s) n += step_count(s, h, true, more);
        return n;
    }
    for (int s = need - D + 1; s < kt; ++s)
        n += s >= 0 ? step_count(s, h, first, more) : step_count(s + 16, h, false, true);
    return n;
}
// snake_in (SIN) variant: one wave issues every W piece (16 per K-tile), so before barrier kt
// the W pieces newer than W(kt) are those of K-tiles kt+1 .. kt+D−1 already issued
__host__ __device__ constexpr int w_newer(int kt, bool more) {
    int n = 0;
    for (int j = kt + 1; j < kt + D; ++j)
        if (j <= 15 || more) n += 16;
    return n;
}
// window pieces per step in the SIN variant (loads issued in step s, snaked and written to LDS in
// step s + 1): chunk 1 of the current tile (steps 0-3, not the block's first tile), chunk 0 of
// the next tile (steps 7-12), the first part of its chunk 1 (steps 14-15) — the same ranges as
// the DMA schedule above
}  // namespace ru8

// vmcnt(N) with N a template constant (N ≤ 63)
template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt field");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// helper h's window pieces q ∈ [P0, P1), q ≡ h (mod 2), of 64-channel chunk cc for the tile at m0
template <int P0, int P1>
__device__ __forceinline__ void ru8_win(const ConvArgs &a, uint32_t buf, int64_t m0, uint32_t voff, int lane, int h) {
    const char *base = (const char *)(a.in + (m0 - 3 * a.dil) * 128);
    asm volatile("" : "+s"(base));
#pragma unroll
    for (int q = P0; q < P1; ++q) {
        if ((q & 1) != h) continue;
        if (q * 8 + 8 <= ru8::WROWS || (lane >> 3) < ru8::WROWS - q * 8)
            ru_dma(base + q * 8 * 256, buf + q * 1024, voff);
    }
}
// helper h's 8 pieces (q ≡ h mod 2) of W K-tile kt into the ring slot at LDS address `slot`
// (the source base passes through an opaque asm per call: otherwise hipcc hoists the 128
// loop-invariant (K-tile, piece) addresses of the unrolled step sequence into SGPRs and spills them)
__device__ __forceinline__ void ru8_w(const ResUnitArgs &u, uint32_t slot, int kt, int h, uint32_t voff1,
                                      uint32_t voff2) {
    const char *w1 = (const char *)u.c1.W, *w2 = (const char *)u.W2p;
    asm volatile("" : "+s"(w1), "+s"(w2));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int q = h + 2 * i;
        if (kt < 14) {
            const int cc = kt >= 7 ? 1 : 0, tap = kt - 7 * cc;
            ru_dma(w1 + q * 8 * 1792 + tap * 256 + cc * 128, slot + q * 1024, voff1);
        } else {
            ru_dma(w2 + q * 8 * 256 + (kt - 14) * 128, slot + q * 1024, voff2);
        }
    }
}

// timing experiments only (wrong results): epilogue 2 without the next Snake / without the
// snaked store when the raw one is kept
#ifndef RU8_X_NOSNAKE2
#define RU8_X_NOSNAKE2 0
#endif
#ifndef RU8_X_NOSTORE_S
#define RU8_X_NOSTORE_S 0
#endif
#ifndef RU8_X_NOLOADX
#define RU8_X_NOLOADX 0    // the residual rows not loaded (zeros): what their re-read from beyond L2 costs
#endif
// SIN window rows: loaded RU8_WLEAD helper steps before their Snake + LDS write (2: the rows come
// from HBM — the previous unit's output — and one step, ≈ 0.6 µs, left the helpers waiting on
// them at most barriers; 1: the previous schedule, A/B).  Deadlines with lead 2: chunk 1 of a tile
// written by step 5 (read from K-tile 7), chunk 0 of the next by step 14 (read from K-tile 0'),
// the first part of its chunk 1 at steps 0' / 1' (buffer 1 free since K-tile 13)
#ifndef RU8_WLEAD
#define RU8_WLEAD 2
#endif
// window helpers' Snake in packed f32 (v_pk_mul / v_pk_fma) or scalar: the helpers issue beside
// an MFMA wave on their SIMD, where the guide prices packed f32 VALU as an anti-lever
#ifndef RU8_WPACKED
#define RU8_WPACKED 0
#endif
// residual prefetch distance in row fragments: fragment i's x rows are loaded while fragment
// i − RU8_XDIST is in epilogue 2 (the first RU8_XDIST during K-tile 15)
#ifndef RU8_XDIST
#define RU8_XDIST 2
#endif
// RU8_STAMPS (diagnostic builds only, tools/ru8_stamps.py): shader-clock stamps of each block's
// second tile (steady state).  Role 0, MFMA wave 0: before / after every K-tile barrier (slots
// 2kt, 2kt+1), after the K loop (32), after epilogue 2 (33), real time at the tile's first
// barrier and its end (34, 35).  Role 1, the W helper (SIN wave 4, else helper 0): before / after
// its pre-barrier vmcnt wait (2kt, 2kt+1) — kept in registers and stored after its last wait, so
// no store of its own sits among the DMAs its counted waits track.  Role 2, window helper 0 (SIN
// wave 5): before / after its pre-barrier lgkmcnt wait.
#ifdef RU8_STAMPS
constexpr int RST_BLK = 1024, RST_SLOTS = 36, RST_LDS = 4 * RST_SLOTS * 8;   // + a dummy role
__device__ unsigned long long g_ru8_stamps[RST_BLK * 3 * RST_SLOTS];
// stamps go to LDS past the kernel's own bytes (an LDS write leaves vmcnt alone, so the helpers'
// counted waits stay exact); each role copies its slots to global memory as it exits
__device__ __forceinline__ void ru8_stamp(char *lds, int role, int i, unsigned long long v) {
    if ((threadIdx.x & 63) == 0) ((unsigned long long *)(lds + ru8::LDS))[role * RST_SLOTS + i] = v;
}
__device__ __forceinline__ void ru8_stamp_flush(const char *lds, int role) {
    if (blockIdx.x < RST_BLK && (threadIdx.x & 63) == 0)
        for (int i = 0; i < RST_SLOTS; ++i)
            g_ru8_stamps[(blockIdx.x * 3 + role) * RST_SLOTS + i] =
                ((const unsigned long long *)(lds + ru8::LDS))[role * RST_SLOTS + i];
}
#define RU8_STAMP(role, i, v) ru8_stamp(lds, role, i, v)
#define RU8_STAMP_FLUSH(role) ru8_stamp_flush(lds, role)
#else
constexpr int RST_LDS = 0;
#define RU8_STAMP(role, i, v) do {} while (0)
#define RU8_STAMP_FLUSH(role) do {} while (0)
#endif
__device__ __forceinline__ unsigned long long ru8_now() {
#ifdef RU8_STAMPS
    return __builtin_amdgcn_s_memtime();
#else
    return 0;
#endif
}

// SIN window helpers: RU8_NWH waves (one per SIMD beside its MFMA wave with the W helper on the
// fourth; the stamps showed two helpers' Snake VALU arriving 700-1450 cycles after the MFMA waves
// at most K-tile barriers).  RU8_NWH=2 (A/B): the previous two.
#ifndef RU8_NWH
#define RU8_NWH 3
#endif
namespace ru8 {
constexpr int NWH = RU8_NWH;
static_assert(NWH == 2 || NWH == 3, "window helpers");
}  // namespace ru8
// SIN window helper H (pieces q ≡ H mod NWH): global 16-B loads of raw x into registers,
// Snake (the unit's first, sa_in / sib_in), bf16, LDS — the same image the LDS-DMA would write
// from x_s.  Plain loads: hipcc counts them and waits for the data of step s only where step
// s + 1 writes it out (inline-asm loads would leave a register copy of an unlanded destination
// possible between the load and its wait).
__host__ __device__ constexpr int win_share(int p0, int p1, int h) {
    int n = 0;
    for (int q = p0; q < p1; ++q) n += q % ru8::NWH == h;
    return n;
}
template <int H, int P0, int P1>
__device__ __forceinline__ void sin_issue(const char *src, uint32_t goff, int l3, uint4 (&ld)[4]) {
    static_assert(win_share(P0, P1, H) <= 4, "a helper's pieces per step fit its load registers");
    int k = 0;
#pragma unroll
    for (int q = P0; q < P1; ++q) {
        if (q % ru8::NWH != H) continue;
        if (q * 8 + 8 <= ru8::WROWS || l3 < ru8::WROWS - q * 8) ld[k] = *(const uint4 *)(src + (int64_t)q * 8 * 256 + goff);
        ++k;
    }
}
template <int H, int P0, int P1>
__device__ __forceinline__ void sin_write(char *buf, uint32_t loff, int l3, const uint4 (&ld)[4], const float (&sa)[8],
                                          const float (&sb)[8]) {
    int k = 0;
#pragma unroll
    for (int q = P0; q < P1; ++q) {
        if (q % ru8::NWH != H) continue;
        if (q * 8 + 8 <= ru8::WROWS || l3 < ru8::WROWS - q * 8) {
            float x[8], y[8];
            unpack8(ld[k], x);
            if (RU8_WPACKED) {
                snake_n<8>(x, sa, sb, y);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) y[e] = snake1(x[e], sa[e], sb[e]);
            }
            *(uint4 *)(buf + q * 1024 + loff) = pack8(y);
        }
        ++k;
    }
}

template <bool RAW, bool SIN = false>
__global__ __launch_bounds__(SIN ? 320 + 64 * ru8::NWH : 384, 1) void ru8_kernel(ResUnitArgs u, int64_t ntiles) {
    constexpr int RBM = ru8::BM, WINB = ru8::WINB, WT = ru8::WT;
    __shared__ __attribute__((aligned(16))) char lds[ru8::LDS + RST_LDS];
    const ConvArgs &a = u.c1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    if (t0 >= t1) return;
    char *par = lds, *win = lds + ru8::PAR, *wr = win + 2 * WINB;
    const uint32_t win3 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)lds + ru8::PAR;
    const uint32_t wr3 = win3 + 2 * WINB;
    float *psa2 = (float *)par, *psib2 = psa2 + 128, *psan = psa2 + 256, *psibn = psa2 + 384;
    bf16_t *pb1 = (bf16_t *)(par + 2048), *pb2 = (bf16_t *)(par + 2304);

    if (SIN && wave == 4) {
        // ---- SIN: one helper wave issues every W piece ----
        const int l3 = lane >> 3, lc = ((lane & 7) ^ l3) * 16;
        const uint32_t vk1 = l3 * 1792 + lc, vk2 = l3 * 256 + lc;
#pragma unroll
        for (int k = 0; k < ru8::D; ++k) {
            ru8_w(u, wr3 + k * WT, k, 0, vk1, vk2);
            ru8_w(u, wr3 + k * WT, k, 1, vk1, vk2);
        }
        int slot = 0;
        for (int64_t t = t0; t < t1; ++t) {
            const bool more = t + 1 < t1;
            sfor<0, 16>([&](auto KT) __attribute__((always_inline)) {
                constexpr int kt = decltype(KT)::value;
                if (t == t0 + 1) RU8_STAMP(1, 2 * kt, ru8_now());
                if (more) vm_wait<ru8::w_newer(kt, true)>();
                else vm_wait<ru8::w_newer(kt, false)>();
                if (t == t0 + 1) RU8_STAMP(1, 2 * kt + 1, ru8_now());
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                const int sp = slot == 0 ? ru8::NSLOT - 1 : slot - 1;
                if constexpr (kt + ru8::D <= 15) {
                    ru8_w(u, wr3 + sp * WT, kt + ru8::D, 0, vk1, vk2);
                    ru8_w(u, wr3 + sp * WT, kt + ru8::D, 1, vk1, vk2);
                } else if (more) {
                    ru8_w(u, wr3 + sp * WT, kt + ru8::D - 16, 0, vk1, vk2);
                    ru8_w(u, wr3 + sp * WT, kt + ru8::D - 16, 1, vk1, vk2);
                }
                slot = slot + 1 == ru8::NSLOT ? 0 : slot + 1;
            });
        }
        vm_wait<0>();
        RU8_STAMP_FLUSH(1);
        return;
    }
    if (SIN && wave >= 5) {
        // ---- SIN: two window helpers (raw x → Snake → LDS) ----
        auto run = [&](auto HC) __attribute__((always_inline)) {
            constexpr int H = decltype(HC)::value;
            const int l3 = lane >> 3, c = (lane & 7) ^ l3;
            const uint32_t goff = l3 * 256 + c * 16, loff = lane * 16;
            float sa[2][8], sb[2][8];
#pragma unroll
            for (int cc = 0; cc < 2; ++cc)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    sa[cc][e] = u.sa_in[cc * 64 + c * 8 + e];
                    sb[cc][e] = u.sib_in[cc * 64 + c * 8 + e];
                }
            int dl = a.dil;
            asm volatile("" : "+s"(dl));
            auto src_of = [&](int64_t m0, int cc) __attribute__((always_inline)) {
                return (const char *)(a.in + (m0 - 3 * dl) * 128) + cc * 128;
            };
            uint4 ld[2][4];
            // prologue: the block's first tile, both chunks, in batches of ≤ 4 pieces
            {
                const int64_t m0 = t0 * RBM;
                sfor<0, 2>([&](auto CCC) __attribute__((always_inline)) {
                    constexpr int cc = decltype(CCC)::value;
                    sfor<0, 5>([&](auto BC) __attribute__((always_inline)) {
                        constexpr int p0 = decltype(BC)::value * 8, p1 = p0 + 8 < ru8::NPW ? p0 + 8 : ru8::NPW;
                        sin_issue<H, p0, p1>(src_of(m0, cc), goff, l3, ld[0]);
                        sin_write<H, p0, p1>(win + cc * WINB, loff, l3, ld[0], sa[cc], sb[cc]);
                    });
                });
            }
            for (int64_t t = t0; t < t1; ++t) {
                const int64_t m0 = t * RBM;
                const bool first = t == t0, more = t + 1 < t1;
                sfor<0, 16>([&](auto KT) __attribute__((always_inline)) {
                    constexpr int kt = decltype(KT)::value, PB = kt & 1, PP = PB ^ 1;
                    if (H == 0 && t == t0 + 1) RU8_STAMP(2, 2 * kt, ru8_now());
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // this wave's LDS writes landed
                    if (H == 0 && t == t0 + 1) RU8_STAMP(2, 2 * kt + 1, ru8_now());
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
                    auto fin = [&](auto P0C, auto P1C, auto CCC, auto BC) __attribute__((always_inline)) {
                        constexpr int p0 = decltype(P0C)::value, p1 = decltype(P1C)::value, cc = decltype(CCC)::value;
                        sin_write<H, p0, p1>(win + cc * WINB, loff, l3, ld[decltype(BC)::value], sa[cc], sb[cc]);
                    };
                    if constexpr (RU8_WLEAD == 2) {
                        // finish step kt − 2's pieces (Snake, LDS) first: they sit in ld[PB], the
                        // registers step kt issues into next — two steps for their rows to arrive
                        if constexpr (kt >= 2 && kt <= 5) {          // chunk 1 of this tile
                            if (!first) fin(IC7<ru8::c1b_lo(kt - 2)>{}, IC7<ru8::c1b_hi(kt - 2)>{}, IC7<1>{}, IC7<PB>{});
                        } else if constexpr (kt >= 9 && kt <= 14) {  // chunk 0 of the next tile
                            if (more) fin(IC7<ru8::c0_lo(kt - 9)>{}, IC7<ru8::c0_hi(kt - 9)>{}, IC7<0>{}, IC7<PB>{});
                        } else if constexpr (kt <= 1) {              // issued at steps 14 / 15 of the previous tile
                            if (!first) fin(IC7<ru8::c1a_lo(kt)>{}, IC7<ru8::c1a_hi(kt)>{}, IC7<1>{}, IC7<PB>{});
                        }
                    }
                    // issue step kt's loads into ld[PB] (the ranges of the DMA schedule)
                    if constexpr (kt <= 3) {
                        if (!first) sin_issue<H, ru8::c1b_lo(kt), ru8::c1b_hi(kt)>(src_of(m0, 1), goff, l3, ld[PB]);
                    } else if constexpr (kt >= 7 && kt <= 12) {
                        if (more) sin_issue<H, ru8::c0_lo(kt - 7), ru8::c0_hi(kt - 7)>(src_of(m0 + RBM, 0), goff, l3, ld[PB]);
                    } else if constexpr (kt >= 14) {
                        if (more) sin_issue<H, ru8::c1a_lo(kt - 14), ru8::c1a_hi(kt - 14)>(src_of(m0 + RBM, 1), goff, l3, ld[PB]);
                    }
                    if constexpr (RU8_WLEAD == 1) {
                        // finish step kt − 1's pieces (loaded into ld[PP]): Snake, LDS
                        if constexpr (kt >= 1 && kt <= 4) {          // chunk 1 of this tile, issued at kt − 1
                            if (!first) fin(IC7<ru8::c1b_lo(kt - 1)>{}, IC7<ru8::c1b_hi(kt - 1)>{}, IC7<1>{}, IC7<PP>{});
                        } else if constexpr (kt >= 8 && kt <= 13) {  // chunk 0 of the next tile
                            if (more) fin(IC7<ru8::c0_lo(kt - 8)>{}, IC7<ru8::c0_hi(kt - 8)>{}, IC7<0>{}, IC7<PP>{});
                        } else if constexpr (kt == 15) {             // chunk 1 (first part) of the next tile
                            if (more) fin(IC7<ru8::c1a_lo(0)>{}, IC7<ru8::c1a_hi(0)>{}, IC7<1>{}, IC7<PP>{});
                        } else if constexpr (kt == 0) {              // issued at step 15 of the previous tile
                            if (!first) fin(IC7<ru8::c1a_lo(1)>{}, IC7<ru8::c1a_hi(1)>{}, IC7<1>{}, IC7<PP>{});
                        }
                    }
                });
            }
            vm_wait<0>();
            if (H == 0) RU8_STAMP_FLUSH(2);
        };
        if (wave == 5) run(IC7<0>{});
        else if (ru8::NWH == 2 || wave == 6) run(IC7<1>{});
        else run(IC7<2>{});
        return;
    }
    if (!SIN && wave >= 4) {
        // ---- helper waves: every LDS-DMA of the block ----
        const int h = wave - 4;
        const int l3 = lane >> 3, lc = ((lane & 7) ^ l3) * 16;
        const uint32_t vw0 = l3 * 256 + lc, vw1 = vw0 + 128;          // window chunk 0 / 1
        const uint32_t vk1 = l3 * 1792 + lc, vk2 = l3 * 256 + lc;       // W1 / W2 rows
        // prologue: chunk 0, W(0), chunk 1, W(1) … W(D − 1)
        ru8_win<0, ru8::NPW>(a, win3, t0 * RBM, vw0, lane, h);
        ru8_w(u, wr3, 0, h, vk1, vk2);
        ru8_win<0, ru8::NPW>(a, win3 + WINB, t0 * RBM, vw1, lane, h);
#pragma unroll
        for (int k = 1; k < ru8::D; ++k) ru8_w(u, wr3 + k * WT, k, h, vk1, vk2);
        int slot = 0;                       // ring slot of the current K-tile
        for (int64_t t = t0; t < t1; ++t) {
            const int64_t m0 = t * RBM;
            const bool first = t == t0, more = t + 1 < t1;
            sfor<0, 16>([&](auto KT) __attribute__((always_inline)) {
                constexpr int kt = decltype(KT)::value;
                if (h == 0 && t == t0 + 1) RU8_STAMP(1, 2 * kt, ru8_now());
                // pre-barrier kt: W(kt) and everything issued before it landed
                if (h == 0) {
                    if (first) {
                        if (more) vm_wait<ru8::allowed(kt, 0, true, true)>();
                        else vm_wait<ru8::allowed(kt, 0, true, false)>();
                    } else {
                        if (more) vm_wait<ru8::allowed(kt, 0, false, true)>();
                        else vm_wait<ru8::allowed(kt, 0, false, false)>();
                    }
                } else {
                    if (first) {
                        if (more) vm_wait<ru8::allowed(kt, 1, true, true)>();
                        else vm_wait<ru8::allowed(kt, 1, true, false)>();
                    } else {
                        if (more) vm_wait<ru8::allowed(kt, 1, false, true)>();
                        else vm_wait<ru8::allowed(kt, 1, false, false)>();
                    }
                }
                if (h == 0 && t == t0 + 1) RU8_STAMP(1, 2 * kt + 1, ru8_now());
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                // step kt: window pieces, then W
                if constexpr (kt <= 3) {
                    if (!first) ru8_win<ru8::c1b_lo(kt), ru8::c1b_hi(kt)>(a, win3 + WINB, m0, vw1, lane, h);
                }
                if constexpr (kt >= 7 && kt <= 12) {
                    if (more) ru8_win<ru8::c0_lo(kt - 7), ru8::c0_hi(kt - 7)>(a, win3, m0 + RBM, vw0, lane, h);
                }
                if constexpr (kt >= 14) {
                    if (more) ru8_win<ru8::c1a_lo(kt - 14), ru8::c1a_hi(kt - 14)>(a, win3 + WINB, m0 + RBM, vw1, lane, h);
                }
                const int sp = slot == 0 ? ru8::NSLOT - 1 : slot - 1;     // K-tile kt−1's slot = W(kt + D)'s
                if constexpr (kt + ru8::D <= 15) ru8_w(u, wr3 + sp * WT, kt + ru8::D, h, vk1, vk2);
                else if (more) ru8_w(u, wr3 + sp * WT, kt + ru8::D - 16, h, vk1, vk2);
                slot = slot + 1 == ru8::NSLOT ? 0 : slot + 1;
            });
        }
        vm_wait<0>();
        if (h == 0) RU8_STAMP_FLUSH(1);
        return;
    }

    // ---- MFMA waves 0-3: rows 64·wave .. +63 of each tile ----
    if (tid < 128) {
        psa2[tid] = a.sa[tid]; psib2[tid] = a.sib[tid];
        if constexpr (!(SIN && RAW)) {       // the next Snake: only where out_s is written
            psan[tid] = u.sa_next[tid]; psibn[tid] = u.sib_next[tid];
        }
        pb1[tid] = a.bias[tid]; pb2[tid] = u.b2[tid];
    }
    const int fr = lane & 15, fc = lane >> 4;
    const bool odd = fc & 1;
    const int wl[2] = {fr * 128 + ((fc ^ (fr & 7)) << 4), fr * 128 + (((4 + fc) ^ (fr & 7)) << 4)};
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int slot = 0;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t m0 = t * RBM;
        bf16x8 yk[4][2];       // y_s k-steps 2, 3 of each row fragment, for K-tile 15
        u32x4 xv[4][4];
        // x (the residual) rows of row fragment i of this wave
        // (row offsets computed at the load, from an opaque m0: hoisted to the tile start, the
        // 16 offsets stayed live through the K loop and spilled)
        auto load_x = [&](int i) __attribute__((always_inline)) {
            int64_t mx = m0;
            asm volatile("" : "+s"(mx));
            const char *xb = (const char *)(u.x + mx * 128);
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {
                const int r = (int)min((int64_t)(64 * wave + 16 * i + fr), a.M - 1 - mx);
                const uint32_t off = (uint32_t)(r * 128 + (2 * jp + (odd ? 1 : 0)) * 16 + (fc >> 1) * 8) * 2;
                xv[i][jp] = RU8_X_NOLOADX ? u32x4{0u, 0u, 0u, 0u} : *(const u32x4 *)(xb + off);
            }
        };
#ifdef RU8_STAMPS
        // MFMA-wave stamps without a branch (a branch per K-tile broke the unrolled schedule and
        // spilled): every lane of every MFMA wave writes; only wave 0's steady tile to role 0
        unsigned long long *sb = (unsigned long long *)(lds + ru8::LDS) + (wave == 0 && t == t0 + 1 ? 0 : 3 * RST_SLOTS);
#endif
        sfor<0, 16>([&](auto KT) __attribute__((always_inline)) {
            constexpr int kt = decltype(KT)::value;
#ifdef RU8_STAMPS
            sb[2 * kt] = ru8_now();
#endif
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#ifdef RU8_STAMPS
            sb[2 * kt + 1] = ru8_now();
            if constexpr (kt == 0) sb[34] = __builtin_amdgcn_s_memrealtime();
#endif
            // (slot opaque: with 16 % NSLOT == 0 hipcc folds every K-tile's slot to a constant and
            // hoists the 16 fragment bases out of the tile loop, where they spill)
            asm volatile("" : "+s"(slot));
            const char *tb = wr + slot * WT;
            slot = slot + 1 == ru8::NSLOT ? 0 : slot + 1;
            if constexpr (kt < 14) {
                constexpr int cc = kt >= 7 ? 1 : 0, tap = kt - 7 * cc;
                int dl = a.dil;
                asm volatile("" : "+s"(dl));
                const int rb = 64 * wave + fr + tap * dl;
                const char *wb = win + cc * WINB + rb * 128;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int xo = ((4 * ks + fc) ^ (rb & 7)) << 4;
                    bf16x8 xf[4], wf[8];
#pragma unroll
                    for (int i = 0; i < 4; ++i) xf[i] = *(const bf16x8 *)(wb + i * 2048 + xo);
#pragma unroll
                    for (int j = 0; j < 8; ++j) wf[j] = *(const bf16x8 *)(tb + j * 2048 + wl[ks]);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
                }
            } else if constexpr (kt == 14) {
                // per row fragment: epilogue 1 (y_s = snake2(bf16(acc + b1)), the k=1 B fragments
                // as in ru7_kernel), then its k=1 MFMAs over y_s k-steps 0, 1 (W2 half 0); k-steps
                // 2, 3 wait for K-tile 15 — only one fragment's y_s is live at full width
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    // (parameter offsets opaque per fragment: hoisted, the 96 parameter values
                    // would stay live across all four fragments)
                    int pl = 4 * fc;
                    asm volatile("" : "+v"(pl));
                    uint2 yv[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int n = 16 * j + pl;
                        float b[4];
                        unpack4(*(const uint2 *)(pb1 + n), b);
                        const float4 sa = *(const float4 *)(psa2 + n), sb = *(const float4 *)(psib2 + n);
                        const float sav[4] = {sa.x, sa.y, sa.z, sa.w}, sbv[4] = {sb.x, sb.y, sb.z, sb.w};
                        float o[4];
                        float t[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                        add_n<4>(t, b);
                        rbf_n<4>(t);
                        snake_n<4>(t, sav, sbv, o);
                        yv[j] = pack4(o);
                        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    }
                    bf16x8 y[4];
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4)
                        y[s4] = __builtin_bit_cast(bf16x8, make_uint4(yv[2 * s4].x, yv[2 * s4].y, yv[2 * s4 + 1].x,
                                                                       yv[2 * s4 + 1].y));
                    yk[i][0] = y[2];
                    yk[i][1] = y[3];
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks) {
                        bf16x8 wf[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) wf[j] = *(const bf16x8 *)(tb + j * 2048 + wl[ks]);
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], y[ks], acc[i][j], 0, 0, 0);
                    }
                }
            } else {
                load_x(0);
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    bf16x8 wf[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) wf[j] = *(const bf16x8 *)(tb + j * 2048 + wl[ks]);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], yk[i][ks], acc[i][j], 0, 0, 0);
                }
#pragma unroll
                for (int i = 1; i < RU8_XDIST; ++i) load_x(i);
            }
        });
#ifdef RU8_STAMPS
        sb[32] = ru8_now();
#endif
        // epilogue 2: x' = x + bf16(acc + b2) (raw, optional) and snake_next(x') → out_s
        int64_t me = m0;
        asm volatile("" : "+s"(me));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i + RU8_XDIST < 4) load_x(i + RU8_XDIST);     // lands during the epilogues before its own
            int pl2 = (odd ? 16 : 0) + (fc >> 1) * 8;
            asm volatile("" : "+v"(pl2));
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {
                const int n = 32 * jp + pl2;
                float bb[8];
                unpack8(*(const uint4 *)(pb2 + n), bb);
                const float4 a0 = *(const float4 *)(psan + n), a1 = *(const float4 *)(psan + n + 4);
                const float4 s0 = *(const float4 *)(psibn + n), s1 = *(const float4 *)(psibn + n + 4);
                const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
                float o[8], rr[8], sn[8];
                pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
                acc[i][2 * jp] = f32x4{0.f, 0.f, 0.f, 0.f};
                acc[i][2 * jp + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
                unpack8(make_uint4(xv[i][jp].x, xv[i][jp].y, xv[i][jp].z, xv[i][jp].w), rr);
                add_n<8>(o, bb);
                rbf_n<8>(o);
                add_n<8>(o, rr);
                rbf_n<8>(o);
                if constexpr (!(SIN && RAW)) {
                    if (RU8_X_NOSNAKE2) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) sn[r] = o[r];
                    } else {
                        snake_n<8>(o, av, sv, sn);
                    }
                }
                const int64_t m = me + 64 * wave + 16 * i + fr;
                if (m < a.M) {
                    if constexpr (SIN) {
                        // raw x' for the next unit (which snakes it while staging), or the
                        // block's snaked output
                        if constexpr (RAW) *(uint4 *)(u.x_out + m * 128 + n) = pack8(o);
                        else *(uint4 *)(u.out_s + m * 128 + n) = pack8(sn);
                    } else {
                        if constexpr (RAW) *(uint4 *)(u.x + m * 128 + n) = pack8(o);
                        if (!(RAW && RU8_X_NOSTORE_S)) *(uint4 *)(u.out_s + m * 128 + n) = pack8(sn);
                    }
                }
            }
        }
#ifdef RU8_STAMPS
        sb[33] = ru8_now();
        sb[35] = __builtin_amdgcn_s_memrealtime();
#endif
    }
    if (wave == 0) RU8_STAMP_FLUSH(0);
}

__global__ void permute_k1_kernel(const bf16_t *w, bf16_t *wp, int n_rows) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_rows * 128) return;
    const int n = idx >> 7, k = idx & 127;
    const int s = k >> 5, g = (k >> 3) & 3, e = k & 7;
    wp[idx] = w[n * 128 + 32 * s + (e < 4 ? 4 * g + e : 16 + 4 * g + e - 4)];
}

// Final decoder conv (Cout = 2 audio channels, k=7, pad 3, no bias) on the
// already-snaked input; fp32 channels-first output [2][L].  One block = 256
// output positions; the 262-row halo window is staged channel-major in LDS so
// consecutive lanes read consecutive positions.
template <int COUT, int CIN>
__global__ __launch_bounds__(256) void conv_out_kernel(const bf16_t *__restrict__ in, int64_t L,
                                                       const float *__restrict__ w,  // [7][Cin][COUT]
                                                       float *__restrict__ out) {
    constexpr int Cin = CIN;
    // the halo window stays position-major ([262][Cin], 16-B chunks XOR-swizzled by the row so
    // the per-lane row reads of one chunk spread over all banks): 16-B global loads and 16-B
    // LDS writes (the former channel-major transpose was 2-B LDS stores, 700 GB/s)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int P = 256 + 6;
    const int chunks = Cin / 8, cm = chunks - 1;
    // the weights are read straight from global memory at wave-uniform addresses (scalar loads
    // into SGPRs, the v_fma's scalar operand): one LDS read per FMA had made the kernel
    // LDS-issue-bound (2.36 ms per 240 s decode, 1.25 TB/s of its 2.95 GB input)
    char *xs = smem;                                   // [P][Cin] bf16, swizzled chunks
    const int64_t t0 = (int64_t)blockIdx.x * 256;
    // every 16-B load of the window in flight before the first LDS store: a load → wait →
    // store loop paid one full memory latency per chunk (17 per block at Cin = 128)
    constexpr int NCH = P * (CIN / 8), ITER = (NCH + 255) / 256;
    uint4 v[ITER];
    // (straight-line: clamped addresses, out-of-range rows zeroed at the store — a guarded load
    // per chunk made hipcc wait vmcnt(0) at every branch merge)
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
        const int c = min(threadIdx.x + 256 * i, NCH - 1);
        const int64_t pos = t0 - 3 + c / chunks;
        v[i] = *(const uint4 *)(in + min(max(pos, (int64_t)0), L - 1) * Cin + (c % chunks) * 8);
    }
    __builtin_amdgcn_sched_barrier(0);      // every load issued before the first store
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
        const int c = threadIdx.x + 256 * i;
        const int p = c / chunks, ch = c % chunks;
        const int64_t pos = t0 - 3 + p;
        const bool ok = pos >= 0 && pos < L;
        const uint4 x = make_uint4(ok ? v[i].x : 0u, ok ? v[i].y : 0u, ok ? v[i].z : 0u, ok ? v[i].w : 0u);
        if (i + 1 < ITER || c < NCH) *(uint4 *)(xs + (size_t)p * Cin * 2 + ((ch ^ (p & cm)) << 4)) = x;
    }
    __syncthreads();
    const int64_t t = t0 + threadIdx.x;
    if (t >= L) return;
    // both output channels in one packed accumulator: v_pk_fma_f32 (x broadcast, the two
    // channels' weights as the scalar pair) — half the VALU issue of two scalar chains
    static_assert(COUT == 2, "packed pair of output channels");
    f32x2 acc = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const int row = threadIdx.x + k;
        const char *xr = xs + (size_t)row * Cin * 2;
#pragma unroll
        for (int c = 0; c < chunks; ++c) {
            float x[8];
            unpack8(*(const uint4 *)(xr + ((c ^ (row & cm)) << 4)), x);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const f32x2 wv = *(const f32x2 *)(w + 2 * (k * Cin + c * 8 + e));
                acc = __builtin_elementwise_fma(f32x2{x[e], x[e]}, wv, acc);
            }
        }
    }
    // rounded through bf16: the reference decodes with a bf16 VAE (init_service_loader.py:132-134),
    // so decode(z).sample is bf16 and the handler upcasts it (generate_music_decode.py:188-189);
    // the fp32 output holds exactly those values
    out[t] = rbf(acc[0]);
    out[L + t] = rbf(acc[1]);
}

// Encoder first conv: channels-first audio [Cin≤2][N] → NLC [N][Cout] raw + snaked, k=7 pad 3, bias.
__global__ __launch_bounds__(256) void conv_in_kernel(const bf16_t *__restrict__ in, int64_t N, int Cin,
                                                      const float *__restrict__ w,  // [Cout][Cin][7]
                                                      const float *__restrict__ bias, int Cout,
                                                      bf16_t *__restrict__ out, bf16_t *__restrict__ out_s,
                                                      const float *__restrict__ sa,
                                                      const float *__restrict__ sib) {
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= N) return;
    float x[2][7];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const int64_t p = t - 3 + k;
            x[c][k] = (c < Cin && p >= 0 && p < N) ? bf2f(in[(int64_t)c * N + p]) : 0.f;
        }
    for (int o = lane; o < Cout; o += 64) {
        float acc = bias ? bias[o] : 0.f;
        for (int c = 0; c < Cin; ++c)
#pragma unroll
            for (int k = 0; k < 7; ++k) acc += x[c][k] * w[(o * Cin + c) * 7 + k];
        const float v = rbf(acc);
        if (out) out[t * Cout + o] = f2bf(v);
        if (out_s) out_s[t * Cout + o] = f2bf(snake1(v, sa[o], sib[o]));
    }
}

__global__ void cf_to_nlc_kernel(const bf16_t *in, int C, int64_t L, bf16_t *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)C * L) return;
    const int64_t t = i / C;
    const int c = (int)(i % C);
    out[i] = in[(int64_t)c * L + t];
}

// latent_dist.sample() (vae_model.py:285-304): h [T][2C] = (mean | scale) →
// z [C][T] = mean + (softplus(scale) + 1e-4)·eps; eps == null → the mean
__global__ void gauss_sample_kernel(const bf16_t *h, int64_t T, int C, const bf16_t *eps, bf16_t *z) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)C * T) return;
    const int c = (int)(i / T);
    const int64_t t = i % T;
    const float mean = bf2f(h[t * 2 * C + c]);
    float v = mean;
    if (eps) {
        const float sc = bf2f(h[t * 2 * C + C + c]);
        const float sp = sc > 20.f ? sc : log1pf(expf(sc));
        v = mean + rbf(rbf(sp) + 1e-4f) * bf2f(eps[i]);
    }
    z[i] = f2bf(v);
}

// weight-norm fusion: one block per dim-0 row of v (numel_row = d1·k)
__global__ void pack_conv_weight_kernel(const bf16_t *v, const bf16_t *g, int d0, int d1, int k,
                                        int transposed, int stride, bf16_t *Wp) {
    const int i = blockIdx.x;                       // dim-0 index
    const int nr = d1 * k;
    const bf16_t *vr = v + (int64_t)i * nr;
    __shared__ float red[256];
    float ss = 0.f;
    for (int e = threadIdx.x; e < nr; e += 256) {
        const float x = bf2f(vr[e]);
        ss += x * x;
    }
    red[threadIdx.x] = ss;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const float scale = g ? bf2f(g[i]) / sqrtf(red[0]) : 1.0f;
    for (int e = threadIdx.x; e < nr; e += 256) {
        const int j = e / k, kk = e % k;
        const float w = bf2f(vr[e]) * scale;
        if (!transposed) {
            // v [Cout=d0][Cin=d1][k] → Wp[co][tap·Cin + ci]
            Wp[(int64_t)i * nr + (int64_t)kk * d1 + j] = f2bf(w);
        } else {
            // v [Cin=d0][Cout=d1][2s] → phase r = kk % s, tap = (kk < s) ? 1 : 0
            const int s = stride, r = kk % s, tap = kk < s ? 1 : 0;
            const int64_t K = 2 * (int64_t)d0;
            Wp[((int64_t)r * d1 + j) * K + (int64_t)tap * d0 + i] = f2bf(w);
        }
    }
}

__global__ void fuse_conv_f32_kernel(const bf16_t *v, const bf16_t *g, int d0, int d1, int k, int k_major,
                                     float *w) {
    const int i = blockIdx.x;
    const int nr = d1 * k;
    const bf16_t *vr = v + (int64_t)i * nr;
    __shared__ float red[256];
    float ss = 0.f;
    for (int e = threadIdx.x; e < nr; e += 256) {
        const float x = bf2f(vr[e]);
        ss += x * x;
    }
    red[threadIdx.x] = ss;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const float scale = g ? bf2f(g[i]) / sqrtf(red[0]) : 1.0f;
    for (int e = threadIdx.x; e < nr; e += 256) {
        const int j = e / k, kk = e % k;
        const float x = bf2f(vr[e]) * scale;
        if (k_major) w[((int64_t)i * k + kk) * d1 + j] = x;   // [Cout][k][Cin]
        else w[(int64_t)i * nr + e] = x;                       // [Cout][Cin][k]
    }
}

__global__ void snake_params_kernel(const bf16_t *alpha, const bf16_t *beta, int C, float *sa, float *sib) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    sa[c] = expf(bf2f(alpha[c])) * 0.15915494309189535f;   // e^α / (2π): snake1's sine in revolutions
    sib[c] = 1.0f / (expf(bf2f(beta[c])) + 1e-9f);
}

__global__ void cast_bf16_f32_kernel(const bf16_t *s, float *d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = bf2f(s[i]);
}

// ACEHIP_CONV7=0 keeps the k=7 convolutions on the im2col conv_gemm / resunit128
// kernels (A/B knob for the halo-staged conv7_kernel)
bool use_conv7() { return knobs().conv7 != 0; }

// Which of the remaining convs run on the persistent counted-ring convp_kernel:
// default the k = 1 convs (C ≥ 256, residual epilogue), ACEHIP_CONVP=1 every eligible conv,
// =0 none.  Per-kernel rocprof of a 240 s decode (r02): k = 1 convs 4.55 vs 5.01 ms on
// conv_gemm_kernel, the ConvTranspose phases 8.30 vs 7.44 ms (so they stay there)
bool use_convp(const ConvArgs &a, int phases) {
    const int v = knobs().convp;
    return v == 1 || (v == 2 && a.taps == 1 && phases == 1);
}

// C = 128 residual units: ACEHIP_RU7=2 (default) ru8_kernel, 1 ru7_kernel, 0 conv7_kernel<FUSED> (A/B)
bool use_ru7() { return knobs().ru7 != 0; }

int num_cus_conv() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

}  // namespace

int permute_k1_weight(const bf16_t *w, bf16_t *wp, int n_rows, hipStream_t s) {
    permute_k1_kernel<<<(n_rows * 128 + 255) / 256, 256, 0, s>>>(w, wp, n_rows);
    HIP_TRY(hipGetLastError());
    return 0;
}

int conv_gemm(const ConvArgs &a, int phases, hipStream_t s) {
    if (a.M <= 0) return 0;
    if (a.N % BN || a.Cin % BK)
        return fail(-1, "conv_gemm: N%128 and Cin%64 required (N=" + std::to_string(a.N) +
                            " Cin=" + std::to_string(a.Cin) + ")");
    if (!a.out && !a.out_s) return fail(-1, "conv_gemm: no output");
    if (!a.zero) return fail(-1, "conv_gemm: zero page");
    if (a.out_s && (!a.sa || !a.sib)) return fail(-1, "conv_gemm: snake params");
    const bool k7 = phases == 1 && a.taps == 7 && a.a_stride == 1 && a.c_stride == 1 && a.c_off == 0 &&
                    a.a_off == -3 * a.dil && a.dil <= 9 && a.L_out == a.M && a.L_in == a.M && !a.res && !a.out && a.out_s;
    if (k7 && knobs().conv7 == 2 && a.in_halo && a.N % 256 == 0 && 3 * a.dil <= kActPadRows && a.M < (1ll << 31)) {
        // the k = 7 conv as an implicit GEMM on the two-phase ping-pong tile (256 × 256, eight
        // waves; gemm.hip EPI_CONV): its halo rows come from the buffer's zero rows — the front
        // ones are never written, the back ones are cleared here
        HIP_TRY(hipMemsetAsync((void *)(a.in + a.L_in * a.Cin), 0, (size_t)3 * a.dil * a.Cin * 2, s));
        GemmArgs g{};
        g.A = a.in; g.lda = a.Cin;
        g.W = a.W; g.ldw = 7 * a.Cin;
        g.Cs = a.out_s; g.ldc = a.N;
        g.M = (int)a.M; g.N = a.N; g.K = 7 * a.Cin;
        g.epi = EPI_CONV; g.bias = a.bias; g.sa = a.sa; g.sib = a.sib;
        g.conv_cin = a.Cin; g.conv_dil = a.dil; g.conv_a0 = -3 * a.dil;
        g.conv_ostride = 1; g.conv_ooff = 0; g.conv_cout = a.N; g.conv_lout = a.L_out;
        return gemm_conv(g, s);
    }
    // ConvTranspose1d (stride s, kernel 2s): the s phases' two-tap GEMMs side by side along N
    // (N = s·Cout, A — input rows m − 1 and m — read once for all of them), column n → channel
    // n % Cout of phase n / Cout at output row m·s − pad + phase; the same padded input
    if (knobs().convt && a.in_halo && phases > 1 && a.taps == 2 && a.a_stride == 1 && a.a_off == -1 && a.dil == 1 &&
        a.c_stride == phases && a.M == a.L_in + 1 && !a.res && (int64_t)phases * a.N % 256 == 0 &&
        a.w_pstride == (int64_t)a.N * 2 * a.Cin && a.M < (1ll << 31)) {
        HIP_TRY(hipMemsetAsync((void *)(a.in + a.L_in * a.Cin), 0, (size_t)a.Cin * 2, s));
        GemmArgs g{};
        g.A = a.in; g.lda = a.Cin;
        g.W = a.W; g.ldw = 2 * a.Cin;
        g.C = a.out; g.Cs = a.out_s; g.ldc = a.N;
        g.M = (int)a.M; g.N = phases * a.N; g.K = 2 * a.Cin;
        g.epi = EPI_CONV; g.bias = a.bias; g.sa = a.sa; g.sib = a.sib;
        g.conv_cin = a.Cin; g.conv_dil = 1; g.conv_a0 = -1;
        g.conv_ostride = phases; g.conv_ooff = a.c_off; g.conv_cout = a.N; g.conv_lout = a.L_out;
        return gemm_conv(g, s);
    }
    // k = 1 convs (the C ≥ 256 residual units' second conv, with the residual) as a plain GEMM on
    // the ping-pong tile (ACEHIP_CONVP=3)
    if (knobs().convp == 3 && phases == 1 && a.taps == 1 && a.a_stride == 1 && a.a_off == 0 && a.c_stride == 1 &&
        a.c_off == 0 && a.L_in == a.M && a.L_out == a.M && a.N % 256 == 0 && a.M < (1ll << 31)) {
        GemmArgs g{};
        g.A = a.in; g.lda = a.Cin;
        g.W = a.W; g.ldw = a.Cin;
        g.C = a.out; g.Cs = a.out_s; g.ldc = a.N;
        g.res = a.res; g.ldr = a.N;
        g.M = (int)a.M; g.N = a.N; g.K = a.Cin;
        g.epi = EPI_CONV; g.bias = a.bias; g.sa = a.sa; g.sib = a.sib;
        g.conv_cin = a.Cin; g.conv_dil = 1; g.conv_a0 = 0;
        g.conv_ostride = 1; g.conv_ooff = 0; g.conv_cout = a.N; g.conv_lout = a.L_out;
        return gemm_conv(g, s);
    }
    if (use_conv7() && k7) {
        const int64_t t7 = ((a.M + CONV7_BM - 1) / CONV7_BM) * (a.N / 128);
        if (t7 >= (1ll << 31)) return fail(-1, "conv_gemm: grid too large");
        conv7_kernel<CONV7_BM, false, false><<<(unsigned)t7, CONV7_BM * 2, 0, s>>>(a, ResUnitArgs{});
        HIP_TRY(hipGetLastError());
        return 0;
    }
    const int64_t tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
    if (tiles >= (1ll << 31)) return fail(-1, "conv_gemm: grid too large");
    if (use_convp(a, phases) && a.taps * a.Cin / BK >= 3 && a.N <= cp::MAXN) {   // ≥ 3 K-tiles per item (vmcnt bookkeeping)
        const int64_t items = tiles * phases;
        const int nb = (int)std::min<int64_t>(items, num_cus_conv());
        const bool rs = a.res != nullptr, raw = a.out != nullptr, sn = a.out_s != nullptr;
#define L(R, W, S) convp_kernel<R, W, S><<<nb, 512, 0, s>>>(a, items, phases)
        if (rs) {
            if (raw && sn) L(true, true, true); else if (raw) L(true, true, false); else L(true, false, true);
        } else {
            if (raw && sn) L(false, true, true); else if (raw) L(false, true, false); else L(false, false, true);
        }
#undef L
        HIP_TRY(hipGetLastError());
        return 0;
    }
    dim3 grid((unsigned)tiles, phases);
    const bool rs = a.res != nullptr, raw = a.out != nullptr, sn = a.out_s != nullptr;
#define L(R, W, S) conv_gemm_kernel<R, W, S><<<grid, 256, 0, s>>>(a)
    if (rs) {
        if (raw && sn) L(true, true, true); else if (raw) L(true, true, false); else L(true, false, true);
    } else {
        if (raw && sn) L(false, true, true); else if (raw) L(false, true, false); else L(false, false, true);
    }
#undef L
    HIP_TRY(hipGetLastError());
    return 0;
}

int resunit128(const ResUnitArgs &u, hipStream_t s) {
    const ConvArgs &a = u.c1;
    if (a.Cin != 128 || a.N != 128 || a.taps != 7 || !a.zero || !a.bias || !a.sa) return fail(-1, "resunit128: args");
    if (u.x == u.out_s || a.in == u.out_s) return fail(-1, "resunit128: out_s must not alias x / x_s");
    if (u.snake_in && !(knobs().ru7 == 2 && u.W2p && u.in_zero_pad && a.dil <= 9 && a.a_off == -3 * a.dil && a.L_in == a.M))
        return fail(-1, "resunit128: snake_in runs on ru8_kernel only");
    if (knobs().ru7 == 2 && u.W2p && u.in_zero_pad && a.dil <= 9 && a.a_off == -3 * a.dil && a.L_in == a.M) {
        const int64_t nt = (a.M + ru8::BM - 1) / ru8::BM;
        const int nb = (int)std::min<int64_t>(nt, (int64_t)num_cus_conv());
        HIP_TRY(hipMemsetAsync((void *)(a.in + a.L_in * 128), 0, (size_t)kActPadRows * 256, s));
        if (!u.snake_in || !u.keep_raw) {
            if (!u.out_s || !u.sa_next || !u.sib_next) return fail(-1, "resunit128: out_s and the next Snake's parameters");
        }
        if (u.snake_in) {
            if (!u.sa_in || !u.sib_in || (u.keep_raw && (!u.x_out || u.x_out == u.x)) || a.in != u.x)
                return fail(-1, "resunit128: snake_in needs sa_in / sib_in, in == x and a separate x_out");
            if (u.keep_raw) ru8_kernel<true, true><<<nb, 320 + 64 * ru8::NWH, 0, s>>>(u, nt);
            else ru8_kernel<false, true><<<nb, 320 + 64 * ru8::NWH, 0, s>>>(u, nt);
        } else if (u.keep_raw) {
            ru8_kernel<true><<<nb, 384, 0, s>>>(u, nt);
        } else {
            ru8_kernel<false><<<nb, 384, 0, s>>>(u, nt);
        }
        HIP_TRY(hipGetLastError());
        return 0;
    }
    if (use_ru7() && u.W2p && u.in_zero_pad && a.dil <= 9 && a.a_off == -3 * a.dil && a.L_in == a.M) {
        const int64_t nt = (a.M + ru::BM - 1) / ru::BM;
        const int nb = (int)std::min<int64_t>(nt, 2 * (int64_t)num_cus_conv());
        // the k=7 halo past the end reads kActPadRows zero rows behind the input
        HIP_TRY(hipMemsetAsync((void *)(a.in + a.L_in * 128), 0, (size_t)kActPadRows * 256, s));
        if (u.keep_raw) ru7_kernel<true><<<nb, 256, 0, s>>>(u, nt);
        else ru7_kernel<false><<<nb, 256, 0, s>>>(u, nt);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    if (use_conv7() && a.dil <= 9 && a.a_off == -3 * a.dil && a.L_in == a.M) {
        const int64_t t7 = (a.M + CONV7_BM - 1) / CONV7_BM;
        if (u.keep_raw) conv7_kernel<CONV7_BM, true, true><<<(unsigned)t7, CONV7_BM * 2, 0, s>>>(a, u);
        else conv7_kernel<CONV7_BM, true, false><<<(unsigned)t7, CONV7_BM * 2, 0, s>>>(a, u);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    const int64_t tiles = (a.M + 127) / 128;
    if (tiles >= (1ll << 31)) return fail(-1, "resunit128: grid too large");
    if (u.keep_raw) resunit128_kernel<true><<<(unsigned)tiles, 256, 0, s>>>(u);
    else resunit128_kernel<false><<<(unsigned)tiles, 256, 0, s>>>(u);
    HIP_TRY(hipGetLastError());
    return 0;
}

int conv_out(const bf16_t *in_s, int64_t L, int Cin, const float *w, int Cout, float *out, hipStream_t s) {
    if (Cout != 2 || Cin != 128) return fail(-1, "conv_out: Cout = 2, Cin = 128");
    const size_t smem = (size_t)Cin * 262 * 2;
    conv_out_kernel<2, 128><<<(unsigned)((L + 255) / 256), 256, smem, s>>>(in_s, L, w, out);
    HIP_TRY(hipGetLastError());
    return 0;
}

int conv_in(const bf16_t *in, int64_t N, int Cin, const float *w, const float *bias, int Cout, bf16_t *out,
            bf16_t *out_s, const float *sa, const float *sib, hipStream_t s) {
    if (Cin > 2) return fail(-1, "conv_in: at most 2 input channels");
    conv_in_kernel<<<(unsigned)((N + 3) / 4), 256, 0, s>>>(in, N, Cin, w, bias, Cout, out, out_s, sa, sib);
    HIP_TRY(hipGetLastError());
    return 0;
}

int cf_to_nlc(const bf16_t *in, int C, int64_t L, bf16_t *out, hipStream_t s) {
    const int64_t n = (int64_t)C * L;
    cf_to_nlc_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(in, C, L, out);
    HIP_TRY(hipGetLastError());
    return 0;
}

int gauss_sample(const bf16_t *h, int64_t T, int C, const bf16_t *eps, bf16_t *z, hipStream_t s) {
    const int64_t n = (int64_t)C * T;
    gauss_sample_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(h, T, C, eps, z);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pack_conv_weight(const bf16_t *v, const bf16_t *g, int d0, int d1, int k, int transposed, int stride,
                     bf16_t *Wp, hipStream_t s) {
    if (transposed && k != 2 * stride) return fail(-1, "pack_conv_weight: convT kernel must be 2*stride");
    pack_conv_weight_kernel<<<d0, 256, 0, s>>>(v, g, d0, d1, k, transposed, stride, Wp);
    HIP_TRY(hipGetLastError());
    return 0;
}

int fuse_conv_weight_f32(const bf16_t *v, const bf16_t *g, int d0, int d1, int k, int k_major, float *w,
                         hipStream_t s) {
    fuse_conv_f32_kernel<<<d0, 256, 0, s>>>(v, g, d0, d1, k, k_major, w);
    HIP_TRY(hipGetLastError());
    return 0;
}

int snake_params(const bf16_t *alpha, const bf16_t *beta, int C, float *sa, float *sib, hipStream_t s) {
    snake_params_kernel<<<(C + 255) / 256, 256, 0, s>>>(alpha, beta, C, sa, sib);
    HIP_TRY(hipGetLastError());
    return 0;
}

int cast_bf16_f32(const bf16_t *src, float *dst, int64_t n, hipStream_t s) {
    cast_bf16_f32_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(src, dst, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip

#ifdef RU8_STAMPS
extern "C" int acehip_diag_ru8_stamps(void *host) {
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(acehip::g_ru8_stamps), sizeof(acehip::g_ru8_stamps)));
    return 0;
}
extern "C" int acehip_diag_ru8_stamps_clear(void) {
    void *p = nullptr;
    HIP_TRY(hipGetSymbolAddress(&p, HIP_SYMBOL(acehip::g_ru8_stamps)));
    HIP_TRY(hipMemset(p, 0, sizeof(acehip::g_ru8_stamps)));
    return 0;
}
#endif
