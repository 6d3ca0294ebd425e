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
//     blocks share the weight panel in L2;
//   * the production tiles are the ping-pong kernels (gemm_pp_kernel, 256×256
//     and 192×256, two wave groups one barrier apart so MFMA and LDS traffic
//     overlap on every SIMD), picked per shape by gemm_pick_variant.
#include <hip/hip_ext.h>

#include "kernels.h"
#include "headpost.h"

namespace acehip {
namespace {

constexpr int BK = 64;
constexpr int GROUP_M = 8;

// GEMM_STAMPS (diagnostic builds only, tools/gemm_stamps.py): per workgroup and wave group,
// shader-clock stamps at kernel entry, after the prologue, after the main loop and after the
// epilogue, plus the real-time clock and the XCC id — where a tile's time goes
#ifdef GEMM_STAMPS
constexpr int STAMP_WG = 16384;
__device__ unsigned long long g_gemm_stamps[STAMP_WG * 2 * 8];
__device__ __forceinline__ void stamp(int slot, int i, unsigned long long v) {
    if (slot < STAMP_WG * 2) {
        asm volatile("" : "+v"(v));
        g_gemm_stamps[slot * 8 + i] = v;
    }
}
#define GSTAMP(i)                                                                                \
    do {                                                                                         \
        if ((threadIdx.x & 255) == 0 && threadIdx.x < 512) stamp(blockIdx.x * 2 + (threadIdx.x >> 8), i, __builtin_amdgcn_s_memtime()); \
    } while (0)
#define GSTAMP_REAL(i)                                                                           \
    do {                                                                                         \
        if ((threadIdx.x & 255) == 0 && threadIdx.x < 512) stamp(blockIdx.x * 2 + (threadIdx.x >> 8), i, __builtin_amdgcn_s_memrealtime()); \
    } while (0)
#else
#define GSTAMP(i) do {} while (0)
#define GSTAMP_REAL(i) do {} while (0)
#endif

// launch-attached timing events (gemm_ext_events): a hipEventRecord around a launch is its own
// barrier packet — ≈ 5.6 µs of idle GPU before and after the timed kernel on this stack
// (turbo timeline, tools/timeline.py) — while hipExtLaunchKernel stamps the dispatch itself
struct ExtEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
thread_local ExtEvents g_ext_ev;
template <typename... KArgs, typename... Args>
inline void klaunch(void (*kern)(KArgs...), dim3 grid, dim3 block, hipStream_t s, Args... args) {
    if (g_ext_ev.stop) {
        hipEvent_t st = g_ext_ev.start;
        g_ext_ev.start = nullptr;
        hipExtLaunchKernelGGL(kern, grid, block, 0, s, st, g_ext_ev.stop, 0, args...);
    } else {
        kern<<<grid, block, 0, s>>>(args...);
    }
}
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

// Epilogue of one wave's SM×SN grid of 16×16 sub-tiles: lane (fr, fc) holds row
// row0 + 16i + fr, columns col0 + 16j + 4fc .. +3 (the transposed MFMA tile).
// Adjacent sub-tiles j, j+1 are paired and the lane pair (fc, fc ^ 1) swaps four
// accumulators (lane ^ 16), so every lane owns 8 CONTIGUOUS columns of one
// sub-tile: one 16-B load / store per operand instead of two 8-B ones (the
// epilogue is store-issue-bound, MI355X_MICROARCH "attention epilogue store
// tail").  SwiGLU: the wave's columns are whole 64-column panels [32 gate | 32 up].
template <int SM, int SN, int EPI, int CHMAX = 12>
__device__ __forceinline__ void epilogue_tile(const GemmArgs &a, const f32x4 (&acc)[SM][SN], int row0, int col0,
                                              int fr, int fc) {
    static_assert(SN % 2 == 0, "sub-tiles are paired");
    const bool odd = fc & 1;
    const int cpos = (fc >> 1) * 8;          // this lane's 8-column group inside its sub-tile
#pragma unroll
    for (int i = 0; i < SM; ++i) {
        const int m = row0 + i * 16 + fr;
        const bool live = m < a.M;           // rows past M still join the lane exchange
        if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
            for (int pnl = 0; pnl < SN / 4; ++pnl) {
                // silu(gate)·up in the MFMA layout first, then one exchange of the products
                f32x4 p0, p1;
                float o[8];
                // bf16(gate) and bf16(up) of both sub-tiles, pairwise rounded, then silu
                float g8[8], u8[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    g8[r] = acc[i][4 * pnl][r];
                    g8[4 + r] = acc[i][4 * pnl + 1][r];
                    u8[r] = acc[i][4 * pnl + 2][r];
                    u8[4 + r] = acc[i][4 * pnl + 3][r];
                }
                rbf_n<8>(g8);
                rbf_n<8>(u8);
#pragma unroll
                for (int r = 0; r < 8; ++r) g8[r] = silu_f(g8[r]);
                rbf_n<8>(g8);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    p0[r] = g8[r] * u8[r];
                    p1[r] = g8[4 + r] * u8[4 + r];
                }
                pair8(p0, p1, odd, o);
                const int nout = ((col0 + pnl * 64) >> 1) + (odd ? 16 : 0) + cpos;
                if (live) *(uint4 *)(a.C + (int64_t)m * a.ldc + nout) = pack8(o);
            }
        }
    }
    if constexpr (EPI == EPI_CONV) {
        // vmcnt counts loads and stores together, so a load issued after a store is waited with
        // that store: every per-column operand (bias, Snake a / 1/b) is loaded once, before the
        // first store, and each row group's residual before the previous row group's stores.
        // The chunked form of the other epilogues (below) loaded the Snake parameters after each
        // store — one store latency in front of every 16-B parameter load: k = 1 C = 256 tile
        // epilogue 64.6 k → 41.0 k cycles, k = 7 C = 256 → 10.7 k (profiles/r05aq_conv_stamps_
        // before.log, r05ar_conv_stamps_after.log); 240 s decode 34.87 → 32.84 ms, bit-identical
        // (r05ar_ab_vae.log).  What is left of the k = 1 epilogue is its 256 KB of stores per
        // tile (raw x' and its Snake): staging the residual tile in LDS first measured ±0
        // (r05as_ab_env_vae_reslds.log)
        constexpr int NP = SN / 2;
        uint4 bz[NP];
        float sav[NP][8], sbv[NP][8];
        int colv[NP], phv[NP];
#pragma unroll
        for (int jp = 0; jp < NP; ++jp) {
            const int n = col0 + (2 * jp + (odd ? 1 : 0)) * 16 + cpos;
            phv[jp] = n / a.conv_cout;
            colv[jp] = n - phv[jp] * a.conv_cout;
            bz[jp] = a.bias ? *(const uint4 *)(a.bias + colv[jp]) : make_uint4(0, 0, 0, 0);
            if (a.Cs) {
                const float4 a0 = *(const float4 *)(a.sa + colv[jp]), a1 = *(const float4 *)(a.sa + colv[jp] + 4);
                const float4 b0 = *(const float4 *)(a.sib + colv[jp]), b1 = *(const float4 *)(a.sib + colv[jp] + 4);
                sav[jp][0] = a0.x; sav[jp][1] = a0.y; sav[jp][2] = a0.z; sav[jp][3] = a0.w;
                sav[jp][4] = a1.x; sav[jp][5] = a1.y; sav[jp][6] = a1.z; sav[jp][7] = a1.w;
                sbv[jp][0] = b0.x; sbv[jp][1] = b0.y; sbv[jp][2] = b0.z; sbv[jp][3] = b0.w;
                sbv[jp][4] = b1.x; sbv[jp][5] = b1.y; sbv[jp][6] = b1.z; sbv[jp][7] = b1.w;
            }
        }
        // residual (k = 1 convs of the C ≥ 256 residual units; one phase, so the output row is
        // m; res may be C): row group i + 1's loads issued before row group i's stores
        uint4 gv[2][NP];
        auto load_res = [&](int i, uint4 (&g)[NP]) {
            const int m = min(row0 + i * 16 + fr, a.M - 1);
#pragma unroll
            for (int jp = 0; jp < NP; ++jp)
                g[jp] = *(const uint4 *)(a.res + (int64_t)m * a.ldr + col0 + (2 * jp + (odd ? 1 : 0)) * 16 + cpos);
        };
        if (a.res) load_res(0, gv[0]);
#pragma unroll
        for (int i = 0; i < SM; ++i) {
            if (a.res && i + 1 < SM) load_res(i + 1, gv[(i + 1) & 1]);
            const int m = row0 + i * 16 + fr;
            const bool live = m < a.M;           // rows past M still join the lane exchange
#pragma unroll
            for (int jp = 0; jp < NP; ++jp) {
                float o[8];
                pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
                if (a.bias) {
                    float bb[8];
                    unpack8(bz[jp], bb);
                    add_n<8>(o, bb);
                }
                // the conv output rounded to bf16 (raw), then its Snake (conv.hip)
                rbf_n<8>(o);
                if (a.res) {                     // x' = bf16(x + bf16(acc + b))
                    float rr[8];
                    unpack8(gv[i & 1][jp], rr);
                    add_n<8>(o, rr);
                    rbf_n<8>(o);
                }
                const int64_t orow = (int64_t)m * a.conv_ostride + a.conv_ooff + phv[jp];
                const bool ok = live && orow >= 0 && orow < a.conv_lout;
                if (a.C && ok) *(uint4 *)(a.C + orow * a.ldc + colv[jp]) = pack8(o);
                if (a.Cs) {
                    float sn[8];
                    snake_n<8>(o, sav[jp], sbv[jp], sn);
                    if (ok) *(uint4 *)(a.Cs + orow * a.ldc + colv[jp]) = pack8(sn);
                }
            }
        }
    } else if constexpr (EPI != EPI_SWIGLU) {
        // operand loads (residual, gate, bias) of a chunk of CH row groups are all issued
        // before its first store: the stores may alias them (in-place residual: C == res),
        // so the compiler would otherwise wait for every load right after issuing it —
        // one full memory latency per 16-B store, exposed at one wave per SIMD
        constexpr int NP = SN / 2, CH = (CHMAX / NP) < 1 ? 1 : (CHMAX / NP);
#pragma unroll
        for (int c0 = 0; c0 < SM; c0 += CH) {
            uint4 rv[CH][NP], gv[CH][NP];
#pragma unroll
            for (int ii = 0; ii < CH; ++ii) {
                if (c0 + ii >= SM) break;
                const int m = min(row0 + (c0 + ii) * 16 + fr, a.M - 1);
                const int bb_ = (EPI == EPI_GATED_RES) ? m / a.rows_per_batch : 0;
#pragma unroll
                for (int jp = 0; jp < NP; ++jp) {
                    const int n = col0 + (2 * jp + (odd ? 1 : 0)) * 16 + cpos;
                    if constexpr (EPI == EPI_STORE) {
                        if (a.bias) rv[ii][jp] = *(const uint4 *)(a.bias + n);
                    } else {
                        rv[ii][jp] = *(const uint4 *)(a.res + (int64_t)m * a.ldr + n);
                        if constexpr (EPI == EPI_GATED_RES)
                            gv[ii][jp] = *(const uint4 *)(a.gate + (int64_t)bb_ * a.gate_bstride + n);
                    }
                }
            }
#pragma unroll
            for (int ii = 0; ii < CH; ++ii) {
                if (c0 + ii >= SM) break;
                const int i = c0 + ii;
                const int m = row0 + i * 16 + fr;
                const bool live = m < a.M;       // rows past M still join the lane exchange
#pragma unroll
                for (int jp = 0; jp < NP; ++jp) {
                    float o[8];
                    pair8(acc[i][2 * jp], acc[i][2 * jp + 1], odd, o);
                    const int n = col0 + (2 * jp + (odd ? 1 : 0)) * 16 + cpos;
                    if constexpr (EPI == EPI_STORE) {
                        if (a.bias) {
                            float bb[8];
                            unpack8(rv[ii][jp], bb);
#pragma unroll
                            for (int r = 0; r < 8; ++r) o[r] += bb[r];
                        }
                    } else {
                        float rr[8];
                        unpack8(rv[ii][jp], rr);
                        // same roundings as rr + bf16(bf16(o)·g) / rr + bf16(o), pairwise
                        rbf_n<8>(o);
                        if constexpr (EPI == EPI_GATED_RES) {
                            float gg[8];
                            unpack8(gv[ii][jp], gg);
#pragma unroll
                            for (int r = 0; r < 8; ++r) o[r] *= gg[r];
                            rbf_n<8>(o);
                        }
#pragma unroll
                        for (int r = 0; r < 8; ++r) o[r] = rr[r] + o[r];
                    }
                    if (live) *(uint4 *)(a.C + (int64_t)m * a.ldc + n) = pack8(o);
                }
            }
        }
    }
}

// NH > 0: NH helper waves issue every LDS-DMA piece (q ≡ h mod NH) with the same counted
// waits and barriers, so the NW MFMA waves (one per SIMD at NW = 4) carry no DMA in their stream
template <int BM, int BN, int WM, int WN, int STAGES, int EPI, int NH = 0>
__global__ __launch_bounds__(WM *WN * 64 + 64 * NH, 1) void gemm_kernel(GemmArgs a) {
    constexpr int NW = WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;          // wave tile
    constexpr int SM = TM / 16, SN = TN / 16;          // 16×16 sub-tiles per wave
    constexpr int ROWS = BM + BN;                      // rows of one stage image (128 B each)
    constexpr int STAGE = ROWS * 128;
    constexpr int NINS = ROWS / 8;                     // glds instructions per stage
    constexpr int PER_WAVE = NINS / NW;
    static_assert(NINS % NW == 0, "staging must split evenly over waves");
    static_assert(EPI != EPI_SWIGLU || TN % 64 == 0, "SwiGLU pairs 32+32 columns per 64-column panel");
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE];
    // split-K (EPI_PARTIAL): split blockIdx.y covers K-tiles [y·kper, min(nk, (y+1)·kper))
    const int ktile0 = EPI == EPI_PARTIAL ? (int)blockIdx.y * a.kper : 0;

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
    const int nk = EPI == EPI_PARTIAL ? min(a.kper, a.K / BK - ktile0) : a.K / BK;

    if constexpr (NH > 0) {
        if (__builtin_amdgcn_readfirstlane(wave) >= NW) {
            constexpr int PPH = NINS / NH;
            static_assert(NINS % NH == 0 && (STAGES - 1) * PPH < 64, "helper pieces / vmcnt field");
            const int h = wave - NW;
            const bf16_t *hs[PPH];
#pragma unroll
            for (int i = 0; i < PPH; ++i) {
                const int q = h + NH * i, r = q * 8 + (lane >> 3);
                const int c = (lane & 7) ^ ((r >> 1) & 7);
                if (r < BM) hs[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8 + ktile0 * BK;
                else hs[i] = a.W + (int64_t)(n0 + r - BM) * a.ldw + c * 8 + ktile0 * BK;
            }
            auto hst = [&](int buf, int k0) {
#pragma unroll
                for (int i = 0; i < PPH; ++i) glds16(hs[i] + k0, lds + buf * STAGE + (h + NH * i) * 1024);
            };
#pragma unroll
            for (int s2 = 0; s2 < STAGES - 1; ++s2)
                if (s2 < nk) hst(s2, s2 * BK);
            for (int kt = 0; kt < nk; ++kt) {
                if (kt + STAGES - 2 < nk) ring_barrier<(STAGES - 2) * PPH>();
                else ring_barrier<0>();
                if (kt + STAGES - 1 < nk) hst((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return;
        }
    }

    // staging sources: wave issues image rows [8q, 8q+8) for q = wave + NW·i
    const bf16_t *src[PER_WAVE];
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
        const int q = wave + NW * i;
        const int r = q * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        if (r < BM) src[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8 + ktile0 * BK;
        else src[i] = a.W + (int64_t)(n0 + r - BM) * a.ldw + c * 8 + ktile0 * BK;
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

    if constexpr (NH == 0) {
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
            if (s < nk) stage(s, s * BK);
    }
    const int fr = lane & 15, fc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt landed (its own wave's DMAs), leaving STAGES-2 newer tiles in flight
        // every wave's DMA for tile kt landed; tile kt-1 fully read (WAR for the refill below)
        if constexpr (NH > 0) {
            ring_barrier<0>();   // own reads retired (no DMA of its own); the helpers waited
        } else {
            if (kt + STAGES - 2 < nk) ring_barrier<(STAGES - 2) * PER_WAVE>();
            else ring_barrier<0>();
            if (kt + STAGES - 1 < nk) stage((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);
        }
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

    if constexpr (EPI == EPI_PARTIAL) {
        // fp32 partial sums of this split: lane's 4 consecutive columns → one 16-B store
        float *ws = (float *)a.ws + (size_t)blockIdx.y * a.M * a.N;
#pragma unroll
        for (int i = 0; i < SM; ++i) {
            const int m = m0 + wm * TM + i * 16 + fr;
            if (m >= a.M) continue;
#pragma unroll
            for (int j = 0; j < SN; ++j)
                *(f32x4 *)(ws + (int64_t)m * a.N + n0 + wn * TN + j * 16 + fc * 4) = acc[i][j];
        }
        return;
    } else {
        epilogue_tile<SM, SN, EPI>(a, acc, m0 + wm * TM, n0 + wn * TN, fr, fc);
    }
}

// Split-K reduction + the GEMM's epilogue (same rounding as epilogue_tile): the
// splits are summed in order (deterministic); one thread per 4 output columns.
// SwiGLU: packed columns p·64 + [0, 32) gate, p·64 + [32, 64) up → output p·32 + i.
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(GemmArgs a, int splits, bf16_t *out, int64_t ldo) {
    const int nout = a.epi == EPI_SWIGLU ? a.N / 2 : a.N;
    const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (e >= (int64_t)a.M * nout) return;
    const int m = (int)(e / nout), q = (int)(e % nout);
    const float *ws = (const float *)a.ws;
    const size_t plane = (size_t)a.M * a.N;
    auto sum4 = [&](int col) {
        f32x4 t = *(const f32x4 *)(ws + (int64_t)m * a.N + col);
        for (int sp = 1; sp < splits; ++sp) t += *(const f32x4 *)(ws + sp * plane + (int64_t)m * a.N + col);
        return t;
    };
    float o[4];
    if (a.epi == EPI_SWIGLU) {
        const int pnl = q / 32, i = q % 32;
        const f32x4 g = sum4(pnl * 64 + i), u = sum4(pnl * 64 + 32 + i);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = rbf(silu_f(rbf(g[r]))) * rbf(u[r]);
    } else {
        const f32x4 acc = sum4(q);
        if (a.epi == EPI_STORE || a.epi == EPI_HEADPOST) {
            float bb[4] = {0.f, 0.f, 0.f, 0.f};
            if (a.bias && a.epi == EPI_STORE) unpack4(*(const uint2 *)(a.bias + q), bb);
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = acc[r] + bb[r];
        } else {
            float rr[4];
            unpack4(*(const uint2 *)(a.res + (int64_t)m * a.ldr + q), rr);
            if (a.epi == EPI_GATED_RES) {
                float gg[4];
                unpack4(*(const uint2 *)(a.gate + (int64_t)(m / a.rows_per_batch) * a.gate_bstride + q), gg);
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = rr[r] + rbf(rbf(acc[r]) * gg[r]);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = rr[r] + rbf(acc[r]);
            }
        }
    }
    *(uint2 *)(out + (int64_t)m * ldo + q) = pack4(o);
}

// Head-post epilogue of a BM×256 QKV tile (two 128-column heads): bf16(acc) → LDS tile
// [BM][PITCH] (the operand ring is dead; store_acc(st, PITCH) writes the wave's
// accumulators), then one 16-lane group per (row, head): RMSNorm + RoPE + head-major
// store.  A lane's units: a fixed head (hh = sub & 1) and rows r = wave·2 + (sub >> 1)
// + 2·NW·it, so (batch, position) advance incrementally (no integer division per unit)
// and every cos/sin row is loaded BEFORE the first store (a load's vmcnt would
// otherwise also wait for the older stores).  When both heads of every tile are of one
// kind (q / k / v boundaries at even heads: the DiT's 16 | 8 | 8) the kind is a scalar, so
// the norm / RoPE choice is a scalar branch; otherwise (tiny test layouts) per lane.
//
// HPT = 1: a BM×128 tile holds one head; the four 16-lane groups of a wave take four rows.
template <int MODE, int ITER, int RPI, int PITCH>
__device__ __forceinline__ void headpost_rows(const GemmArgs &a, const bf16_t *st, int m0, int r0, int hh, int li,
                                              int d, int b0, int s0, bf16_t *base, int64_t bstride, bool norm,
                                              const float (&w)[8], const uint4 (&cv)[ITER], const uint4 (&sv)[ITER]) {
    // MODE: 0 v heads (scatter), 1 q/k without RoPE, 2 q/k with RoPE, 3 per-lane `norm`
    const HeadPostArgs &h = a.hp;
    int bq = b0, sq = s0;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int r = r0 + RPI * it;
        float x[8], cs[8] = {}, sn[8] = {};
        unpack8(*(const uint4 *)(st + r * PITCH + hh * 128 + d), x);
        if constexpr (MODE >= 2) {
            unpack8(cv[it], cs);
            unpack8(sv[it], sn);
        }
        if constexpr (MODE == 1) head_norm_rope_t<true, false>(x, li, w, cs, sn, h.eps);
        else if constexpr (MODE == 2) head_norm_rope_t<true, true>(x, li, w, cs, sn, h.eps);
        else if constexpr (MODE == 3) head_norm_rope(x, li, norm, w, h.cos != nullptr, cs, sn, h.eps);
        if (m0 + r < a.M) *(uint4 *)(base + (int64_t)bq * bstride + sq * 128) = pack8(x);
        sq += RPI;
        while (sq >= h.S) { sq -= h.S; ++bq; }
    }
}

template <int BM, int NW, int LDS_BYTES, int HPT, typename StoreAcc>
__device__ __forceinline__ void headpost_epilogue(const GemmArgs &a, char *lds, int m0, int n0, int wave, int lane,
                                                  StoreAcc store_acc) {
    static_assert(HPT == 1 || HPT == 2, "one or two heads per tile");
    constexpr int PITCH = 128 * HPT + 8;   // 16-B aligned rows, 2-way conflicts on the 8-B writes
    constexpr int RPW = 4 / HPT;           // rows per wave per iteration
    constexpr int RPI = RPW * NW;          // rows per iteration
    constexpr int ITER = BM / RPI;
    static_assert(BM % RPI == 0, "rows must split evenly over the iterations");
    static_assert(BM * PITCH * 2 <= LDS_BYTES, "head-post staging tile must fit the operand ring");
    const HeadPostArgs &h = a.hp;
    const int sub = lane >> 4, li = lane & 15, d = li * 8, hh = HPT == 2 ? sub & 1 : 0;
    const int head = (n0 >> 7) + hh;
    const int nqk = h.nq + h.nk;
    const bool norm = head < nqk;
    const bool rope = h.cos != nullptr;
    const int r0 = wave * RPW + (HPT == 2 ? sub >> 1 : sub);
    const int mf = min(m0 + r0, a.M - 1) + h.m_off;
    const int b0 = mf / h.S, s0 = mf - b0 * h.S;
    uint4 cv[ITER], sv[ITER];
    if (rope) {
        int sq = s0;
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const int sc = min(sq, h.S - 1);
            cv[it] = *(const uint4 *)(h.cos + (int64_t)sc * 128 + d);
            sv[it] = *(const uint4 *)(h.sin + (int64_t)sc * 128 + d);
            sq += RPI;
            while (sq >= h.S) sq -= h.S;
        }
    }
    // destination of this lane's head at (b = 0, s = 0) + its 8 columns, and the batch stride
    bf16_t *base;
    int64_t bstride;
    const int64_t hs = (int64_t)h.S_dst * 128;
    if (head < h.nq) {
        base = h.q + head * hs;
        bstride = h.nq * hs;
    } else if (head < nqk) {
        base = h.k + (head - h.nq) * hs;
        bstride = h.nk * hs;
    } else {
        base = h.v + (head - nqk) * hs;
        bstride = h.nv * hs;
    }
    base += d;
    float w[8] = {};
    if (norm) unpack8(*(const uint4 *)((head < h.nq ? h.qw : h.kw) + d), w);
    bf16_t *st = (bf16_t *)lds;
    __syncthreads();
    store_acc(st, PITCH);
    __syncthreads();
    const bool uniform = HPT == 1 || (h.nq % 2 == 0 && nqk % 2 == 0);
    if (uniform) {
        if ((n0 >> 7) >= nqk)
            headpost_rows<0, ITER, RPI, PITCH>(a, st, m0, r0, hh, li, d, b0, s0, base, bstride, norm, w, cv, sv);
        else if (!rope)
            headpost_rows<1, ITER, RPI, PITCH>(a, st, m0, r0, hh, li, d, b0, s0, base, bstride, norm, w, cv, sv);
        else
            headpost_rows<2, ITER, RPI, PITCH>(a, st, m0, r0, hh, li, d, b0, s0, base, bstride, norm, w, cv, sv);
    } else {
        headpost_rows<3, ITER, RPI, PITCH>(a, st, m0, r0, hh, li, d, b0, s0, base, bstride, norm, w, cv, sv);
    }
}

// ---------------------------------------------------------------------------
// Ping-pong variant: BM×256 tile, 8 waves as 2 groups (wr = 0/1, A rows
// [wr·BM/2, +BM/2)) × 4 (64 columns each).  The groups run one barrier apart,
// so on every SIMD one wave issues MFMAs while the other issues LDS reads and
// LDS-DMA (s_setprio(1) on the MFMA side).  Per K-tile, two phases of
// [ds_read · (stage) · barrier · MFMA over both 32-deep k-steps · barrier]:
//   phase 0  read the four B sub-tiles + A-half 0     stage A(kt+1) → other buffer
//   phase 1  read A-half 1                             stage B(kt+2) → this buffer's B slots,
//                                                       then vmcnt(#B glds): A(kt+1) landed
// (24 / 32 MFMAs per interval at 192 / 256 rows; reads retire before each barrier).
// WAR: A(kt+1) overwrites tile kt−1's A, last read by group 1's phase 1 of kt−1, retired
// before this phase's opening barrier; B(kt+2) overwrites tile kt's B, last read by group 1's
// phase 0, retired before the barrier that opens phase 1.  RAW: each wave's vmcnt precedes
// the barrier that opens the first read of the tile.  Two LDS tile buffers.
// Round 4 replaced a four-phase schedule (12 / 16 MFMAs per interval, 8
// barriers per K-tile; stamps: the 192-row loop 62 % MFMA-busy, now 80 %): DESIGN.md.
// The body of one ping-pong tile; `bid` = the block's index in this GEMM's grid (the fused
// main + tail launch below runs two GEMMs' grids in one) and `lds` = the kernel's 2·BUF bytes
template <int BM>
constexpr int pp_lds_bytes() { return 2 * (BM + 256) * 128; }
template <int BM, int EPI>
__device__ __forceinline__ void gemm_pp_body(const GemmArgs &a, char *lds, int bid) {
    constexpr int BN = 256, TM = BM / 2, SM = TM / 16, SMH = SM / 2;
    constexpr int ROWS = BM + BN, BUF = ROWS * 128;
    constexpr int NA = BM / 64, NB = BN / 64;                // glds per wave for A / B of one K-tile
    static_assert(SM % 2 == 0, "A half must be whole 16-row sub-tiles");

    GSTAMP(0);
    GSTAMP_REAL(4);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int tilesM = (a.M + BM - 1) / BM, tilesN = a.N / BN;
    const int nwg = tilesM * tilesN;
    const int wg = xcd_remap(bid, nwg);
    const int per_group = GROUP_M * tilesN;
    const int gid = wg / per_group, first_m = gid * GROUP_M;
    const int gsz = min(tilesM - first_m, GROUP_M);
    const int tm = first_m + (wg % per_group) % gsz;
    const int tn = (wg % per_group) / gsz;
    const int m0 = tm * BM, n0 = tn * BN;
#ifdef GEMM_STAMPS
    {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if ((threadIdx.x & 255) == 0) stamp(blockIdx.x * 2 + (threadIdx.x >> 8), 6, ((unsigned long long)wg << 32) | xcc);
    }
#endif

    const bf16_t *srcA[NA], *srcB[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int r = (wave + 8 * i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        srcA[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int r = (wave + 8 * i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (((BM + r) >> 1) & 7);
        srcB[i] = a.W + (int64_t)(n0 + r) * a.ldw + c * 8;
    }
    auto stageA = [&](int buf, int k0) {
        char *b = lds + buf * BUF;
        int ko = k0;
        if constexpr (EPI == EPI_CONV) {
            // implicit-GEMM conv: K-tile k0 = tap·cin + c0 reads the input rows shifted by
            // conv_a0 + tap·dil (zero halo rows around the activation)
            const int cin = a.conv_cin, tap = k0 / cin;
            ko = k0 + tap * (a.conv_dil - 1) * cin + a.conv_a0 * cin;
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) glds16(srcA[i] + ko, b + (wave + 8 * i) * 1024);
    };
    auto stageB = [&](int buf, int k0) {
        char *b = lds + buf * BUF + BM * 128;
#pragma unroll
        for (int i = 0; i < NB; ++i) glds16(srcB[i] + k0, b + (wave + 8 * i) * 1024);
    };
    auto bar = [] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    f32x4 acc[SM][4];
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fc = lane >> 4;
    const int arow = wr * TM, brow = BM + wc * 64;

    const int nk = a.K / BK;
    // prologue: tile 0 complete, B(1) in flight
    stageB(0, 0);
    stageA(0, 0);
    if (nk > 1) {
        stageB(1, BK);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    if (wr == 1) bar();   // group 1 runs one barrier behind
    GSTAMP(1);

    {
    bf16x8 xa[SMH][2], bf[4][2];
    auto readA = [&](const char *b, int h) {
#pragma unroll
        for (int i = 0; i < SMH; ++i)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                xa[i][ks] = *(const bf16x8 *)(b + swz(arow + (h * SMH + i) * 16 + fr, ks * 4 + fc));
    };
    auto mma = [&](int h) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < SMH; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[h * SMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], xa[i][ks], acc[h * SMH + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    for (int kt = 0; kt < nk; ++kt) {
        const char *b = lds + (kt & 1) * BUF;
        // phase 0: B (all four sub-tiles, both k-steps) + A-half 0; A(kt+1) → other buffer
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) bf[j][ks] = *(const bf16x8 *)(b + swz(brow + j * 16 + fr, ks * 4 + fc));
        readA(b, 0);
        if (kt + 1 < nk) stageA((kt + 1) & 1, (kt + 1) * BK);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        mma(0);
        bar();
        // phase 1: A-half 1; B(kt+2) → this buffer's B slots (tile kt's B: last read by the
        // other group in its phase 0, retired before the barrier above), then A(kt+1) landed
        readA(b, 1);
        if (kt + 2 < nk) {
            stageB(kt & 1, (kt + 2) * BK);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NB) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        bar();
        mma(1);
        bar();
    }
    }
    if (wr == 0) bar();   // balance the barrier count
    GSTAMP(2);

    if constexpr (EPI == EPI_HEADPOST && BM == 256) {
        // the 256-row staging tile (135 KB at the padded pitch) exceeds the operand ring: the two
        // wave groups' 128-row halves go through it one after the other (headpost_epilogue's
        // opening barrier keeps half 1's staging behind half 0's row pass)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
            headpost_epilogue<128, 8, 2 * BUF, 2>(a, lds, m0 + hf * 128, n0, wave, lane, [&](bf16_t *st, int pitch) {
                if (wr != hf) return;
#pragma unroll
                for (int i = 0; i < SM; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                        *(uint2 *)(st + (i * 16 + fr) * pitch + wc * 64 + j * 16 + fc * 4) = pack4(o);
                    }
            });
        return;
    } else if constexpr (EPI == EPI_HEADPOST) {
        headpost_epilogue<BM, 8, 2 * BUF, 2>(a, lds, m0, n0, wave, lane, [&](bf16_t *st, int pitch) {
#pragma unroll
            for (int i = 0; i < SM; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                    *(uint2 *)(st + (arow + i * 16 + fr) * pitch + wc * 64 + j * 16 + fc * 4) = pack4(o);
                }
        });
        return;
    }

    epilogue_tile<SM, 4, EPI>(a, acc, m0 + arow, n0 + wc * 64, fr, fc);
#ifdef GEMM_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    GSTAMP(3);
    GSTAMP_REAL(5);
}

template <int BM, int EPI>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[pp_lds_bytes<BM>()];
    gemm_pp_body<BM, EPI>(a, lds, blockIdx.x);
}

// The tail-split GEMM (gemm_tail_split: whole rounds of 256-row tiles + the remaining rows as
// one round of 128-row tiles) in ONE launch: blocks [0, nmain) run the main grid, the rest the
// tail grid, so the tail's blocks start on CUs as the main grid's last round drains instead of
// behind a kernel boundary (ACEHIP_GEMM_TAILFUSE)
template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_pp_split_kernel(GemmArgs a, GemmArgs t, int nmain) {
    __shared__ __attribute__((aligned(16))) char lds[pp_lds_bytes<256>()];
    if ((int)blockIdx.x < nmain) gemm_pp_body<256, EPI>(a, lds, blockIdx.x);
    else gemm_pp_body<128, EPI>(t, lds, blockIdx.x - nmain);
}

// ---------------------------------------------------------------------------
// Four-wave variant: BM×BN tile, one wave per SIMD (2×2 waves, wave tile
// (BM/2)×(BN/2): at the production 192×128, the half-chip M ≈ 3000 shapes, 24
// accumulators of 16×16 in AGPRs), register double-buffered fragments.  Per K-tile kt (two 32-deep k-steps), ONE barrier in the middle:
//   half A   MFMAs of k-step 0 (fragments F0)  ∥ ds_reads of k-step 1 → F1
//   ──────   own LDS-DMA of tile kt+1 retired (vmcnt(0): nothing newer is in
//            flight yet) + own reads retired, barrier: tile kt+1 is visible and
//            every wave has finished reading tile kt
//   half B   LDS-DMA of tile kt+2 into tile kt's buffer, MFMAs of k-step 1 (F1)
//            ∥ ds_reads of tile kt+1's k-step 0 → F0
// so the MFMA pipe never waits for a fragment read, the DMA of a tile has one whole
// K-tile (≈96 MFMAs) of lead, and two LDS buffers suffice.
// NH > 0: NH extra helper waves issue every LDS-DMA piece (pieces q ≡ h mod NH), so the four
// MFMA waves carry no DMA in their instruction stream (one wave per SIMD pays ≈ 60-185 cycles
// per piece there); a helper waits for tile kt+1 before barrier kt and refills tile kt's buffer
// after it, the same ordering as the MFMA waves' own refills
template <int BM, int BN, int EPI, int NH = 0>
__global__ __launch_bounds__(256 + 64 * NH, 1) void gemm_w4_kernel(GemmArgs a) {
    constexpr int TM = BM / 2, TN = BN / 2, SM = TM / 16, SN = TN / 16;
    constexpr int ROWS = BM + BN, STAGE = ROWS * 128;
    // ring depth: 3 tile buffers when they fit (a refill's DMA then has two K-tiles of lead,
    // enough for HBM-cold weights), else 2 (one K-tile of lead)
    constexpr int NS = 3 * STAGE <= 160 * 1024 ? 3 : 2;
    constexpr int PW = ROWS / 32;                              // glds per wave per K-tile
    static_assert(ROWS % 32 == 0, "staging must split evenly over 4 waves");
    __shared__ __attribute__((aligned(16))) char lds[NS * STAGE];

    GSTAMP(0);
    GSTAMP_REAL(4);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tilesM = (a.M + BM - 1) / BM, tilesN = a.N / BN;
    const int nwg = tilesM * tilesN;
    const int wg = xcd_remap(blockIdx.x, nwg);
    const int per_group = GROUP_M * tilesN;
    const int gid = wg / per_group, first_m = gid * GROUP_M;
    const int gsz = min(tilesM - first_m, GROUP_M);
    const int tm = first_m + (wg % per_group) % gsz;
    const int tn = (wg % per_group) / gsz;
    const int m0 = tm * BM, n0 = tn * BN;
    const int nk = a.K / BK;

    if constexpr (NH > 0) {
        if (__builtin_amdgcn_readfirstlane(wave) >= 4) {
            constexpr int PPH = 4 * PW / NH;                        // pieces per helper per K-tile
            static_assert((4 * PW) % NH == 0 && (NS - 1) * PPH < 64, "helper pieces / vmcnt field");
            const int h = wave - 4;
            const bf16_t *hs[PPH];
#pragma unroll
            for (int i = 0; i < PPH; ++i) {
                const int q = h + NH * i, r = q * 8 + (lane >> 3);
                const int c = (lane & 7) ^ ((r >> 1) & 7);
                if (r < BM) hs[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8;
                else hs[i] = a.W + (int64_t)(n0 + r - BM) * a.ldw + c * 8;
            }
            auto fill = [&](int buf, int k0) {
#pragma unroll
                for (int i = 0; i < PPH; ++i) glds16(hs[i] + k0, lds + buf * STAGE + (h + NH * i) * 1024);
            };
            for (int t = 0; t < NS; ++t) fill(t, min(t, nk - 1) * BK);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * PPH) : "memory");
            __builtin_amdgcn_s_barrier();
            for (int kt = 0; kt < nk; ++kt) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * PPH) : "memory");   // tile kt+1 landed
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                fill(kt % NS, min(kt + NS, nk - 1) * BK);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (EPI == EPI_HEADPOST) {   // the head-post epilogue's two block barriers
                __syncthreads();
                __syncthreads();
            }
            return;
        }
    }

    // staging: wave issues image rows [8q, 8q+8) for q = wave + 4i (swizzle on the source)
    const bf16_t *src[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int r = (wave + 4 * i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        if (r < BM) src[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8;
        else src[i] = a.W + (int64_t)(n0 + r - BM) * a.ldw + c * 8;
    }
    auto stage1 = [&](int buf, int k0, int i) { glds16(src[i] + k0, lds + buf * STAGE + (wave + 4 * i) * 1024); };
    f32x4 acc[SM][SN];
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fc = lane >> 4;
    const int xrow = wm * TM + fr, wrow = BM + wn * TN + fr;
    bf16x8 x0[SM], w0[SN], x1[SM], w1[SN];
    auto rd = [&](const char *b, int ks, bf16x8 (&xf)[SM], bf16x8 (&wf)[SN]) {
#pragma unroll
        for (int j = 0; j < SN; ++j) wf[j] = *(const bf16x8 *)(b + swz(wrow + j * 16, ks * 4 + fc));
#pragma unroll
        for (int i = 0; i < SM; ++i) xf[i] = *(const bf16x8 *)(b + swz(xrow + i * 16, ks * 4 + fc));
    };
    // MFMA by inline asm with the accumulator tied in place in AGPRs ("+a"): with the
    // builtin, the register allocator of ROCm 7.2 splits dst from srcC at this register
    // pressure (192 accumulators + 112 fragment registers) and rotates the whole
    // accumulator set through v_accvgpr_mov copies every K-tile
    // hook(n) runs after the n-th MFMA (the LDS-DMA pieces of a refill are spread over
    // the MFMA stream this way: volatile asm and the DMA builtin keep their order)
    auto mm = [&](const bf16x8 (&xf)[SM], const bf16x8 (&wf)[SN], auto hook) {
#pragma unroll
        for (int i = 0; i < SM; ++i)
#pragma unroll
            for (int j = 0; j < SN; ++j) {
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(wf[j]), "v"(xf[i]));
                hook(i * SN + j);
            }
    };
    auto none = [](int) {};
    // the wait is the builtin (vmcnt((NS−2)·PW) expcnt(7) lgkmcnt(0): tile kt+1 landed,
    // the NS−2 newer refills still in flight), so the compiler's own waitcnt pass knows
    // every read before it has retired and adds none after it
    constexpr int VM = (NS - 2) * PW;
    static_assert(VM < 64, "vmcnt field");
    constexpr int WAIT_ENC = 0x0070 | (VM & 15) | ((VM >> 4) << 14);
    auto bar = [] {
        __builtin_amdgcn_s_waitcnt(WAIT_ENC);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // (F0 was read during the previous half B: retire it with a compiler-visible
    // lgkmcnt(0) — vmcnt(63) expcnt(7) — before the next reads are issued, or the
    // compiler waits lgkmcnt(0) for it behind them)
    //
    // ONE straight-line loop body for every K-tile, the last ones included: the refill
    // source is clamped to the last tile (a duplicate load into a buffer nobody reads
    // again) and the last iteration's "next" reads hit a stale buffer (unused).  A
    // second copy of the MFMA code (a peeled tail) makes the register allocator move the
    // accumulators between copies with VALU instructions that the asm MFMAs — opaque
    // to the hazard recognizer — would read without the required wait states.
    // prologue: tiles 0..NS−1 (clamped: duplicates past the last tile keep the count
    // uniform), tile 0 landed
    if constexpr (NH == 0) {
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
            for (int i = 0; i < PW; ++i) stage1(t, min(t, nk - 1) * BK, i);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * PW) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    GSTAMP(1);
    rd(lds, 0, x0, w0);
    // refill pieces: one after every EVERY-th MFMA of half B, from MFMA FIRST on
    constexpr int EVERY = SM * SN / PW, FIRST = 1;
    static_assert(FIRST + EVERY * (PW - 1) < SM * SN, "refill pieces must fit in half B");
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt % NS, nxt = (kt + 1) % NS;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        rd(lds + cur * STAGE, 1, x1, w1);
        mm(x0, w0, none);
        bar();
        // refill of this tile's buffer (every wave is past its reads) with tile kt+NS
        const int kr = min(kt + NS, nk - 1) * BK;
        rd(lds + nxt * STAGE, 0, x0, w0);
        if constexpr (NH == 0) {
            mm(x1, w1, [&](int n) {
                if (n >= FIRST && (n - FIRST) % EVERY == 0 && (n - FIRST) / EVERY < PW) stage1(cur, kr, (n - FIRST) / EVERY);
            });
        } else {
            (void)kr;
            mm(x1, w1, none);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the asm MFMAs are opaque to the hazard recognizer: let the last ones retire
    // before their accumulators are read
    GSTAMP(2);
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    if constexpr (EPI == EPI_HEADPOST) {
        headpost_epilogue<BM, 4, sizeof(lds), BN / 128>(a, lds, m0, n0, wave, lane, [&](bf16_t *st, int pitch) {
#pragma unroll
            for (int i = 0; i < SM; ++i)
#pragma unroll
                for (int j = 0; j < SN; ++j) {
                    float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                    *(uint2 *)(st + (wm * TM + i * 16 + fr) * pitch + wn * TN + j * 16 + fc * 4) = pack4(o);
                }
        });
    } else {
        epilogue_tile<SM, SN, EPI>(a, acc, m0 + wm * TM, n0 + wn * TN, fr, fc);
    }
#ifdef GEMM_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    GSTAMP(3);
    GSTAMP_REAL(5);
}

template <int BM, int BN = 256, int NH = 0>
int launch_w4(const GemmArgs &a, hipStream_t s) {
    if (a.N % BN) return fail(-1, "gemm: N not a multiple of the 4-wave tile");
    const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
    constexpr int NT = 256 + 64 * NH;
    switch (a.epi) {
        case EPI_STORE: gemm_w4_kernel<BM, BN, EPI_STORE, NH><<<tiles, NT, 0, s>>>(a); break;
        case EPI_GATED_RES: gemm_w4_kernel<BM, BN, EPI_GATED_RES, NH><<<tiles, NT, 0, s>>>(a); break;
        case EPI_RES: gemm_w4_kernel<BM, BN, EPI_RES, NH><<<tiles, NT, 0, s>>>(a); break;
        case EPI_SWIGLU: klaunch(gemm_w4_kernel<BM, BN, EPI_SWIGLU, NH>, dim3(tiles), dim3(NT), s, a); break;
        case EPI_HEADPOST:
            if constexpr (BM == 192 && (BN == 256 || BN == 128)) {
                gemm_w4_kernel<BM, BN, EPI_HEADPOST, NH><<<tiles, NT, 0, s>>>(a);
                break;
            }
            return fail(-1, "gemm: the head-post epilogue needs the 192-row tile");
        default: return fail(-1, "gemm: bad epilogue for the 4-wave variant");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

template <int BM>
int launch_pp(const GemmArgs &a, hipStream_t s) {
    if (a.N % 256) return fail(-1, "gemm: N not a multiple of 256");
    const int tiles = ((a.M + BM - 1) / BM) * (a.N / 256);
    switch (a.epi) {
        case EPI_STORE: gemm_pp_kernel<BM, EPI_STORE><<<tiles, 512, 0, s>>>(a); break;
        case EPI_GATED_RES: gemm_pp_kernel<BM, EPI_GATED_RES><<<tiles, 512, 0, s>>>(a); break;
        case EPI_RES: gemm_pp_kernel<BM, EPI_RES><<<tiles, 512, 0, s>>>(a); break;
        case EPI_SWIGLU: klaunch(gemm_pp_kernel<BM, EPI_SWIGLU>, dim3(tiles), dim3(512), s, a); break;
        case EPI_CONV:
            if constexpr (BM == 256 || BM == 128) {
                gemm_pp_kernel<BM, EPI_CONV><<<tiles, 512, 0, s>>>(a);
                break;
            }
            return fail(-1, "gemm: the conv epilogue runs on the 256- or 128-row ping-pong tile");
        case EPI_HEADPOST:
            if constexpr (BM == 256 || BM == 192 || BM == 128) {
                gemm_pp_kernel<BM, EPI_HEADPOST><<<tiles, 512, 0, s>>>(a);
                break;
            }
            return fail(-1, "gemm: head-post epilogue needs the 256-, 192- or 128-row ping-pong tile");
        default: return fail(-1, "gemm: bad epilogue");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

template <int BM, int BN, int WM, int WN, int STAGES, int NH = 0>
int launch(const GemmArgs &a, hipStream_t s) {
    if (a.N % BN) return fail(-1, "gemm: N not a multiple of the tile");
    const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
    constexpr int NT = WM * WN * 64 + 64 * NH;
    switch (a.epi) {
        case EPI_STORE: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_STORE, NH><<<tiles, NT, 0, s>>>(a); break;
        case EPI_GATED_RES: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_GATED_RES, NH><<<tiles, NT, 0, s>>>(a); break;
        case EPI_RES: gemm_kernel<BM, BN, WM, WN, STAGES, EPI_RES, NH><<<tiles, NT, 0, s>>>(a); break;
        case EPI_SWIGLU: klaunch(gemm_kernel<BM, BN, WM, WN, STAGES, EPI_SWIGLU, NH>, dim3(tiles), dim3(NT), s, a); break;
        default: return fail(-1, "gemm: bad epilogue for this variant");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace

int gemm_variant(const GemmArgs &a, int variant, hipStream_t s) {
    switch (variant) {
        case 0: return launch<128, 128, 2, 2, 2>(a, s);   // 4 waves, 2-stage (2 blocks/CU): half-chip grids, tails
        // two-phase ping-pong tiles: 256x256 (128 KiB), 192x256 (112 KiB), 128x256 (96 KiB)
        case 7: return launch_pp<256>(a, s);
        case 8: return launch_pp<192>(a, s);
        case 9: return launch_pp<128>(a, s);
        // 4 MFMA waves, 96x64 wave tiles, + 2 LDS-DMA helper waves (M≈3000 shapes: 1 round;
        // ACEHIP_GEMM_HELPERS=0: without, A/B)
        case 13: return knobs().gemm_helpers ? launch_w4<192, 128, 2>(a, s) : launch_w4<192, 128>(a, s);
        case 16: return launch<128, 64, 4, 1, 4>(a, s);   // 4 waves × 32 rows × 64 columns, 4-stage: M ≤ 128 SwiGLU
        case 17: return launch<128, 64, 4, 1, 4, 2>(a, s);  // 16 + two LDS-DMA helper waves (M ≤ 128 SwiGLU)
        default: return fail(-1, "gemm: bad variant (0, 7, 8, 9, 13, 16, 17)");
    }
}

#ifdef GEMM_STAMPS
}  // namespace acehip
extern "C" int acehip_diag_gemm_stamps(void *host, int n_wg) {
    n_wg = std::min(n_wg, acehip::STAMP_WG);
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(acehip::g_gemm_stamps), (size_t)n_wg * 2 * 8 * 8));
    return 0;
}
extern "C" int acehip_diag_gemm_stamps_clear(void) {
    void *p = nullptr;
    HIP_TRY(hipGetSymbolAddress(&p, HIP_SYMBOL(acehip::g_gemm_stamps)));
    HIP_TRY(hipMemset(p, 0, sizeof(acehip::g_gemm_stamps)));
    return 0;
}
namespace acehip {
#endif

bool gemm_ext_events(hipEvent_t start, hipEvent_t stop) {
    const bool consumed = g_ext_ev.stop && !g_ext_ev.start;
    g_ext_ev.start = start;
    g_ext_ev.stop = stop;
    return consumed;
}

static int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

// Half-chip grids (M ≈ 3000: the conditional rows' cross-Q / cross-O): the four-wave
// 192×128 tile with a 3-deep ring fills the chip in one round (16 × 16 tiles at
// N = 2048) where the 128² tile runs 0.75 of a 2-blocks-per-CU round: 34–35 → 31 µs,
// hot or cold weights (tools/bench_gemm.py, r02).  ACEHIP_GEMM_W4S=0 disables it.
static bool use_w4s(int64_t M, int N) {
    if (knobs().gemm_w4s != 1 || N % 128) return false;
    const int cus = num_cus();
    const int64_t t = ((M + 191) / 192) * (N / 128);
    return t <= cus && t * 4 >= (int64_t)cus * 3;
}

// Tile choice from a one-block-per-CU cost model fitted on MI355X
// (tools/bench_gemm.py): time ∝ ⌈tiles / CUs⌉ × per-tile time, with a 256×256
// ping-pong tile costing 1.093× a 192×256 one (it does 1.33× the work).  The
// model reproduces the measured v7/v8 ratios on all four DiT shapes to 2 %.
// Grids that fill at most half the chip fall back to 128×128 (2 blocks/CU): at
// M = 3000, N = 2048 (the cross-O GEMM of the conditional rows) 37 µs vs 46 µs.
int gemm_pick_variant(int64_t M, int N) {
    if (use_w4s(M, N) && (N % 256 || ((M + 191) / 192) * (N / 256) <= num_cus() / 2)) return 13;
    if (N % 256) return 0;
    const int cus = num_cus();
    const int64_t t7 = ((M + 255) / 256) * (N / 256), t8 = ((M + 191) / 192) * (N / 256);
    if (t8 <= cus / 2) return 0;
    // one partial round of 192-row tiles (M ≈ 500: the 20 s song's CFG batch, the lyric
    // encoder's SwiGLU): 128-row tiles still fit one round and finish sooner (ACEHIP_GEMM_PP128)
    const int64_t t9 = ((M + 127) / 128) * (N / 256);
    if (knobs().gemm_pp128 && t8 <= cus && t9 <= cus) return 9;
    const double c7 = (double)((t7 + cus - 1) / cus) * 1.093, c8 = (double)((t8 + cus - 1) / cus);
    return c7 < c8 ? 7 : 8;
}

// Split-K for grids that cannot fill half the chip even with 128×128 tiles (short
// songs / turbo: M = Bc·S of a few hundred rows): the K range is split so the grid
// reaches ~1 block per CU (at least 4 K-tiles per split), every split stores fp32
// partials, and the epilogue is either folded into the consumer (head_post for the
// head-post case; the next rmsnorm_mod for residual epilogues, gemm(…, defer)) or run
// by splitk_epilogue_kernel.  Ring depth (tools/ab_splitk.py, M = 125): 3 stages for
// N ≤ 4096 (down / QKV / O: 20.1 → 19.0, 18.3 → 17.4, 15.1 → 14.9 µs), 2 for the wide
// SwiGLU (26.2 vs 28.3 µs).
static int splitk_finish(const GemmArgs &a, const GemmArgs &p, int splits, hipStream_t s);

// split-K tile width: 64-column tiles double the grid at a given split count (half the splits
// and partial bytes for ~1 block per CU).  Round 3 kept 128 where N and K < 4096 (O at M = 125
// measured 18.7 → 25.3 µs on 64); round 4 measured every shape faster on 64 (O 16.0 → 14.7, QKV
// 15.4 → 14.8, `profiles/r04h2_small_m.log`) and the songs too (turbo 10 s DiT 25.6 → 24.6 ms,
// base 10 s 96.9 → 93.9, `profiles/r04h3_ab_turbo.log`): 64 everywhere.  ACEHIP_SPLITK_BN =
// 128 | 64 forces one (A/B)
static int splitk_bn(const GemmArgs &) {
    const int f = knobs().splitk_bn;
    if (f) return f == 64 ? 64 : 128;
    return 64;
}
static void fill_defer(const GemmArgs &a, int splits, RowAdd *defer);
static int gemm_splitk(const GemmArgs &a, int splits, hipStream_t s, RowAdd *defer = nullptr) {
    GemmArgs p = a;
    const int nk = a.K / BK;
    p.kper = (nk + splits - 1) / splits;
    splits = (nk + p.kper - 1) / p.kper;
    const int bn = splitk_bn(a);
    const int tiles = ((a.M + 127) / 128) * (a.N / bn);
    // (helper waves measured no gain here: 2 MFMA waves / SIMD already cover the DMA issue)
    if (bn == 64) gemm_kernel<128, 64, 4, 1, 3, EPI_PARTIAL><<<dim3(tiles, splits), 256, 0, s>>>(p);
    else if (a.N <= 4096) gemm_kernel<128, 128, 2, 2, 3, EPI_PARTIAL><<<dim3(tiles, splits), 256, 0, s>>>(p);
    else gemm_kernel<128, 128, 2, 2, 2, EPI_PARTIAL><<<dim3(tiles, splits), 256, 0, s>>>(p);
    HIP_TRY(hipGetLastError());
    if (defer) {
        fill_defer(a, splits, defer);
        return 0;
    }
    return splitk_finish(a, p, splits, s);
}

// the residual epilogue is left to the consumer norm (in place: C == res)
static void fill_defer(const GemmArgs &a, int splits, RowAdd *defer) {
    defer->xw = a.C;
    defer->part = (const float *)a.ws;
    defer->splits = splits;
    defer->prows = a.M;
    defer->plane = (int64_t)a.M * a.N;
    defer->gate = a.epi == EPI_GATED_RES ? a.gate : nullptr;
    defer->gate_bstride = a.gate_bstride;
    defer->gate_rpb = a.epi == EPI_GATED_RES ? a.rows_per_batch : 1;
}

// sum the fp32 split partials in order + the GEMM's epilogue (head-post: staged bf16
// projection + the standalone head_post kernel, or head_post reading the partials itself)
static int splitk_finish(const GemmArgs &a, const GemmArgs &p, int splits, hipStream_t s) {
    if (a.epi == EPI_HEADPOST && knobs().splitk_fuse) {
        // head_post reads the partials itself (one launch, no bf16 staging round trip)
        HeadPostArgs h = a.hp;
        h.part = (const float *)a.ws;
        h.splits = splits;
        h.plane = (int64_t)a.M * a.N;
        h.ld_src = a.N;
        return head_post(h, s);
    }
    bf16_t *out = a.C;
    int64_t ldo = a.ldc;
    if (a.epi == EPI_HEADPOST) {   // bf16 projection staged after the partials
        out = (bf16_t *)((char *)a.ws + (size_t)splits * a.M * a.N * 4);
        ldo = a.N;
    }
    const int nout = a.epi == EPI_SWIGLU ? a.N / 2 : a.N;
    const int64_t thr = (int64_t)a.M * nout / 4;
    splitk_epilogue_kernel<<<(unsigned)((thr + 255) / 256), 256, 0, s>>>(p, splits, out, ldo);
    HIP_TRY(hipGetLastError());
    if (a.epi == EPI_HEADPOST) {
        HeadPostArgs h = a.hp;
        h.src = out;
        h.ld_src = a.N;
        return head_post(h, s);
    }
    return 0;
}

// Tail split for ping-pong grids whose last round is a small fraction of the chip
// (SwiGLU gate/up at 240 s: 24 × 48 = 1152 tiles of 256² on 256 CUs = 4.5 rounds, the
// last half-round costing a whole tile time): rows [0, M1) keep the big tile with
// M1 chosen so their grid is whole rounds (less at most one row of tiles), and the
// remaining rows run as one round of 128×128 tiles (2 blocks/CU).  Row-local
// epilogues only (store / SwiGLU; the gated residual indexes its batch by row).
// ACEHIP_GEMM_TAILSPLIT=0 disables it.  Returns 1 when not applicable.
static int gemm_tail_split(const GemmArgs &a, int v, hipStream_t s) {
    if (a.epi != EPI_SWIGLU && a.epi != EPI_STORE && a.epi != EPI_HEADPOST) return 1;
    if (!knobs().gemm_tailsplit) return 1;
    const int BMv = v == 7 ? 256 : 192, cus = num_cus();   // v = 7 or 8
    const int64_t nN = a.N / 256, tiles = (int64_t)((a.M + BMv - 1) / BMv) * nN;
    const int64_t full = tiles / cus, rem = tiles - full * cus;
    if (full < 1 || rem == 0 || rem * 5 > (int64_t)cus * 3) return 1;   // last round > 60 % full
    const int64_t M1 = (full * cus / nN) * BMv;
    if (M1 <= 0 || M1 >= a.M) return 1;
    if (((a.M - M1 + 127) / 128) * (a.N / 128) > 2 * (int64_t)cus) return 1;
    GemmArgs hd = a;
    hd.M = (int)M1;
    GemmArgs tl = a;
    tl.M = a.M - (int)M1;
    tl.A = a.A + M1 * a.lda;
    if (a.epi == EPI_HEADPOST) tl.hp.m_off += (int)M1;   // C unused: rows scatter by (b, s)
    else tl.C = a.C + M1 * a.ldc;
    // ACEHIP_GEMM_TAIL=1: the tail as one round of 128×256 two-phase ping-pong tiles
    const bool pp128 = knobs().gemm_tail == 1 && a.N % 256 == 0 && ((tl.M + 127) / 128) * nN <= cus;
    if (a.epi == EPI_HEADPOST && !pp128) return 1;   // the 128×128 tail tile has no head-post epilogue
    if (pp128 && v == 7 && knobs().gemm_tailfuse) {
        // both grids in one launch (the main grid's block count is a multiple of 8, so the tail
        // blocks' XCD is their own index mod 8, as in a launch of their own)
        const int nmain = (int)(full * cus / nN * nN), ntail = ((tl.M + 127) / 128) * (int)nN;
        if (nmain % 8 == 0 && nmain == (hd.M / 256) * (int)nN && hd.M % 256 == 0) {
            if (a.epi == EPI_SWIGLU) klaunch(gemm_pp_split_kernel<EPI_SWIGLU>, dim3(nmain + ntail), dim3(512), s, hd, tl, nmain);
            else if (a.epi == EPI_HEADPOST) gemm_pp_split_kernel<EPI_HEADPOST><<<nmain + ntail, 512, 0, s>>>(hd, tl, nmain);
            else gemm_pp_split_kernel<EPI_STORE><<<nmain + ntail, 512, 0, s>>>(hd, tl, nmain);
            HIP_TRY(hipGetLastError());
            return 0;
        }
    }
    int rc = gemm_variant(hd, v, s);
    if (rc) return rc;
    return gemm_variant(tl, pp128 ? 9 : 0, s);
}

// the conv epilogue on 64-row ping-pong tiles
static int launch_conv64(const GemmArgs &a, hipStream_t s) {
    const int tiles = ((a.M + 63) / 64) * (a.N / 256);
    gemm_pp_kernel<64, EPI_CONV><<<tiles, 512, 0, s>>>(a);
    HIP_TRY(hipGetLastError());
    return 0;
}

int gemm_conv(const GemmArgs &a, hipStream_t s) {
    if (a.epi != EPI_CONV || (!a.C && !a.Cs) || (a.Cs && (!a.sa || !a.sib)) || a.conv_cin <= 0 || a.conv_dil < 1 ||
        a.conv_ostride < 1 || a.conv_cout <= 0 || a.conv_cout % 8 || a.N % a.conv_cout || a.conv_lout <= 0 || a.M <= 0)
        return fail(-1, "gemm_conv: EPI_CONV with an output, snake parameters and conv geometry required");
    if (a.N % 256 || a.conv_cin % BK || a.K % a.conv_cin || a.lda != a.conv_cin || a.ldw != a.K || a.ldc != a.conv_cout)
        return fail(-1, "gemm_conv: N % 256, cin % 64, K = taps·cin and dense layouts required");
    if (a.res && (a.N != a.conv_cout || a.ldr != a.N || a.conv_ostride != 1 || a.conv_ooff != 0 || a.conv_lout != a.M))
        return fail(-1, "gemm_conv: a residual needs one phase with output row = m");
    if ((int64_t)((a.M + 255) / 256) * (a.N / 256) >= (1ll << 31)) return fail(-1, "gemm_conv: grid too large");
    // short activations (a 10 s decode's C = 1024 / 512 blocks: 40 / 118 tiles of 256 rows on
    // 256 CUs): 128-row tiles double the grid, 64-row tiles (80 KB of LDS, 118 VGPRs: two blocks
    // per CU) quadruple it.  10 s decode 2.13 → 1.96 (128) → 1.91 ms (64 below a quarter of the
    // chip), bit-identical (profiles/r05az_ab_vae_small_tiles.log; ACEHIP_CONV_BM128)
    const int64_t t256 = (int64_t)((a.M + 255) / 256) * (a.N / 256);
    if (knobs().conv_bm128 == 2 && t256 * 4 <= num_cus()) return launch_conv64(a, s);
    if (knobs().conv_bm128 && t256 * 2 <= num_cus()) return launch_pp<128>(a, s);
    return launch_pp<256>(a, s);
}

int gemm(const GemmArgs &a, hipStream_t s, RowAdd *defer) {
    if (defer) defer->part = nullptr;
    if (a.M <= 0) return 0;
    // argument checks shared by every path (split-K included)
    if (a.N % 128 || a.K % BK || a.K <= 0)
        return fail(-1, "gemm: N%128 / K%64 violated (M=" + std::to_string(a.M) + " N=" +
                            std::to_string(a.N) + " K=" + std::to_string(a.K) + ")");
    if ((a.lda | a.ldw | a.ldc) % 8) return fail(-1, "gemm: leading dims must be multiples of 8");
    if (a.epi == EPI_GATED_RES && (!a.gate || a.rows_per_batch <= 0)) return fail(-1, "gemm: gate");
    if ((a.epi == EPI_GATED_RES || a.epi == EPI_RES) && !a.res) return fail(-1, "gemm: res");
    if (a.epi == EPI_HEADPOST) {
        const HeadPostArgs &h = a.hp;
        if (a.N % 256 || h.S <= 0 || (int64_t)h.B * h.S != a.M || (h.nq + h.nk + h.nv) * 128 != a.N ||
            h.S_dst < h.S || (h.nq && !h.qw) || (h.nk && !h.kw) || (h.cos == nullptr) != (h.sin == nullptr))
            return fail(-1, "gemm: head-post arguments inconsistent with the GEMM shape");
    }
    const Knobs &kn = knobs();
    // a deferred epilogue needs the in-place residual form the consumer norm applies
    const bool dfr = defer && kn.splitk_fuse && (a.epi == EPI_GATED_RES || a.epi == EPI_RES) && a.res == a.C &&
                     a.ldr == a.ldc && a.ldc == a.N;
    // SwiGLU of one 128-row chunk (turbo / short songs, M ≤ 128): whole-K 128×64 tiles with the
    // SwiGLU epilogue fused (variant 16: no fp32 partials, no second launch) — M = 125, cold
    // weights: 26.1 → 19.0 µs (tools/bench_small_m.py).  ACEHIP_SMALLM_WHOLEK=0: split-K (A/B)
    if (a.epi == EPI_SWIGLU && a.M <= 128 && a.N % 64 == 0 && kn.smallm_wholek) return gemm_variant(a, kn.smallm_wholek == 2 ? 17 : 16, s);
    if (a.ws && a.N % 128 == 0 && a.K % BK == 0 && (a.N % 256 == 0 || a.epi != EPI_HEADPOST)) {
        const int cus = num_cus();
        const int64_t tiles = ((a.M + 127) / 128) * (a.N / 128);
        const int nk = a.K / BK;
        if (tiles * 2 <= cus && nk >= 8) {
            const int64_t tb = ((a.M + 127) / 128) * (a.N / splitk_bn(a));   // grid tiles of the split kernel
            int splits = (int)std::min<int64_t>(std::min<int64_t>(16, nk / 4), (cus + tb - 1) / tb);
            const size_t need = (size_t)splits * a.M * a.N * 4 + (size_t)a.M * a.N * 2;
            if (splits >= 2 && need <= a.ws_bytes) return gemm_splitk(a, splits, s, dfr ? defer : nullptr);
        }
    }
    if (a.epi == EPI_HEADPOST) {
        // a 192×256 grid that fills at most half the chip (cross-Q of the conditional rows,
        // M = 3000) runs as 192×128 tiles — one head each — with the same fused epilogue;
        // ACEHIP_GEMM_HP128=2: those tiles into the staging buffer + the standalone
        // head_post kernel (the previous path), =0: the 192×256 grid regardless
        const int64_t t192 = (int64_t)((a.M + 191) / 192) * (a.N / 256);
        const bool small = t192 * 2 <= num_cus() && kn.gemm_hp128 != 0;
        if (small && use_w4s(a.M, a.N) && kn.gemm_hp128 != 2) return gemm_variant(a, 13, s);
        if (small && a.ws && (size_t)a.M * a.N * 2 <= a.ws_bytes) {
            GemmArgs st = a;
            st.epi = EPI_STORE;
            st.bias = nullptr;
            st.C = (bf16_t *)a.ws;
            st.ldc = a.N;
            int rc = gemm_variant(st, use_w4s(a.M, a.N) ? 13 : 0, s);
            if (rc) return rc;
            HeadPostArgs hh = a.hp;
            hh.src = st.C;
            hh.ld_src = a.N;
            return head_post(hh, s);
        }
        // whole rounds of 256-row tiles + one round of 128-row tiles where that costs less than
        // the 192-row rounds (cost model of gemm_pick_variant, a 128×256 tile ≈ 0.6 of a 192×256
        // one): QKV at 240 s, 32 × 16 = 2 rounds of 192 → 1 round of 256 + 1 of 128
        if (kn.gemm_hp_tail && a.N % 256 == 0) {
            const int cus = num_cus();
            const int64_t nN = a.N / 256, t7 = ((a.M + 255) / 256) * nN, t8 = ((a.M + 191) / 192) * nN;
            const double c_split = (double)(t7 / cus) * 1.093 + 0.6, c8 = (double)((t8 + cus - 1) / cus);
            if (t7 >= cus && c_split < c8) {
                const int rc = gemm_tail_split(a, 7, s);
                if (rc <= 0) return rc;
            }
        }
        return gemm_variant(a, 8, s);
    }
    const int v = gemm_pick_variant(a.M, a.N);
    if (v == 7 || v == 8) {
        const int rc = gemm_tail_split(a, v, s);
        if (rc <= 0) return rc;   // split done (0) or failed (< 0); 1 = not applicable
    }
    return gemm_variant(a, v, s);
}

}  // namespace acehip
