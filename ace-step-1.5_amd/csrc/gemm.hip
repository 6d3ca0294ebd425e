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
#ifndef W4_DMA_EVERY
#define W4_DMA_EVERY 0     // 4-wave GEMM refill spacing in MFMAs (0: spread over half B)
#endif
#ifndef W4_DMA_FIRST
#define W4_DMA_FIRST 1     // MFMA index of the first refill piece (−1: all before the reads)
#endif
#ifndef W4_COST
#define W4_COST 0.92       // 4-wave 192×256 tile time relative to the ping-pong one (cost model)
#endif
#ifndef PP_SCHED
#define PP_SCHED -1        // ping-pong main loop: -1 per tile (256 rows: 1, 192 rows: 0); 0 12/4/8/0-read phases, 1 8/4/8/4, 2 two phases
#endif

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
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    p0[r] = rbf(silu_f(rbf(acc[i][4 * pnl][r]))) * rbf(acc[i][4 * pnl + 2][r]);
                    p1[r] = rbf(silu_f(rbf(acc[i][4 * pnl + 1][r]))) * rbf(acc[i][4 * pnl + 3][r]);
                }
                pair8(p0, p1, odd, o);
                const int nout = ((col0 + pnl * 64) >> 1) + (odd ? 16 : 0) + cpos;
                if (live) *(uint4 *)(a.C + (int64_t)m * a.ldc + nout) = pack8(o);
            }
        }
    }
    if constexpr (EPI != EPI_SWIGLU) {
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
                        if constexpr (EPI == EPI_GATED_RES) {
                            float gg[8];
                            unpack8(gv[ii][jp], gg);
#pragma unroll
                            for (int r = 0; r < 8; ++r) o[r] = rr[r] + rbf(rbf(o[r]) * gg[r]);
                        } else {
#pragma unroll
                            for (int r = 0; r < 8; ++r) o[r] = rr[r] + rbf(o[r]);
                        }
                    }
                    if (live) *(uint4 *)(a.C + (int64_t)m * a.ldc + n) = pack8(o);
                }
            }
        }
    }
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

    const int nk = EPI == EPI_PARTIAL ? min(a.kper, a.K / BK - ktile0) : a.K / BK;
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

// ---------------------------------------------------------------------------
// Weight-streaming ("skinny") GEMM for M ≤ 128 rows per chunk: turbo / short songs
// (M = Bc·S = 125 at 10 s turbo) where every projection is a read of W with a few
// FLOPs per byte (SwiGLU at M = 125: 120 flop/B, far below the 312 flop/B ridge).
// No LDS staging and no barrier in the main loop: each block owns BN = 16·NT columns
// (an N-slab) and one K-range (split), its 4 waves take interleaved 32-deep K-steps
// (wave w: steps w, w+4, ...), and every operand fragment goes straight from memory
// to the MFMA's registers by buffer_load_dwordx4 (W fragment = 16 rows × 64 B, the
// X fragment likewise): W is read exactly once chip-wide, X (≤ 0.5 MB at K = 2048)
// from L2.  Rows past M read zeros (the buffer range check), so no clamping.  The
// four waves' partial accumulators are summed through LDS and the block stores its
// fp32 partial tile [split][M][N] (the split-K workspace layout); the caller's
// splitk_epilogue_kernel sums the splits in order and applies the epilogue.
// Block order: units (slab, split) with equal index mod 8 share an XCD, so with
// splits = 8 every XCD's blocks read one K-slice of X (L2-resident); the row chunks
// of one unit are 8 block ids apart (same XCD: the second chunk's W comes from L2).
template <int MT, int NT, int D>
__global__ __launch_bounds__(256, 1) void skinny_kernel(GemmArgs a, int kper, int splits, int nchunk) {
    __shared__ f32x4 red[4][MT][NT][64];
    const int lane = threadIdx.x & 63;
    // wave-uniform values made provably uniform (readfirstlane), so the buffer
    // descriptors live in SGPRs and no load is wrapped in a waterfall loop (T20)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 15, q = lane >> 4;
    const int U = gridDim.x / nchunk, L = blockIdx.x;
    int u, chunk;
    if ((U & 7) == 0) {
        const int g = L / (8 * nchunk), rem = L % (8 * nchunk);
        chunk = rem >> 3;
        u = g * 8 + (rem & 7);
    } else {
        u = L % U;
        chunk = L / U;
    }
    const int slab = u / splits, split = u % splits;
    const int n0 = slab * 16 * NT, m0 = chunk * 16 * MT;
    const int kb = split * kper, nst = (min(a.K, kb + kper) - kb) / 32;
    const int spw = (nst - wave + 3) / 4;               // this wave's K-steps: wave + 4t, t < spw
    // buffer descriptors as SGPR quads (base, stride 0, num_records, gfx9 dword3),
    // built from provably wave-uniform values
    auto srd = [](const void *p, int64_t bytes) {
        const uint64_t v = (uint64_t)p;
        u32x4 d;
        d[0] = __builtin_amdgcn_readfirstlane((uint32_t)v);
        d[1] = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
        d[2] = __builtin_amdgcn_readfirstlane((uint32_t)bytes);
        d[3] = 0x00020000;
        return d;
    };
    const u32x4 rx = srd(a.A + (int64_t)m0 * a.lda, (int64_t)(a.M - m0) * a.lda * 2);
    const u32x4 rw = srd(a.W + (int64_t)n0 * a.ldw, (int64_t)16 * NT * a.ldw * 2);
    const u32x4 rz = srd(a.W, 0);   // every load out of range: zeros
    int ox[MT], ow[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) ox[i] = ((16 * i + r) * (int)a.lda + q * 8) * 2;
#pragma unroll
    for (int j = 0; j < NT; ++j) ow[j] = ((16 * j + r) * (int)a.ldw + q * 8) * 2;

    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // K-step t of this wave into (x, w): inline-asm buffer loads, so the only vector-
    // memory operations of the loop are these (MT + NT per step) and the waits below
    // count them exactly (hipcc's own waitcnt placement drained the ring at the loop
    // join); past the wave's steps the zero descriptor is used, so a padded step adds
    // exact zeros with no branch around the loads or the MFMAs
    u32x4 xs[D][MT], wsr[D][NT];
    auto load = [&](u32x4(&x)[MT], u32x4(&w)[NT], int t) {
        const bool ok = t < spw;
        const u32x4 sw = ok ? rw : rz, sx = ok ? rx : rz;
        const int ko = __builtin_amdgcn_readfirstlane((kb + (wave + 4 * t) * 32) * 2);
#pragma unroll
        for (int j = 0; j < NT; ++j)
            asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(w[j]) : "v"(ow[j]), "s"(sw), "s"(ko));
#pragma unroll
        for (int i = 0; i < MT; ++i)
            asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(x[i]) : "v"(ox[i]), "s"(sx), "s"(ko));
    };
    // MFMAs by inline asm with the accumulators tied to AGPRs ("+a"): with the builtin,
    // hipcc keeps them in VGPRs beside the operand ring and shuffles ~200 registers
    // through v_accvgpr_* every iteration
    auto mma = [&](const u32x4(&x)[MT], const u32x4(&w)[NT]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(w[j]), "v"(x[i]));
    };
    // D-slot register ring: D−1 K-steps in flight while one is multiplied
#pragma unroll
    for (int d = 0; d < D - 1; ++d) load(xs[d], wsr[d], d);
    const int niter = (spw + D - 1) / D;
    for (int it = 0; it < niter; ++it) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int t = it * D + d;
            load(xs[(d + D - 1) % D], wsr[(d + D - 1) % D], t + D - 1);
            // slot d landed: only the D−1 younger steps' loads may still be in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * (MT + NT)) : "memory");
            mma(xs[d], wsr[d]);
        }
    }
    // the ring's last (zero) loads land before their registers can be reused: hipcc does
    // not know they are in flight, so the ring stays live (empty asm uses) until the wait;
    // XDL write → VALU read (v_accvgpr_read) hazard: hipcc does not pad after asm MFMAs
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int i = 0; i < MT; ++i) asm volatile("" ::"v"(xs[d][i]));
#pragma unroll
        for (int j = 0; j < NT; ++j) asm volatile("" ::"v"(wsr[d][j]));
    }
    // sum the four waves' partials: every wave parks its accumulators, then wave w
    // reduces the (i, j) sub-tiles with (i·NT + j) % 4 == w and stores them
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) red[wave][i][j][lane] = acc[i][j];
    __syncthreads();
    float *ws = (float *)a.ws + (size_t)split * a.M * a.N;
#pragma unroll
    for (int t = 0; t < MT * NT; ++t) {
        if (t % 4 != wave) continue;
        const int i = t / NT, j = t % NT;
        const f32x4 v = red[0][i][j][lane] + red[1][i][j][lane] + red[2][i][j][lane] + red[3][i][j][lane];
        const int m = m0 + 16 * i + r;
        if (m < a.M) *(f32x4 *)(ws + (int64_t)m * a.N + n0 + 16 * j + 4 * q) = v;
    }
}

// Head-post epilogue of a BM×256 QKV tile (two 128-column heads): bf16(acc) → LDS tile
// [BM][PITCH] (the operand ring is dead; store_acc(st, PITCH) writes the wave's
// accumulators), then one 16-lane group per (row, head): RMSNorm + RoPE + head-major
// store.  A lane's units: a fixed head (hh = sub & 1) and rows r = wave·2 + (sub >> 1)
// + 2·NW·it, so (batch, position) advance incrementally (no integer division per unit)
// and every cos/sin row is loaded BEFORE the first store (a load's vmcnt would
// otherwise also wait for the older stores).
//
// HPT = 1: a BM×128 tile holds one head; the four 16-lane groups of a wave take four rows.
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
    const bool norm = head < h.nq + h.nk;
    const bool rope = h.cos != nullptr;
    const int r0 = wave * RPW + (HPT == 2 ? sub >> 1 : sub);
    const int mf = min(m0 + r0, a.M - 1);
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
    float w[8] = {};
    if (norm) unpack8(*(const uint4 *)((head < h.nq ? h.qw : h.kw) + d), w);
    bf16_t *st = (bf16_t *)lds;
    __syncthreads();
    store_acc(st, PITCH);
    __syncthreads();
    int bq = b0, sq = s0;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int r = r0 + RPI * it;
        float x[8], cs[8] = {}, sn[8] = {};
        unpack8(*(const uint4 *)(st + r * PITCH + hh * 128 + d), x);
        if (rope) {
            unpack8(cv[it], cs);
            unpack8(sv[it], sn);
        }
        const bf16_t *nw;
        bf16_t *dst = head_dst(h, head, bq, sq, nw);
        head_norm_rope(x, li, norm, w, rope, cs, sn, h.eps);
        if (m0 + r < a.M && dst) *(uint4 *)(dst + d) = pack8(x);
        sq += RPI;
        while (sq >= h.S) { sq -= h.S; ++bq; }
    }
}

// ---------------------------------------------------------------------------
// Ping-pong variant: BM×256 tile, 8 waves as 2 groups (wr = 0/1, A rows
// [wr·BM/2, +BM/2)) × 4 (64 columns each).  The groups run one barrier apart,
// so on every SIMD one wave issues MFMAs while the other issues LDS reads and
// LDS-DMA (s_setprio(1) on the MFMA side).  Per K-tile, 4 phases of
// [ds_read · (stage) · barrier · MFMA · barrier]:
//   phase 0  read A-half0 + B0          stage A(kt+1) → other buffer
//   phase 1  read B1
//   phase 2  read A-half1
//   phase 3  (B0, B1 still in regs)     stage B(kt+2) → this buffer's B slots,
//                                        then vmcnt(#B glds): A(kt+1) landed
// WAR: A(kt+1) overwrites tile kt−1's A, last read (group 1, phase 2) two
// barriers earlier; B(kt+2) overwrites tile kt's B, last read in phase 1.
// RAW: each wave's vmcnt precedes the barrier that opens the first read of
// the tile (barrier 8kt+8 for group 0).  Two LDS tile buffers, ~1 tile of
// DMA lead for A and ~1.25 for B.
// DBG (diagnostic variants 20-22 only, results meaningless): bit 0 drops the main-loop
// LDS-DMA, bit 1 the main-loop fragment reads (SCHED 1).
// SPL (SCHED 1 only): how the LDS-DMA pieces of a K-tile are spread over its phases —
//   0  A(kt+1) all in phase 0, B(kt+2) all in phase 3
//   1  A(kt+1) half in phase 0, half in phase 1; B(kt+2) all in phase 3
//   2  A(kt+1) half in phase 0, half in phase 1; B(kt+2) first half in phase 3, second
//      half in the next K-tile's phase 0 (as B(kt+1))
//   3  as 2, but B(kt+1)'s second half in phase 1 (phase 0 carries only its 8 reads + 2);
//      the 256-row default: interleaved 5-round medians (tools/bench_gemm.py ROUNDS=5, cold
//      weights) SwiGLU 251.3 vs 257.3 µs, QKV 91.7 vs 95.0, down 128.6 vs 133.4 against 0
//      (the ablation behind it: without the main-loop DMA the 256² tile ran 22 % faster,
//      without the fragment reads 18 %, without both 37 %)
// SCHED 0 takes SPL 1 only: A(kt+1) split between phases 0 and 1 (phase 3 has no reads)
template <int BM, int EPI, int DBG = 0, int SPL = (BM == 256 ? 3 : 0), int SCH = -1>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmArgs a) {
    constexpr int BN = 256, TM = BM / 2, SM = TM / 16, SMH = SM / 2;
    constexpr int ROWS = BM + BN, BUF = ROWS * 128;
    constexpr int NA = BM / 64, NB = BN / 64;                // glds per wave for A / B of one K-tile
    static_assert(SM % 2 == 0, "A half must be whole 16-row sub-tiles");
    __shared__ __attribute__((aligned(16))) char lds[2 * BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int tilesM = (a.M + BM - 1) / BM, tilesN = a.N / BN;
    const int nwg = tilesM * tilesN;
    const int wg = xcd_remap(blockIdx.x, nwg);
    const int per_group = GROUP_M * tilesN;
    const int gid = wg / per_group, first_m = gid * GROUP_M;
    const int gsz = min(tilesM - first_m, GROUP_M);
    const int tm = first_m + (wg % per_group) % gsz;
    const int tn = (wg % per_group) / gsz;
    const int m0 = tm * BM, n0 = tn * BN;

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
#pragma unroll
        for (int i = 0; i < NA; ++i) glds16(srcA[i] + k0, b + (wave + 8 * i) * 1024);
    };
    auto stageB = [&](int buf, int k0) {
        char *b = lds + buf * BUF + BM * 128;
#pragma unroll
        for (int i = 0; i < NB; ++i) glds16(srcB[i] + k0, b + (wave + 8 * i) * 1024);
    };
    auto stageAp = [&](int buf, int k0, int i0, int i1) {
        char *b = lds + buf * BUF;
#pragma unroll
        for (int i = i0; i < i1; ++i) glds16(srcA[i] + k0, b + (wave + 8 * i) * 1024);
    };
    auto stageBp = [&](int buf, int k0, int i0, int i1) {
        char *b = lds + buf * BUF + BM * 128;
#pragma unroll
        for (int i = i0; i < i1; ++i) glds16(srcB[i] + k0, b + (wave + 8 * i) * 1024);
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
    if (SPL >= 2 && nk > 1) {
        stageBp(1, BK, 0, NB / 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB / 2) : "memory");
    } else if (nk > 1) {
        stageB(1, BK);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    if (wr == 1) bar();   // group 1 runs one barrier behind

    constexpr int SCHED = SCH >= 0 ? SCH : PP_SCHED >= 0 ? PP_SCHED : (BM == 256 ? 1 : 0);
    static_assert(SPL == 0 || SCHED == 1 || (SCHED == 0 && SPL == 1), "LDS-DMA spread: SCHED 1, or SPL 1 on SCHED 0");
    if constexpr (SCHED == 2) {
    // Two phases per K-tile (k-step 0, k-step 1; 32 MFMAs each): half the barriers of
    // the 4-phase schedules.  Phase 0 stages the whole next tile (A and B) into the
    // other buffer, whose last reads (the partner group's phase 1 of tile kt−1)
    // completed before this window's opening barrier; phase 1 waits for its own DMAs.
    bf16x8 xk[2 * SMH], bk[4];
    auto readA2 = [&](const char *b, int ks) {
#pragma unroll
        for (int i = 0; i < 2 * SMH; ++i) xk[i] = *(const bf16x8 *)(b + swz(arow + i * 16 + fr, ks * 4 + fc));
    };
    auto readB2 = [&](const char *b, int ks) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bk[j] = *(const bf16x8 *)(b + swz(brow + j * 16 + fr, ks * 4 + fc));
    };
    auto mma2 = [&] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2 * SMH; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bk[j], xk[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    for (int kt = 0; kt < nk; ++kt) {
        const char *b = lds + (kt & 1) * BUF;
        readB2(b, 0);
        readA2(b, 0);
        if (kt + 1 < nk) {
            stageA((kt + 1) & 1, (kt + 1) * BK);
            if (kt >= 1) stageB((kt + 1) & 1, (kt + 1) * BK);   // B(1) came with the prologue
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        mma2();
        bar();
        readB2(b, 1);
        readA2(b, 1);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        bar();
        mma2();
        bar();
    }
    } else if constexpr (SCHED == 1) {
    // Balanced schedule: phase p multiplies A-half (p & 1) by all four B sub-tiles at
    // k-step (p >> 1), so a loader wave issues 8, 4, 8, 4 ds_read_b128 per phase (the
    // 12-read first phase of the schedule below, plus the A(kt+1) DMA, saturates the
    // 256 B/clk LDS array against a 256-cycle MFMA phase) and holds 8 operand
    // fragments instead of 16.  Reads complete (lgkmcnt(0)) BEFORE each barrier, so
    // the WAR margins of the DMAs (A(kt+1) after tile kt−1's phase-3 reads, B(kt+2)
    // after tile kt's phase-2 reads) are one barrier each.
    bf16x8 xk[SMH], bk[4];
    auto readA1 = [&](const char *b, int h, int ks) {
        if constexpr (DBG & 2) return;
#pragma unroll
        for (int i = 0; i < SMH; ++i) xk[i] = *(const bf16x8 *)(b + swz(arow + (h * SMH + i) * 16 + fr, ks * 4 + fc));
    };
    auto readB1 = [&](const char *b, int ks) {
        if constexpr (DBG & 2) return;
#pragma unroll
        for (int j = 0; j < 4; ++j) bk[j] = *(const bf16x8 *)(b + swz(brow + j * 16 + fr, ks * 4 + fc));
    };
    auto mma1 = [&](int h) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < SMH; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[h * SMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bk[j], xk[i], acc[h * SMH + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    for (int kt = 0; kt < nk; ++kt) {
        const char *b = lds + (kt & 1) * BUF;
        readB1(b, 0);
        readA1(b, 0, 0);
        if (!(DBG & 1) && kt + 1 < nk) {
            if constexpr (SPL == 0) stageA((kt + 1) & 1, (kt + 1) * BK);
            else stageAp((kt + 1) & 1, (kt + 1) * BK, 0, NA / 2);
            if constexpr (SPL == 2) stageBp((kt + 1) & 1, (kt + 1) * BK, NB / 2, NB);
        }
        lgkm0();
        bar();
        mma1(0);
        bar();
        readA1(b, 1, 0);
        if (SPL != 0 && !(DBG & 1) && kt + 1 < nk) {
            stageAp((kt + 1) & 1, (kt + 1) * BK, NA / 2, NA);
            if constexpr (SPL == 3) stageBp((kt + 1) & 1, (kt + 1) * BK, NB / 2, NB);
        }
        lgkm0();
        bar();
        mma1(1);
        bar();
        readB1(b, 1);
        readA1(b, 0, 1);
        lgkm0();
        bar();
        mma1(0);
        bar();
        readA1(b, 1, 1);
        if (SPL >= 2 && !(DBG & 1) && kt + 2 < nk) {
            stageBp(kt & 1, (kt + 2) * BK, 0, NB / 2);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NB / 2) : "memory");
        } else if (!(DBG & 1) && kt + 2 < nk) {
            stageB(kt & 1, (kt + 2) * BK);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NB) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        bar();
        mma1(1);
        bar();
    }
    } else {
    bf16x8 xa[SMH][2], b0[2][2], b1[2][2];
    auto readA = [&](const char *b, int h) {
#pragma unroll
        for (int i = 0; i < SMH; ++i)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                xa[i][ks] = *(const bf16x8 *)(b + swz(arow + (h * SMH + i) * 16 + fr, ks * 4 + fc));
    };
    auto readB = [&](const char *b, int q, bf16x8 (&f)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                f[j][ks] = *(const bf16x8 *)(b + swz(brow + (q * 2 + j) * 16 + fr, ks * 4 + fc));
    };
    auto mma = [&](int h, int q, const bf16x8 (&f)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < SMH; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[h * SMH + i][q * 2 + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[j][ks], xa[i][ks], acc[h * SMH + i][q * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    for (int kt = 0; kt < nk; ++kt) {
        const char *b = lds + (kt & 1) * BUF;
        // phase 0
        readB(b, 0, b0);
        readA(b, 0);
        if (kt + 1 < nk) {
            if constexpr (SPL == 1) stageAp((kt + 1) & 1, (kt + 1) * BK, 0, NA / 2);
            else stageA((kt + 1) & 1, (kt + 1) * BK);
        }
        bar();
        mma(0, 0, b0);
        bar();
        // phase 1
        readB(b, 1, b1);
        if (SPL == 1 && kt + 1 < nk) stageAp((kt + 1) & 1, (kt + 1) * BK, NA / 2, NA);
        bar();
        mma(0, 1, b1);
        bar();
        // phase 2
        readA(b, 1);
        bar();
        mma(1, 1, b1);
        bar();
        // phase 3
        if (kt + 2 < nk) {
            stageB(kt & 1, (kt + 2) * BK);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        mma(1, 0, b0);
        bar();
    }
    }
    if (wr == 0) bar();   // balance the barrier count

    if constexpr (EPI == EPI_HEADPOST) {
        headpost_epilogue<BM, 8, sizeof(lds), 2>(a, lds, m0, n0, wave, lane, [&](bf16_t *st, int pitch) {
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
}

// ---------------------------------------------------------------------------
// Four-wave variant: BM×256 tile, one wave per SIMD (2×2 waves, wave tile
// (BM/2)×128: 48 or 64 accumulators of 16×16, in AGPRs), register double-buffered
// fragments.  Per K-tile kt (two 32-deep k-steps), ONE barrier in the middle:
//   half A   MFMAs of k-step 0 (fragments F0)  ∥ ds_reads of k-step 1 → F1
//   ──────   own LDS-DMA of tile kt+1 retired (vmcnt(0): nothing newer is in
//            flight yet) + own reads retired, barrier: tile kt+1 is visible and
//            every wave has finished reading tile kt
//   half B   LDS-DMA of tile kt+2 into tile kt's buffer, MFMAs of k-step 1 (F1)
//            ∥ ds_reads of tile kt+1's k-step 0 → F0
// so the MFMA pipe never waits for a fragment read, the DMA of a tile has one whole
// K-tile (≈96 MFMAs) of lead, and two LDS buffers suffice.
// DBG 1: no main-loop refill (diagnostic 29).
// VG 1: the main-loop refill goes through VGPRs instead of LDS-DMA — each wave holds the
// next refill's PW pieces in registers (buffer_load_dwordx4, issued one K-tile ahead) and
// writes them with ds_write_b128 at the hook points where the DMA pieces were issued (the
// prologue still stages tiles 0..NS−1 by LDS-DMA).  An LDS-DMA piece costs its wave ≈60
// cycles of issue among MFMAs (MI355X_MICROARCH.md, per-instruction constants); the plain
// load + store pair is meant to cost less.
template <int BM, int BN, int EPI, int DBG = 0, int VG = 0>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(GemmArgs a) {
    constexpr int TM = BM / 2, TN = BN / 2, SM = TM / 16, SN = TN / 16;
    constexpr int ROWS = BM + BN, STAGE = ROWS * 128;
    // ring depth: 3 tile buffers when they fit (a refill's DMA then has two K-tiles of lead,
    // enough for HBM-cold weights), else 2 (one K-tile of lead)
    constexpr int NS = 3 * STAGE <= 160 * 1024 ? 3 : 2;
    constexpr int PW = ROWS / 32;                              // glds per wave per K-tile
    static_assert(ROWS % 32 == 0, "staging must split evenly over 4 waves");
    __shared__ __attribute__((aligned(16))) char lds[NS * STAGE];

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
    // VG: buffer resources over this tile's A rows (rows past M read as zeros) and W rows;
    // piece i is 32 image rows below piece i−1, its source column chunk is the same
    // (the swizzle term (r >> 1) & 7 does not change over 32 rows)
    constexpr int PA = BM / 32;                                   // pieces of A rows
    static_assert(BM % 32 == 0, "A pieces must be whole");
    const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.A + (int64_t)m0 * a.lda), 0, (int)min((int64_t)(a.M - m0) * a.lda * 2, (int64_t)0x7fffffff),
        0x00020000);
    const __amdgpu_buffer_rsrc_t rsW =
        __builtin_amdgcn_make_buffer_rsrc((void *)(a.W + (int64_t)n0 * a.ldw), 0, BN * a.ldw * 2, 0x00020000);
    const int vr0 = wave * 8 + (lane >> 3), vc = (lane & 7) ^ ((vr0 >> 1) & 7);
    const int voA = (vr0 * a.lda + vc * 8) * 2, voW = (vr0 * a.ldw + vc * 8) * 2;
    u32x4 stg[VG ? PW : 1];
    auto vload = [&](int k0, int i) {
        if constexpr (VG) {
            if (i < PA) stg[i] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voA + i * 64 * a.lda, k0 * 2, 0);
            else stg[i] = __builtin_amdgcn_raw_buffer_load_b128(rsW, voW + (i - PA) * 64 * a.ldw, k0 * 2, 0);
        }
    };
    auto vstore = [&](int buf, int i) {
        if constexpr (VG) *(u32x4 *)(lds + buf * STAGE + (wave + 4 * i) * 1024 + lane * 16) = stg[i];
    };

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
    // (VG: the PW register loads of the next refill stay in flight across the barrier; the
    // prologue's LDS-DMA of tile kt+1 is older than them)
    constexpr int VM = VG ? PW : (NS - 2) * PW;
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
    const int nk = a.K / BK;
    // prologue: tiles 0..NS−1 (clamped: duplicates past the last tile keep the count
    // uniform), tile 0 landed
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
        for (int i = 0; i < PW; ++i) stage1(t, min(t, nk - 1) * BK, i);
    if constexpr (VG) {
#pragma unroll
        for (int i = 0; i < PW; ++i) vload(min(NS, nk - 1) * BK, i);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS * PW) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * PW) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd(lds, 0, x0, w0);
    // refill pieces: one after every EVERY-th MFMA of half B, from MFMA FIRST on
    constexpr int EVERY = W4_DMA_EVERY > 0 ? W4_DMA_EVERY : SM * SN / PW, FIRST = W4_DMA_FIRST;
    static_assert(FIRST + EVERY * (PW - 1) < SM * SN, "refill pieces must fit in half B");
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt % NS, nxt = (kt + 1) % NS;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        rd(lds + cur * STAGE, 1, x1, w1);
        mm(x0, w0, none);
        bar();
        // refill of this tile's buffer (every wave is past its reads) with tile kt+NS
        const int kr = min(kt + NS, nk - 1) * BK;
        const int kr1 = min(kt + NS + 1, nk - 1) * BK;   // VG: the refill after this one
        if constexpr (FIRST < 0) {
#pragma unroll
            for (int i = 0; i < PW; ++i) {
                if constexpr (VG) {
                    vstore(cur, i);
                    vload(kr1, i);
                } else {
                    stage1(cur, kr, i);
                }
            }
        }
        rd(lds + nxt * STAGE, 0, x0, w0);
        mm(x1, w1, [&](int n) {
            if (!(DBG & 1) && FIRST >= 0 && n >= FIRST && (n - FIRST) % EVERY == 0 && (n - FIRST) / EVERY < PW) {
                if constexpr (VG) {
                    __builtin_amdgcn_sched_barrier(0);
                    vstore(cur, (n - FIRST) / EVERY);
                    vload(kr1, (n - FIRST) / EVERY);
                    __builtin_amdgcn_sched_barrier(0);
                } else {
                    stage1(cur, kr, (n - FIRST) / EVERY);
                }
            }
        });
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the asm MFMAs are opaque to the hazard recognizer: let the last ones retire
    // before their accumulators are read
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
}

template <int BM, int BN = 256>
int launch_w4(const GemmArgs &a, hipStream_t s) {
    if (a.N % BN) return fail(-1, "gemm: N not a multiple of the 4-wave tile");
    const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
    switch (a.epi) {
        case EPI_STORE: gemm_w4_kernel<BM, BN, EPI_STORE><<<tiles, 256, 0, s>>>(a); break;
        case EPI_GATED_RES: gemm_w4_kernel<BM, BN, EPI_GATED_RES><<<tiles, 256, 0, s>>>(a); break;
        case EPI_RES: gemm_w4_kernel<BM, BN, EPI_RES><<<tiles, 256, 0, s>>>(a); break;
        case EPI_SWIGLU: klaunch(gemm_w4_kernel<BM, BN, EPI_SWIGLU>, dim3(tiles), dim3(256), s, a); break;
        case EPI_HEADPOST:
            if constexpr (BM == 192 && (BN == 256 || BN == 128)) {
                gemm_w4_kernel<BM, BN, EPI_HEADPOST><<<tiles, 256, 0, s>>>(a);
                break;
            }
            return fail(-1, "gemm: the head-post epilogue needs the 192-row tile");
        default: return fail(-1, "gemm: bad epilogue for the 4-wave variant");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------------------
// Stream-K variant of the 256×256 ping-pong tile (N ≤ 4096 projections whose grid is not a
// whole number of rounds: down / self-O at M = 6000 are 192 tiles of 256² on 256 CUs — the
// 192×256 tile fills one round but does 0.82× the work per cycle).  The grid is one block
// per CU; the tiles' K-iterations, concatenated in tile order, are split into equal ranges
// (block i: iterations [I·i/G, I·(i+1)/G)), so every CU multiplies the same number of
// K-tiles.  A range is at most: the late part of one tile (it FINISHES that tile), whole
// tiles, and the head (or a middle part) of one more tile (it CONTRIBUTES to it).  Each
// block runs its contribution first — fp32 partial tile to its own workspace slot
// (write-through sc1 stores), then a ready flag — and then its finishing segments; a
// finisher whose tile began in earlier blocks' ranges adds their partials (in block
// order: deterministic) before the tile's epilogue.  Flags are reset by their consumer, so
// the next launch (or a graph replay) starts from zero.  Deadlock-free: a block waits only
// for contributions, which every block issues before any wait, and the grid (one 128-KiB
// block per CU, grid = CU count) is co-resident; the spin is bounded regardless.
struct SkArgs {
    float *part;        // [G][8 waves][32 fragments][64 lanes] f32x4 = 256 KiB per block
    int *flag;          // [G] 1 = that block's partial is published
    int G;              // grid size (= CUs)
    int ktiles;         // K / 64
};

// compile-time loop: f(integral_constant<I>) for I in [I0, I1)
template <int I0, int I1, typename F>
__device__ __forceinline__ void sk_for(F &&f) {
    if constexpr (I0 < I1) {
        f(std::integral_constant<int, I0>{});
        sk_for<I0 + 1, I1>(f);
    }
}
// accumulator fragment (4 AGPRs from number A) → VGPRs
template <int A>
__device__ __forceinline__ f32x4 sk_acc(void) {
    f32x4 r;
    asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                 "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                 : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3])
                 : "n"(A), "n"(A + 1), "n"(A + 2), "n"(A + 3));
    return r;
}

// the asm-operand captures below are required (clang rejects the implicit form) yet
// reported as unused
#pragma clang diagnostic ignored "-Wunused-lambda-capture"
template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_sk_kernel(GemmArgs a, SkArgs sk) {
    constexpr int BM = 256, BN = 256, TM = BM / 2, SM = TM / 16, SMH = SM / 2;
    constexpr int ROWS = BM + BN, BUF = ROWS * 128;
    constexpr int NA = BM / 64, NB = BN / 64;
    __shared__ __attribute__((aligned(16))) char lds[2 * BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int fr = lane & 15, fc = lane >> 4;
    const int arow = wr * TM, brow = BM + wc * 64;
    const int tilesM = (a.M + BM - 1) / BM, tilesN = a.N / BN;
    const int nk = sk.ktiles;
    // tile t of the K-step sequence → (tm, tn) in groups of GROUP_M tile rows (as
    // gemm_pp_kernel): the ~24 consecutive tiles of one XCD's blocks then share 8 A and
    // 3 W panels, and all blocks start at K-tile 0 together (lockstep K-slices in L2)
    auto tile_mn = [&](int t, int &tm, int &tn) {
        const int per_group = GROUP_M * tilesN;
        const int gid = t / per_group, first_m = gid * GROUP_M;
        const int gsz = min(tilesM - first_m, GROUP_M);
        tm = first_m + (t % per_group) % gsz;
        tn = (t % per_group) / gsz;
    };
    const int64_t I = (int64_t)tilesM * (a.N / BN) * nk;
    // logical block index: XCD-contiguous (blocks of one XCD take consecutive ranges, so a
    // contributor and its finisher mostly share the XCD's L2)
    const int blk = xcd_remap(blockIdx.x, sk.G);
    auto range_start = [&](int b) { return (int64_t)b * I / sk.G; };
    const int64_t s0 = range_start(blk), e0 = range_start(blk + 1);

    // Segments in processing order: the contribution (the range ends inside tile tc: its
    // first or a middle part), then the finished tiles from tf1 − 1 DOWN to tf0 (only tf0
    // can start mid-tile: it needs the earlier blocks' partials, published long before).
    // One continuous K-step sequence q = 0 .. e0 − s0 − 1 over all of them, so the LDS-DMA
    // pipeline runs straight across segment boundaries (the next tile's first K-tiles are
    // staged during the previous tile's last ones).
    const int64_t tc = e0 / nk, tf0 = s0 / nk, tf1 = e0 / nk;
    const bool contrib = e0 % nk != 0;
    const int c_kb = contrib ? (int)(max(s0, tc * nk) - tc * nk) : 0;
    const int c_len = contrib ? (int)(e0 - tc * nk) - c_kb : 0;
    const int f_kb = (int)(s0 - tf0 * nk);                   // tf0's first K-tile
    const int Q = (int)(e0 - s0);
    // K-step cursors (tile, K-tile, segment end, segment index), advanced by one step per
    // main-loop iteration with scalar arithmetic: cA for the A staging (step q + 1), cB for
    // the B staging (q + 2), cM for the step being multiplied (q)
    struct Cur { int t, k, ke, sg; };
    auto seg_begin = [&](Cur &c) {
        if (contrib && c.sg == 0) {
            c.t = (int)tc; c.k = c_kb; c.ke = c_kb + c_len;
        } else {
            const int j = c.sg - (contrib ? 1 : 0);
            c.t = (int)(tf1 - 1 - j);
            c.k = (c.t == (int)tf0) ? f_kb : 0;
            c.ke = nk;
        }
    };
    auto advance = [&](Cur &c) {
        if (++c.k == c.ke) { ++c.sg; seg_begin(c); }
    };

    auto bar = [] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // staging sources: per-lane panel-row pointers of the cursor's tile, rebuilt only when
    // the staged step enters a new tile (per stage: one 64-bit add per LDS-DMA)
    const bf16_t *srcA[NA], *srcB[NB];
    int tA = -1, tB = -1;
    auto set_srcA = [&](int t) {
        int tm, tn;
        tile_mn(t, tm, tn);
        const int m0 = tm * BM;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int r = (wave + 8 * i) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            srcA[i] = a.A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 8;
        }
        tA = t;
    };
    auto set_srcB = [&](int t) {
        int tm, tn;
        tile_mn(t, tm, tn);
        const int n0 = tn * BN;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int r = (wave + 8 * i) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (((BM + r) >> 1) & 7);
            srcB[i] = a.W + (int64_t)(n0 + r) * a.ldw + c * 8;
        }
        tB = t;
    };
    auto stageA = [&](int buf, const Cur &c) {
        if (c.t != tA) set_srcA(c.t);
        char *b = lds + buf * BUF;
#pragma unroll
        for (int i = 0; i < NA; ++i) glds16(srcA[i] + c.k * BK, b + (wave + 8 * i) * 1024);
    };
    auto stageB = [&](int buf, const Cur &c) {
        if (c.t != tB) set_srcB(c.t);
        char *b = lds + buf * BUF + BM * 128;
#pragma unroll
        for (int i = 0; i < NB; ++i) glds16(srcB[i] + c.k * BK, b + (wave + 8 * i) * 1024);
    };
    auto lane_l = [&] { int v = lane; asm volatile("" : "+v"(v)); return v; };
    // The accumulators live in a[0:127] BY NUMBER (fragment (i, j) at a[16i + 4j]) and are
    // touched only by inline asm: MFMAs, the zeroing writes and the reads of the segment
    // finish.  hipcc, left with ≤ 128 VGPRs and no MFMA of its own, allocates no AGPR (the
    // a127 clobber makes the kernel descriptor reserve them) — with accumulators as C++
    // values it shuffled them between VGPRs, AGPRs and scratch around the finish code.
    auto acc_zero = [] {
        sk_for<0, 128>([&](auto R) __attribute__((always_inline)) {
            asm volatile("v_accvgpr_write_b32 a%c0, 0" ::"n"(decltype(R)::value));
        });
        asm volatile("s_nop 2" ::: "a0", "a127");   // v_accvgpr_write → MFMA srcC read
    };
    acc_zero();
    bf16x8 xk[SMH], bk[4];
    auto readA1 = [&](const char *b, int h, int ks) {
#pragma unroll
        for (int i = 0; i < SMH; ++i) xk[i] = *(const bf16x8 *)(b + swz(arow + (h * SMH + i) * 16 + fr, ks * 4 + fc));
    };
    auto readB1 = [&](const char *b, int ks) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bk[j] = *(const bf16x8 *)(b + swz(brow + j * 16 + fr, ks * 4 + fc));
    };
    // MFMAs by inline asm with the accumulators tied to AGPRs ("+a"): the segment finish
    // (epilogue / partial store / partial add) then draws on the VGPRs alone — with the
    // builtin, hipcc kept them in VGPRs and spilled ~160 registers around the finish code
    auto mma1 = [&](auto HC) __attribute__((always_inline)) {
        constexpr int h = decltype(HC)::value;
        bf16x8 *bkp = bk, *xkp = xk;
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        sk_for<0, SMH * 4>([bkp, xkp](auto G) __attribute__((always_inline)) {
            constexpr int g = decltype(G)::value, i = g / 4, j = g % 4, A = ((h * SMH + i) * 4 + j) * 4;
            asm volatile("v_mfma_f32_16x16x32_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                         ::"n"(A), "n"(A + 3), "v"(bkp[j]), "v"(xkp[i]));
        });
        __builtin_amdgcn_s_setprio(0);
    };
    auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    // this block's partial slot: fragment f of wave w at lane l = part + ((w·32 + f)·64 + l)·4
    auto slot = [&](int b) { return sk.part + ((int64_t)b * 512 * 32 + (int64_t)(wave * 32) * 64 + lane) * 4; };

    // prologue (as gemm_pp_kernel): step 0 complete, B(1) in flight
    Cur cM{0, 0, 0, 0}, cA{0, 0, 0, 0}, cB{0, 0, 0, 0};
    seg_begin(cM);
    cA = cM;
    cB = cM;
    if (Q > 0) {
        stageB(0, cB);
        stageA(0, cA);
        advance(cA);
        advance(cB);
        if (Q > 1) {
            stageB(1, cB);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        advance(cB);
    }
    bar();
    if (wr == 1) bar();   // group 1 runs one barrier behind
    for (int q = 0; q < Q; ++q) {
        const char *b = lds + (q & 1) * BUF;
        readB1(b, 0);
        readA1(b, 0, 0);
        if (q + 1 < Q) {
            stageA((q + 1) & 1, cA);
            advance(cA);
        }
        lgkm0();
        bar();
        mma1(std::integral_constant<int, 0>{});
        bar();
        readA1(b, 1, 0);
        lgkm0();
        bar();
        mma1(std::integral_constant<int, 1>{});
        bar();
        readB1(b, 1);
        readA1(b, 0, 1);
        lgkm0();
        bar();
        mma1(std::integral_constant<int, 0>{});
        bar();
        readA1(b, 1, 1);
        if (q + 2 < Q) {
            stageB(q & 1, cB);
            advance(cB);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NB) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        bar();
        mma1(std::integral_constant<int, 1>{});
        bar();
        const Cur st = cM;
        advance(cM);
        if (st.k + 1 != st.ke) continue;
        // ---- segment end: both wave groups in step, then the tile's contribution or finish
        if (wr == 0) bar();
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");   // XDL → VALU / store reads of acc
        if (contrib && st.sg == 0) {
            // fp32 partial → this block's slot (write-through), every storing wave drained,
            // then one lane publishes the flag
            float *p = slot(blk);
            // one base pointer per row group (4 fragments, 4 KiB), immediate offsets within
            // (explicit capture: hipcc does not see an implicit capture used only in asm operands)
            sk_for<0, SM>([p](auto IC) __attribute__((always_inline)) {
                constexpr int i = decltype(IC)::value;
                const f32x4 v0 = sk_acc<16 * i>(), v1 = sk_acc<16 * i + 4>(), v2 = sk_acc<16 * i + 8>(),
                            v3 = sk_acc<16 * i + 12>();
                asm volatile("global_store_dwordx4 %0, %1, off sc1\n\t"
                             "global_store_dwordx4 %0, %2, off offset:1024 sc1\n\t"
                             "global_store_dwordx4 %0, %3, off offset:2048 sc1\n\t"
                             "global_store_dwordx4 %0, %4, off offset:3072 sc1"
                             ::"v"(p + i * 4 * 64 * 4), "v"(v0), "v"(v1), "v"(v2), "v"(v3) : "memory");
            });
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(sk.flag + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const int64_t t = st.t;
            const bool fix = t == tf0 && f_kb > 0;
            if (fix) {
                // the tile's first f_kb K-tiles are block blk − 1's contribution (the host
                // admits only splits with one contributor per tile, sk_split_ok)
                if (tid == 0) {
                    int spins = 0;
                    while (__hip_atomic_load(sk.flag + blk - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1 &&
                           ++spins < (1 << 22))
                        __builtin_amdgcn_s_sleep(2);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __syncthreads();
            }
            // epilogue one row group at a time (the fragments read out of the AGPRs, the
            // contributor's partial added first)
            int tm, tn;
            tile_mn((int)t, tm, tn);
            const int row0 = tm * BM + arow, col0 = tn * BN + wc * 64;
            const int ln = lane_l(), frl = ln & 15, fcl = ln >> 4;
            const float *pp = sk.part + ((int64_t)(blk - 1) * 512 * 32 + (int64_t)(wave * 32) * 64 + ln) * 4;
            sk_for<0, SM>([&](auto IC) __attribute__((always_inline)) {
                constexpr int i = decltype(IC)::value;
                f32x4 c[1][4] = {{sk_acc<16 * i>(), sk_acc<16 * i + 4>(), sk_acc<16 * i + 8>(), sk_acc<16 * i + 12>()}};
                if (fix) {
                    const float *pi = pp + i * 4 * 64 * 4;
                    asm volatile("" : "+v"(pi));   // rebuilt here, not hoisted out of the main loop
#pragma unroll
                    for (int j = 0; j < 4; ++j) c[0][j] += *(const f32x4 *)(pi + j * 64 * 4);
                }
                epilogue_tile<1, 4, EPI, 2>(a, c, row0 + 16 * i, col0, frl, fcl);
            });
            if (fix) {
                __syncthreads();   // every wave read the partial before the slot is released
                if (tid == 0) __hip_atomic_store(sk.flag + blk - 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        acc_zero();
        if (wr == 1) bar();   // group 1 one barrier behind again
    }
    if (wr == 0) bar();   // balance the barrier count
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
        case EPI_HEADPOST:
            if constexpr (BM == 192 || BM == 128) {
                gemm_pp_kernel<BM, EPI_HEADPOST><<<tiles, 512, 0, s>>>(a);
                break;
            }
            return fail(-1, "gemm: head-post epilogue needs the 192- or 128-row ping-pong tile");
        default: return fail(-1, "gemm: bad epilogue");
    }
    HIP_TRY(hipGetLastError());
    return 0;
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
        case EPI_SWIGLU: klaunch(gemm_kernel<BM, BN, WM, WN, STAGES, EPI_SWIGLU>, dim3(tiles), dim3(NT), s, a); break;
        default: return fail(-1, "gemm: bad epilogue for this variant");
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
        case 7: return launch_pp<256>(a, s);              // ping-pong 256x256 (128 KiB)
        case 8: return launch_pp<192>(a, s);              // ping-pong 192x256 (112 KiB)
        case 9: return launch<192, 256, 2, 2, 2>(a, s);   // 4 waves (1/SIMD), 96x128 wave tile, acc in AGPRs
        case 10: return launch<256, 256, 2, 2, 2>(a, s);  // 4 waves (1/SIMD), 128x128 wave tile
        case 11: return launch_w4<192>(a, s);             // 4 waves, 96x128 wave tile, pipelined fragments
        case 12: return launch_pp<128>(a, s);             // ping-pong 128x256 (96 KiB), 64x64 wave tiles
        case 13: return launch_w4<192, 128>(a, s);        // 4 waves, 96x64 wave tile (M≈3000 shapes: 1 round)
        // small-M A/B (tools/bench_small_m.py): narrow-N tiles so a whole-K grid reaches the chip
        case 15: return launch<128, 64, 4, 1, 3>(a, s);   // 4 waves × 32 rows × 64 columns, 3-stage (72 KiB)
        case 16: return launch<128, 64, 4, 1, 4>(a, s);   // same, 4-stage (96 KiB)
        case 17: return launch<128, 64, 2, 1, 3>(a, s);   // 2 waves × 64 rows × 64 columns, 3-stage
        case 20: case 21: case 22: case 23: case 24: case 25: case 26: case 27: case 28: case 29: case 30: {
            // diagnostics / A/B: pp store, see gemm_pp_kernel DBG and SPL
            if (a.N % 256 || a.epi != EPI_STORE) return fail(-1, "gemm: diagnostic variant");
            const int tiles = ((a.M + 255) / 256) * (a.N / 256), t192 = ((a.M + 191) / 192) * (a.N / 256);
            if (variant == 20) gemm_pp_kernel<256, EPI_STORE, 1><<<tiles, 512, 0, s>>>(a);
            else if (variant == 21) gemm_pp_kernel<256, EPI_STORE, 2><<<tiles, 512, 0, s>>>(a);
            else if (variant == 22) gemm_pp_kernel<256, EPI_STORE, 3><<<tiles, 512, 0, s>>>(a);
            else if (variant == 23) gemm_pp_kernel<256, EPI_STORE, 0, 0><<<tiles, 512, 0, s>>>(a);
            else if (variant == 24) gemm_pp_kernel<256, EPI_STORE, 0, 2><<<tiles, 512, 0, s>>>(a);
            else if (variant == 25) gemm_pp_kernel<192, EPI_STORE, 0, 1><<<t192, 512, 0, s>>>(a);
            else if (variant == 27) gemm_pp_kernel<256, EPI_STORE, 0, 3><<<tiles, 512, 0, s>>>(a);
            else if (variant == 29) gemm_w4_kernel<192, 256, EPI_STORE, 1><<<t192, 256, 0, s>>>(a);
            else if (variant == 30) gemm_w4_kernel<192, 256, EPI_STORE, 0, 1><<<t192, 256, 0, s>>>(a);
            else if (variant == 28) gemm_pp_kernel<192, EPI_STORE, 0, 3, 1><<<t192, 512, 0, s>>>(a);
            else gemm_pp_kernel<192, EPI_STORE, 0, 2, 1><<<t192, 512, 0, s>>>(a);
            HIP_TRY(hipGetLastError());
            return 0;
        }
        default: return fail(-1, "gemm: bad variant");
    }
}

bool gemm_ext_events(hipEvent_t start, hipEvent_t stop) {
    const bool consumed = g_ext_ev.stop && !g_ext_ev.start;
    g_ext_ev.start = start;
    g_ext_ev.stop = stop;
    return consumed;
}

static int g_variant_override = -1;
void gemm_set_variant(int v) { g_variant_override = v; }

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

// Tile choice from a one-block-per-CU cost model fitted on MI355X
// (tools/bench_gemm.py): time ∝ ⌈tiles / CUs⌉ × per-tile time, with a 256×256
// ping-pong tile costing 1.093× a 192×256 one (it does 1.33× the work).  The
// model reproduces the measured v7/v8 ratios on all four DiT shapes to 2 %.
// Grids that fill at most half the chip fall back to 128×128 (2 blocks/CU): at
// M = 3000, N = 2048 (the cross-O GEMM of the conditional rows) 37 µs vs 46 µs.
// ACEHIP_GEMM_W4=1 runs the 192×256 tile as the four-wave pipelined kernel (variant 11)
// instead of the ping-pong one.  In isolation (store epilogue) it is 0.92–0.98× the
// ping-pong time; inside the DiT (cold weights, residual / head-post epilogues at one
// wave per SIMD) it is 1.05–1.17× (r02 A/B: 0.581 vs 0.562 s/song), so it is off.
static bool use_w4() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("ACEHIP_GEMM_W4");
        v = (e && e[0] == '1') ? 1 : 0;
    }
    return v == 1;
}

// Half-chip grids (M ≈ 3000: the conditional rows' cross-Q / cross-O): the four-wave
// 192×128 tile with a 3-deep ring fills the chip in one round (16 × 16 tiles at
// N = 2048) where the 128² tile runs 0.75 of a 2-blocks-per-CU round: 34–35 → 31 µs,
// hot or cold weights (tools/bench_gemm.py, r02).  ACEHIP_GEMM_W4S=0 disables it.
static bool use_w4s(int64_t M, int N) {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("ACEHIP_GEMM_W4S");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    if (v != 1 || N % 128) return false;
    const int cus = num_cus();
    const int64_t t = ((M + 191) / 192) * (N / 128);
    return t <= cus && t * 4 >= (int64_t)cus * 3;
}

int gemm_pick_variant(int64_t M, int N) {
    if (use_w4s(M, N) && (N % 256 || ((M + 191) / 192) * (N / 256) <= num_cus() / 2)) return 13;
    if (N % 256) return 0;
    const int cus = num_cus();
    const int64_t t7 = ((M + 255) / 256) * (N / 256), t8 = ((M + 191) / 192) * (N / 256);
    if (t8 <= cus / 2) return 0;
    const double c7 = (double)((t7 + cus - 1) / cus) * 1.093, c8 = (double)((t8 + cus - 1) / cus);
    if (use_w4()) return c7 < c8 * W4_COST ? 7 : 11;
    return c7 < c8 ? 7 : 8;
}

// Split-K for grids that cannot fill half the chip even with 128×128 tiles (short
// songs / turbo: M = Bc·S of a few hundred rows): the K range is split so the grid
// reaches ~1 block per CU, every split stores fp32 partials, and one launch sums
// them in order and applies the epilogue (the head-post case then runs the
// standalone head_post kernel on the staged bf16 projection).
// A/B knobs of the split-K path: ACEHIP_SPLITK_STAGES (2 | 3-stage LDS ring),
// ACEHIP_SPLITK_FILL (target blocks per CU)
// Default (tools/ab_splitk.py, M = 125): the 3-stage ring for N <= 4096 (down / QKV / O:
// 20.1 → 19.0, 18.3 → 17.4, 15.1 → 14.9 µs), 2 stages for the wide SwiGLU (26.2 vs 28.3 µs)
static int splitk_stages(int N) {
    const char *e = getenv("ACEHIP_SPLITK_STAGES");
    return e ? atoi(e) : (N <= 4096 ? 3 : 2);
}
static int splitk_min_ktiles() {   // fewest K-tiles per split (ACEHIP_SPLITK_MINK, A/B; read per call)
    const char *e = getenv("ACEHIP_SPLITK_MINK");
    return e ? std::max(1, atoi(e)) : 4;
}
static int splitk_fill() {
    const char *e = getenv("ACEHIP_SPLITK_FILL");
    return e ? std::max(1, atoi(e)) : 1;
}

static int splitk_finish(const GemmArgs &a, const GemmArgs &p, int splits, hipStream_t s);
// the split-K epilogue folded into its consumer (head_post for EPI_HEADPOST; the next
// rmsnorm_mod for the residual epilogues, gemm(..., defer)): ACEHIP_SPLITK_FUSE=0 keeps
// the separate splitk_epilogue_kernel launch (A/B); read per call
static bool splitk_fuse_on() {
    const char *e = getenv("ACEHIP_SPLITK_FUSE");
    return !(e && e[0] == '0');
}
static bool splitk_hp_fused() { return splitk_fuse_on(); }

// Skinny path (M ≤ 256, K % 128 == 0, N % 64 == 0): skinny_kernel<8, 4> over
// ⌈M/128⌉ row chunks × N/64 slabs × `splits` K-ranges, splits chosen so the grid is
// about one block per CU (K-steps per wave ≥ 2), then the split-K epilogue.
// Measured (tools/bench_skinny.py, cold weights, M = 16 / 64 / 125 / 250, one process):
// no faster than the 128×128 split-K path — SwiGLU at M = 125 34 vs 26 µs, down 21 vs 20,
// QKV 17 vs 18, O 16 vs 16; even W-only streaming (M = 16) reaches 2.4 TB/s against
// split-K's 2.9, and every shape carries a ~10 µs floor (two launches, the cold-weight
// first touch) — so it is off by default; ACEHIP_SKINNY=1 selects it (A/B).
static bool use_skinny() {   // read per call (in-process A/B)
    const char *e = getenv("ACEHIP_SKINNY");
    return e && e[0] == '1';
}
static int skinny_depth() {   // register-ring depth (A/B knob ACEHIP_SKINNY_D = 2 | 3 | 4; read per call)
    const char *e = getenv("ACEHIP_SKINNY_D");
    return e ? atoi(e) : 3;
}
static void fill_defer(const GemmArgs &a, int splits, RowAdd *defer);
static int gemm_skinny(const GemmArgs &a, hipStream_t s, int depth = 0, RowAdd *defer = nullptr) {
    constexpr int MT = 8, NT = 4, BN = 16 * NT;
    if (!depth) depth = skinny_depth();
    const int cus = num_cus();
    const int nchunk = (a.M + 16 * MT - 1) / (16 * MT);
    const int slabs = a.N / BN, nk = a.K / 128;         // K in units of 4 waves × 32
    int splits = std::max(1, (int)((cus + slabs * nchunk / 2) / (slabs * nchunk)));
    splits = std::min(splits, std::max(1, nk / 2));
    const int kper = ((nk + splits - 1) / splits) * 128;
    splits = (a.K + kper - 1) / kper;
    const size_t need = (size_t)splits * a.M * a.N * 4 + (a.epi == EPI_HEADPOST ? (size_t)a.M * a.N * 2 : 0);
    if (need > a.ws_bytes) return 1;
    if (depth == 4) skinny_kernel<MT, NT, 4><<<slabs * splits * nchunk, 256, 0, s>>>(a, kper, splits, nchunk);
    else if (depth == 2) skinny_kernel<MT, NT, 2><<<slabs * splits * nchunk, 256, 0, s>>>(a, kper, splits, nchunk);
    else skinny_kernel<MT, NT, 3><<<slabs * splits * nchunk, 256, 0, s>>>(a, kper, splits, nchunk);
    HIP_TRY(hipGetLastError());
    if (defer) {
        fill_defer(a, splits, defer);
        return 0;
    }
    return splitk_finish(a, a, splits, s);
}

// split-K tile width: 64-column tiles double the grid at a given split count (half the splits
// and partial bytes for ~1 block per CU).  Measured at M = 125, cold weights, one process
// (tools/bench_small_m.py, profiles/r03_small_m.log): down (N 2048, K 6144) 19.9 → 17.9 µs,
// QKV (N 4096, K 2048) 18.8 → 17.2, but O (N 2048, K 2048: 4 K-tiles per split) 18.7 → 25.3 —
// so 64 where N or K ≥ 4096.  ACEHIP_SPLITK_BN = 128 | 64 forces one (A/B; read per call)
static int splitk_bn(const GemmArgs &a) {
    const char *e = getenv("ACEHIP_SPLITK_BN");
    if (e) return atoi(e) == 64 ? 64 : 128;
    return (a.N >= 4096 || a.K >= 4096) ? 64 : 128;
}
static int gemm_splitk(const GemmArgs &a, int splits, hipStream_t s, RowAdd *defer = nullptr) {
    GemmArgs p = a;
    const int nk = a.K / BK;
    p.kper = (nk + splits - 1) / splits;
    splits = (nk + p.kper - 1) / p.kper;
    const int bn = splitk_bn(a);
    const int tiles = ((a.M + 127) / 128) * (a.N / bn);
    if (bn == 64) gemm_kernel<128, 64, 4, 1, 3, EPI_PARTIAL><<<dim3(tiles, splits), 256, 0, s>>>(p);
    else if (splitk_stages(a.N) == 3) gemm_kernel<128, 128, 2, 2, 3, EPI_PARTIAL><<<dim3(tiles, splits), 256, 0, s>>>(p);
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
// projection + the standalone head_post kernel)
static int splitk_finish(const GemmArgs &a, const GemmArgs &p, int splits, hipStream_t s) {
    if (a.epi == EPI_HEADPOST && splitk_hp_fused()) {
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
// ACEHIP_GEMM_TAILSPLIT=0 disables it, =<digit> picks the tail variant (A/B).  Returns 1 when not applicable.
static int gemm_tail_split(const GemmArgs &a, int v, hipStream_t s) {
    if (a.epi != EPI_SWIGLU && a.epi != EPI_STORE) return 1;
    const char *e = getenv("ACEHIP_GEMM_TAILSPLIT");
    if (e && e[0] == '0') return 1;
    const int BMv = v == 7 ? 256 : 192, cus = num_cus();   // v = 7, 8 or 11
    const int64_t nN = a.N / 256, tiles = (int64_t)((a.M + BMv - 1) / BMv) * nN;
    const int64_t full = tiles / cus, rem = tiles - full * cus;
    if (full < 1 || rem == 0 || rem * 5 > (int64_t)cus * 3) return 1;   // last round > 60 % full
    const int64_t M1 = (full * cus / nN) * BMv;
    if (M1 <= 0 || M1 >= a.M) return 1;
    const int tv = (e && e[0] >= '2' && e[0] <= '9') ? e[0] - '0' : 0;   // tail variant (A/B)
    const int64_t tail_bn = (tv == 3 || tv == 5 || tv == 6) ? 256 : 128;
    if (((a.M - M1 + 127) / 128) * (a.N / tail_bn) > 2 * (int64_t)cus) return 1;
    GemmArgs hd = a;
    hd.M = (int)M1;
    int rc = gemm_variant(hd, v, s);
    if (rc) return rc;
    GemmArgs tl = a;
    tl.M = a.M - (int)M1;
    tl.A = a.A + M1 * a.lda;
    tl.C = a.C + M1 * a.ldc;
    return gemm_variant(tl, tv, s);
}

// Stream-K dispatch of the 256×256 ping-pong tile (gemm_sk_kernel): needs the handle's
// stream-K workspace (a.sk_part / a.sk_flag) and N % 256 == 0, epilogues that work on one
// finished tile in registers (store, residual, gated residual, SwiGLU).
// ACEHIP_GEMM_SK: 0 off (default), 1 on where the cost model prefers it, 2 forced (A/B).
// Measured (cold weights, µs, tools/bench_gemm.py; v11 = the 192/256 tail-split path):
//   eq_k6144 8192×2048×6144 (256 tiles, no hand-off)  v7 149.4  v14 156.6
//   down  v11 130.7  v14 138.6     qkv  v11 94.8  v14 98.9     o  v11 47.5  v14 59.6
//   swiglu  v11 287.4  v14 302.1 (290.6 vs 300.3 on another box)
// i.e. ~5 % main-loop cost for the cursor bookkeeping + ~20 µs of partial hand-off on
// down (256 KB fp32 per contributor written, then re-read by a latency-bound
// chunked epilogue) — it loses everywhere, so it stays an A/B variant (14).
static int sk_mode() {   // read per call: in-process A/B (tools/ab_env_song.py)
    const char *e = getenv("ACEHIP_GEMM_SK");
    return e ? atoi(e) : 0;
}
// every tile split between at most two blocks (one contributor: the kernel's fixup reads
// block blk − 1 only) and no block range strictly inside one tile
static bool sk_split_ok(int64_t tiles, int nk, int G) {
    const int64_t I = tiles * nk;
    for (int b = 0; b < G; ++b) {
        const int64_t s0 = (int64_t)b * I / G, e0 = (int64_t)(b + 1) * I / G;
        if (e0 <= s0) return false;
        if (s0 % nk && s0 / nk == (e0 - 1) / nk && e0 % nk) return false;     // middle part
        if (s0 % nk && b > 0 && (int64_t)(b - 1) * I / G > (s0 / nk) * nk) return false;   // 2+ contributors
    }
    return true;
}
static int gemm_sk(const GemmArgs &a, hipStream_t s) {
    SkArgs sk{};
    sk.part = a.sk_part;
    sk.flag = a.sk_flag;
    sk.G = std::min(num_cus(), SK_MAX_BLOCKS);
    sk.ktiles = a.K / BK;
    if (!sk_split_ok((int64_t)((a.M + 255) / 256) * (a.N / 256), sk.ktiles, sk.G))
        return fail(-1, "gemm_sk: split with more than one contributor per tile");
    switch (a.epi) {
        case EPI_STORE: gemm_sk_kernel<EPI_STORE><<<sk.G, 512, 0, s>>>(a, sk); break;
        case EPI_GATED_RES: gemm_sk_kernel<EPI_GATED_RES><<<sk.G, 512, 0, s>>>(a, sk); break;
        case EPI_RES: gemm_sk_kernel<EPI_RES><<<sk.G, 512, 0, s>>>(a, sk); break;
        case EPI_SWIGLU: gemm_sk_kernel<EPI_SWIGLU><<<sk.G, 512, 0, s>>>(a, sk); break;
        default: return fail(-1, "gemm_sk: epilogue");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}
int gemm_sk_forced(const GemmArgs &a, hipStream_t s) {
    if (!a.sk_part || !a.sk_flag || a.N % 256 || a.K % BK || a.K < 4 * BK) return fail(-1, "gemm_sk: shape / workspace");
    return gemm_sk(a, s);
}
// stream-K time in 192×256-tile rounds (cost model of gemm_pick_variant: a 256² tile =
// 1.093 of a 192×256 one) + the partial hand-off, vs the chosen variant's rounds
static bool prefer_sk(const GemmArgs &a, int v) {
    const int m = sk_mode();
    if (m == 0 || !a.sk_part || !a.sk_flag || a.N % 256 || a.K < 4 * BK) return false;
    if (a.epi != EPI_STORE && a.epi != EPI_GATED_RES && a.epi != EPI_RES && a.epi != EPI_SWIGLU) return false;
    const int cus = num_cus();
    if (!sk_split_ok((int64_t)((a.M + 255) / 256) * (a.N / 256), a.K / BK, std::min(cus, SK_MAX_BLOCKS))) return false;
    if (m == 2) return true;
    const int64_t t7 = ((a.M + 255) / 256) * (a.N / 256), t8 = ((a.M + 191) / 192) * (a.N / 256);
    if (t7 < cus / 2) return false;
    const double sk = (double)t7 * 1.093 / cus + 0.06;
    const double cur = v == 7 ? (double)((t7 + cus - 1) / cus) * 1.093 : (double)((t8 + cus - 1) / cus);
    return sk < cur * 0.97;
}

// small-M A/B entry (tools/bench_skinny.py): mode 2..4 = the skinny kernel at that ring
// depth, 0 = the 128×128 split-K path; needs a.ws
int gemm_small(const GemmArgs &a, int mode, hipStream_t s) {
    if (!a.ws || a.M > 256 || a.N % 64 || a.K % 128) return fail(-1, "gemm_small: shape / workspace");
    if (mode >= 2 && mode <= 4) {
        const int rc = gemm_skinny(a, s, mode);
        return rc == 1 ? fail(-1, "gemm_small: workspace too small") : rc;
    }
    const int cus = num_cus();
    const int64_t tiles = ((a.M + 127) / 128) * (a.N / 128);
    const int nk = a.K / BK;
    const int splits = (int)std::max<int64_t>(2, std::min<int64_t>(std::min<int64_t>(16, nk / 4),
                                                                   (splitk_fill() * cus + tiles - 1) / tiles));
    return gemm_splitk(a, splits, s);
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
    // a deferred epilogue needs the in-place residual form the consumer norm applies
    const bool dfr = defer && splitk_fuse_on() && (a.epi == EPI_GATED_RES || a.epi == EPI_RES) && a.res == a.C &&
                     a.ldr == a.ldc && a.ldc == a.N;
    if (a.ws && a.M <= 256 && a.N % 64 == 0 && a.K % 128 == 0 && a.K >= 512 && use_skinny() &&
        (a.epi != EPI_SWIGLU || a.N % 64 == 0)) {
        const int rc = gemm_skinny(a, s, 0, dfr ? defer : nullptr);
        if (rc <= 0) return rc;   // done (0) or failed (< 0); 1 = workspace too small
    }
    // SwiGLU of one 128-row chunk (turbo / short songs, M ≤ 128): whole-K 128×64 tiles with the
    // SwiGLU epilogue fused (variant 16: no fp32 partials, no second launch) — M = 125, cold
    // weights: 26.1 → 19.0 µs (tools/bench_small_m.py).  ACEHIP_SMALLM_WHOLEK=0: split-K (A/B)
    if (a.epi == EPI_SWIGLU && a.M <= 128 && a.N % 64 == 0 && g_variant_override < 0) {
        const char *e = getenv("ACEHIP_SMALLM_WHOLEK");
        if (!(e && e[0] == '0')) return gemm_variant(a, 16, s);
    }
    if (a.ws && a.N % 128 == 0 && a.K % BK == 0 && (a.N % 256 == 0 || a.epi != EPI_HEADPOST)) {
        const int cus = num_cus();
        const int64_t tiles = ((a.M + 127) / 128) * (a.N / 128);
        const int nk = a.K / BK;
        if (tiles * 2 <= cus && nk >= 8) {
            const int64_t tb = ((a.M + 127) / 128) * (a.N / splitk_bn(a));   // grid tiles of the split kernel
            int splits = (int)std::min<int64_t>(std::min<int64_t>(16, nk / splitk_min_ktiles()),
                                                (splitk_fill() * cus + tb - 1) / tb);
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
        const char *e = getenv("ACEHIP_GEMM_HP128");
        const bool small = t192 * 2 <= num_cus() && !(e && e[0] == '0');
        if (small && use_w4s(a.M, a.N) && !(e && e[0] == '2')) return launch_w4<192, 128>(a, s);
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
        return use_w4() ? launch_w4<192>(a, s) : launch_pp<192>(a, s);
    }
    int v = g_variant_override;
    if (v < 0) {
        v = gemm_pick_variant(a.M, a.N);
        if ((v == 7 || v == 8 || v == 11) && prefer_sk(a, v)) return gemm_sk(a, s);
        if (v == 7 || v == 8 || v == 11) {
            const int rc = gemm_tail_split(a, v, s);
            if (rc <= 0) return rc;   // split done (0) or failed (< 0); 1 = not applicable
        }
    }
    if ((v == 3 || (v >= 5 && v != 13)) && a.N % 256) v = 0;   // (13 needs N % 128 only)
    return gemm_variant(a, v, s);
}

}  // namespace acehip
