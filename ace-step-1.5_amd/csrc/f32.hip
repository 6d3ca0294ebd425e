// f32.hip — the fp32 parity mode of the DiT forward (an fp32
// build vs the reference's fp32 forward, rel-L2 <= 1e-4).  The reference runs in
// fp32 whenever the device is not cuda/xpu (init_service_orchestrator.py:51), so
// this is the arithmetic of AceStepDiTModel.forward (base:1303-1507) with no bf16
// rounding anywhere: fp32 weights, fp32 activations, fp32 accumulation.
//
// It is a parity mode, not the production path: kernels are simple and exact
// rather than tuned.  The GEMM and attention still run on the matrix cores —
// v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate, exact fp32 FMA chains; the
// 157 TF fp32 peak of MI355X) — everything else is VALU.
//
// MFMA 16x16x4 f32 operand maps (cdna_hip_programming.md): lane l holds
// A[l & 15][k = l >> 4], B[k = l >> 4][l & 15]; the accumulator D[(l >> 4)·4 + r][l & 15].
#include "kernels.h"

namespace acehip {
namespace {

__device__ __forceinline__ float silu_exact(float x) { return x / (1.0f + expf(-x)); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// C[M,N] = A[M,K] · W[N,K]ᵀ with epilogue (see gemm_f32 in kernels.h).
// 64x64 tile, BK 16, 4 waves (2x2) of 32x32, each 2x2 MFMA tiles.
constexpr int FB = 64, FK = 16, FP = FK + 1;   // LDS rows padded: conflict-free column reads
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32Args a) {
    __shared__ float As[FB][FP], Ws[FB][FP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tilesN = (a.N + FB - 1) / FB;
    const int64_t m0 = (int64_t)(blockIdx.x / tilesN) * FB;
    const int n0 = (blockIdx.x % tilesN) * FB;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int lr = tid >> 2, lc = (tid & 3) * 4;     // loader: row 0..63, 4 columns
    for (int k0 = 0; k0 < a.K; k0 += FK) {
        const int64_t am = m0 + lr;
        const int wnr = n0 + lr;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int k = k0 + lc + c;
            As[lr][lc + c] = (am < a.M && k < a.K) ? a.A[am * a.lda + k] : 0.f;
            Ws[lr][lc + c] = (wnr < a.N && k < a.K) ? a.W[(int64_t)wnr * a.ldw + k] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < FK; ks += 4) {
            const int kk = ks + (lane >> 4);
            float av[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) av[i] = As[wm * 32 + i * 16 + (lane & 15)][kk];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = Ws[wn * 32 + j * 16 + (lane & 15)][kk];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
                const int n = n0 + wn * 32 + j * 16 + (lane & 15);
                if (m >= a.M || n >= a.N) continue;
                float v = acc[i][j][r];
                if (a.bias) v += a.bias[n];
                if (a.epi == EPI_GATED_RES) {
                    const int64_t b = m / a.rows_per_batch;
                    v = a.res[m * a.ldr + n] + v * a.gate[b * a.gate_bstride + n];
                } else if (a.epi == EPI_RES) {
                    v = a.res[m * a.ldr + n] + v;
                }
                a.C[m * a.ldc + n] = v;
            }
}

// Qwen3RMSNorm (+ AdaLN): fp32 all the way (modeling_qwen3.py:59-64; base:499,530,1496)
__global__ __launch_bounds__(256) void rmsnorm_f32_kernel(const float *x, const float *w, const float *shift,
                                                          const float *scale, int64_t mod_bstride,
                                                          int rows_per_batch, float *out, int M, int D, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const float *xr = x + (int64_t)row * D;
    float ss = 0.f;
    for (int d = lane; d < D; d += 64) ss += xr[d] * xr[d];
    ss = wave_sum(ss);
    const float r = rsqrtf(ss / (float)D + eps);
    const int64_t b = row / rows_per_batch;
    for (int d = lane; d < D; d += 64) {
        float v = w[d] * (xr[d] * r);
        if (scale) v = v * (1.0f + scale[b * mod_bstride + d]) + shift[b * mod_bstride + d];
        out[(int64_t)row * D + d] = v;
    }
}

// per (row, head): q/k RMSNorm (weight after the norm) + rotate-half RoPE + head-major
// scatter; v heads copied (base:300-345)
__global__ __launch_bounds__(256) void head_post_f32_kernel(HeadPostF32Args a) {
    const int nh = a.nq + a.nk + a.nv;
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (item >= (int64_t)a.B * a.S * nh) return;
    const int64_t row = item / nh;
    const int h = (int)(item % nh);
    const int b = (int)(row / a.S), s = (int)(row % a.S);
    const float *src = a.src + row * a.ld_src + (int64_t)h * 128;
    float x0 = src[lane], x1 = src[lane + 64];
    float *dst;
    const float *w = nullptr;
    if (h < a.nq) {
        dst = a.q + (((int64_t)b * a.nq + h) * a.S_dst + s) * 128;
        w = a.qw;
    } else if (h < a.nq + a.nk) {
        dst = a.k + (((int64_t)b * a.nk + (h - a.nq)) * a.S_dst + s) * 128;
        w = a.kw;
    } else {
        dst = a.v + (((int64_t)b * a.nv + (h - a.nq - a.nk)) * a.S_dst + s) * 128;
    }
    if (w) {
        const float r = rsqrtf(wave_sum(x0 * x0 + x1 * x1) / 128.0f + a.eps);
        x0 = w[lane] * (x0 * r);
        x1 = w[lane + 64] * (x1 * r);
        if (a.cos) {
            const float c0 = a.cos[(int64_t)s * 128 + lane], c1 = a.cos[(int64_t)s * 128 + lane + 64];
            const float s0 = a.sin[(int64_t)s * 128 + lane], s1 = a.sin[(int64_t)s * 128 + lane + 64];
            const float y0 = x0 * c0 + (-x1) * s0;     // rotate_half: [-x[64:], x[:64]]
            const float y1 = x1 * c1 + x0 * s1;
            x0 = y0;
            x1 = y1;
        }
    }
    dst[lane] = x0;
    dst[lane + 64] = x1;
}

// softmax(Q·Kᵀ·scale + band mask)·V, fp32, GQA.  Block = 64 queries of one (b, h):
// 4 waves × 16 query rows; key tiles of 32 staged in LDS; S and O accumulate in
// the same MFMA D layout (row (l>>4)·4 + r), so the online-softmax statistics of a
// row live in the lanes that hold that row of O.  P goes through LDS to become the
// A operand of P·V.
__global__ __launch_bounds__(256) void attention_f32_kernel(AttnF32Args a) {
    __shared__ float Ks[32][129], Vs[32][129], Ps[4][16][33];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qblocks = (a.Sq + 63) / 64;
    const int qb = blockIdx.x % qblocks;
    const int bh = blockIdx.x / qblocks;
    const int b = bh / a.H, h = bh % a.H, kvh = h / (a.H / a.KV);
    const int q0 = qb * 64 + wave * 16;
    const float *Q = a.q + ((int64_t)(b * a.H + h) * a.Sq) * 128;
    const float *K = a.k + ((int64_t)(b * a.KV + kvh) * a.Sk) * 128;
    const float *V = a.v + ((int64_t)(b * a.KV + kvh) * a.Sk) * 128;
    // this lane's Q fragments: Q[q0 + (l & 15)][4·ks + (l >> 4)], 32 k-steps
    float qf[32];
    {
        const int qi = q0 + (lane & 15);
#pragma unroll
        for (int ks = 0; ks < 32; ++ks) qf[ks] = qi < a.Sq ? Q[(int64_t)qi * 128 + 4 * ks + (lane >> 4)] : 0.f;
    }
    f32x4 o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mrow[4], lrow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { mrow[r] = -INFINITY; lrow[r] = 0.f; }
    // key range of the whole block (band: skip tiles outside every row's band)
    int k_lo = 0, k_hi = a.Sk;
    if (a.window >= 0) {
        k_lo = max(0, qb * 64 - a.window);
        k_hi = min(a.Sk, qb * 64 + 64 + a.window);
    }
    k_lo &= ~31;
    for (int k0 = k_lo; k0 < k_hi; k0 += 32) {
        __syncthreads();
        for (int e = tid; e < 32 * 128; e += 256) {
            const int j = e >> 7, d = e & 127;
            const bool in = k0 + j < a.Sk;
            Ks[j][d] = in ? K[(int64_t)(k0 + j) * 128 + d] : 0.f;
            Vs[j][d] = in ? V[(int64_t)(k0 + j) * 128 + d] : 0.f;
        }
        __syncthreads();
        f32x4 sc[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            sc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 32; ++ks)
                sc[kt] = mfma4(qf[ks], Ks[kt * 16 + (lane & 15)][4 * ks + (lane >> 4)], sc[kt]);
        }
        // scale + mask; this lane: rows q0 + (l>>4)·4 + r, keys k0 + 16·kt + (l & 15)
        float tmax[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int qi = q0 + (lane >> 4) * 4 + r;
            tmax[r] = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                const int kj = k0 + kt * 16 + (lane & 15);
                bool ok = kj < a.Sk;
                if (a.window >= 0) ok = ok && abs(qi - kj) <= a.window;
                const float v = ok ? sc[kt][r] * a.scale : -INFINITY;
                sc[kt][r] = v;
                tmax[r] = fmaxf(tmax[r], v);
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) tmax[r] = fmaxf(tmax[r], __shfl_xor(tmax[r], off, 64));
        }
        float alpha[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float mn = fmaxf(mrow[r], tmax[r]);
            alpha[r] = mn == -INFINITY ? 1.f : expf(mrow[r] - mn);
            float psum = 0.f;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                const float p = mn == -INFINITY ? 0.f : expf(sc[kt][r] - mn);
                psum += p;
                Ps[wave][(lane >> 4) * 4 + r][kt * 16 + (lane & 15)] = p;
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) psum += __shfl_xor(psum, off, 64);
            lrow[r] = lrow[r] * alpha[r] + psum;
            mrow[r] = mn;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[t][r] *= alpha[r];
        __builtin_amdgcn_s_barrier();   // Ps of this wave written (wave-local, but keep LDS ordered)
        // O[16 q][128] += P[16][32] · V[32][128]
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const float pa = Ps[wave][lane & 15][4 * ks + (lane >> 4)];
#pragma unroll
            for (int t = 0; t < 8; ++t) o[t] = mfma4(pa, Vs[4 * ks + (lane >> 4)][t * 16 + (lane & 15)], o[t]);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int qi = q0 + (lane >> 4) * 4 + r;
        if (qi >= a.Sq) continue;
        const float inv = 1.0f / lrow[r];
        float *orow = a.o + ((int64_t)b * a.Sq + qi) * a.o_ld + (int64_t)h * 128;
#pragma unroll
        for (int t = 0; t < 8; ++t) orow[t * 16 + (lane & 15)] = o[t][r] * inv;
    }
}

// y[m][n] = Σ_k act(x[m][k])·W[n][k] + b[n]; act 1 = silu (fp32)
__global__ __launch_bounds__(256) void gemv_f32_kernel(const float *x, int64_t ldx, const float *W, const float *bias,
                                                       float *y, int64_t ldy, int M, int N, int K, int act) {
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int m = blockIdx.y;
    if (n >= N) return;
    float acc = 0.f;
    for (int k = lane; k < K; k += 64) {
        const float xv = x[(int64_t)m * ldx + k];
        acc += W[(int64_t)n * K + k] * (act ? silu_exact(xv) : xv);
    }
    acc = wave_sum(acc);
    if (lane == 0) y[(int64_t)m * ldy + n] = acc + (bias ? bias[n] : 0.f);
}

__global__ void sinusoid_f32_kernel(const float *t, const float *t_r, int t_stride, int use_diff, const float *freqs,
                                    float *emb) {
    const int b = blockIdx.x, i = threadIdx.x;
    float tv = t[b * t_stride];
    if (use_diff) tv = tv - t_r[b * t_stride];
    const float arg = (tv * 1000.0f) * freqs[i];
    emb[b * 256 + i] = cosf(arg);
    emb[b * 256 + 128 + i] = sinf(arg);
}

__global__ void add_f32_kernel(const float *a, const float *b, float *o, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = a[i] + b[i];
}

// proj rows: 6 for the layer tables (proj [Bc][6][D]); 1 for norm_out (temb [Bc][D])
__global__ void modulation_f32_kernel(const float *tables, int rows, const float *proj, int proj_rows, int Bc, int D,
                                      float *mod) {
    const int l = blockIdx.z, b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)rows * D) return;
    const int j = (int)(e / D), d = (int)(e % D);
    mod[(((int64_t)l * Bc + b) * rows) * D + e] =
        tables[(int64_t)l * rows * D + e] + proj[((int64_t)b * proj_rows + (j % proj_rows)) * D + d];
}

__global__ void pack_patches_f32_kernel(const float *xt, const float *ctx, int Bx, int T, int S, float *X) {
    const int row = blockIdx.x;
    const int b = row / S, s = row % S, bb = b % Bx;
    for (int i = threadIdx.x; i < 384; i += blockDim.x) {
        const int k = i / 192, c = i % 192, t = 2 * s + k;
        float v = 0.f;
        if (t < T) v = c < 128 ? ctx[((int64_t)bb * T + t) * 128 + c] : xt[((int64_t)bb * T + t) * 64 + (c - 128)];
        X[(int64_t)row * 384 + i] = v;
    }
}

__global__ void crop_f32_kernel(const float *src, int rows_src, int rows_dst, int C, float *dst) {
    const int b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < (int64_t)rows_dst * C) dst[(int64_t)b * rows_dst * C + e] = src[(int64_t)b * rows_src * C + e];
}

__global__ void swiglu_f32_kernel(const float *g, const float *u, float *o, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = silu_exact(g[i]) * u[i];
}

inline unsigned blocks(int64_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

}  // namespace

int gemm_f32(const GemmF32Args &a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0 || a.K <= 0) return fail(-1, "gemm_f32: shape");
    if ((a.epi == EPI_GATED_RES && (!a.gate || !a.res || a.rows_per_batch <= 0)) || (a.epi == EPI_RES && !a.res))
        return fail(-1, "gemm_f32: epilogue operands");
    const int64_t tiles = (int64_t)((a.M + FB - 1) / FB) * ((a.N + FB - 1) / FB);
    gemm_f32_kernel<<<(unsigned)tiles, 256, 0, s>>>(a);
    HIP_TRY(hipGetLastError());
    return 0;
}

int rmsnorm_f32(const float *x, const float *w, const float *shift, const float *scale, int64_t mod_bstride,
                int rows_per_batch, float *out, int M, int D, float eps, hipStream_t s) {
    rmsnorm_f32_kernel<<<blocks(M, 4), 256, 0, s>>>(x, w, shift, scale, mod_bstride, rows_per_batch, out, M, D, eps);
    HIP_TRY(hipGetLastError());
    return 0;
}

int head_post_f32(const HeadPostF32Args &a, hipStream_t s) {
    const int64_t items = (int64_t)a.B * a.S * (a.nq + a.nk + a.nv);
    if (items <= 0) return 0;
    head_post_f32_kernel<<<blocks(items, 4), 256, 0, s>>>(a);
    HIP_TRY(hipGetLastError());
    return 0;
}

int attention_f32(const AttnF32Args &a, hipStream_t s) {
    if (a.H % a.KV) return fail(-1, "attention_f32: heads");
    const int64_t grid = (int64_t)a.B * a.H * ((a.Sq + 63) / 64);
    attention_f32_kernel<<<(unsigned)grid, 256, 0, s>>>(a);
    HIP_TRY(hipGetLastError());
    return 0;
}

int gemv_f32(const float *x, int64_t ldx, const float *W, const float *bias, float *y, int64_t ldy, int M, int N,
             int K, int act, hipStream_t s) {
    gemv_f32_kernel<<<dim3(blocks(N, 4), M), 256, 0, s>>>(x, ldx, W, bias, y, ldy, M, N, K, act);
    HIP_TRY(hipGetLastError());
    return 0;
}

int timestep_sinusoid_f32(const float *t, const float *t_r, int t_stride, int use_diff, int Bc, const float *freqs,
                          float *emb, hipStream_t s) {
    sinusoid_f32_kernel<<<Bc, 128, 0, s>>>(t, t_r, t_stride, use_diff, freqs, emb);
    HIP_TRY(hipGetLastError());
    return 0;
}

int add_f32(const float *a, const float *b, float *o, int64_t n, hipStream_t s) {
    add_f32_kernel<<<blocks(n), 256, 0, s>>>(a, b, o, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int modulation_f32(const float *tables, int n_tables, int rows, const float *proj, int Bc, int D, float *mod,
                   hipStream_t s) {
    const int proj_rows = rows == 6 ? 6 : 1;
    modulation_f32_kernel<<<dim3(blocks((int64_t)rows * D), Bc, n_tables), 256, 0, s>>>(tables, rows, proj, proj_rows,
                                                                                      Bc, D, mod);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pack_patches_f32(const float *xt, const float *ctx, int Bx, int Bc, int T, int S, float *X, hipStream_t s) {
    pack_patches_f32_kernel<<<Bc * S, 128, 0, s>>>(xt, ctx, Bx, T, S, X);
    HIP_TRY(hipGetLastError());
    return 0;
}

int crop_rows_f32(const float *src, int Bc, int rows_src, int rows_dst, int C, float *dst, hipStream_t s) {
    crop_f32_kernel<<<dim3(blocks((int64_t)rows_dst * C), Bc), 256, 0, s>>>(src, rows_src, rows_dst, C, dst);
    HIP_TRY(hipGetLastError());
    return 0;
}

int swiglu_f32(const float *g, const float *u, float *o, int64_t n, hipStream_t s) {
    swiglu_f32_kernel<<<blocks(n), 256, 0, s>>>(g, u, o, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
