// small.hip — the DiT's small / bandwidth-trivial kernels.
//
// timestep embedding (reference base:225-254): the sinusoid of bf16(t·1000)
// and the three tiny-M linears run as a weight-streaming GEMV (M = Bc ≤ 16);
// the per-layer AdaLN tables (base:493-495) are added once per forward for all
// layers; proj_in's concat+pad+patchify (base:1347-1358) becomes a gather
// into the K=384 GEMM operand; proj_out's crop (base:1501) a row copy.
#include "kernels.h"

namespace acehip {
namespace {

__global__ __launch_bounds__(256) void gemv_small_kernel(const bf16_t *__restrict__ x, int64_t ldx,
                                                         const bf16_t *__restrict__ W,
                                                         const bf16_t *__restrict__ bias,
                                                         bf16_t *__restrict__ y, int64_t ldy, int M,
                                                         int N, int K, int act) {
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (n >= N) return;
    float acc[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m] = 0.f;
    const bf16_t *wr = W + (int64_t)n * K;
    // the row's W chunks (K ≤ 2048: ≤ 4 per lane) are all issued before the first FMA: the
    // kernel is a latency chain per wave otherwise (one W round trip per 512 columns)
    uint4 wq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = lane * 8 + c * 512;
        if (k < K) wq[c] = *(const uint4 *)(wr + k);
    }
    for (int c = 0, k = lane * 8; k < K; ++c, k += 512) {
        float wv[8];
        unpack8(c < 4 ? wq[c & 3] : *(const uint4 *)(wr + k), wv);
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            if (m < M) {
                float xv[8];
                unpack8(*(const uint4 *)(x + m * ldx + k), xv);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float xx = act ? rbf(silu_f(xv[j])) : xv[j];
                    acc[m] += wv[j] * xx;
                }
            }
        }
    }
    const float bb = bias ? bf2f(bias[n]) : 0.f;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        if (m < M) {
            const float v = wave_sum(acc[m]);
            if (lane == 0) y[m * ldy + n] = f2bf(v + bb);
        }
    }
}

// y = bf16(silu(x)) for the M ≤ 16 rows of a timestep-MLP input, once (gemv_small's act
// operand; in-kernel it was recomputed for every output column: N·M·K transcendentals)
__global__ __launch_bounds__(256) void silu_rows_kernel(const bf16_t *__restrict__ x, int64_t ldx,
                                                        bf16_t *__restrict__ y, int64_t ldy, int K) {
    const int m = blockIdx.y, k = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (k >= K) return;
    float v[8];
    unpack8(*(const uint4 *)(x + m * ldx + k), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = silu_f(v[j]);
    *(uint4 *)(y + m * ldy + k) = pack8(v);
}

// dst row r (r = blockIdx.y) = src, 16 B per lane
__global__ __launch_bounds__(256) void bcast_rows_kernel(const bf16_t *__restrict__ src, int64_t n,
                                                         bf16_t *__restrict__ dst) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (i < n) *(uint4 *)(dst + blockIdx.y * n + i) = *(const uint4 *)(src + i);
}

__global__ void sinusoid_kernel(const float *t, const float *t_r, int t_stride, int use_diff,
                                const float *freqs, bf16_t *emb) {
    const int b = blockIdx.x, i = threadIdx.x;  // 128 threads
    float tv = t[b * t_stride];
    if (use_diff) tv = rbf(tv - t_r[b * t_stride]);   // (timestep - timestep_r) in bf16
    const float ts = rbf(tv * 1000.0f);                // t * scale in the model dtype
    const float arg = ts * freqs[i];
    emb[b * 256 + i] = f2bf(cosf(arg));
    emb[b * 256 + 128 + i] = f2bf(sinf(arg));
}

__global__ void add_kernel(const bf16_t *a, const bf16_t *b, bf16_t *o, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

// mod[l][b][j][d] = bf16(table[l][j][d] + proj[b][j % proj_rows][d])
__global__ void modulation_kernel(const bf16_t *tables, int rows, const bf16_t *proj, int proj_rows,
                                  int Bc, int D, bf16_t *mod) {
    const int l = blockIdx.z, b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)rows * D) return;
    const int j = (int)(e / D), d = (int)(e % D);
    const float v = bf2f(tables[(int64_t)l * rows * D + e]) +
                    bf2f(proj[((int64_t)b * proj_rows + (j % proj_rows)) * D + d]);
    const bf16_t r = f2bf(v);
    mod[(((int64_t)l * Bc + b) * rows) * D + e] = r;
}

// X[b][s][k*192 + c]: c < 128 → ctx[b%Bx][2s+k][c]; else xt[b%Bx][2s+k][c-128]; 0 past T
__global__ void pack_patches_kernel(const bf16_t *xt, const bf16_t *ctx, int Bx, int T, int S,
                                    bf16_t *X) {
    const int row = blockIdx.x;           // b*S + s
    const int b = row / S, s = row % S;
    const int bb = b % Bx;
    for (int i = threadIdx.x; i < 384 / 8; i += blockDim.x) {
        const int k = (i * 8) / 192, c = (i * 8) % 192;
        const int t = 2 * s + k;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (t < T) {
            if (c < 128) v = *(const uint4 *)(ctx + ((int64_t)bb * T + t) * 128 + c);
            else v = *(const uint4 *)(xt + ((int64_t)bb * T + t) * 64 + (c - 128));
        }
        *(uint4 *)(X + (int64_t)row * 384 + i * 8) = v;
    }
}

__global__ void crop_kernel(const bf16_t *src, int rows_src, int rows_dst, int C, bf16_t *dst) {
    const int b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)rows_dst * C) return;
    dst[(int64_t)b * rows_dst * C + e] = src[(int64_t)b * rows_src * C + e];
}

__global__ void cast_kernel(const float *src, bf16_t *dst, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = f2bf(src[i]);
}

__global__ void copy_cols_kernel(const bf16_t *src, int64_t lds, bf16_t *dst, int64_t ldd, int M, int C) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)M * C) return;
    const int64_t m = e / C, c = e - m * C;
    dst[m * ldd + c] = src[m * lds + c];
}

__global__ void gather_head_row_kernel(const bf16_t *V, int KV, int Le, int H, bf16_t *out) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;   // e = h·128 + d
    if (e >= H * 128) return;
    const int h = e >> 7, d = e & 127;
    out[e] = V[((int64_t)(h / (H / KV)) * Le) * 128 + d];
}

__global__ void add_row_bcast_kernel(bf16_t *X, const bf16_t *c, int64_t n8, int D8) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    float x[8], y[8];
    unpack8(((const uint4 *)X)[i], x);
    unpack8(((const uint4 *)c)[i % D8], y);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += y[j];
    ((uint4 *)X)[i] = pack8(x);
}

__global__ __launch_bounds__(256) void wav_peak_kernel(const float4 *w, int64_t n4, unsigned *peak) {
    const int b = blockIdx.y;
    const float4 *p = w + (int64_t)b * n4;
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 v = p[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        atomicMax(peak + b, __float_as_uint(m));   // non-negative floats order as their bits
    }
}

// One pass for the whole output path of a song:
//  (1) the decode guard (generate_music_decode.py:193-195): divide by the peak when it
//      exceeds 1 (IEEE division, as torch);
//  (2) normalize_audio (audio_utils.py:24-62, inference.py:674-679) when target > 0:
//      gain = target_amp / peak' — a python float over a 0-d tensor, which torch
//      evaluates as reciprocal(peak') * target (Tensor.__rtruediv__) — then x *= gain,
//      skipped when peak' < 1e-6.
// peak' (the peak after (1)) needs no second reduction: division is monotone and
// correctly rounded, so max|x / pk| = fl(pk / pk) = 1 exactly when (1) applied.
__global__ __launch_bounds__(256) void wav_scale_kernel(float4 *w, int64_t n4, const float *peak, int guard,
                                                        float target) {
    const int b = blockIdx.y;
    const float pk = peak[b];
    const bool div = guard && pk > 1.0f;
    const float p2 = div ? 1.0f : pk;
    const bool norm = target > 0.f && !(p2 < 1e-6f);
    if (!div && !norm) return;
    const float gain = (1.0f / p2) * target;
    float4 *p = w + (int64_t)b * n4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 v = p[i];
        if (div) { v.x /= pk; v.y /= pk; v.z /= pk; v.w /= pk; }
        if (norm) { v.x *= gain; v.y *= gain; v.z *= gain; v.w *= gain; }
        p[i] = v;
    }
}

// The output leg's sample conversion fused into the scale pass: after (1)+(2) above, every
// sample is written back (the fp32 tensor the reference returns, inference.py:711) AND packed as
// interleaved PCM16 [N][C] — the frame layout a WAV / FLAC writer consumes (soundfile gets
// [samples, channels], audio_utils.py:173,190) — q = rint(clamp(x, −1, 1) · 32767), libsndfile's
// float → 16-bit conversion (normalised, round-to-nearest-even; identical to its unclipped
// lrintf(x · 0x7FFF) for |x| ≤ 1, which normalize_audio guarantees).  One thread: 4 frames.
template <int C>
__global__ __launch_bounds__(256) void wav_scale_pcm16_kernel(float *w, int64_t N, const float *peak, int guard,
                                                              float target, short *pcm) {
    const int b = blockIdx.y;
    const float pk = peak[b];
    const bool div = guard && pk > 1.0f;
    const float p2 = div ? 1.0f : pk;
    const bool norm = target > 0.f && !(p2 < 1e-6f);
    const float gain = (1.0f / p2) * target;
    float *p = w + (int64_t)b * C * N;
    short *q = pcm + (int64_t)b * C * N;
    const int64_t n4 = N / 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float v[C][4];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float4 x = ((const float4 *)(p + (int64_t)c * N))[i];
            v[c][0] = x.x; v[c][1] = x.y; v[c][2] = x.z; v[c][3] = x.w;
        }
        if (div || norm) {
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (div) v[c][j] /= pk;
                    if (norm) v[c][j] *= gain;
                }
#pragma unroll
            for (int c = 0; c < C; ++c)
                ((float4 *)(p + (int64_t)c * N))[i] = make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
        }
        short o[4 * C];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int c = 0; c < C; ++c)
                o[j * C + c] = (short)__builtin_rintf(fminf(fmaxf(v[c][j], -1.0f), 1.0f) * 32767.0f);
        if constexpr (C == 2) {
            uint4 u;
            u.x = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
            u.y = (uint32_t)(uint16_t)o[2] | ((uint32_t)(uint16_t)o[3] << 16);
            u.z = (uint32_t)(uint16_t)o[4] | ((uint32_t)(uint16_t)o[5] << 16);
            u.w = (uint32_t)(uint16_t)o[6] | ((uint32_t)(uint16_t)o[7] << 16);
            ((uint4 *)q)[i] = u;
        } else {
            uint2 u;
            u.x = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
            u.y = (uint32_t)(uint16_t)o[2] | ((uint32_t)(uint16_t)o[3] << 16);
            ((uint2 *)q)[i] = u;
        }
    }
}

// FSQ (vector_quantize_pytorch FSQ.bound / codes_to_indices, restated; see
// oracle/condenc_oracle.py): fp32 math as the library forces (force_quantization_f32)
__global__ void fsq_quantize_kernel(const bf16_t *z, int64_t ldz, int M, FsqLevels lv, bf16_t *codes, int64_t ldc,
                                    int *idx) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= M) return;
    float index = 0.f, basis = 1.f;
    for (int i = 0; i < lv.n; ++i) {
        const int L = lv.L[i];
        const float half_l = ((float)(L - 1) * 1.001f) / 2.0f;
        const float offset = (L % 2 == 0) ? 0.5f : 0.0f;
        const float shift = atanhf(offset / half_l);
        const float bounded = tanhf(bf2f(z[(int64_t)row * ldz + i]) + shift) * half_l - offset;
        const float hw = (float)(L / 2);
        const float code = rintf(bounded) / hw;                 // torch.round: half to even
        codes[(int64_t)row * ldc + i] = f2bf(code);
        index += (code * hw + hw) * basis;
        basis *= (float)L;
    }
    for (int i = lv.n; i < 64; ++i) codes[(int64_t)row * ldc + i] = 0;   // K padding of project_out
    if (idx) idx[row] = (int)rintf(index);
}

__global__ void fsq_codes_kernel(const int *idx, int M, FsqLevels lv, bf16_t *codes, int64_t ldc) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= M) return;
    int basis = 1;
    for (int i = 0; i < lv.n; ++i) {
        const int L = lv.L[i], hw = L / 2;
        const int level = (idx[row] / basis) % L;
        codes[(int64_t)row * ldc + i] = f2bf((float)(level - hw) / (float)hw);
        basis *= L;
    }
    for (int i = lv.n; i < 64; ++i) codes[(int64_t)row * ldc + i] = 0;
}

}  // namespace

int fsq_quantize(const bf16_t *z, int64_t ldz, int M, const FsqLevels &lv, bf16_t *codes, int64_t ldc, int *idx,
                 hipStream_t s) {
    if (M <= 0) return 0;
    if (lv.n <= 0 || lv.n > 8 || ldc < 64) return fail(-1, "fsq_quantize: 1..8 levels, ldc >= 64");
    fsq_quantize_kernel<<<(M + 255) / 256, 256, 0, s>>>(z, ldz, M, lv, codes, ldc, idx);
    HIP_TRY(hipGetLastError());
    return 0;
}

int fsq_codes_from_indices(const int *idx, int M, const FsqLevels &lv, bf16_t *codes, int64_t ldc, hipStream_t s) {
    if (M <= 0) return 0;
    if (lv.n <= 0 || lv.n > 8 || ldc < 64) return fail(-1, "fsq_codes: 1..8 levels, ldc >= 64");
    fsq_codes_kernel<<<(M + 255) / 256, 256, 0, s>>>(idx, M, lv, codes, ldc);
    HIP_TRY(hipGetLastError());
    return 0;
}

int wav_peak_normalize(float *wav, int B, int64_t n, float *peak, hipStream_t s, float target_amp, int guard) {
    HIP_TRY(hipMemsetAsync(peak, 0, (size_t)B * sizeof(float), s));
    const int64_t n4 = n / 4;
    const unsigned gx = (unsigned)std::min<int64_t>(1024, (n4 + 255) / 256);
    wav_peak_kernel<<<dim3(gx, B), 256, 0, s>>>((const float4 *)wav, n4, (unsigned *)peak);
    HIP_TRY(hipGetLastError());
    wav_scale_kernel<<<dim3(gx, B), 256, 0, s>>>((float4 *)wav, n4, peak, guard, target_amp);
    HIP_TRY(hipGetLastError());
    return 0;
}

int wav_postprocess_pcm16(float *wav, int B, int C, int64_t N, float *peak, hipStream_t s, float target_amp,
                          int guard, short *pcm) {
    HIP_TRY(hipMemsetAsync(peak, 0, (size_t)B * sizeof(float), s));
    const int64_t n4 = N / 4;
    const unsigned gx = (unsigned)std::min<int64_t>(1024, (C * n4 + 255) / 256);
    wav_peak_kernel<<<dim3(gx, B), 256, 0, s>>>((const float4 *)wav, C * n4, (unsigned *)peak);
    HIP_TRY(hipGetLastError());
    const unsigned gp = (unsigned)std::min<int64_t>(1024, (n4 + 255) / 256);
    if (C == 2)
        wav_scale_pcm16_kernel<2><<<dim3(gp, B), 256, 0, s>>>(wav, N, peak, guard, target_amp, pcm);
    else
        wav_scale_pcm16_kernel<1><<<dim3(gp, B), 256, 0, s>>>(wav, N, peak, guard, target_amp, pcm);
    HIP_TRY(hipGetLastError());
    return 0;
}

int gather_head_row(const bf16_t *V, int KV, int Le, int H, bf16_t *out, hipStream_t s) {
    if (KV <= 0 || H % KV) return fail(-1, "gather_head_row: heads");
    gather_head_row_kernel<<<(H * 128 + 255) / 256, 256, 0, s>>>(V, KV, Le, H, out);
    HIP_TRY(hipGetLastError());
    return 0;
}

int add_row_bcast(bf16_t *X, const bf16_t *c, int rows, int D, hipStream_t s) {
    if (rows <= 0) return 0;
    if (D % 8) return fail(-1, "add_row_bcast: D % 8");
    const int64_t n8 = (int64_t)rows * D / 8;
    add_row_bcast_kernel<<<(unsigned)((n8 + 255) / 256), 256, 0, s>>>(X, c, n8, D / 8);
    HIP_TRY(hipGetLastError());
    return 0;
}

int copy_cols(const bf16_t *src, int64_t lds, bf16_t *dst, int64_t ldd, int M, int C, hipStream_t s) {
    if (M <= 0 || C <= 0) return 0;
    copy_cols_kernel<<<(unsigned)(((int64_t)M * C + 255) / 256), 256, 0, s>>>(src, lds, dst, ldd, M, C);
    HIP_TRY(hipGetLastError());
    return 0;
}

int gemv_small(const bf16_t *x, int64_t ldx, const bf16_t *W, const bf16_t *bias, bf16_t *y,
               int64_t ldy, int M, int N, int K, int act, hipStream_t s, bf16_t *act_scratch) {
    if (M > 16 || K % 8 || ldx % 8) return fail(-1, "gemv_small: M<=16, K%8==0 required");
    if (act && act_scratch && M > 0) {
        // bf16(silu(x)) once into the scratch rows (same rounding as the in-kernel rbf(silu))
        silu_rows_kernel<<<dim3((unsigned)((K / 8 + 255) / 256), M), 256, 0, s>>>(x, ldx, act_scratch, K, K);
        HIP_TRY(hipGetLastError());
        x = act_scratch;
        ldx = K;
        act = 0;
    }
    gemv_small_kernel<<<(N + 3) / 4, 256, 0, s>>>(x, ldx, W, bias, y, ldy, M, N, K, act);
    HIP_TRY(hipGetLastError());
    return 0;
}

int bcast_rows(const bf16_t *src, int64_t n, bf16_t *dst, int rows, hipStream_t s) {
    if (n % 8) return fail(-1, "bcast_rows: n % 8");
    bcast_rows_kernel<<<dim3((unsigned)((n / 8 + 255) / 256), rows), 256, 0, s>>>(src, n, dst);
    HIP_TRY(hipGetLastError());
    return 0;
}

int timestep_sinusoid(const float *t, const float *t_r, int t_stride, int use_diff, int Bc,
                      const float *freqs, bf16_t *emb, hipStream_t s) {
    sinusoid_kernel<<<Bc, 128, 0, s>>>(t, t_r, t_stride, use_diff, freqs, emb);
    HIP_TRY(hipGetLastError());
    return 0;
}

int add_bf16(const bf16_t *a, const bf16_t *b, bf16_t *out, int64_t n, hipStream_t s) {
    add_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a, b, out, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int modulation(const bf16_t *tables, int n_tables, int rows, const bf16_t *proj, int Bc, int D,
               bf16_t *mod, hipStream_t s) {
    // proj rows: 6 for the layer tables (proj [Bc][6][D]); 1 for norm_out (temb [Bc][D])
    const int proj_rows = rows == 6 ? 6 : 1;
    dim3 grid((unsigned)(((int64_t)rows * D + 255) / 256), Bc, n_tables);
    modulation_kernel<<<grid, 256, 0, s>>>(tables, rows, proj, proj_rows, Bc, D, mod);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pack_patches(const bf16_t *xt, const bf16_t *ctx, int Bx, int Bc, int T, int S, bf16_t *X,
                 hipStream_t s) {
    pack_patches_kernel<<<Bc * S, 64, 0, s>>>(xt, ctx, Bx, T, S, X);
    HIP_TRY(hipGetLastError());
    return 0;
}

int crop_rows(const bf16_t *src, int Bc, int rows_src, int rows_dst, int C, bf16_t *dst,
              hipStream_t s) {
    dim3 grid((unsigned)(((int64_t)rows_dst * C + 255) / 256), Bc);
    crop_kernel<<<grid, 256, 0, s>>>(src, rows_src, rows_dst, C, dst);
    HIP_TRY(hipGetLastError());
    return 0;
}

int cast_f32_bf16(const float *src, bf16_t *dst, int64_t n, hipStream_t s) {
    cast_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(src, dst, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
