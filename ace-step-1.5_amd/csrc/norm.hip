// norm.hip — RMSNorm (+AdaLN modulation) and per-head q/k RMSNorm + RoPE.
//
// rmsnorm_mod: Qwen3RMSNorm (transformers modeling_qwen3.py:59-64) followed
// by the AdaLN modulation of AceStepDiTLayer (reference base:499, :530, and
// norm_out :1496), reproducing each bf16 rounding of the torch op sequence:
//   n = bf16(x·rsqrt(mean(x²)+eps)); y = bf16(w·n);
//   y = bf16(y·bf16(1+scale)); y = bf16(y+shift)
// One wave per row, 16-byte vector loads (HBM-bound: 2·D bytes in, 2·D out).
//
// head_post: after the fused QKV GEMM, each 128-wide head gets its RMSNorm
// (q_norm / k_norm, base:304,338), RoPE rotate-half with bf16 rounding of
// q·cos, rot(q)·sin and the sum (modeling_qwen3.py:166-170), and is scattered
// into the head-major [B][heads][S][128] layout the attention kernel streams.
#include "kernels.h"

namespace acehip {
namespace {

template <int V>   // elements per vector access (8 → 16 B, 4 → 8 B)
__global__ __launch_bounds__(256) void rmsnorm_mod_kernel(const bf16_t *__restrict__ x,
                                                          const bf16_t *__restrict__ w,
                                                          const bf16_t *__restrict__ shift,
                                                          const bf16_t *__restrict__ scale,
                                                          int64_t mod_bstride, int rows_per_batch,
                                                          bf16_t *__restrict__ out, int M, int D,
                                                          float eps) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const bf16_t *xr = x + (int64_t)row * D;
    constexpr int MAXV = 64 / V;  // up to D=4096
    float v[MAXV][V];
    const int nv = D / (64 * V);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (i < nv) {
            const int e = (i * 64 + lane) * V;
            if constexpr (V == 8) unpack8(*(const uint4 *)(xr + e), v[i]);
            else unpack4(*(const uint2 *)(xr + e), v[i]);
#pragma unroll
            for (int j = 0; j < V; ++j) ss += v[i][j] * v[i][j];
        }
    }
    ss = wave_sum(ss);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
    const int b = row / rows_per_batch;
    const bf16_t *sh = shift ? shift + (int64_t)b * mod_bstride : nullptr;
    const bf16_t *sc = scale ? scale + (int64_t)b * mod_bstride : nullptr;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (i < nv) {
            const int e = (i * 64 + lane) * V;
            float wv[V], o[V];
            if constexpr (V == 8) unpack8(*(const uint4 *)(w + e), wv);
            else unpack4(*(const uint2 *)(w + e), wv);
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = rbf(wv[j] * rbf(v[i][j] * r));
            if (sc) {
                float s1[V], s2[V];
                if constexpr (V == 8) { unpack8(*(const uint4 *)(sc + e), s1); unpack8(*(const uint4 *)(sh + e), s2); }
                else { unpack4(*(const uint2 *)(sc + e), s1); unpack4(*(const uint2 *)(sh + e), s2); }
#pragma unroll
                for (int j = 0; j < V; ++j) o[j] = rbf(o[j] * rbf(1.0f + s1[j])) + s2[j];
            }
            if constexpr (V == 8) *(uint4 *)(out + (int64_t)row * D + e) = pack8(o);
            else *(uint2 *)(out + (int64_t)row * D + e) = pack4(o);
        }
    }
}

__global__ __launch_bounds__(256) void head_post_kernel(HeadPostArgs a) {
    const int row = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = row / a.S, s = row % a.S;
    const int units = a.nq + a.nk + a.nv;
    const bf16_t *src = a.src + (int64_t)row * a.ld_src;
    const int d = lane * 2;
    float cs0 = 0, cs1 = 0, sn0 = 0, sn1 = 0;
    if (a.cos) {
        const uint32_t c = *(const uint32_t *)(a.cos + (int64_t)s * 128 + d);
        const uint32_t n = *(const uint32_t *)(a.sin + (int64_t)s * 128 + d);
        cs0 = bf2f(c & 0xffff); cs1 = bf2f(c >> 16);
        sn0 = bf2f(n & 0xffff); sn1 = bf2f(n >> 16);
    }
    for (int u = wave; u < units; u += 4) {
        const uint32_t raw = *(const uint32_t *)(src + u * 128 + d);
        float x0 = bf2f(raw & 0xffff), x1 = bf2f(raw >> 16);
        bf16_t *dst;
        const bf16_t *nw = nullptr;
        if (u < a.nq) {
            dst = a.q + (((int64_t)b * a.nq + u) * a.S_dst + s) * 128;
            nw = a.qw;
        } else if (u < a.nq + a.nk) {
            dst = a.k + (((int64_t)b * a.nk + (u - a.nq)) * a.S_dst + s) * 128;
            nw = a.kw;
        } else {
            dst = a.v + (((int64_t)b * a.nv + (u - a.nq - a.nk)) * a.S_dst + s) * 128;
        }
        if (nw) {
            const float ss = wave_sum(x0 * x0 + x1 * x1);
            const float r = 1.0f / sqrtf(ss * (1.0f / 128.0f) + a.eps);
            const uint32_t wr = *(const uint32_t *)(nw + d);
            x0 = rbf(bf2f(wr & 0xffff) * rbf(x0 * r));
            x1 = rbf(bf2f(wr >> 16) * rbf(x1 * r));
            if (a.cos) {
                // rotate_half: out[d] = x[d]cos[d] + (d<64 ? -x[d+64] : x[d-64]) sin[d]
                float p0 = __shfl_xor(x0, 32, 64), p1 = __shfl_xor(x1, 32, 64);
                if (lane < 32) { p0 = -p0; p1 = -p1; }
                x0 = rbf(x0 * cs0) + rbf(p0 * sn0);
                x1 = rbf(x1 * cs1) + rbf(p1 * sn1);
            }
        }
        *(uint32_t *)(dst + d) = (uint32_t)f2bf(x0) | ((uint32_t)f2bf(x1) << 16);
    }
}

}  // namespace

int rmsnorm_mod(const bf16_t *x, const bf16_t *w, const bf16_t *shift, const bf16_t *scale,
                int64_t mod_bstride, int rows_per_batch, bf16_t *out, int M, int D, float eps,
                hipStream_t s) {
    if (M <= 0) return 0;
    if (D % 256 || D > 4096) return fail(-1, "rmsnorm: D must be a multiple of 256, <= 4096");
    if ((shift == nullptr) != (scale == nullptr)) return fail(-1, "rmsnorm: shift/scale");
    const int grid = (M + 3) / 4;
    if (D % 512 == 0)
        rmsnorm_mod_kernel<8><<<grid, 256, 0, s>>>(x, w, shift, scale, mod_bstride,
                                                   rows_per_batch > 0 ? rows_per_batch : M, out, M, D, eps);
    else
        rmsnorm_mod_kernel<4><<<grid, 256, 0, s>>>(x, w, shift, scale, mod_bstride,
                                                   rows_per_batch > 0 ? rows_per_batch : M, out, M, D, eps);
    HIP_TRY(hipGetLastError());
    return 0;
}

int head_post(const HeadPostArgs &a, hipStream_t s) {
    if (a.B * a.S <= 0) return 0;
    head_post_kernel<<<a.B * a.S, 256, 0, s>>>(a);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
