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

template <int V, int NV>   // elements per vector access (8 → 16 B, 4 → 8 B); vectors per lane (D = 64·V·NV)
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
    constexpr int MAXV = NV;
    float v[MAXV][V];
    constexpr int nv = NV;
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
    const int b = row / rows_per_batch;
    const bf16_t *sh = shift ? shift + (int64_t)b * mod_bstride : nullptr;
    const bf16_t *sc = scale ? scale + (int64_t)b * mod_bstride : nullptr;
    // issue the weight / modulation loads before the reduction (independent of it)
    typedef __attribute__((ext_vector_type(V / 2))) uint32_t vec_t;
    vec_t wr[MAXV], s1r[MAXV], s2r[MAXV];
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (i < nv) {
            const int e = (i * 64 + lane) * V;
            wr[i] = *(const vec_t *)(w + e);
            if (sc) {
                s1r[i] = *(const vec_t *)(sc + e);
                s2r[i] = *(const vec_t *)(sh + e);
            }
        }
    }
    ss = wave_sum(ss);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (i < nv) {
            const int e = (i * 64 + lane) * V;
            float wv[V], o[V];
            if constexpr (V == 8) unpack8(*(const uint4 *)&wr[i], wv);
            else unpack4(*(const uint2 *)&wr[i], wv);
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = rbf(wv[j] * rbf(v[i][j] * r));
            if (sc) {
                float s1[V], s2[V];
                if constexpr (V == 8) { unpack8(*(const uint4 *)&s1r[i], s1); unpack8(*(const uint4 *)&s2r[i], s2); }
                else { unpack4(*(const uint2 *)&s1r[i], s1); unpack4(*(const uint2 *)&s2r[i], s2); }
#pragma unroll
                for (int j = 0; j < V; ++j) o[j] = rbf(o[j] * rbf(1.0f + s1[j])) + s2[j];
            }
            if constexpr (V == 8) *(uint4 *)(out + (int64_t)row * D + e) = pack8(o);
            else *(uint2 *)(out + (int64_t)row * D + e) = pack4(o);
        }
    }
}

// 16 lanes per 128-wide head (8 elements = one 16-B load each), 4 heads per
// wave in flight; the rotate-half partner of element d is d±64 → lane ^ 8.
__global__ __launch_bounds__(256) void head_post_kernel(HeadPostArgs a) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = lane >> 4, li = lane & 15;      // head slot within the wave, lane within the head
    const int row = blockIdx.x;
    const int b = row / a.S, s = row % a.S;
    const int units = a.nq + a.nk + a.nv;
    const bf16_t *src = a.src + (int64_t)row * a.ld_src;
    const int d = li * 8;
    float cs[8], sn[8];
    if (a.cos) {
        unpack8(*(const uint4 *)(a.cos + (int64_t)s * 128 + d), cs);
        unpack8(*(const uint4 *)(a.sin + (int64_t)s * 128 + d), sn);
    }
    for (int u0 = wave * 4; u0 < units; u0 += 16) {
        const int u = u0 + sub;
        const bool act = u < units;
        float x[8];
        if (act) unpack8(*(const uint4 *)(src + u * 128 + d), x);
        else
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = 0.f;
        bf16_t *dst = nullptr;
        const bf16_t *nw = nullptr;
        if (u < a.nq) {
            dst = a.q + (((int64_t)b * a.nq + u) * a.S_dst + s) * 128;
            nw = a.qw;
        } else if (u < a.nq + a.nk) {
            dst = a.k + (((int64_t)b * a.nk + (u - a.nq)) * a.S_dst + s) * 128;
            nw = a.kw;
        } else if (act) {
            dst = a.v + (((int64_t)b * a.nv + (u - a.nq - a.nk)) * a.S_dst + s) * 128;
        }
        // per-head RMSNorm over 16 lanes (all lanes shuffle; inactive ones carry zeros)
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
        if (nw) {
            const float r = 1.0f / sqrtf(ss * (1.0f / 128.0f) + a.eps);
            float w[8];
            unpack8(*(const uint4 *)(nw + d), w);
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = rbf(w[j] * rbf(x[j] * r));
        }
        if (a.cos) {
            float p[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) p[j] = __shfl_xor(x[j], 8, 64);
            if (nw) {
                const float sg = li < 8 ? -1.0f : 1.0f;
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = rbf(x[j] * cs[j]) + rbf(sg * p[j] * sn[j]);
            }
        }
        if (act) *(uint4 *)(dst + d) = pack8(x);
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
    const int rpb = rows_per_batch > 0 ? rows_per_batch : M;
#define RMS_LAUNCH(V_, NV_)                                                                        \
    rmsnorm_mod_kernel<V_, NV_><<<grid, 256, 0, s>>>(x, w, shift, scale, mod_bstride, rpb, out, M, D, eps)
    if (D % 512 == 0) {
        switch (D / 512) {
            case 1: RMS_LAUNCH(8, 1); break;
            case 2: RMS_LAUNCH(8, 2); break;
            case 3: RMS_LAUNCH(8, 3); break;
            case 4: RMS_LAUNCH(8, 4); break;
            case 5: RMS_LAUNCH(8, 5); break;
            case 6: RMS_LAUNCH(8, 6); break;
            case 7: RMS_LAUNCH(8, 7); break;
            default: RMS_LAUNCH(8, 8); break;
        }
    } else {
        switch (D / 256) {
            case 1: RMS_LAUNCH(4, 1); break;
            case 3: RMS_LAUNCH(4, 3); break;
            case 5: RMS_LAUNCH(4, 5); break;
            case 7: RMS_LAUNCH(4, 7); break;
            case 9: RMS_LAUNCH(4, 9); break;
            case 11: RMS_LAUNCH(4, 11); break;
            case 13: RMS_LAUNCH(4, 13); break;
            default: RMS_LAUNCH(4, 15); break;
        }
    }
#undef RMS_LAUNCH
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
