// headpost.h — the per-head q/k RMSNorm + RoPE transform shared by the
// standalone head_post kernel (norm.hip) and the fused QKV / cross-Q GEMM
// epilogue (gemm.hip, EPI_HEADPOST), so both paths round identically.
//
// Reference: q = q_norm(q_proj(x).view(.., 128)), k = k_norm(...) (base:304,338),
// Qwen3RMSNorm (transformers modeling_qwen3.py:59-64: w · bf16(x·rsqrt(mean x²+eps))),
// then rotate-half RoPE q·cos + rot(q)·sin with each product rounded to bf16
// (modeling_qwen3.py:166-170).
#pragma once
#include "kernels.h"

namespace acehip {

// One 128-wide head is held by 16 consecutive lanes, 8 elements each
// (d = 8·li, li = lane & 15).  Every lane of the wave must call this (it
// shuffles); norm == false leaves x unchanged (v heads).  `rope` must be
// uniform over the wave; w is this lane's 8 norm weights, cs/sn its 8 cos/sin.
// 16-lane row rotations by DPP (row_ror:n, a VALU move): __shfl_xor compiled to
// ds_bpermute — 12 LDS round trips per (row, head) unit, 4 of them a dependent chain
template <int N>
__device__ __forceinline__ float row_ror(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + N, 0xF, 0xF, false));
}

// NORM: q / k head (RMSNorm, then RoPE when ROPE); a v head passes through unchanged.
// rsqrt by v_rsq_f32 (the reference's torch.rsqrt; the IEEE 1/sqrtf expansion was ~35 VALU
// per head row); the rotate-half sign folds into one fma: x·cos + sg·bf16(p·sin), sg·t exact
template <bool NORM, bool ROPE>
__device__ __forceinline__ void head_norm_rope_t(float (&x)[8], int li, const float (&w)[8], const float (&cs)[8],
                                                 const float (&sn)[8], float eps) {
    if constexpr (NORM) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
        // all-reduce over the 16 lanes of the head: rotations by 8, 4, 2, 1 within the row
        ss += row_ror<8>(ss);
        ss += row_ror<4>(ss);
        ss += row_ror<2>(ss);
        ss += row_ror<1>(ss);
        // (bf16 roundings two at a time, rbf_n: the same values as per-element rbf)
        const float r = __builtin_amdgcn_rsqf(ss * (1.0f / 128.0f) + eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] *= r;
        rbf_n<8>(x);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] *= w[j];
        rbf_n<8>(x);
        if constexpr (ROPE) {
            float p[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) p[j] = row_ror<8>(x[j]) * sn[j];   // rotate-half partner d ± 64 (lane ^ 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] *= cs[j];
            rbf_n<8>(x);
            rbf_n<8>(p);
            const float sg = li < 8 ? -1.0f : 1.0f;
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = __builtin_fmaf(sg, p[j], x[j]);
        }
    }
}

// runtime-flag form (the standalone head_post kernel, mixed-type tiles): every lane of the wave
// must call it (it shuffles); `rope` must be uniform over the wave
__device__ __forceinline__ void head_norm_rope(float (&x)[8], int li, bool norm, const float (&w)[8], bool rope,
                                               const float (&cs)[8], const float (&sn)[8], float eps) {
    // the lane reductions run unmasked: a v head's lanes compute and discard
    float y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = x[j];
    if (rope) head_norm_rope_t<true, true>(y, li, w, cs, sn, eps);
    else head_norm_rope_t<true, false>(y, li, w, cs, sn, eps);
    if (norm) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = y[j];
    }
}

// destination row of head `u` (q | k | v order) for token (b, s); nullptr for u past the end
__device__ __forceinline__ bf16_t *head_dst(const HeadPostArgs &a, int u, int b, int s, const bf16_t *&nw) {
    nw = nullptr;
    if (u < a.nq) {
        nw = a.qw;
        return a.q + (((int64_t)b * a.nq + u) * a.S_dst + s) * 128;
    }
    if (u < a.nq + a.nk) {
        nw = a.kw;
        return a.k + (((int64_t)b * a.nk + (u - a.nq)) * a.S_dst + s) * 128;
    }
    if (u < a.nq + a.nk + a.nv) return a.v + (((int64_t)b * a.nv + (u - a.nq - a.nk)) * a.S_dst + s) * 128;
    return nullptr;
}

}  // namespace acehip
