// common.h — shared device/host helpers for libacehip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

// ------------------------------------------------------------- bf16 math ---
__host__ __device__ __forceinline__ float bf2f(bf16_t v) {
    union { uint32_t u; float f; } x;
    x.u = ((uint32_t)v) << 16;
    return x.f;
}
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// fp32 → bf16, round-to-nearest-even (torch's rounding for every bf16 op
// output).  On the device this is gfx950's v_cvt_pk_bf16_f32 (RNE, one
// instruction for two values); the host keeps the integer formulation — the
// two agree on every non-NaN input, NaN stays NaN (payload may differ).
__host__ __device__ __forceinline__ bf16_t f2bf(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(bf16_t, (__bf16)f);
#else
    union { uint32_t u; float f; } x;
    x.f = f;
    if ((x.u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((x.u >> 16) | 0x40);
    uint32_t r = x.u + 0x7fffu + ((x.u >> 16) & 1u);
    return (bf16_t)(r >> 16);
#endif
}
// round an fp32 value through bf16 (models one torch bf16 op's output rounding)
__host__ __device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }
// rbf over an array, two values per v_cvt_pk_bf16_f32 (+ a shift and a mask to widen them
// back): the same rounding as N calls of rbf, half the conversions
template <int N>
__device__ __forceinline__ void rbf_n(float *x) {
    static_assert(N % 2 == 0, "pairs");
#pragma unroll
    for (int i = 0; i < N; i += 2) {
        const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x[i], x[i + 1]}, bf16x2));
        x[i] = __builtin_bit_cast(float, u << 16);
        x[i + 1] = __builtin_bit_cast(float, u & 0xffff0000u);
    }
}
// two fp32 → packed bf16 pair (low half = a)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}

// silu = x·σ(x) = x / (1 + e^−x); the reciprocal by v_rcp_f32 (1 ulp) instead of the IEEE
// division sequence (div_scale ×2, rcp, 5 FMAs, div_fmas, div_fixup): the SwiGLU epilogue is
// VALU-bound and the result is rounded to bf16 right after
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// Snake of a value already rounded to bf16: x + 1/(e^β+1e-9)·sin(e^α x)².  `a` is e^α/(2π)
// (snake_params_kernel folds the 1/(2π) in): v_sin_f32 takes its argument in revolutions, so
// the sine is one multiply and one v_sin (|α·x| stays small for Oobleck activations, and the
// result is rounded to bf16 anyway)
__device__ __forceinline__ float snake1(float x, float a, float ib) {
    const float s = __builtin_amdgcn_sinf(a * x);
    return __builtin_fmaf(ib * s, s, x);
}
// the same on a pair (v_pk_mul_f32 / v_pk_fma_f32: two values per VALU slot; IEEE-identical
// to two snake1 calls)
__device__ __forceinline__ f32x2 snake2(f32x2 x, f32x2 a, f32x2 ib) {
    const f32x2 t = a * x;
    const f32x2 s = {__builtin_amdgcn_sinf(t.x), __builtin_amdgcn_sinf(t.y)};
    return __builtin_elementwise_fma(ib * s, s, x);
}
// array forms over pairs (N even): y = snake(x), o += v
template <int N>
__device__ __forceinline__ void snake_n(const float *x, const float *a, const float *ib, float *y) {
#pragma unroll
    for (int i = 0; i < N; i += 2) {
        const f32x2 r = snake2(f32x2{x[i], x[i + 1]}, f32x2{a[i], a[i + 1]}, f32x2{ib[i], ib[i + 1]});
        y[i] = r.x;
        y[i + 1] = r.y;
    }
}
template <int N>
__device__ __forceinline__ void add_n(float *o, const float *v) {
#pragma unroll
    for (int i = 0; i < N; i += 2) {
        const f32x2 r = f32x2{o[i], o[i + 1]} + f32x2{v[i], v[i + 1]};
        o[i] = r.x;
        o[i + 1] = r.y;
    }
}

// pack/unpack 8 bf16 in a uint4
__device__ __forceinline__ void unpack8(const uint4 &u, float *f) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = bf2f((bf16_t)(w[i] & 0xffff));
        f[2 * i + 1] = bf2f((bf16_t)(w[i] >> 16));
    }
}
__device__ __forceinline__ uint4 pack8(const float *f) {
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}
__device__ __forceinline__ uint2 pack4(const float *f) {
    return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
}
__device__ __forceinline__ void unpack4(const uint2 &u, float *f) {
    f[0] = bf2f((bf16_t)(u.x & 0xffff)); f[1] = bf2f((bf16_t)(u.x >> 16));
    f[2] = bf2f((bf16_t)(u.y & 0xffff)); f[3] = bf2f((bf16_t)(u.y >> 16));
}

// 16×16 MFMA output tiles (transposed layout: lane (fr = lane & 15, fc = lane >> 4) holds
// row fr, columns 4fc..4fc+3): pair sub-tiles lo (cols c..c+15) and hi (c+16..c+31) so
// that lane (fr, fc) ends up with 8 CONTIGUOUS columns — of lo if fc is even, of hi if odd —
// at offset 8·(fc >> 1): one 4-value swap with lane ^ 16.  Turns an epilogue's 8-B
// accesses into 16-B ones (the store tail is issue-bound).
__device__ __forceinline__ void pair8(const f32x4 &lo, const f32x4 &hi, bool odd, float (&v)[8]) {
    // v_permlane16_swap_b32 (VALU, no LDS round trip): the odd 16-lane rows of its first operand
    // trade with the even rows of its second — with (lo, hi) that hands the even rows their odd
    // partner's lo and the odd rows their even partner's hi, so v = (first, second) in every
    // lane.  Both lanes of a pair must be active.  Inline asm: ROCm 7.2's
    // __builtin_amdgcn_permlane16_swap folds the four calls into the first one's result
    // (every r got r = 0's values); the s_nop 1 is the VALU-write → permlane-read wait the
    // compiler does not insert for asm.
    (void)odd;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float a = lo[r], b = hi[r];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
        v[r] = a;
        v[4 + r] = b;
    }
}

// ------------------------------------------------------- wave reductions ---
// Σ_{sp < splits} p[sp·plane + 0..7] summed in split order (the split-K epilogue's own
// order, so a consumer that folds it in rounds identically); four splits' loads in flight at
// a time from clamped indices, the extra ones dropped by a select (no branch around a load)
__device__ __forceinline__ void sum_parts8(const float *p, int64_t plane, int splits, float (&acc)[8]) {
    f32x4 a0 = *(const f32x4 *)p, a1 = *(const f32x4 *)(p + 4);
    for (int s0 = 1; s0 < splits; s0 += 4) {
        f32x4 v0[4], v1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float *q = p + (int64_t)min(s0 + i, splits - 1) * plane;
            v0[i] = *(const f32x4 *)q;
            v1[i] = *(const f32x4 *)(q + 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool ok = s0 + i < splits;
            a0 = ok ? a0 + v0[i] : a0;
            a1 = ok ? a1 + v1[i] : a1;
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        acc[c] = a0[c];
        acc[4 + c] = a1[c];
    }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// --------------------------------------------------------- LDS-DMA (glds) --
// 16 bytes per lane, global → LDS; the LDS destination is lds_base + lane*16
// (wave-uniform base).  gfx950 global_load_lds_dwordx4.
__device__ __forceinline__ void glds16(const void *gsrc, void *lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)gsrc,
                                     (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

// bijective XCD-aware block remap (cdna_hip_programming.md §5 template)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ------------------------------------------------------------ host side ---
namespace acehip {
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
}  // namespace acehip

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return acehip::fail(-3, std::string(#expr) + ": " + hipGetErrorString(_e));  \
    } while (0)
