// norm.hip — RMSNorm (+AdaLN modulation) and per-head q/k RMSNorm + RoPE.
//
// rmsnorm_mod: Qwen3RMSNorm (transformers modeling_qwen3.py:59-64) followed
// by the AdaLN modulation of AceStepDiTLayer (reference base:499, :530, and
// norm_out :1496), reproducing each bf16 rounding of the torch op sequence:
//   n = bf16(x·rsqrt(mean(x²)+eps)); y = bf16(w·n);
//   y = bf16(y·bf16(1+scale)); y = bf16(y+shift)
// R rows per wave, 16-byte vector loads (HBM-bound: 2·D bytes in, 2·D out).
//
// head_post: after the fused QKV GEMM, each 128-wide head gets its RMSNorm
// (q_norm / k_norm, base:304,338), RoPE rotate-half with bf16 rounding of
// q·cos, rot(q)·sin and the sum (modeling_qwen3.py:166-170), and is scattered
// into the head-major [B][heads][S][128] layout the attention kernel streams.
#include "kernels.h"
#include "headpost.h"

namespace acehip {
namespace {

template <int V> struct VecOf;
template <> struct VecOf<8> { typedef uint4 T; };
template <> struct VecOf<4> { typedef uint2 T; };

template <int V>
__device__ __forceinline__ void unpackv(const typename VecOf<V>::T &u, float *f) {
    if constexpr (V == 8) unpack8(u, f);
    else unpack4(u, f);
}
template <int V>
__device__ __forceinline__ typename VecOf<V>::T packv(const float *f) {
    if constexpr (V == 8) return pack8(f);
    else return pack4(f);
}

// V elements per vector access (8 → 16 B, 4 → 8 B), NV vectors per lane
// (D = 64·V·NV), R consecutive rows per wave: the R rows' loads are all in
// flight before the first reduction, and the norm weight / AdaLN scale+shift
// vectors are loaded once per wave (re-loaded only when the rows cross a
// batch boundary).
template <int V, int NV, int R>
__global__ __launch_bounds__(256) void rmsnorm_mod_kernel(const bf16_t *x,   // not restrict: RowAdd writes it (ra.xw)
                                                          const bf16_t *__restrict__ w,
                                                          const bf16_t *__restrict__ shift,
                                                          const bf16_t *__restrict__ scale,
                                                          int64_t mod_bstride, int rows_per_batch,
                                                          bf16_t *__restrict__ out, int M, int D,
                                                          float eps, RowAdd ra) {
    typedef typename VecOf<V>::T vec_t;
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
    if (row0 >= M) return;
    vec_t xr[R][NV];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bf16_t *xp = x + (int64_t)min(row0 + r, M - 1) * D;
#pragma unroll
        for (int i = 0; i < NV; ++i) xr[r][i] = *(const vec_t *)(xp + (i * 64 + lane) * V);
    }
    // weight / modulation loads are independent of the row-add and the reductions: issued with
    // the x loads, before any store of the row add (vmcnt also counts stores, so a load issued
    // after them would make its wait cover their completion too)
    vec_t wr[NV], s1r[NV], s2r[NV];
    int cur_b = row0 / rows_per_batch;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int e = (i * 64 + lane) * V;
        wr[i] = *(const vec_t *)(w + e);
        if (scale) {
            s1r[i] = *(const vec_t *)(scale + (int64_t)cur_b * mod_bstride + e);
            s2r[i] = *(const vec_t *)(shift + (int64_t)cur_b * mod_bstride + e);
        }
    }
    // rows < ra.prows first get the deferred split-K residual epilogue of the GEMM that
    // produced them (gemm(..., defer)): x = bf16(x + bf16(bf16(Σ partials)·gate)) or
    // bf16(x + bf16(Σ partials)), summed in split order as splitk_epilogue_kernel does
    if (ra.part) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = row0 + r;
            if (row >= M || row >= ra.prows) continue;   // wave-uniform
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int e = (i * 64 + lane) * V;
                float xv[V], acc[V];
                unpackv<V>(xr[r][i], xv);
                const float *pp = ra.part + (int64_t)row * D + e;
                if constexpr (V == 8) {
                    sum_parts8(pp, ra.plane, ra.splits, acc);
                } else {
                    f32x4 t = *(const f32x4 *)pp;
                    for (int sp = 1; sp < ra.splits; ++sp) t += *(const f32x4 *)(pp + sp * ra.plane);
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[c] = t[c];
                }
                if (ra.gate) {
                    float gg[V];
                    unpackv<V>(*(const vec_t *)(ra.gate + (int64_t)(row / ra.gate_rpb) * ra.gate_bstride + e), gg);
#pragma unroll
                    for (int j = 0; j < V; ++j) xv[j] = xv[j] + rbf(rbf(acc[j]) * gg[j]);
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) xv[j] = xv[j] + rbf(acc[j]);
                }
                xr[r][i] = packv<V>(xv);
                *(vec_t *)(ra.xw + (int64_t)row * D + e) = xr[r][i];
            }
        }
    }
    // rows >= ra.from first get x = bf16(x + v), written back (the CFG null rows' constant
    // cross-attention output, add_row_bcast folded into this pass)
    if (ra.v) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = row0 + r;
            if (row >= M || row < ra.from) continue;   // wave-uniform
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int e = (i * 64 + lane) * V;
                float xv[V], av[V];
                unpackv<V>(xr[r][i], xv);
                unpackv<V>(*(const vec_t *)(ra.v + e), av);
#pragma unroll
                for (int j = 0; j < V; ++j) xv[j] += av[j];
                xr[r][i] = packv<V>(xv);
                *(vec_t *)(ra.xw + (int64_t)row * D + e) = xr[r][i];
            }
        }
    }
    float rs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            float f[V];
            unpackv<V>(xr[r][i], f);
#pragma unroll
            for (int j = 0; j < V; ++j) ss += f[j] * f[j];
        }
        rs[r] = ss;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int r = 0; r < R; ++r) rs[r] += __shfl_xor(rs[r], o, 64);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        if (row >= M) break;
        if (scale && row / rows_per_batch != cur_b) {   // wave-uniform, rare
            cur_b = row / rows_per_batch;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int e = (i * 64 + lane) * V;
                s1r[i] = *(const vec_t *)(scale + (int64_t)cur_b * mod_bstride + e);
                s2r[i] = *(const vec_t *)(shift + (int64_t)cur_b * mod_bstride + e);
            }
        }
        const float rn = 1.0f / sqrtf(rs[r] / (float)D + eps);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = (i * 64 + lane) * V;
            float xv[V], wv[V], o[V];
            unpackv<V>(xr[r][i], xv);
            unpackv<V>(wr[i], wv);
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = rbf(wv[j] * rbf(xv[j] * rn));
            if (scale) {
                float s1[V], s2[V];
                unpackv<V>(s1r[i], s1);
                unpackv<V>(s2r[i], s2);
#pragma unroll
                for (int j = 0; j < V; ++j) o[j] = rbf(o[j] * rbf(1.0f + s1[j])) + s2[j];
            }
            *(vec_t *)(out + (int64_t)row * D + e) = packv<V>(o);
        }
    }
}

// WPR waves per row (D = 512·NV·WPR, 16-B accesses): more waves in flight
// for the same bytes; the row's sum of squares is combined through LDS.
// RowAdd (partials / row constant) as in rmsnorm_mod_kernel: the short-song path (few rows,
// split-K partials to fold in) uses this kernel with WPR = 4 for more loads in flight per row
template <int NV, int WPR>
__global__ __launch_bounds__(256) void rmsnorm_split_kernel(const bf16_t *x,   // not restrict: RowAdd writes it
                                                            const bf16_t *__restrict__ w,
                                                            const bf16_t *__restrict__ shift,
                                                            const bf16_t *__restrict__ scale,
                                                            int64_t mod_bstride, int rows_per_batch,
                                                            bf16_t *__restrict__ out, int M, int D,
                                                            float eps, RowAdd ra) {
    constexpr int RPB = 4 / WPR;   // rows per 256-thread block
    __shared__ float run[4][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rl = wave / WPR, wp = wave % WPR;
    const bool live = blockIdx.x * RPB + rl < M;
    const int row = min(blockIdx.x * RPB + rl, M - 1);
    const int b = row / rows_per_batch;
    const bf16_t *xp = x + (int64_t)row * D;
    uint4 xr[NV], wr[NV], s1r[NV], s2r[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) xr[i] = *(const uint4 *)(xp + ((wp * NV + i) * 64 + lane) * 8);
    // weight / modulation vectors with the x loads, before the row add's stores (see rmsnorm_mod_kernel)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int e = ((wp * NV + i) * 64 + lane) * 8;
        wr[i] = *(const uint4 *)(w + e);
        if (scale) {
            s1r[i] = *(const uint4 *)(scale + (int64_t)b * mod_bstride + e);
            s2r[i] = *(const uint4 *)(shift + (int64_t)b * mod_bstride + e);
        }
    }
    if (ra.part && row < ra.prows) {               // wave-uniform
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = ((wp * NV + i) * 64 + lane) * 8;
            float xv[8], acc[8];
            unpack8(xr[i], xv);
            sum_parts8(ra.part + (int64_t)row * D + e, ra.plane, ra.splits, acc);
            if (ra.gate) {
                float gg[8];
                unpack8(*(const uint4 *)(ra.gate + (int64_t)(row / ra.gate_rpb) * ra.gate_bstride + e), gg);
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = xv[j] + rbf(rbf(acc[j]) * gg[j]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = xv[j] + rbf(acc[j]);
            }
            xr[i] = pack8(xv);
            if (live) *(uint4 *)(ra.xw + (int64_t)row * D + e) = xr[i];
        }
    }
    if (ra.v && row >= ra.from) {                  // wave-uniform
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = ((wp * NV + i) * 64 + lane) * 8;
            float xv[8], av[8];
            unpack8(xr[i], xv);
            unpack8(*(const uint4 *)(ra.v + e), av);
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] += av[j];
            xr[i] = pack8(xv);
            if (live) *(uint4 *)(ra.xw + (int64_t)row * D + e) = xr[i];
        }
    }
    // lane L's running sum of squares continues across the row's waves in element order
    // (wave wp holds the lane's elements wp·NV·512 + …), then the same xor tree: exactly the
    // fma sequence of the one-wave-per-row kernel, so both round identically
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < WPR; ++k) {
        if (wp == k) {                             // wave-uniform
            ss = k == 0 ? 0.f : run[rl * WPR + k - 1][lane];
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                float f[8];
                unpack8(xr[i], f);
#pragma unroll
                for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
            }
            run[rl * WPR + k][lane] = ss;
        }
        __syncthreads();
    }
    ss = run[rl * WPR + WPR - 1][lane];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (blockIdx.x * RPB + rl >= M) return;
    const float rn = 1.0f / sqrtf(ss / (float)D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int e = ((wp * NV + i) * 64 + lane) * 8;
        float xv[8], wv[8], o[8];
        unpack8(xr[i], xv);
        unpack8(wr[i], wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rbf(wv[j] * rbf(xv[j] * rn));
        if (scale) {
            float s1[8], s2[8];
            unpack8(s1r[i], s1);
            unpack8(s2r[i], s2);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = rbf(o[j] * rbf(1.0f + s1[j])) + s2[j];
        }
        *(uint4 *)(out + (int64_t)row * D + e) = pack8(o);
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
    const float *psrc = a.part ? a.part + (int64_t)row * a.ld_src : nullptr;
    const int d = li * 8;
    float cs[8] = {}, sn[8] = {};
    if (a.cos) {
        unpack8(*(const uint4 *)(a.cos + (int64_t)s * 128 + d), cs);
        unpack8(*(const uint4 *)(a.sin + (int64_t)s * 128 + d), sn);
    }
    for (int u0 = blockIdx.y * 16 + wave * 4; u0 < units; u0 += 16 * gridDim.y) {
        const int u = u0 + sub;
        float x[8] = {};
        if (u < units) {
            if (psrc) {
                // split-K partials summed in split order, + 0 and bf16-rounded exactly as
                // splitk_epilogue_kernel stages them (EPI_HEADPOST: no bias)
                float acc[8];
                sum_parts8(psrc + u * 128 + d, a.plane, a.splits, acc);
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = rbf(acc[j] + 0.f);
            } else {
                unpack8(*(const uint4 *)(src + u * 128 + d), x);
            }
        }
        const bf16_t *nw;
        bf16_t *dst = head_dst(a, u, b, s, nw);
        float w[8] = {};
        if (nw) unpack8(*(const uint4 *)(nw + d), w);
        head_norm_rope(x, li, nw != nullptr, w, a.cos != nullptr, cs, sn, a.eps);
        if (dst) *(uint4 *)(dst + d) = pack8(x);
    }
}

}  // namespace

template <int R>
static void rms_launch(const bf16_t *x, const bf16_t *w, const bf16_t *shift, const bf16_t *scale,
                       int64_t mbs, int rpb, bf16_t *out, int M, int D, float eps, RowAdd ra, hipStream_t s) {
    const int grid = (M + 4 * R - 1) / (4 * R);
#define RMS_LAUNCH(V_, NV_) \
    rmsnorm_mod_kernel<V_, NV_, R><<<grid, 256, 0, s>>>(x, w, shift, scale, mbs, rpb, out, M, D, eps, ra)
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
}

int rmsnorm_mod(const bf16_t *x, const bf16_t *w, const bf16_t *shift, const bf16_t *scale,
                int64_t mod_bstride, int rows_per_batch, bf16_t *out, int M, int D, float eps,
                hipStream_t s, RowAdd ra, int rows_per_wave) {
    if (M <= 0) return 0;
    if ((ra.v || ra.part) && (!ra.xw || ra.xw != x)) return fail(-1, "rmsnorm: row add must write back to x");
    if (ra.part && (ra.splits < 1 || ra.prows > M || ra.plane < (int64_t)ra.prows * D || ra.gate_rpb <= 0))
        return fail(-1, "rmsnorm: deferred split-K epilogue arguments");
    if (D % 256 || D > 4096) return fail(-1, "rmsnorm: D must be a multiple of 256, <= 4096");
    if ((shift == nullptr) != (scale == nullptr)) return fail(-1, "rmsnorm: shift/scale");
    const int rpb = rows_per_batch > 0 ? rows_per_batch : M;
    // a deferred split-K epilogue (few rows, up to 16 partial slabs per row): 4 waves per row
    const int R = rows_per_wave ? rows_per_wave : !ra.part ? 1 : D % 2048 == 0 ? -4 : D % 1024 == 0 ? -2 : 1;
    if (R < 0 && D % (512 * -R) == 0 && D / (512 * -R) <= 4) {   // -WPR: WPR waves per row
        const int WPR = -R, nv = D / (512 * WPR), grid = (M + 4 / WPR - 1) / (4 / WPR);
#define SPLIT(NV_, W_) \
    rmsnorm_split_kernel<NV_, W_><<<grid, 256, 0, s>>>(x, w, shift, scale, mod_bstride, rpb, out, M, D, eps, ra)
        if (WPR == 2) {
            if (nv == 1) SPLIT(1, 2); else if (nv == 2) SPLIT(2, 2); else if (nv == 3) SPLIT(3, 2); else SPLIT(4, 2);
        } else {
            if (nv == 1) SPLIT(1, 4); else if (nv == 2) SPLIT(2, 4); else if (nv == 3) SPLIT(3, 4); else SPLIT(4, 4);
        }
#undef SPLIT
        HIP_TRY(hipGetLastError());
        return 0;
    }
    switch (R < 0 ? 1 : R) {
        case 1: rms_launch<1>(x, w, shift, scale, mod_bstride, rpb, out, M, D, eps, ra, s); break;
        case 2: rms_launch<2>(x, w, shift, scale, mod_bstride, rpb, out, M, D, eps, ra, s); break;
        default: rms_launch<4>(x, w, shift, scale, mod_bstride, rpb, out, M, D, eps, ra, s); break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

int head_post(const HeadPostArgs &a, hipStream_t s) {
    if (a.B * a.S <= 0) return 0;
    // reading split-K partials: one block per (row, 16 heads), more loads in flight per row
    const int units = a.nq + a.nk + a.nv;
    head_post_kernel<<<dim3(a.B * a.S, a.part ? (units + 15) / 16 : 1), 256, 0, s>>>(a);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
