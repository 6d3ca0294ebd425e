// sampler.hip — one fused base/sft sampler step per song.
//
// Restates reference base:1943-1979 with apg_forward / MomentumBuffer /
// project (acestep/models/base/apg_guidance.py:5-56):
//   diff = cond − uncond; ra = diff + (−0.75)·ra            (bf16 ops)
//   ‖ra‖₂ over T per channel → bf16; sf = min(1, bf16(bf16(1/‖ra‖)·2.5)); v0 = bf16(ra·sf)
//   v1 = cond/max(‖cond‖,1e-12); par = Σ(v0·v1)·v1; orth = v0 − par   (float64)
//   vt = bf16(cond + bf16((g−1)·bf16(orth)));  xt = bf16(xt − bf16(vt·dt))
// Storage type S = bf16 (production: every op output rounded to bf16 as torch
// does) or float (the fp32 parity mode: the same chain with no rounding).
// The norms are global per-(song, channel) reductions over T: three launches
// (see apg_phase_kernel), L2-resident passes, no host sync.  2.3 MB per song
// at 240 s.  The chunk-partial workspace is one per device: calls on
// different streams of one device must not overlap.
#include "kernels.h"

#include <map>
#include <mutex>

namespace acehip {
namespace {

// 8 consecutive elements of a row: bf16 (16 B) or fp32 (32 B); R = the storage
// type's rounding of one op output (torch's bf16 op semantics / none in fp32)
__device__ __forceinline__ void ld8(const bf16_t *p, float *f) { unpack8(*(const uint4 *)p, f); }
__device__ __forceinline__ void ld8(const float *p, float *f) {
    const float4 a = *(const float4 *)p, b = *(const float4 *)(p + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t *p, const float *f) { *(uint4 *)p = pack8(f); }
__device__ __forceinline__ void st8(float *p, const float *f) {
    *(float4 *)p = make_float4(f[0], f[1], f[2], f[3]);
    *(float4 *)(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}
template <class S> __device__ __forceinline__ float R(float x) { return rbf(x); }
template <> __device__ __forceinline__ float R<float>(float x) { return x; }
__device__ __forceinline__ float ld1(const bf16_t *p) { return bf2f(*p); }
__device__ __forceinline__ float ld1(const float *p) { return *p; }
__device__ __forceinline__ void st1(bf16_t *p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void st1(float *p, float v) { *p = v; }

// The norms are reductions over all T rows of a (song, channel), so the step
// runs as three launches over grid (8 channel groups, ⌈T/256⌉ row chunks, B
// songs), one row per thread (8 channels = one 16-B access), with per-chunk
// partial sums in a small workspace combined in chunk order (deterministic):
//   phase 1  ra update (written), Σ ra² (fp32) and Σ cond² (fp64) per chunk
//   phase 2  sf, ‖cond‖ from the phase-1 partials; Σ v0·v1 (fp64) per chunk
//   phase 3  dot from the phase-2 partials; vt and the Euler update
// (one workgroup per channel group walking all T rows was 78 µs per step at
// T = 6000 on 8 CUs; the three launches spread it over 192 workgroups)
constexpr int APG_TC = 256;
struct ApgPart {
    float ss[8];
    double cs[8];
    double dot[8];
};

// chunk partials of one (song, channel group) summed in chunk order, then over
// the block: thread j < 8 owns channel j; results broadcast through LDS
template <int PHASE>
__device__ __forceinline__ void apg_totals(const ApgPart *p, int nch, float *sf, double *denom, double *dot) {
    __shared__ float s_sf[8];
    __shared__ double s_den[8], s_dot[8];
    const int j = threadIdx.x;
    if (j < 8) {
        float a = 0.f;
        double c = 0.0, d = 0.0;
        for (int ch = 0; ch < nch; ++ch) {
            a += p[ch].ss[j];
            c += p[ch].cs[j];
            if (PHASE == 3) d += p[ch].dot[j];
        }
        s_sf[j] = a;
        s_den[j] = c;
        s_dot[j] = d;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sf[k] = s_sf[k];
        denom[k] = s_den[k];
        dot[k] = s_dot[k];
    }
}

template <class S, int PHASE>
__global__ __launch_bounds__(APG_TC) void apg_phase_kernel(const S *__restrict__ vt, S *__restrict__ xt,
                                                         S *__restrict__ ra, int B, int T, float guidance,
                                                         float dt, int first_step, int out_mode,
                                                         ApgPart *__restrict__ part) {
    constexpr int C = 64, CG = 8, NW = APG_TC / 64;
    __shared__ float s_ss[NW][CG];
    __shared__ double s_cs[NW][CG];
    const int cg = blockIdx.x, ch = blockIdx.y, b = blockIdx.z, nch = gridDim.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int t = ch * APG_TC + tid;
    const int64_t base = (int64_t)b * T * C + cg * CG, i = base + (int64_t)t * C;
    const S *cond = vt, *unc = vt + (int64_t)B * T * C;
    ApgPart *pp = part + (int64_t)(b * CG + cg) * nch;
    float sf[8];
    double denom[8], dot[8];
    if (PHASE > 1) {
        apg_totals<PHASE>(pp, nch, sf, denom, dot);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float nrm = R<S>(sqrtf(sf[j]));
            // norm_threshold / diff_norm (apg_guidance.py:47) is a python float over a
            // tensor: torch evaluates __rtruediv__ as reciprocal(diff_norm) * 2.5, each
            // rounded to the tensor dtype — not bf16(2.5 / n) (differs for ~1 in 4 norms)
            sf[j] = fminf(1.0f, R<S>(R<S>(1.0f / nrm) * 2.5f));
            denom[j] = fmax(sqrt(denom[j]), 1e-12);
        }
    }
    float ss[8];
    double cs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { ss[j] = 0.f; cs[j] = 0.0; }
    if (t < T) {
        float c8[8], r8[8];
        ld8(cond + i, c8);
        if (PHASE == 1) {
            float u8[8];
            ld8(unc + i, u8);
            if (!first_step) ld8(ra + i, r8);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float diff = R<S>(c8[j] - u8[j]);
                r8[j] = first_step ? diff : R<S>(diff + R<S>(-0.75f * r8[j]));
                ss[j] = r8[j] * r8[j];
                cs[j] = (double)c8[j] * (double)c8[j];
            }
            st8(ra + i, r8);
        } else if (PHASE == 2) {
            ld8(ra + i, r8);
#pragma unroll
            for (int j = 0; j < 8; ++j) cs[j] = (double)R<S>(r8[j] * sf[j]) * ((double)c8[j] / denom[j]);
        } else {
            float x8[8];
            ld8(ra + i, r8);
            if (!out_mode) ld8(xt + i, x8);
            const float gm1 = guidance - 1.0f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const double v0 = (double)R<S>(r8[j] * sf[j]);
                const double v1 = (double)c8[j] / denom[j];
                const float orth = R<S>((float)(v0 - dot[j] * v1));
                const float g = R<S>(c8[j] + R<S>(gm1 * orth));
                x8[j] = out_mode ? g : R<S>(x8[j] - R<S>(g * dt));
            }
            st8(xt + i, x8);
        }
    }
    if (PHASE == 3) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (PHASE == 1) ss[j] = wave_sum(ss[j]);
        cs[j] = wave_sum_d(cs[j]);
    }
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < 8; ++j) { s_ss[wave][j] = ss[j]; s_cs[wave][j] = cs[j]; }
    __syncthreads();
    if (tid < 8) {
        float a = 0.f;
        double c = 0.0;
        for (int w = 0; w < NW; ++w) { a += s_ss[w][tid]; c += s_cs[w][tid]; }
        if (PHASE == 1) {
            pp[ch].ss[tid] = a;
            pp[ch].cs[tid] = c;
        } else {
            pp[ch].dot[tid] = c;
        }
    }
}

// outside the CFG interval (vt = cond) or without CFG: the Euler update alone
template <class S>
__global__ __launch_bounds__(APG_TC) void euler_rows_kernel(const S *__restrict__ vt, S *__restrict__ xt, int T,
                                                          float dt, int out_mode) {
    constexpr int C = 64;
    const int t = blockIdx.y * APG_TC + threadIdx.x;
    if (t >= T) return;
    const int64_t i = (int64_t)blockIdx.z * T * C + blockIdx.x * 8 + (int64_t)t * C;
    float c8[8], x8[8];
    ld8(vt + i, c8);
    if (out_mode) { st8(xt + i, c8); return; }
    ld8(xt + i, x8);
#pragma unroll
    for (int j = 0; j < 8; ++j) x8[j] = R<S>(x8[j] - R<S>(c8[j] * dt));
    st8(xt + i, x8);
}

template <class S>
__global__ void axpy_kernel(const S *vt, S *xt, int64_t n, float sc) {
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i + 8 <= n) {
        float v[8], x[8];
        ld8(vt + i, v);
        ld8(xt + i, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = R<S>(x[j] - R<S>(v[j] * sc));
        st8(xt + i, x);
    } else {
        for (int64_t k = i; k < n; ++k) st1(xt + k, R<S>(ld1(xt + k) - R<S>(ld1(vt + k) * sc)));
    }
}


// ADG (Angle-based Dynamic Guidance, apg_guidance.py:107-180, apply_norm =
// False, apply_clip = True) fused with the Euler update.  Row-local over the
// 64 channels: one wave per (song, frame) row, lane = channel.  Precision
// chain of the reference: hats / diff in bf16; the angle in float64
// (call_cos_tensor on .to(float): per-element divide by the norm, then the
// dot); the perpendicular split in float32; the recombination in float64
// (masks applied by multiplication, so a 0/0 stays NaN exactly as in torch);
// the result cast float64 → float32 → bf16 (c10's double → BFloat16 path).
template <class S>
__global__ __launch_bounds__(256) void adg_euler_kernel(const S *__restrict__ vt,
                                                        S *__restrict__ xt, int B, int T,
                                                        float guidance, float sigma, float dt,
                                                        int out_mode) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= (int64_t)B * T) return;
    const int64_t i = row * 64 + lane;
    const float x = ld1(xt + i);
    const float vc = ld1(vt + i);
    const float vu = ld1(vt + (int64_t)B * T * 64 + i);
    const float ht = R<S>(x - R<S>(sigma * vc));
    const float hu = R<S>(x - R<S>(sigma * vu));
    const float diff = R<S>(ht - hu);
    // angle, float64
    const double na = sqrt(wave_sum_d((double)ht * (double)ht));
    const double nb = sqrt(wave_sum_d((double)hu * (double)hu));
    const double cs = wave_sum_d(((double)ht / na) * ((double)hu / nb));
    double w = (double)guidance - 1.0;
    w = w * (w > 0.0 ? 1.0 : 0.0) + 1e-3;
    const double clip = 3.14 / 6;
    const double th = acos(cs);
    const double thn = fmin(fmax(w * th, -clip), clip);
    // perpendicular component, float32
    const float dot = wave_sum(diff * hu);
    const float nsq = wave_sum(hu * hu);
    const float perp = diff - (dot / (nsq + 1e-8f)) * hu;
    // recombination, float64
    const double st = sin(th), sn = sin(thn);
    const double v_new = cos(thn) * (double)ht;
    const double p1 = (double)perp * sn / st * (st > 1e-3 ? 1.0 : 0.0);
    const float p2 = perp * (float)w * (st <= 1e-3 ? 1.0f : 0.0f);
    const double nw = v_new + (p1 + (double)p2);
    const float v = R<S>((float)(((double)x - nw) / (double)sigma));
    st1(xt + i, out_mode ? v : R<S>(x - R<S>(v * dt)));
}

}  // namespace

int adg_euler(const void *vt, void *xt, int B, int T, int C, float guidance, float sigma, float dt, int out_mode,
              bool f32, hipStream_t s) {
    if (C != 64) return fail(-1, "adg_euler: C must be 64");
    if (B <= 0 || T <= 0) return 0;
    const int64_t rows = (int64_t)B * T;
    const unsigned g = (unsigned)((rows + 3) / 4);
    if (f32) adg_euler_kernel<float><<<g, 256, 0, s>>>((const float *)vt, (float *)xt, B, T, guidance, sigma, dt, out_mode);
    else adg_euler_kernel<bf16_t><<<g, 256, 0, s>>>((const bf16_t *)vt, (bf16_t *)xt, B, T, guidance, sigma, dt, out_mode);
    HIP_TRY(hipGetLastError());
    return 0;
}

// Chunk partials of the APG norms: one buffer per (device, stream), so calls on different
// streams (or from different host threads, each on its own stream) never share scratch;
// the map is guarded.  A buffer only grows (hipFree waits for the device first).
static ApgPart *apg_workspace(size_t n, hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::pair<ApgPart *, size_t>> by_key;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto &e = by_key[{dev, s}];
    if (e.second < n) {
        if (e.first) (void)hipFree(e.first);
        e.first = nullptr;
        e.second = 0;
        if (hipMalloc(&e.first, n * sizeof(ApgPart)) != hipSuccess) return nullptr;
        e.second = n;
    }
    return e.first;
}

int apg_euler(const void *vt, void *xt, void *ra, int B, int T, int C, float guidance, float dt, int apply_cfg,
              int first_step, int out_mode, bool f32, hipStream_t s) {
    if (C != 64) return fail(-1, "apg_euler: C must be 64");
    if (B <= 0 || T <= 0) return 0;
    const int nch = (T + APG_TC - 1) / APG_TC;
    const dim3 g(C / 8, nch, B);
    if (apply_cfg <= 0) {
        if (f32) euler_rows_kernel<float><<<g, APG_TC, 0, s>>>((const float *)vt, (float *)xt, T, dt, out_mode);
        else euler_rows_kernel<bf16_t><<<g, APG_TC, 0, s>>>((const bf16_t *)vt, (bf16_t *)xt, T, dt, out_mode);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    ApgPart *part = apg_workspace((size_t)B * (C / 8) * nch, s);
    if (!part) return fail(-1, "apg_euler: workspace allocation failed");
#define APG_PHASES(S_)                                                                                       \
    apg_phase_kernel<S_, 1><<<g, APG_TC, 0, s>>>((const S_ *)vt, (S_ *)xt, (S_ *)ra, B, T, guidance, dt,     \
                                                 first_step, out_mode, part);                               \
    apg_phase_kernel<S_, 2><<<g, APG_TC, 0, s>>>((const S_ *)vt, (S_ *)xt, (S_ *)ra, B, T, guidance, dt,     \
                                                 first_step, out_mode, part);                               \
    apg_phase_kernel<S_, 3><<<g, APG_TC, 0, s>>>((const S_ *)vt, (S_ *)xt, (S_ *)ra, B, T, guidance, dt,     \
                                                 first_step, out_mode, part)
    if (f32) { APG_PHASES(float); }
    else { APG_PHASES(bf16_t); }
#undef APG_PHASES
    HIP_TRY(hipGetLastError());
    return 0;
}

int axpy(const void *vt, void *xt, int64_t n, float sc, bool f32, hipStream_t s) {
    if (n <= 0) return 0;
    const int64_t threads = (n + 7) / 8;
    const unsigned g = (unsigned)((threads + 255) / 256);
    if (f32) axpy_kernel<float><<<g, 256, 0, s>>>((const float *)vt, (float *)xt, n, sc);
    else axpy_kernel<bf16_t><<<g, 256, 0, s>>>((const bf16_t *)vt, (bf16_t *)xt, n, sc);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
