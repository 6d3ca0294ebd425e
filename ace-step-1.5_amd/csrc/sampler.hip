// sampler.hip — one fused base/sft sampler step per song.
//
// Restates reference base:1943-1979 with apg_forward / MomentumBuffer /
// project (acestep/models/base/apg_guidance.py:5-56):
//   diff = cond − uncond; ra = diff + (−0.75)·ra            (bf16 ops)
//   ‖ra‖₂ over T per channel → bf16; sf = min(1, bf16(2.5/‖ra‖)); v0 = bf16(ra·sf)
//   v1 = cond/max(‖cond‖,1e-12); par = Σ(v0·v1)·v1; orth = v0 − par   (float64)
//   vt = bf16(cond + bf16((g−1)·bf16(orth)));  xt = bf16(xt − bf16(vt·dt))
// The norms are global per-(song, channel) reductions over T, so one 1024-
// thread workgroup owns a song (64 channels × 16 row groups) and runs three
// L2-resident passes with LDS reductions in between: no host sync, no extra
// launches.  Data per song is 2.3 MB at 240 s — bandwidth-trivial.
#include "kernels.h"

namespace acehip {
namespace {

__global__ __launch_bounds__(1024) void apg_euler_kernel(const bf16_t *__restrict__ vt,
                                                         bf16_t *__restrict__ xt,
                                                         bf16_t *__restrict__ ra, int B, int T,
                                                         float guidance, float dt, int apply_cfg,
                                                         int first_step, int out_mode) {
    constexpr int C = 64, RG = 16;
    __shared__ float s_ss[RG][C];
    __shared__ double s_cs[RG][C];
    __shared__ double s_dot[RG][C];
    const int b = blockIdx.x;
    const int c = threadIdx.x & (C - 1), rg = threadIdx.x / C;
    const int64_t base = (int64_t)b * T * C;
    const bf16_t *cond = vt + base;
    const bf16_t *unc = vt + (int64_t)B * T * C + base;
    bf16_t *x = xt + base;
    if (apply_cfg <= 0) {
        // no CFG (vt is [B,T,C]) or outside the CFG interval (vt = cond)
        for (int t = rg; t < T; t += RG) {
            const int64_t i = (int64_t)t * C + c;
            const float v = bf2f(cond[i]);
            x[i] = out_mode ? cond[i] : f2bf(bf2f(x[i]) - rbf(v * dt));
        }
        return;
    }
    bf16_t *rab = ra + base;
    float ss = 0.f;
    double cs = 0.0;
    for (int t = rg; t < T; t += RG) {
        const int64_t i = (int64_t)t * C + c;
        const float cv = bf2f(cond[i]);
        const float diff = rbf(cv - bf2f(unc[i]));
        const float r = first_step ? diff : rbf(diff + rbf(-0.75f * bf2f(rab[i])));
        rab[i] = f2bf(r);
        const float rr = rbf(r);
        ss += rr * rr;
        cs += (double)cv * (double)cv;
    }
    s_ss[rg][c] = ss;
    s_cs[rg][c] = cs;
    __syncthreads();
    ss = 0.f;
    cs = 0.0;
#pragma unroll
    for (int g = 0; g < RG; ++g) { ss += s_ss[g][c]; cs += s_cs[g][c]; }
    const float nrm = rbf(sqrtf(ss));
    const float sf = fminf(1.0f, rbf(2.5f / nrm));
    const double denom = fmax(sqrt(cs), 1e-12);
    double dot = 0.0;
    for (int t = rg; t < T; t += RG) {
        const int64_t i = (int64_t)t * C + c;
        const double v0 = (double)rbf(bf2f(rab[i]) * sf);
        dot += v0 * ((double)bf2f(cond[i]) / denom);
    }
    s_dot[rg][c] = dot;
    __syncthreads();
    dot = 0.0;
#pragma unroll
    for (int g = 0; g < RG; ++g) dot += s_dot[g][c];
    const float gm1 = guidance - 1.0f;
    for (int t = rg; t < T; t += RG) {
        const int64_t i = (int64_t)t * C + c;
        const float cv = bf2f(cond[i]);
        const double v0 = (double)rbf(bf2f(rab[i]) * sf);
        const double v1 = (double)cv / denom;
        const float orth = rbf((float)(v0 - dot * v1));
        const float g = rbf(cv + rbf(gm1 * orth));
        x[i] = out_mode ? f2bf(g) : f2bf(bf2f(x[i]) - rbf(g * dt));
    }
}

__global__ void axpy_kernel(const bf16_t *vt, bf16_t *xt, int64_t n, float sc) {
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i + 8 <= n) {
        float v[8], x[8];
        unpack8(*(const uint4 *)(vt + i), v);
        unpack8(*(const uint4 *)(xt + i), x);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = x[j] - rbf(v[j] * sc);
        *(uint4 *)(xt + i) = pack8(x);
    } else {
        for (int64_t k = i; k < n; ++k) xt[k] = f2bf(bf2f(xt[k]) - rbf(bf2f(vt[k]) * sc));
    }
}

}  // namespace

int apg_euler(const bf16_t *vt, bf16_t *xt, bf16_t *ra, int B, int T, int C, float guidance,
              float dt, int apply_cfg, int first_step, int out_mode, hipStream_t s) {
    if (C != 64) return fail(-1, "apg_euler: C must be 64");
    if (B <= 0 || T <= 0) return 0;
    apg_euler_kernel<<<B, 1024, 0, s>>>(vt, xt, ra, B, T, guidance, dt, apply_cfg, first_step, out_mode);
    HIP_TRY(hipGetLastError());
    return 0;
}

int axpy_bf16(const bf16_t *vt, bf16_t *xt, int64_t n, float sc, hipStream_t s) {
    if (n <= 0) return 0;
    const int64_t threads = (n + 7) / 8;
    axpy_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(vt, xt, n, sc);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
