// conv.h — implicit-GEMM convolution arguments (see conv.hip).
#pragma once
#include "common.h"

namespace acehip {

// out[m·c_stride + c_off + phase][n] = Σ_{tap,ci} in[m·a_stride + tap·dil + a_off][ci] · W_phase[n][tap·Cin + ci] (+bias[n]) (+res)
// epilogue writes the raw value to `out` and/or Snake(raw) (params sa = e^α/(2π),
// sib = 1/(e^β+1e-9)) to `out_s` — the activation the NEXT convolution consumes.
struct ConvArgs {
    const bf16_t *in; int64_t L_in; int Cin;     // NLC input [L_in][Cin]
    const bf16_t *W; int64_t w_pstride;          // packed [phases][N][taps·Cin]
    const bf16_t *bias;                          // [N] or null
    bf16_t *out;                                 // raw output [L_out][N] or null
    bf16_t *out_s; const float *sa, *sib;        // snaked output or null
    const bf16_t *res;                           // residual [L_out][N] or null (may alias out)
    int64_t L_out; int N;
    int64_t M;                                   // GEMM rows per phase
    int taps, dil, a_stride, a_off, c_stride, c_off;
    const bf16_t *zero;                          // ≥ 128 B of zeros (im2col padding source)
    // in is a VAE activation buffer: ≥ kActPadRows zero rows before row 0 and addressable rows
    // after L_in (the k = 7 conv may then run as an implicit GEMM on the ping-pong tile, which
    // reads its halo rows from there; ACEHIP_CONV7=2)
    int in_halo = 0;
};
// fused residual unit at C = 128: c1 = the k=7 conv (in = x_s, sa/sib = snake2,
// bias = b1); then x' = x + (W2·y_s + b2), written raw into x (keep_raw) and
// snaked (sa_next/sib_next) into out_s
// zero rows (of the widest stage, 2048 channels) kept in front of the VAE activation buffers:
// the persistent residual-unit kernel reads the k=7 halo rows before the start from them
constexpr int kActPadRows = 32;
// rows past L that a C = 128 residual-unit window may read (ru8_kernel: a 310-row window from
// m0 - 3·dil of the last 256-row tile, so up to L + 306): the back pad of every activation
// buffer covers at least this many 128-channel rows whatever the widest stage is
constexpr int kResWindowBackRows = 320;
struct ResUnitArgs {
    ConvArgs c1;
    const bf16_t *W2, *b2;
    const bf16_t *W2p;                           // W2 with columns permuted (permute_k1_weight) or null
    int in_zero_pad;                             // c1.in is preceded by ≥ kActPadRows zero rows (ru7_kernel)
    bf16_t *x;
    bf16_t *out_s;
    const float *sa_next, *sib_next;
    int keep_raw;
    // snake_in (ru8_kernel only): c1.in is the RAW x (= x); the unit's first Snake (sa_in / sib_in)
    // is applied while the window is staged, so no x_s tensor exists; keep_raw then writes x' to
    // x_out (a different buffer: neighbouring tiles' windows still read x), else out_s as usual
    int snake_in = 0;
    const float *sa_in = nullptr, *sib_in = nullptr;
    bf16_t *x_out = nullptr;
};
int resunit128(const ResUnitArgs &u, hipStream_t s);
// W2 [n_rows][128] → columns permuted within each 32-block so that the k=7 accumulator
// layout is the k=1 MFMA's B operand (ru7_kernel): new 8g+e ← old e<4 ? 4g+e : 16+4g+e−4
int permute_k1_weight(const bf16_t *w, bf16_t *wp, int n_rows, hipStream_t s);
int conv_gemm(const ConvArgs &a, int phases, hipStream_t s);
// final decoder conv: snaked NLC [L][Cin] → fp32 channels-first [Cout=2][L], k 7, no bias;
// w [7][Cin][2] (the two output channels adjacent), Cin = 128
int conv_out(const bf16_t *in_s, int64_t L, int Cin, const float *w, int Cout, float *out, hipStream_t s);
// encoder first conv: channels-first [Cin≤2][N] → raw + snaked NLC [N][Cout], k 7, bias
int conv_in(const bf16_t *in, int64_t N, int Cin, const float *w, const float *bias, int Cout,
            bf16_t *out, bf16_t *out_s, const float *sa, const float *sib, hipStream_t s);
int cf_to_nlc(const bf16_t *in, int C, int64_t L, bf16_t *out, hipStream_t s);
int gauss_sample(const bf16_t *h, int64_t T, int C, const bf16_t *eps, bf16_t *z, hipStream_t s);
// weight-norm fusion + implicit-GEMM packing: w = g·v/‖v‖ (norm over all dims but 0)
//   conv  v [Cout][Cin][k]  → Wp[co][tap·Cin+ci]
//   convT v [Cin][Cout][2s] → Wp[r][co][tap·Cin+ci], tap0 = kernel r+s (input m−1), tap1 = kernel r
int pack_conv_weight(const bf16_t *v, const bf16_t *g, int d0, int d1, int k, int transposed,
                     int stride, bf16_t *Wp, hipStream_t s);
// same fusion into fp32 [Cout][k][Cin] (for conv_out) or [Cout][Cin][k] (conv_in) layouts
int fuse_conv_weight_f32(const bf16_t *v, const bf16_t *g, int d0, int d1, int k, int k_major,
                         float *w, hipStream_t s);
int snake_params(const bf16_t *alpha, const bf16_t *beta, int C, float *sa, float *sib, hipStream_t s);
int cast_bf16_f32(const bf16_t *src, float *dst, int64_t n, hipStream_t s);

}  // namespace acehip
