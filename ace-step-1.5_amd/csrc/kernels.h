// kernels.h — launchers for every device kernel of libacehip (internal C++ API).
#pragma once
#include "common.h"

namespace acehip {

// ----------------------------------------------------------------- knobs ---
// A/B switches (knobs.hip): read from the ACEHIP_* environment once, on first use or by
// acehip_reload_knobs(); gen counts reloads (part of the DiT graph key)
struct Knobs {
    int gemm_tailsplit = 1;   // ACEHIP_GEMM_TAILSPLIT: 0 off, 1 on
    int gemm_tail = 1;        // ACEHIP_GEMM_TAIL: tail-split tile (1: 128×256 ping-pong, 0: 128×128)
    int gemm_helpers = 1;     // ACEHIP_GEMM_HELPERS: LDS-DMA helper waves in the half-chip 4-wave tile
    int gemm_w4s = 1;         // ACEHIP_GEMM_W4S: half-chip grids on the four-wave 192×128 tile
    int gemm_hp128 = 1;       // ACEHIP_GEMM_HP128: 0 / 2 alternative cross-Q head-post paths
    int splitk_fuse = 1;      // ACEHIP_SPLITK_FUSE: split-K epilogues folded into their consumers
    int splitk_bn = 0;        // ACEHIP_SPLITK_BN: 0 auto, 64 / 128 forced
    int smallm_wholek = 2;    // ACEHIP_SMALLM_WHOLEK: M ≤ 128 SwiGLU on whole-K 128×64 tiles (2: + DMA helper waves, 1: without, 0: split-K)
    int attn_pw = 2;          // ACEHIP_ATTN_PW: layer kinds on attn_pw_kernel (1 full, 2 band, 4 cross)
    int attn_persist = 1;     // ACEHIP_ATTN_PERSIST: persistent band units
    int attn_pw_split = 24;   // ACEHIP_ATTN_PW_SPLIT: shortest KV loop whose tail units are split
    int attn_small = 1;       // ACEHIP_ATTN_SMALL: few-unit unmasked full / cross attention on attn_small_kernel (1 with KV parts, 2 without, 0 off)
    int attn_small_mask = 1;  // ACEHIP_ATTN_SMALL_MASK: key-padding-masked full attention (condition encoders) on attn_small_kernel too
    int attn_small_causal = 1; // ACEHIP_ATTN_SMALL_CAUSAL: unmasked causal attention (the text encoder) on attn_small_kernel too
    int attn_short_tpp = 3;   // ACEHIP_ATTN_SHORT_TPP: KV tiles per part of the short split
    int attn_cus = 0;         // ACEHIP_ATTN_CUS: CU count the splits plan for (0: the device's)
    int attn_streamk = 1;     // ACEHIP_ATTN_STREAMK: stream-K rounds for unmasked full / cross layers
    int fuse_rowadd = 1;      // ACEHIP_FUSE_ROWADD: null-row constant added in the MLP norm
    int dit_dedup = 1;        // ACEHIP_DIT_DEDUP: layer-0 CFG row dedup
    int dit_graph = 0;        // ACEHIP_DIT_GRAPH: HIP-graph replay of the forward body
    int attn_prio = 0;        // ACEHIP_ATTN_PRIO: attn_fwd_kernel<2> waves 4-7 at s_setprio 1 (the guide's static priority)
    int gemm_pp128 = 1;       // ACEHIP_GEMM_PP128: a one-round 192-row grid whose 128-row grid also fits one round runs on 128-row tiles
    int gemm_tailfuse = 1;    // ACEHIP_GEMM_TAILFUSE: the tail-split GEMM's main and tail grids in one launch
    int gemm_hp_tail = 1;     // ACEHIP_GEMM_HPTAIL: head-post GEMMs as a tail split (256-row main rounds + a 128-row tail round) where the cost model prefers it
    int convt = 1;            // ACEHIP_CONVT: 1 ConvTranspose (N % 256 == 0, padded input) as an implicit GEMM, 0 conv_gemm_kernel
    int conv7 = 2;            // ACEHIP_CONV7: k = 7 VAE convs — 2 implicit GEMM on the ping-pong tile (C ≥ 256, padded input), 1 halo-staged conv7_kernel
    int conv_bm128 = 2;       // ACEHIP_CONV_BM128: GEMM convs whose 256-row grid fills ≤ 1/2 of the chip on 128-row tiles, ≤ 1/4 on 64-row (2; 1: 128 only; 0: 256 always)
    int convp = 3;            // ACEHIP_CONVP: 0 none, 1 all, 2 k = 1 convs on convp_kernel, 3 k = 1 convs with N % 256 == 0 on the ping-pong GEMM (the rest on conv_gemm_kernel)
    int ru7 = 2;              // ACEHIP_RU7: C = 128 residual unit — 2 ru8_kernel (256-row tiles), 1 ru7_kernel, 0 conv7
    int vae_snake_in = 1;     // ACEHIP_VAE_SNAKE_IN: C = 128 decoder blocks without x_s tensors (ru8 SIN)
    int kv_group_kib = 262144; // ACEHIP_KV_GROUP_KIB: cross-K/V scratch bound at dit_create (tests force small groups)
    unsigned gen = 0;
};
const Knobs &knobs();

// ------------------------------------------------------------------ GEMM ---
// per-head post-projection: q/k RMSNorm (+RoPE) and scatter to head-major layouts
struct HeadPostArgs {
    const bf16_t *src; int64_t ld_src;   // rows [B*S]
    int B, S;
    int nq, nk, nv;                      // heads of each kind in the row (q | k | v)
    const bf16_t *qw, *kw;               // norm weights [128]
    const bf16_t *cos, *sin;             // [S][128] bf16 or null (no RoPE)
    bf16_t *q, *k, *v;                   // [B][nq|nk|nv][S_dst][128]
    int S_dst;
    float eps;
    // split-K input (gemm's small-M path): the projection is Σ_s part[s·plane + row·ld_src + col]
    // (fp32 partials summed in split order, then rounded to bf16) instead of src
    const float *part = nullptr; int splits = 0; int64_t plane = 0;
    int m_off = 0;                       // row of the full projection that GEMM row 0 is (tail-split grids)
};
enum GemmEpi {
    EPI_STORE = 0,       // C = bf16(acc + bias)
    EPI_GATED_RES = 1,   // C = bf16(res + bf16(bf16(acc) * gate[b][n]))   (AdaLN-Zero gated residual)
    EPI_RES = 2,         // C = bf16(res + bf16(acc))                       (plain residual)
    EPI_SWIGLU = 3,      // packed [gate|up] blocks of 32 rows → C[M, N/2] = bf16(silu(g)·u)
    EPI_HEADPOST = 4,    // bf16(acc) staged in LDS, then per-128-column head: q/k RMSNorm (+RoPE) and
                         // scatter to head-major [B][heads][S][128] (GemmArgs::hp); C unused
};


struct GemmArgs {
    const bf16_t *A; int64_t lda;   // [M, K]
    const bf16_t *W; int64_t ldw;   // [N, K]  (nn.Linear weight layout)
    bf16_t *C; int64_t ldc;         // output
    int M, N, K;
    int epi;
    const bf16_t *bias;             // [N] or null
    const bf16_t *res; int64_t ldr; // residual (may alias C)
    const bf16_t *gate; int64_t gate_bstride; int rows_per_batch;
    HeadPostArgs hp;                // EPI_HEADPOST only (rows of hp.B·hp.S; hp.src/ld_src unused)
    // split-K workspace (grids too small to fill the chip): fp32 partials [splits][M][N]
    // + a bf16 [M][N] staging tile for the head-post case; null disables split-K
    void *ws; size_t ws_bytes;
    int kper;                       // internal: K-tiles per split (EPI_PARTIAL launches)
    // EPI_CONV (gemm_conv only): a VAE convolution as an implicit GEMM.  Tap t = k / conv_cin
    // reads A(m, k) = in[m + conv_a0 + t·conv_dil][k % conv_cin] (A = in, lda = conv_cin; the
    // caller provides zero rows around the input).  Column n is output channel n % conv_cout of
    // phase p = n / conv_cout (a ConvTranspose's phases side by side: W = the packed
    // [phases][conv_cout][taps·cin] taps); row m lands on output row m·conv_ostride + conv_ooff + p
    // when that lies in [0, conv_lout): raw bf16(acc + bias) — or bf16(res + bf16(acc + bias)) with
    // a residual (one phase; res may alias C) — to C (if set), its Snake (sa / sib) to Cs (if
    // set), both with row pitch ldc = conv_cout
    const float *sa, *sib;
    bf16_t *Cs;
    int conv_cin, conv_dil, conv_a0, conv_ostride, conv_ooff, conv_cout;
    int64_t conv_lout;
};
constexpr int EPI_PARTIAL = 5;                       // internal: fp32 partials of split blockIdx.y → ws
constexpr int EPI_CONV = 6;                          // the VAE's implicit-GEMM convs (gemm_conv)
constexpr size_t GEMM_WS_BYTES = (size_t)48 << 20;   // runtimes' split-K workspace
struct RowAdd;
// defer != null: a residual-epilogue GEMM (EPI_GATED_RES / EPI_RES) that takes the small-M
// split-K path leaves its fp32 partials in a.ws and describes its epilogue in *defer (the
// consumer rmsnorm_mod applies it, one launch fewer); defer->part stays null otherwise
int gemm(const GemmArgs &a, hipStream_t s, RowAdd *defer = nullptr);
int gemm_variant(const GemmArgs &a, int variant, hipStream_t s);   // tuning / tests
// VAE convolutions (k = 7 dilated, ConvTranspose phases) on the two-phase ping-pong tile
// (EPI_CONV; the caller provides the input's zero halo rows)
int gemm_conv(const GemmArgs &a, hipStream_t s);
// Launch-attached timing events for the next GEMM of this thread (the SwiGLU paths: ping-pong,
// generic and four-wave tiles): its first launch takes `start`, every launch `stop` (the last
// completion wins), by hipExtLaunchKernel — no separate event packets in the stream.
// gemm_ext_events(nullptr, nullptr) disarms; it returns whether `start` was consumed.
bool gemm_ext_events(hipEvent_t start, hipEvent_t stop);

// --------------------------------------------------------------- small ops --
// y[m][n] = bf16(Σ_k act(x[m][k])·W[n][k] + b[n]); act: 0 none, 1 bf16(silu(x)); M ≤ 16
// act_scratch (≥ M·K elements): with act, bf16(silu(x)) is formed there once first
int gemv_small(const bf16_t *x, int64_t ldx, const bf16_t *W, const bf16_t *bias, bf16_t *y,
               int64_t ldy, int M, int N, int K, int act, hipStream_t s, bf16_t *act_scratch = nullptr);
// sinusoid of bf16(t*1000): emb[b][0:128]=cos, [128:256]=sin, as bf16 (base:225-246)
// dst[r][0..n) = src[0..n) for r < rows (n % 8 == 0)
int bcast_rows(const bf16_t *src, int64_t n, bf16_t *dst, int rows, hipStream_t s);
int timestep_sinusoid(const float *t, const float *t_r, int t_stride, int use_diff, int Bc,
                      const float *freqs, bf16_t *emb, hipStream_t s);
// out = bf16(a + b) elementwise
int add_bf16(const bf16_t *a, const bf16_t *b, bf16_t *out, int64_t n, hipStream_t s);
// mod[l][b][j][d] = bf16(table[l][j][d] + proj[b][j][d]) for all layers
int modulation(const bf16_t *tables, int n_tables, int rows, const bf16_t *proj, int Bc, int D,
               bf16_t *mod, hipStream_t s);
// proj_in input pack: X[b][s][k*192+c] = (c<128 ? ctx : xt)[b % Bx][2s+k][..] or 0
int pack_patches(const bf16_t *xt, const bf16_t *ctx, int Bx, int Bc, int T, int S, bf16_t *X,
                 hipStream_t s);
// out[h·128 + d] = V[h / (H/KV)][0][d]  (row 0 of each KV head, V [KV][Le][128])
int gather_head_row(const bf16_t *V, int KV, int Le, int H, bf16_t *out, hipStream_t s);
// X[r][:] = bf16(X[r][:] + c[:]) for rows r < rows (c bf16 [D])
int add_row_bcast(bf16_t *X, const bf16_t *c, int rows, int D, hipStream_t s);
// dst[m][0:C] = src[m][0:C] (row-strided column block copy)
int copy_cols(const bf16_t *src, int64_t lds, bf16_t *dst, int64_t ldd, int M, int C, hipStream_t s);
// crop [Bc][2S][64] → [Bc][T][64]
int crop_rows(const bf16_t *src, int Bc, int rows_src, int rows_dst, int C, bf16_t *dst,
              hipStream_t s);

// ---------------------------------------------------------------- norms ----
// out[m] = AdaLN or plain RMSNorm of x[m] (rows of D):
//   plain: bf16(w · bf16(x·rsqrt(mean x²+eps)))
//   mod:   bf16(bf16(plain · bf16(1+scale[b])) + shift[b])
// optional row add fused into rmsnorm_mod: rows >= from first become x = bf16(x + v[D]),
// written back to xw (== x)
struct RowAdd {
    bf16_t *xw = nullptr;
    const bf16_t *v = nullptr;
    int from = 0;
    // deferred split-K residual epilogue (gemm(..., defer)): rows < prows first become
    // x = bf16(x + bf16(bf16(acc)·gate[row / gate_rpb])) (gate != null) or bf16(x + bf16(acc)),
    // acc = Σ_s part[s·plane + row·D + col] in split order — the splitk epilogue's arithmetic
    const float *part = nullptr;
    int splits = 0, prows = 0;
    int64_t plane = 0;
    const bf16_t *gate = nullptr;
    int64_t gate_bstride = 0;
    int gate_rpb = 1;
};
// rows_per_wave: kernel variant (tests / micro-bench: 1, 2, 4 rows per wave, −2 / −4 waves
// per row); 0 = the default (1)
int rmsnorm_mod(const bf16_t *x, const bf16_t *w, const bf16_t *shift, const bf16_t *scale,
                int64_t mod_bstride, int rows_per_batch, bf16_t *out, int M, int D, float eps,
                hipStream_t s, RowAdd ra = RowAdd{}, int rows_per_wave = 0);
int head_post(const HeadPostArgs &a, hipStream_t s);

// ------------------------------------------------------------- attention ---
// ws: attention_ws_bytes() of zero-initialised device memory (tail-split partials
// + self-resetting counters), or null to disable tail balancing.
// kmask: optional key-padding mask [B][Sk] (1 = attend), encoder semantics (attention.hip header)
// window: < 0 full, >= 0 band |i−j| <= window, ATTN_CAUSAL keys j <= i (Qwen3 text encoder)
constexpr int ATTN_CAUSAL = -2;
int attention(const bf16_t *q, const bf16_t *k, const bf16_t *v, bf16_t *o, int B, int H, int KV,
              int Sq, int Sk, int window, float scale, int64_t o_ld, void *ws, hipStream_t s,
              const uint8_t *kmask = nullptr);
size_t attention_ws_bytes();

// --------------------------------------------------------------- sampler ---
// element type bf16 (f32 = false) or fp32 (the parity mode)
int apg_euler(const void *vt, void *xt, void *ra, int B, int T, int C, float guidance, float dt, int apply_cfg,
              int first_step, int out_mode, bool f32, hipStream_t s);
int axpy(const void *vt, void *xt, int64_t n, float sc, bool f32, hipStream_t s);
int adg_euler(const void *vt, void *xt, int B, int T, int C, float guidance, float sigma, float dt, int out_mode,
              bool f32, hipStream_t s);

// ------------------------------------------------------------------ FSQ ----
struct FsqLevels { int n; int L[8]; };
// z [M][ldz] bf16 (first n columns) → codes [M][ldc ≥ 64] bf16 (columns ≥ n zeroed), idx [M] (or null)
int fsq_quantize(const bf16_t *z, int64_t ldz, int M, const FsqLevels &lv, bf16_t *codes, int64_t ldc, int *idx,
                 hipStream_t s);
int fsq_codes_from_indices(const int *idx, int M, const FsqLevels &lv, bf16_t *codes, int64_t ldc, hipStream_t s);

// ------------------------------------------------------ fp32 parity mode ---
// (f32.hip) the DiT forward with no bf16 rounding, SURVEY §8c(iii)
struct GemmF32Args {
    const float *A; int64_t lda;     // [M, K]
    const float *W; int64_t ldw;     // [N, K]
    float *C; int64_t ldc;
    int M, N, K;
    int epi;                          // EPI_STORE / EPI_GATED_RES / EPI_RES
    const float *bias;
    const float *res; int64_t ldr;
    const float *gate; int64_t gate_bstride; int rows_per_batch;
};
int gemm_f32(const GemmF32Args &a, hipStream_t s);
struct HeadPostF32Args {
    const float *src; int64_t ld_src;
    int B, S, nq, nk, nv;
    const float *qw, *kw, *cos, *sin;
    float *q, *k, *v;
    int S_dst;
    float eps;
};
int head_post_f32(const HeadPostF32Args &a, hipStream_t s);
struct AttnF32Args {
    const float *q, *k, *v;           // [B][H|KV][S][128]
    float *o; int64_t o_ld;           // [B][Sq][o_ld], head h at column h·128
    int B, H, KV, Sq, Sk, window;
    float scale;
};
int attention_f32(const AttnF32Args &a, hipStream_t s);
int rmsnorm_f32(const float *x, const float *w, const float *shift, const float *scale, int64_t mod_bstride,
                int rows_per_batch, float *out, int M, int D, float eps, hipStream_t s);
int gemv_f32(const float *x, int64_t ldx, const float *W, const float *bias, float *y, int64_t ldy, int M, int N,
             int K, int act, hipStream_t s);
int timestep_sinusoid_f32(const float *t, const float *t_r, int t_stride, int use_diff, int Bc, const float *freqs,
                          float *emb, hipStream_t s);
int add_f32(const float *a, const float *b, float *o, int64_t n, hipStream_t s);
int modulation_f32(const float *tables, int n_tables, int rows, const float *proj, int Bc, int D, float *mod,
                   hipStream_t s);
int pack_patches_f32(const float *xt, const float *ctx, int Bx, int Bc, int T, int S, float *X, hipStream_t s);
int crop_rows_f32(const float *src, int Bc, int rows_src, int rows_dst, int C, float *dst, hipStream_t s);
int swiglu_f32(const float *g, const float *u, float *o, int64_t n, hipStream_t s);

// ----------------------------------------------------------------- misc ----
// per song b: peak = max |wav[b]|; if peak > 1, wav[b] /= peak (n samples per song, n % 4 == 0)
// decode guard (when guard != 0) then normalize_audio (when target_amp > 0), see small.hip
int wav_peak_normalize(float *wav, int B, int64_t n, float *peak, hipStream_t s, float target_amp = 0.f,
                       int guard = 1);
int wav_postprocess_pcm16(float *wav, int B, int C, int64_t N, float *peak, hipStream_t s, float target_amp,
                          int guard, short *pcm);
int cast_f32_bf16(const float *src, bf16_t *dst, int64_t n, hipStream_t s);

}  // namespace acehip
