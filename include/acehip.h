/*
 * acehip.h — C ABI of libacehip.so, the MI355X (gfx950) implementation of the
 * ACE-Step 1.5 hot path: the DiT flow-matching denoise step and the Oobleck
 * VAE decode/encode.
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes. No
 * torch types cross this boundary.  All tensors are caller-owned, contiguous,
 * device-resident buffers (e.g. torch.Tensor.data_ptr()); the library owns the
 * packed weights, the cross-attention K/V cache and the workspace (sized at
 * create time from the max_* fields).  Nothing is allocated inside
 * forward/decode/encode calls.  Two calls allocate, once, outside the hot loop:
 *   - acehip_sampler_apg_euler keeps its norm partials in a library-owned
 *     workspace per (device, stream), allocated on the first call on that stream
 *     and grown (hipFree + hipMalloc) only when a larger B*T arrives;
 *   - acehip_dit_set_timesteps uses buffers allocated at finalize for 64 steps;
 *     a longer schedule (the reference builds <= 60) synchronises the stream and
 *     grows them once.
 * Work is enqueued on the caller's stream (hipStream_t passed as void*); apart from
 * that growth no entry point synchronises the host.
 *
 * Threading: a handle is bound to one device and is not re-entrant; every
 * entry point calls hipSetDevice(handle->device) first because callers (the
 * reference API server's ThreadPoolExecutor, reference
 * acestep/api_server.py:1291-1292) may call from any thread.
 *
 * Errors: 0 = ok; negative = error class; acehip_last_error() returns the
 * thread-local message of the last failing call.
 *
 * Each entry point names the reference interface it replaces (file:line in
 * the reference checkout).
 */
#ifndef ACEHIP_H
#define ACEHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 100: round-1 ABI.  200: dtype argument on acehip_dit_forward and the three sampler
 * entry points, acehip_dit_cfg.fp32 (round 2).  300: acehip_vae_encode accepts any
 * N in [hop, max_T*hop] (latents = floor(N/hop) frames).  Callers check
 * acehip_get_version() == ACEHIP_VERSION before binding (acehip/_ffi.py does). */
#define ACEHIP_VERSION 400

enum acehip_status {
    ACEHIP_OK = 0,
    ACEHIP_E_ARG = -1,          /* bad argument / shape */
    ACEHIP_E_OOM = -2,          /* device allocation failed */
    ACEHIP_E_HIP = -3,          /* HIP runtime error */
    ACEHIP_E_STATE = -4,        /* not finalized / condition not set */
    ACEHIP_E_NAME = -5          /* unknown weight name */
};

enum acehip_dtype { ACEHIP_F32 = 0, ACEHIP_BF16 = 1 };

int acehip_get_version(void);
/* Re-read the ACEHIP_* A/B switches from the environment (they are read once, on first
 * use, otherwise).  Tests and A/B tools only: call while no other thread is inside the
 * library; a DiT handle re-captures its HIP graph after a reload. */
int acehip_reload_knobs(void);
const char *acehip_last_error(void);
/* Content hash of the native sources the library was built from (the .hip and .h files under
 * csrc/ and include/; ace-step-1.5_amd/csrc/native_hash.py).  acehip/_ffi.py refuses a library whose
 * hash differs from the sources beside it, so a shipped binary is provably the tree's. */
const char *acehip_build_hash(void);

/* ---------------------------------------------------------------- DiT ---- */

/* Hyper-parameters (reference AceStepConfig,
 * acestep/models/base/configuration_acestep_v15.py:148-260). */
typedef struct acehip_dit_cfg {
    int hidden;          /* 2048 */
    int intermediate;    /* 6144 */
    int heads;           /* 16 */
    int kv_heads;        /* 8 */
    int head_dim;        /* 128 (the kernels require 128) */
    int layers;          /* 24 */
    int window;          /* 128: sliding layers attend |i-j| <= window */
    int patch;           /* 2 */
    int in_channels;     /* 192 = context 128 + latent 64 */
    int out_channels;    /* 64 */
    float eps;           /* 1e-6 */
    float rope_theta;    /* 1e6 */
    int max_S;           /* max tokens per batch row (T/patch) */
    int max_Bc;          /* max DiT batch (2x songs with CFG) */
    int max_Lenc;        /* max encoder sequence length */
    const uint8_t *sliding; /* [layers] 1 = sliding layer; NULL = even idx */
    int fp32;            /* 0: the bf16 production path; 1: the fp32 parity mode (SURVEY
                          * §8c(iii)) — fp32 weights, activations and accumulation, the
                          * reference's fp32 forward (init_service_orchestrator.py:51 runs
                          * fp32 off cuda/xpu); set_condition / forward then take fp32 */
} acehip_dit_cfg;

typedef struct acehip_dit acehip_dit;

/* replaces: AutoModel.from_pretrained(...).to(device).to(dtype)
 * (acestep/core/generation/handler/init_service_loader.py:56-89) */
int acehip_dit_create(int device, const acehip_dit_cfg *cfg, acehip_dit **out);

/* One reference state-dict tensor by its HF name without the "decoder."
 * prefix (e.g. "layers.3.mlp.gate_proj.weight").  Copies and
 * repacks; the caller keeps ownership of ptr.  dtype: ACEHIP_F32/BF16.
 * Precedent: acestep/models/mlx/dit_convert.py:11-66. */
int acehip_dit_set_weight(acehip_dit *h, const char *name, const void *ptr, int dtype,
                          int ndim, const int64_t *shape, int on_device);

/* Validates that every tensor is present; builds fused layouts. */
int acehip_dit_finalize(acehip_dit *h);

/* condition_embedder + per-layer cross-attention K/V cache.
 * replaces: the first-step branch of AceStepAttention.forward
 * (acestep/models/base/modeling_acestep_v15_base.py:310-325, :1359).
 * enc: [Bc, Lenc, hidden] in the handle's dtype (CFG: cond rows then null rows). */
int acehip_dit_set_condition(acehip_dit *h, const void *enc, int Bc, int Lenc, void *stream);

/* Declare batch rows [first_row, Bc) of the current condition uniform: their
 * encoder sequence is ONE vector repeated (the CFG null rows,
 * null_condition_emb.expand_as, base:1907).  The decoder never masks encoder
 * positions (base:1384-1385), so such a row's cross-attention softmax is
 * exactly uniform and its output is V row 0 for every query; forward then
 * skips the cross-Q projection / attention / cross-O GEMM for those rows and
 * adds the per-layer constant cross-O output (precomputed here).  first_row ==
 * Bc turns it off; set_condition resets it. */
int acehip_dit_set_uniform_rows(acehip_dit *h, int first_row, void *stream);

/* One decoder forward: AceStepDiTModel.forward
 * (acestep/models/base/modeling_acestep_v15_base.py:1303-1507).
 * xt: bf16 [Bx, T, 64]; ctx: bf16 [Bx, T, 128]; batch row b of the DiT reads
 * xt/ctx row (b % Bx) — CFG's cat([xt, xt]) without a copy (base:1929).
 * t, t_r: device fp32 [Bc] holding model-dtype values; t_stride 0
 * broadcasts element 0.  vt_out: [Bc, T, 64].  dtype is the
 * element type of xt / ctx / vt_out and must be the handle's: ACEHIP_BF16
 * (production) or ACEHIP_F32 (a handle created with cfg.fp32 = 1). */
int acehip_dit_forward(acehip_dit *h, const void *xt, const void *ctx, int Bx,
                       const float *t, const float *t_r, int t_stride, int Bc, int T,
                       int dtype, void *vt_out, void *stream);

/* Timestep MLPs of a whole schedule at once: t, t_r are device fp32 arrays of n_steps
 * entries, one broadcast timestep pair per step (the t-dependent part of
 * AceStepDiTModel.forward, base:1340-1344, evaluated for every step of the sampler loop
 * base:1936 / turbo:1968 up front).  acehip_dit_forward_step(step) is then
 * acehip_dit_forward with t = t[step], t_r = t_r[step], t_stride 0, except that the ~108 MB
 * of timestep-MLP weights are read once per schedule instead of once per step — bit-
 * identical (each MLP row is computed by the same instruction sequence).  bf16 handles. */
int acehip_dit_set_timesteps(acehip_dit *h, const float *t, const float *t_r, int n_steps, void *stream);
int acehip_dit_forward_step(acehip_dit *h, const void *xt, const void *ctx, int Bx, int step, int Bc, int T,
                            int dtype, void *vt_out, void *stream);

/* Replay the pointer-independent middle of acehip_dit_forward (timestep MLPs,
 * modulation, proj_in, the layer stack, norm_out) as one HIP graph, captured
 * once per (Bc, S, Lenc, uniform rows) and re-captured when they change or
 * after finalize.  Default off (ACEHIP_DIT_GRAPH=1 turns it on at create):
 * measured neutral on MI355X (0.600 vs 0.602 s/song, turbo 10 s 38.8 vs
 * 39.2 ms) — kernel-to-kernel gaps are not launch-bound here.  Profiling runs
 * the eager path.  Results are bit-identical either way. */
int acehip_dit_set_graph(acehip_dit *h, int enable);

int acehip_dit_destroy(acehip_dit *h);

/* Per-kernel HIP-event timing inside acehip_dit_forward (for the bench's
 * roofline numbers).  enable != 0 clears the counters and starts recording
 * an event pair around every launch of the listed kernel families on the
 * forward's stream; read after the caller synchronised that stream.
 * kind: 0 SwiGLU gate/up GEMM, 1 down GEMM, 2 QKV GEMM, 3 O/cross-O GEMMs,
 *       4 full self-attention, 5 band self-attention, 6 cross-attention. */
int acehip_dit_profile(acehip_dit *h, int enable);
int acehip_dit_profile_read(acehip_dit *h, int kind, int *launches, float *total_ms);
/* Restrict recording to the kinds whose bit is set (default 0x7f = all): the
 * bench times only the roofline kernel inside its timed region. */
int acehip_dit_profile_kinds(acehip_dit *h, unsigned mask);

/* --------------------------------------------------- condition encoders ---- */

/* One stack of AceStepEncoderLayer (reference base:374-440) with its
 * embed_tokens Linear, final Qwen3RMSNorm and optional proj_out Linear — the
 * shape shared by AceStepLyricEncoder (base:577-731), AceStepTimbreEncoder
 * (base:997-1178), AttentionPooler (base:734-859) and AudioTokenDetokenizer
 * (base:862-994).  The host composes them into AceStepConditionEncoder
 * (base:1509-1554; pack_sequences base:138-169 is index plumbing). */
typedef struct acehip_enc_cfg {
    int hidden;          /* 2048 */
    int intermediate;    /* 6144 */
    int heads;           /* 16 */
    int kv_heads;        /* 8 */
    int head_dim;        /* 128 */
    int layers;          /* lyric 8, timbre 4, pooler/detokenizer 2 */
    int window;          /* 128 (sliding layers: |i-j| <= window) */
    int in_dim;          /* embed_tokens in-features (lyric/text 1024, timbre 64, pooler 2048) */
    int embed_bias;      /* 1: embed_tokens has a bias */
    int out_dim;         /* proj_out out-features (detokenizer 64), 0 = none; <= 128 */
    float eps;           /* 1e-6 */
    float rope_theta;    /* 1e6 */
    int max_tokens;      /* max B*S per forward */
    int max_S;           /* max sequence length */
    const uint8_t *sliding; /* [layers] 1 = sliding layer, 2 = causal (Qwen3
                             * text encoder, Qwen3Model's default mask); NULL = even idx */
} acehip_enc_cfg;

typedef struct acehip_enc acehip_enc;

int acehip_enc_create(int device, const acehip_enc_cfg *cfg, acehip_enc **out);
/* Names relative to the module, as in its state dict: "embed_tokens.weight",
 * "layers.3.self_attn.q_proj.weight", "layers.3.input_layernorm.weight",
 * "norm.weight", "proj_out.bias" ...  dtype ACEHIP_F32/BF16. */
int acehip_enc_set_weight(acehip_enc *h, const char *name, const void *ptr, int dtype, int ndim,
                          const int64_t *shape, int on_device);
int acehip_enc_finalize(acehip_enc *h);
/* embed_tokens: out bf16 [M, hidden] = x bf16 [M, in_dim] · Wᵀ (+ b)
 * (base:623, :1085, :766, :895). */
int acehip_enc_embed(acehip_enc *h, const void *x, int M, void *out, void *stream);
/* layers + norm (+ proj_out): x bf16 [B, S, hidden] (not modified) →
 * out bf16 [B, S, out_dim ? out_dim : hidden].  kmask: device uint8 [B, S]
 * key-padding mask (1 = attend; create_4d_mask semantics, base:56-135) or
 * NULL (no padding mask).  RoPE positions 0..S-1 per sequence. */
int acehip_enc_forward(acehip_enc *h, const void *x, const uint8_t *kmask, int B, int S, void *out,
                       void *stream);
int acehip_enc_destroy(acehip_enc *h);

/* FSQ quantizer of the audio tokenizer (ResidualFSQ, 1 quantizer, levels
 * {8,8,8,5,5,5}: base:1196-1200; vector_quantize_pytorch FSQ restated, see
 * oracle/condenc_oracle.py): z bf16 [M, ldz] (the project_in output, first
 * n_levels columns) → codes bf16 [M, ldc >= 64] (columns >= n_levels zeroed, so
 * the padded project_out GEMM can consume them) and int32 indices [M] (or NULL). */
int acehip_fsq_quantize(const void *z, int ldz, int M, const int *levels, int n_levels, void *codes, int ldc,
                        int32_t *indices, void *stream);
/* FSQ.indices_to_codes (quantizer.get_output_from_indices before project_out,
 * acestep/core/generation/handler/audio_codes.py:62). */
int acehip_fsq_codes_from_indices(const int32_t *indices, int M, const int *levels, int n_levels, void *codes,
                                  int ldc, void *stream);

/* ------------------------------------------------------------ sampler ---- */

/* One base/sft CFG step: cond/uncond split + APG (momentum -0.75, norm clip
 * 2.5 over T, float64 projection) + Euler ODE update, fused.
 * replaces: base:1943-1979 + acestep/models/base/apg_guidance.py:5-56.
 * vt: bf16 [2B, T, 64] (cond rows then uncond rows); xt: bf16 [B, T, 64]
 * updated in place; ra: bf16 [B, T, 64] momentum state (first_step != 0
 * means running_average == 0); apply_cfg == 0 → vt = cond (no momentum
 * update), apply_cfg < 0 → no CFG (vt is [B,T,64]).  dt: bf16 value.
 * out_mode 0: xt = bf16(xt − bf16(v·dt)) (ODE);  out_mode 1: xt = v (the
 * guided velocity, for the caller's SDE branch, base:1968-1973).
 * dtype: ACEHIP_BF16 (every op rounded to bf16 as torch does) or ACEHIP_F32 (the
 * fp32 parity mode: the same chain unrounded) for vt / xt / ra.
 * The norms' chunk partials live in a library-owned workspace per (device,
 * stream), allocated on first use under a lock: concurrent calls on different
 * streams are independent; calls on one stream are ordered by that stream. */
int acehip_sampler_apg_euler(const void *vt, void *xt, void *ra, int B, int T, int C,
                             float guidance, float dt, int apply_cfg, int first_step,
                             int out_mode, int dtype, void *stream);

/* One base/sft CFG step with ADG guidance (use_adg=True) + Euler, fused.
 * replaces: base:1958-1964 + adg_forward (apg_guidance.py:107-180, angle clip
 * pi/6, no norm).  vt: bf16 [2B, T, 64] cond then uncond; xt: bf16 [B, T, 64]
 * updated in place; sigma: t_curr (bf16 value).  Row-local (no reduction over
 * T).  The reference only supports B == 1 (its [N*T,1] x [N,T,C] broadcast);
 * this computes the per-row generalisation for any B.  out_mode as above. */
int acehip_sampler_adg_euler(const void *vt, void *xt, int B, int T, int C, float guidance,
                             float sigma, float dt, int out_mode, int dtype, void *stream);

/* xt = bf16(xt - bf16(vt * s)) on [n] elements — Euler ODE (turbo:1985-1991)
 * and the final x0 = xt - vt*t (turbo:1975-1977); dtype as above. */
int acehip_sampler_axpy(const void *vt, void *xt, int64_t n, float s, int dtype, void *stream);

/* ---------------------------------------------------------------- VAE ---- */

/* diffusers AutoencoderOobleck config (acestep/models/mlx/vae_model.py:251-281) */
typedef struct acehip_vae_cfg {
    int encoder_hidden;  /* 128 */
    int decoder_channels;/* 128 */
    int latent_channels; /* 64 */
    int audio_channels;  /* 2 */
    int n_blocks;        /* 5 */
    int ratios[8];       /* downsampling ratios, e.g. {2,4,4,6,10} */
    int multiples[8];    /* channel multiples, e.g. {1,2,4,8,16} */
    int max_T;           /* max latent frames per decode */
    int max_B;
    int with_encoder;
} acehip_vae_cfg;

typedef struct acehip_vae acehip_vae;

/* replaces: AutoencoderOobleck.from_pretrained (init_service_loader.py:123-144) */
int acehip_vae_create(int device, const acehip_vae_cfg *cfg, acehip_vae **out);
/* diffusers names: "decoder.block.2.res_unit1.conv1.weight_g" etc.; both the
 * weight_g/weight_v and parametrizations.weight.original{0,1} spellings. */
int acehip_vae_set_weight(acehip_vae *h, const char *name, const void *ptr, int dtype,
                          int ndim, const int64_t *shape, int on_device);
/* fuses weight_g·v/||v|| and repacks every conv into implicit-GEMM layout */
int acehip_vae_finalize(acehip_vae *h);

/* vae.decode(z).sample (acestep/core/generation/handler/vae_decode_chunks.py:42)
 * z: bf16 [B, 64, T] → wav fp32 [B, 2, T*hop]; untiled (the decoder's
 * receptive field is < the reference's 64-frame overlap). */
int acehip_vae_decode(acehip_vae *h, const void *z, int B, int T, void *wav, void *stream);
/* Test entry (block-level parity): the first launches of acehip_vae_decode for ONE song
 * (z bf16 [1, 64, T]) — conv1 and decoder blocks 0 .. n_blocks-1 — and a copy of the
 * activation they leave: channels-last bf16 [L][C] (L = T·Π strides so far), already passed
 * through the NEXT Snake (block n_blocks' snake1, or decoder.snake1 after the last block),
 * i.e. exactly the input of the next stage (vae_model.py:119-142, 190-230). */
int acehip_vae_decode_blocks(acehip_vae *h, const void *z, int T, int n_blocks, void *act, void *stream);

/* vae.encode(x).latent_dist.sample() (vae_encode.py:65) — and, untiled, the
 * handler's tiled_encode (vae_encode.py:15-82: the encoder's receptive field is
 * inside the reference's 2 s overlap, tiled == untiled).
 * wav: bf16 [B, 2, N], hop <= N <= max_T*hop; T = floor(N/hop) latent frames
 * (every strided conv maps L to floor(L/s), as AutoencoderOobleck's does);
 * eps: bf16 [B, 64, T] or NULL (NULL → the mean); z_out: bf16 [B, 64, T]. */
int acehip_vae_encode(acehip_vae *h, const void *wav, int B, int N, const void *eps,
                      void *z_out, void *stream);

int acehip_vae_destroy(acehip_vae *h);

/* Unit-level parity hooks (no reference counterpart: the per-conv checks of the
 * Oobleck layers, acestep/models/mlx/vae_model.py:24-230, against fp32
 * torch.nn.functional.conv1d / conv_transpose1d).  Both run the production weight
 * packing and kernel selection on channels-last bf16 tensors and synchronise `stream`.
 * acehip_vae_conv: kind 0 Conv1d(k, dilation dil, padding dil·(k−1)/2); kind 1
 * ConvTranspose1d(k = 2s, stride s, padding ⌈s/2⌉) (decoder blocks); kind 2 Conv1d(k = 2s,
 * stride s, padding ⌈s/2⌉) (encoder blocks).  in [L_in][Cin]; w bf16 in torch layout
 * ([Cout][Cin][k]; kind 1: [Cin][Cout][k]); bias [Cout] or NULL; res [L_out][Cout] or NULL
 * (out = bf16(res + bf16(conv + bias))); out [L_out][Cout] or NULL; alpha/beta [Cout]
 * (Snake1d, log-scale) with out_s = Snake(out) or NULL.  Cin % 64 == 0, Cout % 128 == 0.
 * acehip_vae_resunit: one C = 128 OobleckResidualUnit (vae_model.py:62-87) as the decoder
 * runs it: x, x_s = bf16(snake1(x)) [L][128] → x_out = x + conv2(snake2(conv1(x_s))) (or
 * NULL) and xs_out = bf16(snake_next(x_out)); w1 [128][128][7] (dilation dil ≤ 9), w2
 * [128][128][1]. */
int acehip_vae_conv(int kind, const void *in, int64_t L_in, int Cin, const void *w, const void *bias,
                    const void *res, int Cout, int k, int stride, int dil, void *out, const void *alpha,
                    const void *beta, void *out_s, void *stream);
int acehip_vae_resunit(const void *x, const void *x_s, int64_t L, int C, int dil, const void *w1, const void *b1,
                       const void *alpha2, const void *beta2, const void *w2, const void *b2, const void *alpha_n,
                       const void *beta_n, void *x_out, void *xs_out, void *stream);

/* The decode output guard of _decode_generate_music_pred_latents
 * (acestep/core/generation/handler/generate_music_decode.py:190-192):
 * per song, peak = max |wav|; if peak > 1 the song is divided by its peak.
 * wav fp32 [B, n] in place (n = channels·samples, n % 4 == 0); peak: device
 * scratch of B floats (receives the peaks). */
int acehip_wav_peak_normalize(float *wav, int B, int64_t n, float *peak, void *stream);

/* The guard above (guard != 0) fused with the product's loudness step,
 * normalize_audio (acestep/audio_utils.py:24-62, applied per song at
 * acestep/inference.py:674-679 when enable_normalization and normalization_db
 * <= 0): after the guard, gain = (1 / peak) * target_amp (fp32, the order torch
 * evaluates float / tensor in), wav *= gain,
 * skipped for songs whose peak < 1e-6.  target_amp = fp32(10^(normalization_db/20));
 * 0 = no normalization.  Bit-identical to the reference steps it replaces; one
 * peak pass + one scale pass. */
int acehip_wav_postprocess(float *wav, int B, int64_t n, float *peak, int guard, float target_amp,
                           void *stream);
/* The postprocess pass pair above with the output leg's sample conversion fused in (audio_utils.py
 * AudioSaver.save_audio → soundfile PCM_16, the default FLAC / WAV subtype): wav fp32 [B][C][N]
 * (C = 1 or 2, N % 4 == 0) is updated in place exactly as acehip_wav_postprocess does, and every
 * sample is also written to pcm int16 [B][N][C] (interleaved frames) as
 * rint(clamp(x, -1, 1) * 32767).  Halves the device→host bytes of the leg. */
int acehip_wav_postprocess_pcm16(float *wav, int B, int C, int64_t N, float *peak, int guard, float target_amp,
                                 int16_t *pcm, void *stream);

/* ------------------------------------------------------------ kernels ---- */
/* Single-kernel entry points used by the parity tests and the profiler
 * (same code the runtimes above launch). */

/* C[M,N] = A[M,K] · W[N,K]^T (+bias) — bf16 MFMA, fp32 accumulate. */
int acehip_gemm_bf16(const void *A, int lda, const void *W, int ldw, void *C, int ldc,
                     int M, int N, int K, const void *bias, void *stream);

/* Same with an explicit epilogue (0 store+bias, 2 residual add into C,
 * 3 SwiGLU: W rows packed [32 gate; 32 up] per 64-row panel, C is [M][N/2])
 * and tile variant (0: 128x128 2-stage, 7: 256x256 ping-pong, 8: 192x256
 * ping-pong, 9: 128x256 ping-pong (7-9: N % 256 == 0), 13: four-wave 192x128
 * + DMA helper waves (N % 128 == 0), 16: 128x64 4-stage, 17: 16 + two DMA
 * helper waves (N % 64 == 0);
 * -1: the production choice, including the tail split and split-K for grids that
 * cannot fill half the chip) — tuning and tests. */
int acehip_gemm_bf16_ex(const void *A, int lda, const void *W, int ldw, void *C, int ldc,
                        int M, int N, int K, const void *bias, int epi, int variant, void *stream);

/* Flash attention, head_dim 128, GQA: q [B,H,Sq,128], k/v [B,KV,Sk,128] →
 * o [B,Sq,H*128]; window -1 = full, >= 0 |i-j| <= window, -2 = causal
 * (keys j <= i; the Qwen3 text encoder's default mask). */
int acehip_attention_bf16(const void *q, const void *k, const void *v, void *o, int B, int H,
                          int KV, int Sq, int Sk, int window, float scale, void *stream);
/* Same with a key-padding mask kmask uint8 [B, Sk] (1 = attend), encoder semantics. */
int acehip_attention_masked_bf16(const void *q, const void *k, const void *v, void *o, int B,
                                 int H, int KV, int Sq, int Sk, int window, float scale,
                                 const uint8_t *kmask, void *stream);

/* Qwen3RMSNorm (+ AdaLN modulation when shift/scale are given) over rows of D
 * (transformers modeling_qwen3.py:59-64; reference base:499,530,1496):
 * out = bf16(bf16(bf16(w·bf16(x·rsqrt(mean x²+eps)))·bf16(1+scale[b])) + shift[b]),
 * b = row / rows_per_batch, shift/scale rows mod_bstride apart.
 * rows_per_wave: 0 = default, 1/2/4 rows per wave, -2/-4 = 2/4 waves per row (tuning, tests). */
int acehip_rmsnorm_bf16(const void *x, const void *w, const void *shift, const void *scale,
                        int64_t mod_bstride, int rows_per_batch, void *out, int M, int D, float eps,
                        int rows_per_wave, void *stream);

/* Projection GEMM with the q/k RMSNorm + RoPE + head-major scatter epilogue
 * (reference base:300-345 q_proj/k_proj/v_proj → q_norm/k_norm → apply_rotary_pos_emb):
 * rows [B·S] of A · W[N,K]ᵀ, N = (nq+nk+nv)·128, split into heads q | k | v and written
 * to q [B,nq,S,128], k [B,nk,S,128], v [B,nv,S,128]; cos/sin [S,128] or NULL (no RoPE). */
int acehip_gemm_headpost_bf16(const void *A, int lda, const void *W, int K, int B, int S, int nq,
                              int nk, int nv, const void *qw, const void *kw, const void *cos,
                              const void *sin, float eps, void *q, void *k, void *v, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* ACEHIP_H */
