// encoder.hip — the condition-encoder runtime behind acehip_enc_* (C ABI in
// include/acehip.h).
//
// One handle = one stack of AceStepEncoderLayer (reference base:374-440)
// between an embed_tokens Linear and a final Qwen3RMSNorm, with an optional
// proj_out Linear.  That single shape covers the lyric encoder (base:577-731,
// 8 layers, key-padding mask), the timbre encoder (base:997-1178, 4 layers,
// no mask), the attention pooler (base:734-859) and the detokenizer
// (base:862-994); the host composes them into AceStepConditionEncoder
// (base:1509-1554).  With every layer causal (sliding[l] == 2) and no embed
// Linear it is also the Qwen3-Embedding-0.6B text encoder (Qwen3Model, the
// reference's infer_text_embeddings, conditioning_embed.py:71-74).  The layer reuses the DiT's kernels unchanged:
//
//   XN = RMSNorm(X)                              rmsnorm_mod (plain)
//   q|k|v = XN·Wqkvᵀ → q/k RMSNorm + RoPE → head-major     gemm EPI_HEADPOST
//   AO = attention(q, k, v; band or full; key-padding mask)   attention
//   X  = bf16(X + bf16(AO·Woᵀ))                  gemm EPI_RES   (base:416-427)
//   XN = RMSNorm(X);  H = silu(XN·Wgᵀ)·(XN·Wuᵀ)  gemm EPI_SWIGLU
//   X  = bf16(X + bf16(H·Wdᵀ))                   gemm EPI_RES   (base:430-433)
//
// Runs once per song (twice in the reference, service_generate_execute.py:123
// and base:1820), so it is launch-count-light rather than tuned: every GEMM
// is the DiT's MFMA GEMM, every attention the DiT's flash kernel.
#include <cmath>
#include <map>
#include <vector>

#include "kernels.h"
#include "../../include/acehip.h"

using namespace acehip;

struct acehip_enc {
    int device = 0;
    acehip_enc_cfg cfg{};
    std::vector<uint8_t> sliding;
    int D = 0, F = 0, qd = 0, kvd = 0, L = 0;
    bool finalized = false;
    std::vector<void *> allocs;
    struct Slot {
        bf16_t *dst;
        std::vector<int64_t> shape;
        int kind;   // 0 copy, 1 gate (interleave), 2 up (interleave), 3 proj_out rows padded to 128
        bool set;
    };
    std::map<std::string, Slot> slots;
    struct Layer { bf16_t *ln1, *ln2, *wqkv, *wo, *qn, *kn, *wgu, *wdown; };
    std::vector<Layer> layers;
    bf16_t *wemb = nullptr, *bemb = nullptr, *norm = nullptr, *wout = nullptr, *bout = nullptr;
    bf16_t *rope_cos = nullptr, *rope_sin = nullptr;
    std::vector<float> inv_freq_override;
    // workspace
    bf16_t *X, *XN, *Qh, *Kh, *Vh, *AO, *Hb, *O128;
    void *attn_ws = nullptr;
    void *gemm_ws = nullptr;   // split-K partials for small-M GEMMs
};

// every GEMM of this runtime may use the handle's split-K workspace (small-M grids)
static inline int hgemm(acehip_enc *h, GemmArgs g, hipStream_t s, RowAdd *defer = nullptr) {
    g.ws = h->gemm_ws;
    g.ws_bytes = h->gemm_ws ? GEMM_WS_BYTES : 0;
    return gemm(g, s, defer);
}

namespace {

bf16_t *enc_alloc(acehip_enc *h, size_t elems) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(elems, 1) * 2) != hipSuccess) return nullptr;
    h->allocs.push_back(p);
    return (bf16_t *)p;
}

int enc_build_rope(acehip_enc *h) {
    const int hd = h->cfg.head_dim, S = h->cfg.max_S;
    std::vector<float> inv(hd / 2);
    for (int i = 0; i < hd / 2; ++i) {
        const float v = h->inv_freq_override.empty() ? 1.0f / powf(h->cfg.rope_theta, (float)(2 * i) / (float)hd)
                                                     : h->inv_freq_override[i];
        inv[i] = bf2f(f2bf(v));   // model.to(bf16) casts the rotary inv_freq buffer too (see dit.hip)
    }
    std::vector<bf16_t> c((size_t)S * hd), s((size_t)S * hd);
    for (int p = 0; p < S; ++p)
        for (int i = 0; i < hd; ++i) {
            const float f = (float)p * inv[i % (hd / 2)];
            c[(size_t)p * hd + i] = f2bf((float)cos((double)f));
            s[(size_t)p * hd + i] = f2bf((float)sin((double)f));
        }
    HIP_TRY(hipMemcpy(h->rope_cos, c.data(), c.size() * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->rope_sin, s.data(), s.size() * 2, hipMemcpyHostToDevice));
    return 0;
}

}  // namespace

extern "C" {

int acehip_enc_destroy(acehip_enc *h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    for (void *p : h->allocs) (void)hipFree(p);
    delete h;
    return 0;
}

int acehip_enc_create(int device, const acehip_enc_cfg *cfg, acehip_enc **out) {
    if (!cfg || !out) return fail(ACEHIP_E_ARG, "enc_create: null argument");
    if (cfg->head_dim != 128) return fail(ACEHIP_E_ARG, "enc_create: head_dim must be 128");
    if (cfg->hidden % 256 || cfg->intermediate % 64 || cfg->kv_heads <= 0 || cfg->heads % cfg->kv_heads ||
        cfg->heads / cfg->kv_heads > 2 || ((cfg->heads + 2 * cfg->kv_heads) * 128) % 256)
        return fail(ACEHIP_E_ARG, "enc_create: unsupported dims");
    if (cfg->in_dim < 0 || (cfg->in_dim && cfg->in_dim % 64) || cfg->out_dim < 0 || cfg->out_dim > 128 ||
        cfg->layers < 0 || cfg->max_tokens <= 0 || cfg->max_S <= 0)
        return fail(ACEHIP_E_ARG, "enc_create: in_dim % 64, out_dim <= 128, max_tokens/max_S > 0");
    HIP_TRY(hipSetDevice(device));
    auto *h = new acehip_enc();
    h->device = device;
    h->cfg = *cfg;
    h->D = cfg->hidden; h->F = cfg->intermediate; h->L = cfg->layers;
    h->qd = cfg->heads * 128; h->kvd = cfg->kv_heads * 128;
    h->sliding.resize(h->L);
    for (int i = 0; i < h->L; ++i) h->sliding[i] = cfg->sliding ? cfg->sliding[i] : ((i + 1) % 2);
    h->cfg.sliding = nullptr;
    const int D = h->D, F = h->F, qd = h->qd, kvd = h->kvd;
    bool ok = true;
    auto A = [&](size_t n) { bf16_t *p = enc_alloc(h, n); ok = ok && p; return p; };
    auto slot = [&](const std::string &n, bf16_t *dst, std::vector<int64_t> shape, int kind = 0) {
        h->slots[n] = acehip_enc::Slot{dst, std::move(shape), kind, false};
    };
    h->layers.resize(h->L);
    for (int i = 0; i < h->L && ok; ++i) {
        auto &ly = h->layers[i];
        ly.ln1 = A(D); ly.ln2 = A(D); ly.qn = A(128); ly.kn = A(128);
        ly.wqkv = A((size_t)(qd + 2 * kvd) * D); ly.wo = A((size_t)D * qd);
        ly.wgu = A((size_t)2 * F * D); ly.wdown = A((size_t)D * F);
        if (!ok) break;
        const std::string p = "layers." + std::to_string(i);
        slot(p + ".input_layernorm.weight", ly.ln1, {D});
        slot(p + ".post_attention_layernorm.weight", ly.ln2, {D});
        slot(p + ".self_attn.q_proj.weight", ly.wqkv, {qd, D});
        slot(p + ".self_attn.k_proj.weight", ly.wqkv + (size_t)qd * D, {kvd, D});
        slot(p + ".self_attn.v_proj.weight", ly.wqkv + (size_t)(qd + kvd) * D, {kvd, D});
        slot(p + ".self_attn.o_proj.weight", ly.wo, {D, qd});
        slot(p + ".self_attn.q_norm.weight", ly.qn, {128});
        slot(p + ".self_attn.k_norm.weight", ly.kn, {128});
        slot(p + ".mlp.gate_proj.weight", ly.wgu, {F, D}, 1);
        slot(p + ".mlp.up_proj.weight", ly.wgu, {F, D}, 2);
        slot(p + ".mlp.down_proj.weight", ly.wdown, {D, F});
    }
    if (ok && cfg->in_dim) {
        h->wemb = A((size_t)D * cfg->in_dim);
        slot("embed_tokens.weight", h->wemb, {D, cfg->in_dim});
        if (cfg->embed_bias) {
            h->bemb = A(D);
            slot("embed_tokens.bias", h->bemb, {D});
        }
    }
    h->norm = A(D);
    if (ok) slot("norm.weight", h->norm, {D});
    if (ok && cfg->out_dim) {
        h->wout = A((size_t)128 * D);   // rows past out_dim stay zero
        h->bout = A(128);
        if (ok) {
            HIP_TRY(hipMemset(h->wout, 0, (size_t)128 * D * 2));
            HIP_TRY(hipMemset(h->bout, 0, 256));
            slot("proj_out.weight", h->wout, {cfg->out_dim, D});
            slot("proj_out.bias", h->bout, {cfg->out_dim});
        }
    }
    const size_t M = cfg->max_tokens;
    h->X = A(M * D); h->XN = A(M * D);
    h->Qh = A(M * qd); h->Kh = A(M * kvd); h->Vh = A(M * kvd); h->AO = A(M * qd);
    h->Hb = A(M * F);
    h->O128 = cfg->out_dim ? A(M * 128) : nullptr;
    h->gemm_ws = A(GEMM_WS_BYTES / 2);
    h->rope_cos = A((size_t)cfg->max_S * 128); h->rope_sin = A((size_t)cfg->max_S * 128);
    if (ok) {
        const size_t wb = attention_ws_bytes();
        h->attn_ws = enc_alloc(h, (wb + 1) / 2);
        ok = h->attn_ws && hipMemset(h->attn_ws, 0, wb) == hipSuccess;
    }
    if (!ok) {
        acehip_enc_destroy(h);
        return fail(ACEHIP_E_OOM, "enc_create: device allocation failed");
    }
    *out = h;
    return 0;
}

int acehip_enc_set_weight(acehip_enc *h, const char *name, const void *ptr, int dtype, int ndim,
                          const int64_t *shape, int on_device) {
    if (!h || !name || !ptr || !shape || ndim <= 0) return fail(ACEHIP_E_ARG, "enc_set_weight: null argument");
    if (dtype != ACEHIP_F32 && dtype != ACEHIP_BF16) return fail(ACEHIP_E_ARG, "enc_set_weight: dtype");
    HIP_TRY(hipSetDevice(h->device));
    const std::string nm(name);
    if (nm == "_rope_inv_freq") {   // the caller's torch fp32 inv_freq (exact reference constant)
        if (dtype != ACEHIP_F32 || shape[0] != 64) return fail(ACEHIP_E_ARG, "_rope_inv_freq: fp32 [64]");
        h->inv_freq_override.resize(64);
        HIP_TRY(hipMemcpy(h->inv_freq_override.data(), ptr, 256,
                          on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
        return 0;
    }
    if (nm == "rotary_emb.inv_freq") return 0;   // non-persistent buffer, recomputed
    auto it = h->slots.find(nm);
    if (it == h->slots.end()) return fail(ACEHIP_E_NAME, "enc_set_weight: unknown weight " + nm);
    auto &s = it->second;
    if (std::vector<int64_t>(shape, shape + ndim) != s.shape)
        return fail(ACEHIP_E_ARG, "enc_set_weight: shape mismatch for " + nm);
    int64_t n = 1;
    for (auto v : s.shape) n *= v;
    // stage through the host as bf16 (load time only; RNE like torch's .to(bfloat16))
    std::vector<bf16_t> hb(n);
    const hipMemcpyKind k = on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost;
    if (dtype == ACEHIP_F32) {
        std::vector<float> f(n);
        HIP_TRY(hipMemcpy(f.data(), ptr, n * 4, k));
        for (int64_t i = 0; i < n; ++i) hb[i] = f2bf(f[i]);
    } else {
        HIP_TRY(hipMemcpy(hb.data(), ptr, n * 2, k));
    }
    if (s.kind == 1 || s.kind == 2) {   // gate/up interleaved in 32-row panels (SwiGLU epilogue layout)
        const int64_t F = s.shape[0], K = s.shape[1];
        bf16_t *dst = s.dst + (s.kind == 2 ? 32 * K : 0);
        HIP_TRY(hipMemcpy2D(dst, 64 * K * 2, hb.data(), 32 * K * 2, 32 * K * 2, F / 32, hipMemcpyHostToDevice));
    } else {
        HIP_TRY(hipMemcpy(s.dst, hb.data(), n * 2, hipMemcpyHostToDevice));
    }
    s.set = true;
    return 0;
}

int acehip_enc_finalize(acehip_enc *h) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    HIP_TRY(hipSetDevice(h->device));
    std::string missing;
    for (auto &kv : h->slots)
        if (!kv.second.set) missing += kv.first + " ";
    if (!missing.empty()) return fail(ACEHIP_E_STATE, "enc_finalize: missing weights: " + missing.substr(0, 400));
    if (h->F % 32) return fail(ACEHIP_E_ARG, "intermediate must be a multiple of 32");
    const int rc = enc_build_rope(h);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    h->finalized = true;
    return 0;
}

int acehip_enc_embed(acehip_enc *h, const void *x, int M, void *out, void *stream) {
    if (!h || !x || !out) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized || !h->wemb) return fail(ACEHIP_E_STATE, "enc_embed: not finalized / no embed_tokens");
    if (M <= 0) return M == 0 ? 0 : fail(ACEHIP_E_ARG, "enc_embed: M");
    HIP_TRY(hipSetDevice(h->device));
    GemmArgs g{};
    g.A = (const bf16_t *)x; g.lda = h->cfg.in_dim; g.W = h->wemb; g.ldw = h->cfg.in_dim;
    g.C = (bf16_t *)out; g.ldc = h->D; g.M = M; g.N = h->D; g.K = h->cfg.in_dim;
    g.epi = EPI_STORE; g.bias = h->bemb;
    return gemm(g, (hipStream_t)stream);
}

int acehip_enc_forward(acehip_enc *h, const void *x, const uint8_t *kmask, int B, int S, void *out, void *stream) {
    if (!h || !x || !out) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized) return fail(ACEHIP_E_STATE, "enc_forward before finalize");
    if (B <= 0 || S <= 0 || S > h->cfg.max_S || (int64_t)B * S > h->cfg.max_tokens)
        return fail(ACEHIP_E_ARG, "enc_forward: B*S / S out of range");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const int D = h->D, F = h->F, qd = h->qd, kvd = h->kvd, M = B * S;
    const int H = h->cfg.heads, KV = h->cfg.kv_heads;
    const float eps = h->cfg.eps, scale = 1.0f / sqrtf(128.0f);
    int rc;
#define RUN(e) do { if ((rc = (e))) return rc; } while (0)
    HIP_TRY(hipMemcpyAsync(h->X, x, (size_t)M * D * 2, hipMemcpyDeviceToDevice, s));
    // few tokens (text / lyric encoders): the O and down GEMMs take gemm's split-K path and
    // leave their residual epilogue to the next norm (`pend`, as in the DiT forward)
    RowAdd pend{};
    for (int l = 0; l < h->L; ++l) {
        const auto &ly = h->layers[l];
        RUN(rmsnorm_mod(h->X, ly.ln1, nullptr, nullptr, 0, S, h->XN, M, D, eps, s, pend));
        pend = RowAdd{};
        GemmArgs q{};
        q.A = h->XN; q.lda = D; q.W = ly.wqkv; q.ldw = D;
        q.M = M; q.N = qd + 2 * kvd; q.K = D; q.epi = EPI_HEADPOST;
        q.hp.B = B; q.hp.S = S; q.hp.nq = H; q.hp.nk = KV; q.hp.nv = KV; q.hp.qw = ly.qn; q.hp.kw = ly.kn;
        q.hp.cos = h->rope_cos; q.hp.sin = h->rope_sin;
        q.hp.q = h->Qh; q.hp.k = h->Kh; q.hp.v = h->Vh; q.hp.S_dst = S; q.hp.eps = eps;
        RUN(hgemm(h, q, s));
        // layer kind: 0 full, 1 band |i−j| <= window, 2 causal (the Qwen3 text encoder)
        const int win = h->sliding[l] == 2 ? ATTN_CAUSAL : h->sliding[l] ? h->cfg.window : -1;
        RUN(attention(h->Qh, h->Kh, h->Vh, h->AO, B, H, KV, S, S, win, scale, qd, h->attn_ws, s, kmask));
        GemmArgs o{};
        o.A = h->AO; o.lda = qd; o.W = ly.wo; o.ldw = qd; o.C = h->X; o.ldc = D;
        o.M = M; o.N = D; o.K = qd; o.epi = EPI_RES; o.res = h->X; o.ldr = D;
        RUN(hgemm(h, o, s, &pend));
        RUN(rmsnorm_mod(h->X, ly.ln2, nullptr, nullptr, 0, S, h->XN, M, D, eps, s, pend));
        pend = RowAdd{};
        GemmArgs gu{};
        gu.A = h->XN; gu.lda = D; gu.W = ly.wgu; gu.ldw = D; gu.C = h->Hb; gu.ldc = F;
        gu.M = M; gu.N = 2 * F; gu.K = D; gu.epi = EPI_SWIGLU;
        RUN(hgemm(h, gu, s));
        GemmArgs dn{};
        dn.A = h->Hb; dn.lda = F; dn.W = ly.wdown; dn.ldw = F; dn.C = h->X; dn.ldc = D;
        dn.M = M; dn.N = D; dn.K = F; dn.epi = EPI_RES; dn.res = h->X; dn.ldr = D;
        RUN(hgemm(h, dn, s, &pend));
    }
    if (!h->cfg.out_dim) {
        RUN(rmsnorm_mod(h->X, h->norm, nullptr, nullptr, 0, S, (bf16_t *)out, M, D, eps, s, pend));
        return 0;
    }
    // detokenizer proj_out (base:991): rows padded to 128 with zeros, then the used columns
    RUN(rmsnorm_mod(h->X, h->norm, nullptr, nullptr, 0, S, h->XN, M, D, eps, s, pend));
    GemmArgs po{};
    po.A = h->XN; po.lda = D; po.W = h->wout; po.ldw = D; po.C = h->O128; po.ldc = 128;
    po.M = M; po.N = 128; po.K = D; po.epi = EPI_STORE; po.bias = h->bout;
    RUN(hgemm(h, po, s));
    RUN(copy_cols(h->O128, 128, (bf16_t *)out, h->cfg.out_dim, M, h->cfg.out_dim, s));
#undef RUN
    return 0;
}

int acehip_fsq_quantize(const void *z, int ldz, int M, const int *levels, int n_levels, void *codes, int ldc,
                        int32_t *indices, void *stream) {
    if (!z || !codes || !levels || n_levels <= 0 || n_levels > 8 || ldz < n_levels)
        return fail(ACEHIP_E_ARG, "fsq_quantize: argument");
    FsqLevels lv{n_levels, {}};
    for (int i = 0; i < n_levels; ++i) lv.L[i] = levels[i];
    return fsq_quantize((const bf16_t *)z, ldz, M, lv, (bf16_t *)codes, ldc, indices, (hipStream_t)stream);
}

int acehip_fsq_codes_from_indices(const int32_t *indices, int M, const int *levels, int n_levels, void *codes,
                                  int ldc, void *stream) {
    if (!indices || !codes || !levels || n_levels <= 0 || n_levels > 8) return fail(ACEHIP_E_ARG, "fsq_codes: argument");
    FsqLevels lv{n_levels, {}};
    for (int i = 0; i < n_levels; ++i) lv.L[i] = levels[i];
    return fsq_codes_from_indices(indices, M, lv, (bf16_t *)codes, ldc, (hipStream_t)stream);
}

}  // extern "C"
