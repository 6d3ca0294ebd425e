// vae.hip — the Oobleck VAE runtime behind acehip_vae_* (include/acehip.h).
//
// Replaces diffusers AutoencoderOobleck.decode/encode as called by the
// reference handler (acestep/core/generation/handler/vae_decode_chunks.py:42,
// vae_encode.py:65); structure per acestep/models/mlx/vae_model.py:94-230.
// set_weight keeps raw (weight_g, weight_v) copies; finalize fuses
// w = g·v/‖v‖ (vae_convert.py:18-34) straight into implicit-GEMM layouts.
//
// Decode runs untiled, one song at a time, with three activation buffers of
// max(L·C) elements: X (raw residual stream) and two snaked buffers that
// alternate as the k=7 conv input / k=1 conv input.  Every conv writes the
// Snake of its output for its consumer (conv.hip), so the residual unit is
//   y_s = snake2(conv7(x_s)) ;  x = x + conv1(y_s), x_s = snake_next(x)
// with no separate activation passes.
#include <map>
#include <vector>

#include "kernels.h"
#include "conv.h"
#include "../../include/acehip.h"

using namespace acehip;

namespace {

struct Raw {
    bf16_t *p = nullptr;
    std::vector<int64_t> shape;
};
struct ConvL {
    bf16_t *Wp = nullptr;
    bf16_t *bias = nullptr;
    int cin = 0, cout = 0, k = 0, stride = 1, transposed = 0;
};
struct SnakeP {
    float *a = nullptr, *ib = nullptr;
};
struct ResU {
    SnakeP s1, s2;
    ConvL c1, c2;
    bf16_t *W2p = nullptr;   // C = 128: c2 weights permuted for ru7_kernel
    int dil = 1;
};
struct DecBlk {
    SnakeP snake;
    ConvL convT;
    ResU res[3];
    int cin, cout, stride;
};
struct EncBlk {
    ResU res[3];
    SnakeP snake;
    ConvL conv;
    int cin, cout, stride;
};

}  // namespace

struct acehip_vae {
    int device = 0;
    acehip_vae_cfg cfg{};
    int hop = 1;
    std::vector<void *> allocs;
    std::map<std::string, Raw> raw;
    bool finalized = false;
    // decoder
    ConvL dconv1;
    std::vector<DecBlk> dec;
    SnakeP dsnake;
    float *dconv2_w = nullptr;  // [7][C][2] (output channel innermost)
    // encoder
    float *econv1_w = nullptr, *econv1_b = nullptr;  // [C][2][7], [C]
    std::vector<EncBlk> enc;
    SnakeP esnake;
    ConvL econv2;
    // buffers
    bf16_t *X = nullptr, *P = nullptr, *Q = nullptr;
    bf16_t *zero = nullptr;     // zero page: im2col padding source
    int64_t buf_elems = 0;
};

namespace {

void *valloc(acehip_vae *h, size_t bytes) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
    h->allocs.push_back(p);
    return p;
}

std::string norm_name(std::string n) {
    const std::string o0 = ".parametrizations.weight.original0", o1 = ".parametrizations.weight.original1";
    size_t k;
    if ((k = n.find(o0)) != std::string::npos) n = n.substr(0, k) + ".weight_g";
    else if ((k = n.find(o1)) != std::string::npos) n = n.substr(0, k) + ".weight_v";
    if (n.rfind("vae.", 0) == 0) n = n.substr(4);
    return n;
}

Raw *find(acehip_vae *h, const std::string &n) {
    auto it = h->raw.find(n);
    return it == h->raw.end() ? nullptr : &it->second;
}

int make_conv(acehip_vae *h, const std::string &name, int cin, int cout, int k, int stride, bool transposed,
              bool bias, ConvL &out) {
    Raw *v = find(h, name + ".weight_v");
    Raw *g = find(h, name + ".weight_g");
    if (!v) v = find(h, name + ".weight");
    if (!v) return fail(ACEHIP_E_STATE, "vae_finalize: missing " + name + ".weight_v");
    const int d0 = transposed ? cin : cout, d1 = transposed ? cout : cin;
    if (v->shape != std::vector<int64_t>{d0, d1, k})
        return fail(ACEHIP_E_ARG, "vae_finalize: bad shape for " + name);
    out.cin = cin; out.cout = cout; out.k = k; out.stride = stride; out.transposed = transposed;
    const size_t n = (size_t)cin * cout * k;
    out.Wp = (bf16_t *)valloc(h, n * 2);
    if (!out.Wp) return fail(ACEHIP_E_OOM, "vae_finalize: oom");
    int rc = pack_conv_weight(v->p, g ? g->p : nullptr, d0, d1, k, transposed ? 1 : 0, stride, out.Wp, 0);
    if (rc) return rc;
    if (bias) {
        Raw *b = find(h, name + ".bias");
        if (!b) return fail(ACEHIP_E_STATE, "vae_finalize: missing " + name + ".bias");
        out.bias = b->p;   // kept (raw buffer stays alive)
    }
    return 0;
}

int make_snake(acehip_vae *h, const std::string &name, int C, SnakeP &s) {
    Raw *a = find(h, name + ".alpha"), *b = find(h, name + ".beta");
    if (!a || !b) return fail(ACEHIP_E_STATE, "vae_finalize: missing " + name + ".alpha/.beta");
    s.a = (float *)valloc(h, C * 4);
    s.ib = (float *)valloc(h, C * 4);
    if (!s.a || !s.ib) return fail(ACEHIP_E_OOM, "vae_finalize: oom");
    return snake_params(a->p, b->p, C, s.a, s.ib, 0);
}

int make_res(acehip_vae *h, const std::string &p, int C, int dil, ResU &r) {
    int rc;
    r.dil = dil;
    if ((rc = make_snake(h, p + ".snake1", C, r.s1))) return rc;
    if ((rc = make_snake(h, p + ".snake2", C, r.s2))) return rc;
    if ((rc = make_conv(h, p + ".conv1", C, C, 7, 1, false, true, r.c1))) return rc;
    if ((rc = make_conv(h, p + ".conv2", C, C, 1, 1, false, true, r.c2))) return rc;
    if (C == 128) {
        r.W2p = (bf16_t *)valloc(h, (size_t)C * C * 2);
        if (!r.W2p) return fail(ACEHIP_E_OOM, "vae_finalize: oom");
        return permute_k1_weight(r.c2.Wp, r.W2p, C, 0);
    }
    return 0;
}

// one implicit-GEMM conv launch; `zero` = the caller's zero page (the handle's own, so two
// handles on different devices or threads never share launch state)
int run_conv(const bf16_t *zero, const ConvL &c, const bf16_t *in, int64_t L_in, int64_t M, int taps, int dil, int a_stride,
             int a_off, int c_stride, int c_off, int64_t L_out, bf16_t *out, bf16_t *out_s, const SnakeP *sn,
             const bf16_t *res, int phases, hipStream_t s, int in_halo = 0) {
    ConvArgs a{};
    a.in_halo = in_halo;
    a.in = in; a.L_in = L_in; a.Cin = c.cin;
    a.W = c.Wp; a.w_pstride = (int64_t)c.cout * taps * c.cin;
    a.bias = c.bias; a.out = out; a.out_s = out_s;
    a.sa = sn ? sn->a : nullptr; a.sib = sn ? sn->ib : nullptr;
    a.res = res; a.L_out = L_out; a.N = c.cout; a.M = M;
    a.taps = taps; a.dil = dil; a.a_stride = a_stride; a.a_off = a_off; a.c_stride = c_stride; a.c_off = c_off;
    a.zero = zero;
    return conv_gemm(a, phases, s);
}

// residual unit on (x raw in X, x_s in cur): leaves x in X (if keep_raw) and next-snaked x in cur
int res_unit(const bf16_t *zero, const ResU &r, int64_t L, bf16_t *X, bf16_t *cur, bf16_t *other, const SnakeP &next, bool keep_raw,
             hipStream_t s) {
    int rc;
    if (r.c1.cin == 128) {
        // fused k=7 → Snake → k=1 → residual; y_s never leaves LDS
        ResUnitArgs u{};
        ConvArgs &a = u.c1;
        a.in = cur; a.L_in = L; a.Cin = 128; a.W = r.c1.Wp; a.bias = r.c1.bias;
        a.sa = r.s2.a; a.sib = r.s2.ib; a.L_out = L; a.N = 128; a.M = L;
        a.taps = 7; a.dil = r.dil; a.a_stride = 1; a.a_off = -3 * r.dil; a.c_stride = 1; a.c_off = 0;
        a.zero = zero;
        u.W2 = r.c2.Wp; u.W2p = r.W2p; u.b2 = r.c2.bias; u.x = X; u.out_s = other;
        u.in_zero_pad = 1;   // cur is h->P or h->Q
        u.sa_next = next.a; u.sib_next = next.ib; u.keep_raw = keep_raw ? 1 : 0;
        if ((rc = resunit128(u, s))) return rc;
        // the snaked output is in `other`: copy-free hand-back by swapping roles is done by the caller
        return 1;   // signals "output in other"
    }
    // (cur is one of the padded activation buffers: in_halo)
    if ((rc = run_conv(zero, r.c1, cur, L, L, 7, r.dil, 1, -3 * r.dil, 1, 0, L, nullptr, other, &r.s2, nullptr, 1, s, 1)))
        return rc;
    return run_conv(zero, r.c2, other, L, L, 1, 1, 1, 0, 1, 0, L, keep_raw ? X : nullptr, cur, &next, X, 1, s);
}

// ACEHIP_VAE_SNAKE_IN: the C = 128 residual units of a decoder block take RAW x and apply their
// first Snake while staging the window (ru8_kernel<·, SIN>), so the block's x_s tensors are
// never written or read (ConvTranspose writes raw x only, units 1-2 write raw x' only)
bool snake_in_block(const DecBlk &bk) {
    return knobs().vae_snake_in && knobs().ru7 == 2 && bk.cout == 128 && bk.res[0].W2p && bk.res[1].W2p &&
           bk.res[2].W2p;
}

// decoder block j on the snake-in path: in = the block input (snaked), X / cur / other the three
// buffers (cur = in); returns with the snaked block output in `cur` and X / other free
int dec_block_snake_in(acehip_vae *h, int j, int64_t &L, bf16_t *&X, bf16_t *&cur, bf16_t *&other, hipStream_t s) {
    const auto &bk = h->dec[j];
    const int n = h->cfg.n_blocks, st = bk.stride, pad = (st + 1) / 2;
    int rc;
    // ConvTranspose1d → raw x only
    if ((rc = run_conv(h->zero, bk.convT, cur, L, L + 1, 2, 1, 1, -1, st, -pad, L * st, X, nullptr, nullptr, nullptr,
                       st, s, 1)))
        return rc;
    L *= st;
    bf16_t *bufs[3] = {X, cur, other};          // raw x in bufs[0]; unit u: in bufs[u] → out bufs[u + 1 mod 3]
    for (int u = 0; u < 3; ++u) {
        const ResU &r = bk.res[u];
        const SnakeP &next = j + 1 < n ? h->dec[j + 1].snake : h->dsnake;
        bf16_t *in = bufs[u], *out = bufs[(u + 1) % 3];
        ResUnitArgs ua{};
        ConvArgs &a = ua.c1;
        a.in = in; a.L_in = L; a.Cin = 128; a.W = r.c1.Wp; a.bias = r.c1.bias;
        a.sa = r.s2.a; a.sib = r.s2.ib; a.L_out = L; a.N = 128; a.M = L;
        a.taps = 7; a.dil = r.dil; a.a_stride = 1; a.a_off = -3 * r.dil; a.c_stride = 1; a.c_off = 0;
        a.zero = h->zero;
        ua.W2 = r.c2.Wp; ua.W2p = r.W2p; ua.b2 = r.c2.bias; ua.x = in;
        ua.in_zero_pad = 1;
        ua.snake_in = 1; ua.sa_in = r.s1.a; ua.sib_in = r.s1.ib;
        ua.keep_raw = u < 2 ? 1 : 0;
        ua.sa_next = next.a; ua.sib_next = next.ib;     // read only by the last unit (out_s)
        if (u < 2) ua.x_out = out;
        else ua.out_s = out;
        if ((rc = resunit128(ua, s))) return rc;
    }
    // the snaked output is in bufs[0] (unit 2: bufs[2] → bufs[0])
    cur = bufs[0];
    X = bufs[1];
    other = bufs[2];
    return 0;
}

}  // namespace

extern "C" {

int acehip_vae_create(int device, const acehip_vae_cfg *cfg, acehip_vae **out) {
    if (!cfg || !out) return fail(ACEHIP_E_ARG, "vae_create: null argument");
    if (cfg->n_blocks < 1 || cfg->n_blocks > 8 || cfg->max_T <= 0 || cfg->max_B <= 0)
        return fail(ACEHIP_E_ARG, "vae_create: bad config");
    if (cfg->audio_channels != 2) return fail(ACEHIP_E_ARG, "vae_create: stereo (2 channels) required");
    HIP_TRY(hipSetDevice(device));
    auto *h = new acehip_vae();
    h->device = device;
    h->cfg = *cfg;
    const int n = cfg->n_blocks;
    int hop = 1;
    for (int i = 0; i < n; ++i) hop *= cfg->ratios[i];
    h->hop = hop;
    // decoder blocks: strides reversed, channels C·cm[n−i] → C·cm[n−i−1] with cm = [1] + multiples
    std::vector<int> cm(n + 1);
    cm[0] = 1;
    for (int i = 0; i < n; ++i) cm[i + 1] = cfg->multiples[i];
    h->dec.resize(n);
    for (int i = 0; i < n; ++i) {
        h->dec[i].cin = cfg->decoder_channels * cm[n - i];
        h->dec[i].cout = cfg->decoder_channels * cm[n - i - 1];
        h->dec[i].stride = cfg->ratios[n - 1 - i];
    }
    h->enc.resize(n);
    for (int i = 0; i < n; ++i) {
        h->enc[i].cin = cfg->encoder_hidden * cm[i];
        h->enc[i].cout = cfg->encoder_hidden * cm[i + 1];
        h->enc[i].stride = cfg->ratios[i];
    }
    // activation buffer size: max over all stages of L·C
    int64_t mx = (int64_t)cfg->max_T * std::max(cfg->latent_channels, h->dec[0].cin);
    int64_t L = cfg->max_T;
    for (int i = 0; i < n; ++i) {
        L *= h->dec[i].stride;
        mx = std::max(mx, L * (int64_t)h->dec[i].cout);
    }
    if (cfg->with_encoder) {
        int64_t Le = (int64_t)cfg->max_T * hop;
        mx = std::max(mx, Le * (int64_t)cfg->encoder_hidden);
        for (int i = 0; i < n; ++i) {
            mx = std::max(mx, Le * (int64_t)h->enc[i].cin);
            Le /= h->enc[i].stride;
            mx = std::max(mx, Le * (int64_t)h->enc[i].cout);
        }
    }
    h->buf_elems = mx;
    // each activation buffer carries kActPadRows zero rows (at the widest stage's row pitch) in
    // front and as many addressable rows behind: the persistent residual-unit kernel reads its
    // halo rows before the start from the front ones and whole windows past the end from the
    // back ones (resunit128 zeroes the first kActPadRows rows past L before each launch)
    const size_t pad = std::max((size_t)kActPadRows * std::max(h->dec[0].cin, cfg->encoder_hidden * cm[n]) * 2,
                                (size_t)kResWindowBackRows * 128 * 2);
    bf16_t **bufs[3] = {&h->X, &h->P, &h->Q};
    for (bf16_t **b : bufs) {
        char *p = (char *)valloc(h, (size_t)mx * 2 + 2 * pad);
        if (p && hipMemset(p, 0, pad) != hipSuccess) p = nullptr;
        *b = p ? (bf16_t *)(p + pad) : nullptr;
    }
    h->zero = (bf16_t *)valloc(h, 4096);
    if (h->zero && hipMemset(h->zero, 0, 4096) != hipSuccess) h->zero = nullptr;
    if (!h->X || !h->P || !h->Q || !h->zero) {
        acehip_vae_destroy(h);
        return fail(ACEHIP_E_OOM, "vae_create: activation buffers (" + std::to_string(3 * mx * 2 >> 20) + " MiB)");
    }
    *out = h;
    return 0;
}

int acehip_vae_set_weight(acehip_vae *h, const char *name, const void *ptr, int dtype, int ndim,
                          const int64_t *shape, int on_device) {
    if (!h || !name || !ptr || !shape) return fail(ACEHIP_E_ARG, "vae_set_weight: null argument");
    HIP_TRY(hipSetDevice(h->device));
    const std::string nm = norm_name(name);
    int64_t n = 1;
    std::vector<int64_t> sh;
    for (int i = 0; i < ndim; ++i) {
        n *= shape[i];
        sh.push_back(shape[i]);
    }
    // snake params [1,C,1] and weight_g [d0,1,1] are stored flat
    Raw r;
    r.shape = sh;
    r.p = (bf16_t *)valloc(h, (size_t)n * 2);
    if (!r.p) return fail(ACEHIP_E_OOM, "vae_set_weight: oom");
    const hipMemcpyKind kd = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (dtype == ACEHIP_BF16) {
        HIP_TRY(hipMemcpy(r.p, ptr, n * 2, kd));
    } else if (dtype == ACEHIP_F32) {
        float *tmp = (float *)valloc(h, (size_t)n * 4);
        if (!tmp) return fail(ACEHIP_E_OOM, "vae_set_weight: oom");
        HIP_TRY(hipMemcpy(tmp, ptr, n * 4, kd));
        int rc = cast_f32_bf16(tmp, r.p, n, 0);
        if (rc) return rc;
        HIP_TRY(hipDeviceSynchronize());
    } else {
        return fail(ACEHIP_E_ARG, "vae_set_weight: dtype");
    }
    h->raw[nm] = r;
    return 0;
}

int acehip_vae_finalize(acehip_vae *h) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    HIP_TRY(hipSetDevice(h->device));
    const auto &c = h->cfg;
    const int n = c.n_blocks;
    int rc;
    if ((rc = make_conv(h, "decoder.conv1", c.latent_channels, h->dec[0].cin, 7, 1, false, true, h->dconv1))) return rc;
    for (int j = 0; j < n; ++j) {
        auto &b = h->dec[j];
        const std::string p = "decoder.block." + std::to_string(j);
        if ((rc = make_snake(h, p + ".snake1", b.cin, b.snake))) return rc;
        if ((rc = make_conv(h, p + ".conv_t1", b.cin, b.cout, 2 * b.stride, b.stride, true, true, b.convT))) return rc;
        const int dil[3] = {1, 3, 9};
        for (int u = 0; u < 3; ++u)
            if ((rc = make_res(h, p + ".res_unit" + std::to_string(u + 1), b.cout, dil[u], b.res[u]))) return rc;
    }
    if ((rc = make_snake(h, "decoder.snake1", c.decoder_channels, h->dsnake))) return rc;
    {
        Raw *v = find(h, "decoder.conv2.weight_v"), *g = find(h, "decoder.conv2.weight_g");
        if (!v) v = find(h, "decoder.conv2.weight");
        if (!v) return fail(ACEHIP_E_STATE, "vae_finalize: missing decoder.conv2");
        h->dconv2_w = (float *)valloc(h, (size_t)c.audio_channels * 7 * c.decoder_channels * 4);
        if ((rc = fuse_conv_weight_f32(v->p, g ? g->p : nullptr, c.audio_channels, c.decoder_channels, 7, 1,
                                       h->dconv2_w, 0)))
            return rc;
        // conv_out reads the two output channels' weights as adjacent pairs [7][C][2]
        const size_t n = (size_t)c.audio_channels * 7 * c.decoder_channels;
        std::vector<float> w(n), wp(n);
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(w.data(), h->dconv2_w, n * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n / 2; ++i) {
            wp[2 * i] = w[i];
            wp[2 * i + 1] = w[n / 2 + i];
        }
        HIP_TRY(hipMemcpy(h->dconv2_w, wp.data(), n * 4, hipMemcpyHostToDevice));
    }
    if (c.with_encoder) {
        Raw *v = find(h, "encoder.conv1.weight_v"), *g = find(h, "encoder.conv1.weight_g");
        Raw *b = find(h, "encoder.conv1.bias");
        if (!v) v = find(h, "encoder.conv1.weight");
        if (!v || !b) return fail(ACEHIP_E_STATE, "vae_finalize: missing encoder.conv1");
        h->econv1_w = (float *)valloc(h, (size_t)c.encoder_hidden * c.audio_channels * 7 * 4);
        h->econv1_b = (float *)valloc(h, (size_t)c.encoder_hidden * 4);
        if ((rc = fuse_conv_weight_f32(v->p, g ? g->p : nullptr, c.encoder_hidden, c.audio_channels, 7, 0,
                                       h->econv1_w, 0)))
            return rc;
        if ((rc = cast_bf16_f32(b->p, h->econv1_b, c.encoder_hidden, 0))) return rc;
        for (int j = 0; j < n; ++j) {
            auto &e = h->enc[j];
            const std::string p = "encoder.block." + std::to_string(j);
            const int dil[3] = {1, 3, 9};
            for (int u = 0; u < 3; ++u)
                if ((rc = make_res(h, p + ".res_unit" + std::to_string(u + 1), e.cin, dil[u], e.res[u]))) return rc;
            if ((rc = make_snake(h, p + ".snake1", e.cin, e.snake))) return rc;
            if ((rc = make_conv(h, p + ".conv1", e.cin, e.cout, 2 * e.stride, e.stride, false, true, e.conv))) return rc;
        }
        const int dm = h->enc[n - 1].cout;
        if ((rc = make_snake(h, "encoder.snake1", dm, h->esnake))) return rc;
        if ((rc = make_conv(h, "encoder.conv2", dm, c.encoder_hidden, 3, 1, false, true, h->econv2))) return rc;
    }
    HIP_TRY(hipDeviceSynchronize());
    h->finalized = true;
    return 0;
}

int acehip_vae_decode(acehip_vae *h, const void *z, int B, int T, void *wav, void *stream) {
    if (!h || !z || !wav) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized) return fail(ACEHIP_E_STATE, "vae_decode before finalize");
    if (B <= 0 || T <= 0 || T > h->cfg.max_T) return fail(ACEHIP_E_ARG, "vae_decode: T out of range");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const int n = h->cfg.n_blocks, Cz = h->cfg.latent_channels;
    const int64_t Lout = (int64_t)T * h->hop;
    int rc;
    for (int b = 0; b < B; ++b) {
        const bf16_t *zb = (const bf16_t *)z + (int64_t)b * Cz * T;
        float *wb = (float *)wav + (int64_t)b * h->cfg.audio_channels * Lout;
        bf16_t *X = h->X, *cur = h->P, *other = h->Q;
        if ((rc = cf_to_nlc(zb, Cz, T, X, s))) return rc;
        // conv1 (k7) → snaked by block 0's snake1
        if ((rc = run_conv(h->zero, h->dconv1, X, T, T, 7, 1, 1, -3, 1, 0, T, nullptr, cur, &h->dec[0].snake, nullptr, 1, s)))
            return rc;
        int64_t L = T;
        for (int j = 0; j < n; ++j) {
            const auto &bk = h->dec[j];
            const int st = bk.stride, pad = (st + 1) / 2;
            if (snake_in_block(bk)) {
                if ((rc = dec_block_snake_in(h, j, L, X, cur, other, s))) return rc;
                continue;
            }
            // ConvTranspose1d as `st` phase GEMMs → raw x (residual) + snaked x for res_unit1
            if ((rc = run_conv(h->zero, bk.convT, cur, L, L + 1, 2, 1, 1, -1, st, -pad, L * st, X, other, &bk.res[0].s1,
                               nullptr, st, s, 1)))
                return rc;
            L *= st;
            std::swap(cur, other);
            for (int u = 0; u < 3; ++u) {
                const SnakeP &next = u < 2 ? bk.res[u + 1].s1 : (j + 1 < n ? h->dec[j + 1].snake : h->dsnake);
                rc = res_unit(h->zero, bk.res[u], L, X, cur, other, next, u < 2, s);
                if (rc == 1) std::swap(cur, other);
                else if (rc) return rc;
            }
        }
        if ((rc = conv_out(cur, L, h->cfg.decoder_channels, h->dconv2_w, h->cfg.audio_channels, wb, s))) return rc;
    }
    return 0;
}

int acehip_vae_decode_blocks(acehip_vae *h, const void *z, int T, int n_blocks, void *act, void *stream) {
    if (!h || !z || !act) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized) return fail(ACEHIP_E_STATE, "vae_decode_blocks before finalize");
    const int n = h->cfg.n_blocks, Cz = h->cfg.latent_channels;
    if (T <= 0 || T > h->cfg.max_T || n_blocks < 0 || n_blocks > n)
        return fail(ACEHIP_E_ARG, "vae_decode_blocks: T or n_blocks out of range");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    int rc;
    // the same launches as acehip_vae_decode, stopped after block n_blocks
    bf16_t *X = h->X, *cur = h->P, *other = h->Q;
    if ((rc = cf_to_nlc((const bf16_t *)z, Cz, T, X, s))) return rc;
    if ((rc = run_conv(h->zero, h->dconv1, X, T, T, 7, 1, 1, -3, 1, 0, T, nullptr, cur, &h->dec[0].snake, nullptr, 1, s)))
        return rc;
    int64_t L = T, C = h->dec[0].cin;
    for (int j = 0; j < n_blocks; ++j) {
        const auto &bk = h->dec[j];
        const int st = bk.stride, pad = (st + 1) / 2;
        if (snake_in_block(bk)) {
            if ((rc = dec_block_snake_in(h, j, L, X, cur, other, s))) return rc;
            C = bk.cout;
            continue;
        }
        if ((rc = run_conv(h->zero, bk.convT, cur, L, L + 1, 2, 1, 1, -1, st, -pad, L * st, X, other, &bk.res[0].s1,
                           nullptr, st, s, 1)))
            return rc;
        L *= st;
        C = bk.cout;
        std::swap(cur, other);
        for (int u = 0; u < 3; ++u) {
            const SnakeP &next = u < 2 ? bk.res[u + 1].s1 : (j + 1 < n ? h->dec[j + 1].snake : h->dsnake);
            rc = res_unit(h->zero, bk.res[u], L, X, cur, other, next, u < 2, s);
            if (rc == 1) std::swap(cur, other);
            else if (rc) return rc;
        }
    }
    HIP_TRY(hipMemcpyAsync(act, cur, (size_t)L * C * 2, hipMemcpyDeviceToDevice, s));
    return 0;
}

int acehip_vae_encode(acehip_vae *h, const void *wav, int B, int N, const void *eps, void *z_out, void *stream) {
    if (!h || !wav || !z_out) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized || !h->cfg.with_encoder) return fail(ACEHIP_E_STATE, "vae_encode: encoder not loaded");
    // any N >= hop: every strided conv (k = 2s, pad ceil(s/2)) maps L to floor(L / s), so the
    // latent length is floor(N / hop) as in AutoencoderOobleck.encode; the samples past
    // hop·floor(N / hop) still feed the last frames through the convs' right halo
    if (B <= 0 || N < h->hop || (int64_t)N > (int64_t)h->cfg.max_T * h->hop)
        return fail(ACEHIP_E_ARG, "vae_encode: N must be in [hop, max_T * hop]");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const int n = h->cfg.n_blocks, Cz = h->cfg.latent_channels, T = N / h->hop;
    int rc;
    for (int b = 0; b < B; ++b) {
        const bf16_t *wb = (const bf16_t *)wav + (int64_t)b * h->cfg.audio_channels * N;
        bf16_t *zb = (bf16_t *)z_out + (int64_t)b * Cz * T;
        const bf16_t *eb = eps ? (const bf16_t *)eps + (int64_t)b * Cz * T : nullptr;
        bf16_t *X = h->X, *cur = h->P, *other = h->Q;
        if ((rc = conv_in(wb, N, h->cfg.audio_channels, h->econv1_w, h->econv1_b, h->cfg.encoder_hidden, X, cur,
                          h->enc[0].res[0].s1.a, h->enc[0].res[0].s1.ib, s)))
            return rc;
        int64_t L = N;
        for (int j = 0; j < n; ++j) {
            const auto &bk = h->enc[j];
            for (int u = 0; u < 3; ++u) {
                const SnakeP &next = u < 2 ? bk.res[u + 1].s1 : bk.snake;
                rc = res_unit(h->zero, bk.res[u], L, X, cur, other, next, u < 2, s);
                if (rc == 1) std::swap(cur, other);
                else if (rc) return rc;
            }
            const int st = bk.stride, pad = (st + 1) / 2;
            const SnakeP &next = j + 1 < n ? h->enc[j + 1].res[0].s1 : h->esnake;
            if ((rc = run_conv(h->zero, bk.conv, cur, L, L / st, 2 * st, 1, st, -pad, 1, 0, L / st, j + 1 < n ? X : nullptr,
                               other, &next, nullptr, 1, s)))
                return rc;
            L /= st;
            std::swap(cur, other);
        }
        // conv2 (k3, pad 1) → h [T][2·Cz] (mean | scale), then the Gaussian sample
        if ((rc = run_conv(h->zero, h->econv2, cur, L, L, 3, 1, 1, -1, 1, 0, L, X, nullptr, nullptr, nullptr, 1, s))) return rc;
        if ((rc = gauss_sample(X, T, Cz, eb, zb, s))) return rc;
    }
    return 0;
}

// ---- unit-level parity hooks (single convs / one residual unit, production kernels) ----
namespace {
struct Tmp {   // scratch for the parity hooks, freed on scope exit (after a stream sync)
    std::vector<void *> p;
    void *get(size_t bytes) {
        void *q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        p.push_back(q);
        return q;
    }
    ~Tmp() {
        for (void *q : p) (void)hipFree(q);
    }
};
const bf16_t *hook_zero_page() {
    // one zero page for the unit hooks, created once (thread-safe static init)
    static bf16_t *const z = [] {
        bf16_t *p = nullptr;
        if (hipMalloc(&p, 4096) != hipSuccess) return (bf16_t *)nullptr;
        if (hipMemset(p, 0, 4096) != hipSuccess) return (bf16_t *)nullptr;
        return p;
    }();
    return z;
}
}  // namespace

int acehip_vae_conv(int kind, const void *in, int64_t L_in, int Cin, const void *w, const void *bias,
                    const void *res, int Cout, int k, int stride, int dil, void *out, const void *alpha,
                    const void *beta, void *out_s, void *stream) {
    if (!in || !w || (!out && !out_s) || (out_s && (!alpha || !beta))) return fail(ACEHIP_E_ARG, "vae_conv: null argument");
    if (L_in <= 0 || Cin % 64 || Cout % 128 || kind < 0 || kind > 2 || stride < 1 || dil < 1)
        return fail(ACEHIP_E_ARG, "vae_conv: Cin % 64, Cout % 128, kind 0..2");
    if ((kind == 0 && (k % 2 == 0 || stride != 1)) || (kind > 0 && k != 2 * stride) || (kind == 2 && L_in % stride))
        return fail(ACEHIP_E_ARG, "vae_conv: kernel / stride inconsistent with the kind");
    hipStream_t s = (hipStream_t)stream;
    const bf16_t *zero = hook_zero_page();
    if (!zero) return fail(ACEHIP_E_OOM, "vae_conv: zero page");
    Tmp t;
    ConvL c;
    c.cin = Cin; c.cout = Cout; c.k = k; c.stride = stride; c.transposed = kind == 1;
    c.Wp = (bf16_t *)t.get((size_t)Cin * Cout * k * 2);
    c.bias = (bf16_t *)bias;
    SnakeP sn;
    if (out_s) {
        sn.a = (float *)t.get((size_t)Cout * 4);
        sn.ib = (float *)t.get((size_t)Cout * 4);
    }
    if (!c.Wp || (out_s && (!sn.a || !sn.ib))) return fail(ACEHIP_E_OOM, "vae_conv: oom");
    int rc;
    if ((rc = pack_conv_weight((const bf16_t *)w, nullptr, kind == 1 ? Cin : Cout, kind == 1 ? Cout : Cin, k,
                               kind == 1, stride, c.Wp, s)))
        return rc;
    if (out_s && (rc = snake_params((const bf16_t *)alpha, (const bf16_t *)beta, Cout, sn.a, sn.ib, s))) return rc;
    const SnakeP *snp = out_s ? &sn : nullptr;
    bf16_t *o = (bf16_t *)out, *os = (bf16_t *)out_s;
    const bf16_t *x = (const bf16_t *)in, *r = (const bf16_t *)res;
    const int pad = (stride + 1) / 2;
    int halo = 0;
    if ((kind == 0 && k == 7 && knobs().conv7 == 2) || (kind == 1 && knobs().convt)) {
        // stage the input the way the decoder's activation buffers hold it (zero rows around
        // it), so the unit test exercises the implicit-GEMM paths (ACEHIP_CONV7=2, ACEHIP_CONVT=1)
        const size_t rowb = (size_t)Cin * 2, padb = (size_t)kActPadRows * rowb;
        char *xp = (char *)t.get((size_t)L_in * rowb + 2 * padb);
        if (!xp) return fail(ACEHIP_E_OOM, "vae_conv: oom");
        HIP_TRY(hipMemsetAsync(xp, 0, padb, s));
        HIP_TRY(hipMemcpyAsync(xp + padb, in, (size_t)L_in * rowb, hipMemcpyDeviceToDevice, s));
        x = (const bf16_t *)(xp + padb);
        halo = 1;
    }
    if (kind == 0) rc = run_conv(zero, c, x, L_in, L_in, k, dil, 1, -dil * (k - 1) / 2, 1, 0, L_in, o, os, snp, r, 1, s, halo);
    else if (kind == 1)
        rc = run_conv(zero, c, x, L_in, L_in + 1, 2, 1, 1, -1, stride, -pad, L_in * stride, o, os, snp, r, stride, s, halo);
    else rc = run_conv(zero, c, x, L_in, L_in / stride, k, 1, stride, -pad, 1, 0, L_in / stride, o, os, snp, r, 1, s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
}

int acehip_vae_resunit(const void *x, const void *x_s, int64_t L, int C, int dil, const void *w1, const void *b1,
                       const void *alpha2, const void *beta2, const void *w2, const void *b2, const void *alpha_n,
                       const void *beta_n, void *x_out, void *xs_out, void *stream) {
    if (!x || !x_s || !w1 || !b1 || !alpha2 || !beta2 || !w2 || !b2 || !alpha_n || !beta_n || !xs_out)
        return fail(ACEHIP_E_ARG, "vae_resunit: null argument");
    if (C != 128 || L <= 0 || dil < 1 || dil > 9) return fail(ACEHIP_E_ARG, "vae_resunit: C = 128, dilation 1..9");
    hipStream_t s = (hipStream_t)stream;
    const bf16_t *zero = hook_zero_page();
    if (!zero) return fail(ACEHIP_E_OOM, "vae_resunit: zero page");
    Tmp t;
    // the decoder's activation layout: kActPadRows zero rows in front, addressable rows behind
    const size_t rowb = (size_t)C * 2, pad = std::max((size_t)kActPadRows * 2048 * 2, (size_t)kResWindowBackRows * 128 * 2);
    char *xs_pad = (char *)t.get((size_t)L * rowb + 2 * pad);
    bf16_t *xr = (bf16_t *)t.get((size_t)L * rowb);
    ResU r;
    r.dil = dil;
    r.c1.cin = r.c1.cout = C; r.c1.k = 7;
    r.c2.cin = r.c2.cout = C; r.c2.k = 1;
    r.c1.Wp = (bf16_t *)t.get((size_t)C * C * 7 * 2);
    r.c2.Wp = (bf16_t *)t.get((size_t)C * C * 2);
    r.W2p = (bf16_t *)t.get((size_t)C * C * 2);
    r.c1.bias = (bf16_t *)b1;
    r.c2.bias = (bf16_t *)b2;
    r.s2.a = (float *)t.get(C * 4); r.s2.ib = (float *)t.get(C * 4);
    SnakeP nx;
    nx.a = (float *)t.get(C * 4); nx.ib = (float *)t.get(C * 4);
    bf16_t *other = (bf16_t *)t.get((size_t)L * rowb);
    if (!xs_pad || !xr || !r.c1.Wp || !r.c2.Wp || !r.W2p || !r.s2.a || !r.s2.ib || !nx.a || !nx.ib || !other)
        return fail(ACEHIP_E_OOM, "vae_resunit: oom");
    bf16_t *cur = (bf16_t *)(xs_pad + pad);
    HIP_TRY(hipMemsetAsync(xs_pad, 0, pad, s));
    HIP_TRY(hipMemcpyAsync(cur, x_s, (size_t)L * rowb, hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemcpyAsync(xr, x, (size_t)L * rowb, hipMemcpyDeviceToDevice, s));
    int rc;
    if ((rc = pack_conv_weight((const bf16_t *)w1, nullptr, C, C, 7, 0, 1, r.c1.Wp, s))) return rc;
    if ((rc = pack_conv_weight((const bf16_t *)w2, nullptr, C, C, 1, 0, 1, r.c2.Wp, s))) return rc;
    if ((rc = permute_k1_weight(r.c2.Wp, r.W2p, C, s))) return rc;
    if ((rc = snake_params((const bf16_t *)alpha2, (const bf16_t *)beta2, C, r.s2.a, r.s2.ib, s))) return rc;
    if ((rc = snake_params((const bf16_t *)alpha_n, (const bf16_t *)beta_n, C, nx.a, nx.ib, s))) return rc;
    rc = res_unit(zero, r, L, xr, cur, other, nx, x_out != nullptr, s);
    if (rc < 0 || rc > 1) return rc;
    HIP_TRY(hipMemcpyAsync(xs_out, rc == 1 ? other : cur, (size_t)L * rowb, hipMemcpyDeviceToDevice, s));
    if (x_out) HIP_TRY(hipMemcpyAsync(x_out, xr, (size_t)L * rowb, hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
}

int acehip_vae_destroy(acehip_vae *h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    for (void *p : h->allocs) (void)hipFree(p);
    delete h;
    return 0;
}

// _decode_generate_music_pred_latents' output guard (generate_music_decode.py:190-192):
// peak = |wav|.amax over (channels, samples) per song; if any peak > 1 every song
// is divided by max(peak, 1) — per song that is "divide by peak when peak > 1",
// IEEE division as torch does it.  wav fp32 [B][n] in place; peak: [B] scratch.
int acehip_wav_peak_normalize(float *wav, int B, int64_t n, float *peak, void *stream) {
    if (!wav || !peak || B <= 0 || n <= 0) return fail(ACEHIP_E_ARG, "wav_peak_normalize: argument");
    if (n % 4) return fail(ACEHIP_E_ARG, "wav_peak_normalize: samples per song must be a multiple of 4");
    return wav_peak_normalize(wav, B, n, peak, (hipStream_t)stream);
}

// the guard above fused with normalize_audio(target_db) of acestep/inference.py:674-679
// (audio_utils.py:24-62): one read pass (peak) + one read-write pass per song
int acehip_wav_postprocess(float *wav, int B, int64_t n, float *peak, int guard, float target_amp, void *stream) {
    if (!wav || !peak || B <= 0 || n <= 0) return fail(ACEHIP_E_ARG, "wav_postprocess: argument");
    if (n % 4) return fail(ACEHIP_E_ARG, "wav_postprocess: samples per song must be a multiple of 4");
    if (!(target_amp >= 0.f)) return fail(ACEHIP_E_ARG, "wav_postprocess: target_amp must be >= 0");
    return wav_peak_normalize(wav, B, n, peak, (hipStream_t)stream, target_amp, guard);
}

// the same pass pair with the sample conversion of the output leg fused in: wav fp32 [B][C][N]
// (channels-first, updated in place as above) → pcm int16 [B][N][C] (interleaved frames), ready
// for a WAV / FLAC writer after one device→host copy of half the fp32 bytes
int acehip_wav_postprocess_pcm16(float *wav, int B, int C, int64_t N, float *peak, int guard, float target_amp,
                                 int16_t *pcm, void *stream) {
    if (!wav || !peak || !pcm || B <= 0 || N <= 0) return fail(ACEHIP_E_ARG, "wav_postprocess_pcm16: argument");
    if (C != 1 && C != 2) return fail(ACEHIP_E_ARG, "wav_postprocess_pcm16: 1 or 2 channels");
    if (N % 4) return fail(ACEHIP_E_ARG, "wav_postprocess_pcm16: samples per channel must be a multiple of 4");
    if (!(target_amp >= 0.f)) return fail(ACEHIP_E_ARG, "wav_postprocess_pcm16: target_amp must be >= 0");
    return wav_postprocess_pcm16(wav, B, C, N, peak, (hipStream_t)stream, target_amp, guard, (short *)pcm);
}

}  // extern "C"
