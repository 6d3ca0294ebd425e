// dit.hip — the DiT runtime behind acehip_dit_* (C ABI in include/acehip.h).
//
// Owns the packed bf16 weights, the cross-attention K/V cache and a
// workspace sized at create time; acehip_dit_forward enqueues one whole
// AceStepDiTModel.forward (reference base:1303-1507) on the caller's stream
// with no allocation and no host synchronisation.
//
// Weight packing (from the reference state-dict names):
//   self q|k|v rows concatenated → one QKV GEMM (N = q + 2kv)
//   cross k|v rows concatenated → one GEMM per layer at set_condition
//   gate/up interleaved in 32-row panels → one GEMM with a SwiGLU epilogue
//   proj_in  Conv1d [D][192][2]  → [D][2·192] (k-major) so the patch GEMM
//            reads [T][192] rows pairwise with no im2col copy
//   proj_out ConvT  [D][64][2]   → [2·64][D] so the GEMM output [S][128] is
//            the de-patchified [2S][64] sequence in place
//   scale_shift_tables of all layers contiguous → one modulation launch
#include <unistd.h>
#include <map>
#include <mutex>
#include <cmath>
#include <vector>
#include <cstring>

#include "kernels.h"
#include "../../include/acehip.h"

using namespace acehip;

namespace {

enum PackKind { P_COPY, P_GU_GATE, P_GU_UP, P_PROJ_IN, P_PROJ_OUT_W, P_PROJ_OUT_B,
                // fp32 parity mode: fp32 destinations, reference layouts except the patch convs
                P_F32, P_F32_PROJ_IN, P_F32_PROJ_OUT_W, P_F32_PROJ_OUT_B };

struct Slot {
    bf16_t *dst = nullptr;
    std::vector<int64_t> shape;
    PackKind kind = P_COPY;
    bool set = false;
    float *dst_f32 = nullptr;
};

}  // namespace

struct acehip_dit {
    int device = 0;
    acehip_dit_cfg cfg{};
    std::vector<uint8_t> sliding;
    int D = 0, F = 0, qd = 0, kvd = 0, L = 0;
    bool finalized = false, have_cond = false;
    int cond_Bc = 0, cond_Lenc = 0;

    std::vector<void *> allocs;
    std::map<std::string, Slot> slots;

    // weights
    bf16_t *tables = nullptr;   // [L][6][D]
    struct Layer {
        bf16_t *n_sa, *n_ca, *n_mlp, *wqkv, *wo, *qn, *kn, *cqn, *ckn, *wcq, *wckv, *wco, *wgu, *wdown;
    };
    std::vector<Layer> layers;
    bf16_t *sst_out, *win, *bin, *wce, *bce, *norm_out, *wout, *bout;
    bf16_t *te_l1[2], *te_b1[2], *te_l2[2], *te_b2[2], *te_tp[2], *te_btp[2];
    float *freqs = nullptr;          // [128] sinusoid frequencies
    float *inv_freq_host = nullptr;  // optional override, [hd/2]
    std::vector<float> inv_freq_override;
    bf16_t *attn_ws = nullptr;  // attention tail-split workspace (attention_ws_bytes())
    bf16_t *rope_cos = nullptr, *rope_sin = nullptr;   // [max_S][hd]

    // workspace
    bf16_t *X, *XN, *Qh, *Kh, *Vh, *AO, *Hb, *Xin, *O2;
    bf16_t *emb[2], *h1, *temb_e[2], *proj_e[2], *temb, *proj, *mod, *mod_out;
    bf16_t *Kc, *Vc, *E, *KVtmp;
    int kv_group = 1;                  // layers per cross-K/V GEMM at set_condition (KVtmp holds that many)
    bf16_t *wckv_all = nullptr;        // every layer's cross K/V projection, [L][2·kvd][D] (one GEMM)
    bf16_t *gemv_act = nullptr;        // 16 × D: bf16(silu(x)) rows of the timestep MLPs (gemv_small)
    // CFG null rows (acehip_dit_set_uniform_rows): batch rows >= uniform_from have an
    // encoder sequence that is one vector repeated, so their cross-attention is the
    // constant V row and their cross-O output the per-layer constant cnull[l]
    int uniform_from = 1 << 30;
    bf16_t *cnull = nullptr, *vnull = nullptr;   // [L][D], [q_dim]
    // timestep MLP outputs of a whole schedule (acehip_dit_set_timesteps): row i = step i's
    // temb [D] and proj [6D]; ts_scratch holds the batched MLP intermediates
    int ts_n = 0, ts_cap = 0;
    bf16_t *ts_temb = nullptr, *ts_proj = nullptr, *ts_scratch = nullptr;
    bf16_t *tmp;   // weight staging (fp32 → bf16 casts, host repacks)
    void *gemm_ws = nullptr;   // split-K partials for small-M GEMMs (short songs / turbo)
    size_t tmp_elems = 0;

    // optional per-kernel event timing (acehip_dit_profile)
    static constexpr int NKIND = 7, NPAIR = 16384;
    bool prof = false;
    unsigned prof_mask = 0x7f;         // kinds recorded while profiling (acehip_dit_profile_kinds)
    std::vector<hipEvent_t> ev;        // 2·NPAIR events
    std::vector<int> ev_kind;          // kind of each recorded pair
    int ev_used = 0;

    // HIP graph of the forward's pointer-independent middle (acehip_dit_set_graph): the
    // timestep MLPs, modulation, proj_in and the layer stack read and write only handle
    // buffers, so one capture per (Bc, S, Lenc, uniform_from) replays for every step
    bool graph_on = false;
    hipStream_t cap_stream = nullptr;
    hipGraphExec_t gexec = nullptr;
    int gkey[6] = {-1, -1, -1, -1, -1, -1};

    // fp32 parity mode (acehip_dit_cfg.fp32): fp32 weights and workspace,
    // the kernels of f32.hip; the bf16 buffers above are not allocated
    bool f32 = false;
    struct F32 {
        struct Layer {
            float *n_sa, *n_ca, *n_mlp, *wqkv, *wo, *qn, *kn, *cqn, *ckn, *wcq, *wckv, *wco, *wg, *wu, *wdown;
        };
        std::vector<Layer> layers;
        float *tables, *sst_out, *win, *bin, *wce, *bce, *norm_out, *wout, *bout;
        float *te_l1[2], *te_b1[2], *te_l2[2], *te_b2[2], *te_tp[2], *te_btp[2];
        float *rope_cos, *rope_sin;
        float *X, *XN, *QKV, *Qh, *Kh, *Vh, *AO, *G, *U, *Hb, *Xin, *O2;
        float *emb[2], *h1, *temb_e[2], *proj_e[2], *temb, *proj, *mod, *mod_out;
        float *Kc, *Vc, *E, *KVtmp;
    } f{};
};

static int forward_body(acehip_dit *h, int Bc, int S, bool dup, bool ts_cached, hipStream_t s);
static int timestep_mlps(acehip_dit *h, const bf16_t *const emb[2], int rows, bf16_t *h1, bf16_t *const temb_e[2],
                         bf16_t *const proj_e[2], bf16_t *temb, bf16_t *proj, hipStream_t s);
static int forward_bf16(acehip_dit *h, const void *xt, const void *ctx, int Bx, const float *t, const float *t_r,
                        int t_stride, int step, int Bc, int T, void *vt_out, hipStream_t s);
static int create_f32(acehip_dit *h);
static int set_weight_f32(acehip_dit *h, Slot &s, const void *ptr, int dtype, int64_t n, int on_device);
static int build_rope_f32(acehip_dit *h);
static int set_condition_f32(acehip_dit *h, const float *enc, int Bc, int Lenc, hipStream_t s);
static int forward_f32(acehip_dit *h, const float *xt, const float *ctx, int Bx, const float *t, const float *t_r,
                       int t_stride, int Bc, int T, float *vt_out, hipStream_t s);

// every GEMM of this runtime may use the handle's split-K workspace (small-M grids)
static inline int hgemm(acehip_dit *h, GemmArgs g, hipStream_t s, RowAdd *defer = nullptr) {
    g.ws = h->gemm_ws;
    g.ws_bytes = h->gemm_ws ? GEMM_WS_BYTES : 0;
    return gemm(g, s, defer);
}

namespace {

thread_local std::string g_err;

bf16_t *dalloc(acehip_dit *h, size_t elems) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(elems, 1) * 2) != hipSuccess) return nullptr;
    h->allocs.push_back(p);
    return (bf16_t *)p;
}

void add_slot(acehip_dit *h, const std::string &name, bf16_t *dst, std::vector<int64_t> shape,
              PackKind kind = P_COPY) {
    Slot s;
    s.dst = dst;
    s.shape = std::move(shape);
    s.kind = kind;
    h->slots[name] = s;
}

int64_t numel(const std::vector<int64_t> &s) {
    int64_t n = 1;
    for (auto v : s) n *= v;
    return n;
}

// host-side bf16 rounding (same as device f2bf)
inline bf16_t hf2bf(float f) { return f2bf(f); }

int build_rope(acehip_dit *h) {
    const int hd = h->cfg.head_dim, S = h->cfg.max_S;
    std::vector<float> inv(hd / 2);
    for (int i = 0; i < hd / 2; ++i) {
        float v;
        if (!h->inv_freq_override.empty()) v = h->inv_freq_override[i];
        else v = 1.0f / powf(h->cfg.rope_theta, (float)(2 * i) / (float)hd);
        inv[i] = bf2f(hf2bf(v));   // model.to(bf16) casts the inv_freq buffer (init_service_loader.py:81-89)
    }
    std::vector<bf16_t> c((size_t)S * hd), s((size_t)S * hd);
    for (int p = 0; p < S; ++p)
        for (int i = 0; i < hd; ++i) {
            const float f = (float)p * inv[i % (hd / 2)];
            c[(size_t)p * hd + i] = hf2bf((float)cos((double)f));
            s[(size_t)p * hd + i] = hf2bf((float)sin((double)f));
        }
    HIP_TRY(hipMemcpy(h->rope_cos, c.data(), c.size() * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->rope_sin, s.data(), s.size() * 2, hipMemcpyHostToDevice));
    return 0;
}

// record an event pair around `launch` when profiling is on
template <class F>
int timed(acehip_dit *h, int kind, hipStream_t s, F &&launch) {
    if (!h->prof || !((h->prof_mask >> kind) & 1u) || h->ev_used >= acehip_dit::NPAIR) return launch();
    const int i = h->ev_used++;
    h->ev_kind[i] = kind;
    if (kind == 0) {
        // the SwiGLU GEMM (the bench's roofline kernel, timed inside the measured song): the
        // events ride on its launches (gemm_ext_events) instead of two event packets that
        // would idle the GPU ≈ 5.6 µs each; a path without launch events drops the sample
        gemm_ext_events(h->ev[2 * i], h->ev[2 * i + 1]);
        const int rc = launch();
        if (!gemm_ext_events(nullptr, nullptr)) h->ev_kind[i] = -1;
        return rc;
    }
    HIP_TRY(hipEventRecord(h->ev[2 * i], s));
    const int rc = launch();
    HIP_TRY(hipEventRecord(h->ev[2 * i + 1], s));
    return rc;
}

}  // namespace

namespace acehip {
void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
}  // namespace acehip

extern "C" {

int acehip_get_version(void) { return ACEHIP_VERSION; }
const char *acehip_last_error(void) { return g_err.c_str(); }

int acehip_dit_create(int device, const acehip_dit_cfg *cfg, acehip_dit **out) {
    if (!cfg || !out) return fail(ACEHIP_E_ARG, "dit_create: null argument");
    if (cfg->head_dim != 128) return fail(ACEHIP_E_ARG, "dit_create: head_dim must be 128");
    if (cfg->hidden % 256 || cfg->intermediate % 64 || cfg->heads % cfg->kv_heads)
        return fail(ACEHIP_E_ARG, "dit_create: unsupported dims");
    if (cfg->patch != 2 || cfg->in_channels != 192 || cfg->out_channels != 64)
        return fail(ACEHIP_E_ARG, "dit_create: patch 2 / 192 in / 64 out required");
    if (cfg->max_Bc > 16 || cfg->max_Bc <= 0 || cfg->max_S <= 0 || cfg->max_Lenc <= 0)
        return fail(ACEHIP_E_ARG, "dit_create: max_Bc in [1,16], max_S/max_Lenc > 0");
    HIP_TRY(hipSetDevice(device));
    auto *h = new acehip_dit();
    h->device = device;
    h->cfg = *cfg;
    h->D = cfg->hidden; h->F = cfg->intermediate; h->L = cfg->layers;
    h->qd = cfg->heads * cfg->head_dim; h->kvd = cfg->kv_heads * cfg->head_dim;
    h->sliding.resize(h->L);
    for (int i = 0; i < h->L; ++i) h->sliding[i] = cfg->sliding ? cfg->sliding[i] : ((i + 1) % 2);
    h->cfg.sliding = nullptr;
    h->graph_on = knobs().dit_graph == 1;
    if (cfg->fp32) {
        h->f32 = true;
        h->graph_on = false;
        const int rc = create_f32(h);
        if (rc) {
            const std::string e = acehip_last_error();
            acehip_dit_destroy(h);
            return fail(rc, e);
        }
        *out = h;
        return 0;
    }
    const int D = h->D, F = h->F, qd = h->qd, kvd = h->kvd, L = h->L;
    bool ok = true;
    auto A = [&](size_t n) { bf16_t *p = dalloc(h, n); ok = ok && p; return p; };

    h->tables = A((size_t)L * 6 * D);
    h->layers.resize(L);
    // the layers' cross K/V projections side by side: set_condition runs them as ONE GEMM
    // (N = L·2·kvd) instead of L small-M ones
    h->wckv_all = A((size_t)L * 2 * kvd * D);
    for (int i = 0; i < L; ++i) {
        auto &ly = h->layers[i];
        ly.n_sa = A(D); ly.n_ca = A(D); ly.n_mlp = A(D);
        ly.wqkv = A((size_t)(qd + 2 * kvd) * D); ly.wo = A((size_t)D * qd);
        ly.qn = A(128); ly.kn = A(128); ly.cqn = A(128); ly.ckn = A(128);
        ly.wcq = A((size_t)qd * D); ly.wckv = h->wckv_all ? h->wckv_all + (size_t)i * 2 * kvd * D : nullptr;
        ly.wco = A((size_t)D * qd);
        ly.wgu = A((size_t)2 * F * D); ly.wdown = A((size_t)D * F);
        if (!ok) break;
        const std::string p = "layers." + std::to_string(i);
        add_slot(h, p + ".scale_shift_table", h->tables + (size_t)i * 6 * D, {1, 6, D});
        add_slot(h, p + ".self_attn_norm.weight", ly.n_sa, {D});
        add_slot(h, p + ".cross_attn_norm.weight", ly.n_ca, {D});
        add_slot(h, p + ".mlp_norm.weight", ly.n_mlp, {D});
        add_slot(h, p + ".self_attn.q_proj.weight", ly.wqkv, {qd, D});
        add_slot(h, p + ".self_attn.k_proj.weight", ly.wqkv + (size_t)qd * D, {kvd, D});
        add_slot(h, p + ".self_attn.v_proj.weight", ly.wqkv + (size_t)(qd + kvd) * D, {kvd, D});
        add_slot(h, p + ".self_attn.o_proj.weight", ly.wo, {D, qd});
        add_slot(h, p + ".self_attn.q_norm.weight", ly.qn, {128});
        add_slot(h, p + ".self_attn.k_norm.weight", ly.kn, {128});
        add_slot(h, p + ".cross_attn.q_proj.weight", ly.wcq, {qd, D});
        add_slot(h, p + ".cross_attn.k_proj.weight", ly.wckv, {kvd, D});
        add_slot(h, p + ".cross_attn.v_proj.weight", ly.wckv + (size_t)kvd * D, {kvd, D});
        add_slot(h, p + ".cross_attn.o_proj.weight", ly.wco, {D, qd});
        add_slot(h, p + ".cross_attn.q_norm.weight", ly.cqn, {128});
        add_slot(h, p + ".cross_attn.k_norm.weight", ly.ckn, {128});
        add_slot(h, p + ".mlp.gate_proj.weight", ly.wgu, {F, D}, P_GU_GATE);
        add_slot(h, p + ".mlp.up_proj.weight", ly.wgu, {F, D}, P_GU_UP);
        add_slot(h, p + ".mlp.down_proj.weight", ly.wdown, {D, F});
    }
    h->sst_out = A(2 * D); h->win = A((size_t)D * 384); h->bin = A(D);
    h->wce = A((size_t)D * D); h->bce = A(D); h->norm_out = A(D);
    h->wout = A((size_t)128 * D); h->bout = A(128);
    const char *te_names[2] = {"time_embed", "time_embed_r"};
    for (int e = 0; e < 2; ++e) {
        h->te_l1[e] = A((size_t)D * 256); h->te_b1[e] = A(D);
        h->te_l2[e] = A((size_t)D * D); h->te_b2[e] = A(D);
        h->te_tp[e] = A((size_t)6 * D * D); h->te_btp[e] = A(6 * D);
        if (!ok) break;
        const std::string p = te_names[e];
        add_slot(h, p + ".linear_1.weight", h->te_l1[e], {D, 256});
        add_slot(h, p + ".linear_1.bias", h->te_b1[e], {D});
        add_slot(h, p + ".linear_2.weight", h->te_l2[e], {D, D});
        add_slot(h, p + ".linear_2.bias", h->te_b2[e], {D});
        add_slot(h, p + ".time_proj.weight", h->te_tp[e], {6 * D, D});
        add_slot(h, p + ".time_proj.bias", h->te_btp[e], {6 * D});
    }
    if (ok) {
        add_slot(h, "scale_shift_table", h->sst_out, {1, 2, D});
        add_slot(h, "proj_in.1.weight", h->win, {D, 192, 2}, P_PROJ_IN);
        add_slot(h, "proj_in.1.bias", h->bin, {D});
        add_slot(h, "condition_embedder.weight", h->wce, {D, D});
        add_slot(h, "condition_embedder.bias", h->bce, {D});
        add_slot(h, "norm_out.weight", h->norm_out, {D});
        add_slot(h, "proj_out.1.weight", h->wout, {D, 64, 2}, P_PROJ_OUT_W);
        add_slot(h, "proj_out.1.bias", h->bout, {64}, P_PROJ_OUT_B);
    }
    // workspace
    const size_t S = cfg->max_S, Bc = cfg->max_Bc, M = S * Bc, Le = cfg->max_Lenc;
    h->X = A(M * D); h->XN = A(M * D);
    h->Qh = A(M * qd); h->Kh = A(M * kvd); h->Vh = A(M * kvd); h->AO = A(M * qd);
    h->Hb = A(M * F); h->Xin = A(M * 384); h->O2 = A(M * 128);
    for (int e = 0; e < 2; ++e) {
        h->emb[e] = A(Bc * 256); h->temb_e[e] = A(Bc * D); h->proj_e[e] = A(Bc * 6 * D);
    }
    h->h1 = A(Bc * D); h->temb = A(Bc * D); h->proj = A(Bc * 6 * D);
    h->mod = A((size_t)L * Bc * 6 * D); h->mod_out = A(Bc * 2 * D);
    h->Kc = A((size_t)L * Bc * kvd * Le); h->Vc = A((size_t)L * Bc * kvd * Le);
    // cross K/V scratch: the layers' K/V projections run as GEMMs over groups of kv_group layers
    // (N = kv_group·2·kvd), the group sized so the scratch stays ≤ 256 MiB at max_Bc·max_Lenc
    // (all 24 layers in one GEMM for a CFG song, one layer per GEMM at the 16 × 2048 maximum)
    {
        const size_t per_layer = Bc * Le * 2 * kvd * 2;
        const size_t bound = (size_t)knobs().kv_group_kib << 10;      // 256 MiB by default
        h->kv_group = (int)std::max<size_t>(1, std::min<size_t>((size_t)L, bound / per_layer));
    }
    h->E = A(Bc * Le * D); h->KVtmp = A(Bc * Le * 2 * kvd * (size_t)h->kv_group);
    h->cnull = A((size_t)L * D); h->vnull = A(qd);
    h->gemv_act = A((size_t)16 * D);
    h->gemm_ws = A(GEMM_WS_BYTES / 2);
    h->rope_cos = A(S * 128); h->rope_sin = A(S * 128);
    h->tmp_elems = std::max<size_t>((size_t)6 * D * D, (size_t)D * 384);
    h->tmp = A(h->tmp_elems * 2);   // room for an fp32 staging copy
    {   // attention tail-split partials + self-resetting counters (zeroed once)
        const size_t wb = attention_ws_bytes();
        h->attn_ws = A((wb + 1) / 2);
        if (h->attn_ws && hipMemset(h->attn_ws, 0, wb) != hipSuccess) ok = false;
    }
    void *fr = nullptr;
    if (ok && hipMalloc(&fr, 128 * sizeof(float)) == hipSuccess) {
        h->allocs.push_back(fr);
        h->freqs = (float *)fr;
        float f[128];
        for (int i = 0; i < 128; ++i)   // torch: exp(-ln(1e4) * arange(128, f32) / 128) in fp32 (base:239-241)
            f[i] = expf((-9.210340371976184f * (float)i) / 128.0f);
        ok = hipMemcpy(h->freqs, f, sizeof(f), hipMemcpyHostToDevice) == hipSuccess;
    } else {
        ok = false;
    }
    if (!ok) {
        acehip_dit_destroy(h);
        return fail(ACEHIP_E_OOM, "dit_create: device allocation failed");
    }
    *out = h;
    return 0;
}

int acehip_dit_set_weight(acehip_dit *h, const char *name, const void *ptr, int dtype, int ndim,
                          const int64_t *shape, int on_device) {
    if (!h || !name || !ptr || !shape) return fail(ACEHIP_E_ARG, "dit_set_weight: null argument");
    HIP_TRY(hipSetDevice(h->device));
    std::string nm(name);
    if (nm.rfind("decoder.", 0) == 0) nm = nm.substr(8);
    if (nm == "_timestep_freqs" || nm == "_rope_inv_freq") {
        // optional overrides computed by the caller's torch (exact reference constants), fp32
        if (dtype != ACEHIP_F32) return fail(ACEHIP_E_ARG, nm + ": fp32 required");
        const int n = (int)shape[0];
        std::vector<float> v(n);
        HIP_TRY(hipMemcpy(v.data(), ptr, n * 4, on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
        if (nm == "_timestep_freqs") {
            if (n != 128) return fail(ACEHIP_E_ARG, "_timestep_freqs must have 128 entries");
            HIP_TRY(hipMemcpy(h->freqs, v.data(), 512, hipMemcpyHostToDevice));
        } else {
            if (n != h->cfg.head_dim / 2) return fail(ACEHIP_E_ARG, "_rope_inv_freq size");
            h->inv_freq_override = v;
        }
        return 0;
    }
    if (nm == "rotary_emb.inv_freq") return 0;  // non-persistent buffer; recomputed
    auto it = h->slots.find(nm);
    if (it == h->slots.end()) return fail(ACEHIP_E_NAME, "dit_set_weight: unknown weight " + nm);
    Slot &s = it->second;
    std::vector<int64_t> sh(shape, shape + ndim);
    if (sh != s.shape) {
        std::string e = "dit_set_weight: shape mismatch for " + nm + " got [";
        for (auto v : sh) e += std::to_string(v) + ",";
        e += "] want [";
        for (auto v : s.shape) e += std::to_string(v) + ",";
        return fail(ACEHIP_E_ARG, e + "]");
    }
    const int64_t n = numel(sh);
    if (dtype != ACEHIP_F32 && dtype != ACEHIP_BF16) return fail(ACEHIP_E_ARG, "dtype");
    if (h->f32) return set_weight_f32(h, s, ptr, dtype, n, on_device);
    // bring to a contiguous bf16 device source
    const bf16_t *src = nullptr;
    std::vector<bf16_t> hb;
    if (s.kind == P_PROJ_IN || s.kind == P_PROJ_OUT_W || s.kind == P_PROJ_OUT_B) {
        // small: repack on host
        std::vector<float> f(n);
        if (dtype == ACEHIP_F32) {
            HIP_TRY(hipMemcpy(f.data(), ptr, n * 4, on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
        } else {
            std::vector<bf16_t> b(n);
            HIP_TRY(hipMemcpy(b.data(), ptr, n * 2, on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
            for (int64_t i = 0; i < n; ++i) f[i] = bf2f(b[i]);
        }
        hb.resize(s.kind == P_PROJ_OUT_B ? 128 : n);
        if (s.kind == P_PROJ_IN) {         // [D][192][2] → [D][k*192 + c]
            const int64_t D = sh[0];
            for (int64_t o = 0; o < D; ++o)
                for (int c = 0; c < 192; ++c)
                    for (int k = 0; k < 2; ++k) hb[o * 384 + k * 192 + c] = hf2bf(f[(o * 192 + c) * 2 + k]);
        } else if (s.kind == P_PROJ_OUT_W) {   // [D][64][2] → [k*64 + o][D]
            const int64_t D = sh[0];
            for (int64_t c = 0; c < D; ++c)
                for (int o = 0; o < 64; ++o)
                    for (int k = 0; k < 2; ++k) hb[(k * 64 + o) * D + c] = hf2bf(f[(c * 64 + o) * 2 + k]);
        } else {                               // bias [64] → [k*64 + o]
            for (int k = 0; k < 2; ++k)
                for (int o = 0; o < 64; ++o) hb[k * 64 + o] = hf2bf(f[o]);
        }
        HIP_TRY(hipMemcpy(s.dst, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
        s.set = true;
        return 0;
    }
    if (dtype == ACEHIP_F32) {
        // cast through the staging buffer in chunks
        // tmp holds tmp_elems floats (4·tmp_elems bytes)
        const float *fsrc = (const float *)ptr;
        float *fstage = (float *)h->tmp;
        if (s.kind == P_COPY) {
            // chunked cast straight into the destination
            const int64_t chunk = (int64_t)h->tmp_elems;
            for (int64_t off = 0; off < n; off += chunk) {
                const int64_t c = std::min(chunk, n - off);
                HIP_TRY(hipMemcpy(fstage, fsrc + off, c * 4, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
                int rc = cast_f32_bf16(fstage, s.dst + off, c, 0);
                if (rc) return rc;
                HIP_TRY(hipDeviceSynchronize());
            }
            s.set = true;
            return 0;
        }
        if ((size_t)n * 6 > h->tmp_elems * 4) return fail(ACEHIP_E_ARG, "fp32 weight too large for staging; pass bf16");
        HIP_TRY(hipMemcpy(fstage, fsrc, n * 4, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
        bf16_t *b16 = h->tmp + n * 2;   // bf16 copy right after the fp32 staging
        int rc = cast_f32_bf16(fstage, b16, n, 0);
        if (rc) return rc;
        HIP_TRY(hipDeviceSynchronize());
        src = b16;
    } else {
        if (s.kind == P_COPY) {
            HIP_TRY(hipMemcpy(s.dst, ptr, n * 2, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
            s.set = true;
            return 0;
        }
        src = (const bf16_t *)ptr;
    }
    const hipMemcpyKind kind = (dtype == ACEHIP_F32 || on_device) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (s.kind == P_GU_GATE || s.kind == P_GU_UP) {
        const int64_t F = sh[0], K = sh[1];
        bf16_t *dst = s.dst + (s.kind == P_GU_UP ? 32 * K : 0);
        HIP_TRY(hipMemcpy2D(dst, 64 * K * 2, src, 32 * K * 2, 32 * K * 2, F / 32, kind));
        s.set = true;
        return 0;
    }
    return fail(ACEHIP_E_ARG, "dit_set_weight: unhandled pack kind");
}

// Buffers of acehip_dit_set_timesteps for `cap` steps: allocated at finalize for kTsCap
// steps (every schedule the reference builds: ≤ 60 base/sft steps, ≤ 20 turbo), grown only
// by a longer schedule (the header documents that exception to "no allocation in calls").
static constexpr int kTsCap = 64;
static int alloc_timesteps(acehip_dit *h, int n_steps) {
    for (bf16_t *p : {h->ts_temb, h->ts_proj, h->ts_scratch})
        if (p) (void)hipFree(p);
    h->ts_temb = h->ts_proj = h->ts_scratch = nullptr;
    h->ts_cap = h->ts_n = 0;
    const int D = h->D;
    const int cap = std::max(n_steps, kTsCap);
    // scratch: emb [2][cap][256], h1 [cap][D], temb_e [2][cap][D], proj_e [2][cap][6D]
    const size_t scratch = (size_t)cap * (2 * 256 + D + 2 * D + 2 * 6 * D);
    HIP_TRY(hipMalloc(&h->ts_temb, (size_t)cap * D * 2));
    HIP_TRY(hipMalloc(&h->ts_proj, (size_t)cap * 6 * D * 2));
    HIP_TRY(hipMalloc(&h->ts_scratch, scratch * 2));
    h->ts_cap = cap;
    return 0;
}

int acehip_dit_finalize(acehip_dit *h) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    HIP_TRY(hipSetDevice(h->device));
    if (h->gexec) { HIP_TRY(hipGraphExecDestroy(h->gexec)); h->gexec = nullptr; }   // re-capture
    std::string missing;
    for (auto &kv : h->slots)
        if (!kv.second.set) missing += kv.first + " ";
    if (!missing.empty()) return fail(ACEHIP_E_STATE, "dit_finalize: missing weights: " + missing.substr(0, 400));
    if (h->F % 32) return fail(ACEHIP_E_ARG, "intermediate must be a multiple of 32");
    int rc = h->f32 ? build_rope_f32(h) : build_rope(h);
    if (rc) return rc;
    if (!h->f32 && h->ts_cap < kTsCap && (rc = alloc_timesteps(h, kTsCap))) return rc;
    HIP_TRY(hipDeviceSynchronize());
    h->finalized = true;
    return 0;
}

int acehip_dit_set_condition(acehip_dit *h, const void *enc, int Bc, int Lenc, void *stream) {
    if (!h || !enc) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized) return fail(ACEHIP_E_STATE, "set_condition before finalize");
    if (Bc <= 0 || Bc > h->cfg.max_Bc || Lenc <= 0 || Lenc > h->cfg.max_Lenc)
        return fail(ACEHIP_E_ARG, "set_condition: Bc/Lenc out of range");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    if (h->f32) return set_condition_f32(h, (const float *)enc, Bc, Lenc, s);
    const int D = h->D, kvd = h->kvd, M = Bc * Lenc;
    GemmArgs g{};
    g.A = (const bf16_t *)enc; g.lda = D; g.W = h->wce; g.ldw = D; g.C = h->E; g.ldc = D;
    g.M = M; g.N = D; g.K = D; g.epi = EPI_STORE; g.bias = h->bce;
    int rc = hgemm(h, g, s);
    if (rc) return rc;
    const size_t per = (size_t)Bc * kvd * Lenc;
    // the layers' K/V projections in GEMMs over groups of kv_group layers: M = Bc·Lenc rows ×
    // N = kv_group·2·kvd (turbo 10 s: 641 × 49152 in one GEMM — a full-chip grid, where L
    // separate N = 2048 GEMMs were small-M split-K launches + their epilogues); the k-norm /
    // head-major scatter stays per layer
    const int G = h->kv_group;
    const int64_t ldkv = (int64_t)G * 2 * kvd;
    for (int l = 0; l < h->L; ++l) {
        const int lg = l % G;
        if (lg == 0) {
            const int nl = std::min(G, h->L - l);
            GemmArgs k{};
            k.A = h->E; k.lda = D; k.W = h->wckv_all + (size_t)l * 2 * kvd * D; k.ldw = D; k.C = h->KVtmp;
            k.ldc = ldkv; k.M = M; k.N = nl * 2 * kvd; k.K = D; k.epi = EPI_STORE;
            if ((rc = hgemm(h, k, s))) return rc;
        }
        HeadPostArgs p{};
        p.src = h->KVtmp + (size_t)lg * 2 * kvd; p.ld_src = ldkv; p.B = Bc; p.S = Lenc;
        p.nq = 0; p.nk = h->cfg.kv_heads; p.nv = h->cfg.kv_heads;
        p.kw = h->layers[l].ckn; p.k = h->Kc + l * per; p.v = h->Vc + l * per;
        p.S_dst = Lenc; p.eps = h->cfg.eps;
        if ((rc = head_post(p, s))) return rc;
    }
    h->have_cond = true;
    h->cond_Bc = Bc;
    h->cond_Lenc = Lenc;
    h->uniform_from = 1 << 30;
    return 0;
}

int acehip_dit_set_uniform_rows(acehip_dit *h, int first_row, void *stream) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    if (!h->have_cond) return fail(ACEHIP_E_STATE, "set_uniform_rows before set_condition");
    if (first_row < 0 || first_row > h->cond_Bc) return fail(ACEHIP_E_ARG, "set_uniform_rows: first_row in [0, Bc]");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    h->uniform_from = 1 << 30;
    if (first_row == h->cond_Bc) return 0;   // none uniform
    if (h->f32) return 0;                    // parity mode: every row computed in full
    const int D = h->D, qd = h->qd, kvd = h->kvd, Le = h->cond_Lenc;
    const size_t per = (size_t)h->cond_Bc * kvd * Le;
    for (int l = 0; l < h->L; ++l) {
        // softmax over identical keys is uniform: every query's output is V row 0 of its
        // KV head (bit-exact: Σ of Lenc equal terms and the division are exact in fp32)
        int rc = gather_head_row(h->Vc + l * per + (size_t)first_row * kvd * Le, h->cfg.kv_heads, Le, h->cfg.heads,
                                 h->vnull, s);
        if (rc) return rc;
        GemmArgs g{};
        g.A = h->vnull; g.lda = qd; g.W = h->layers[l].wco; g.ldw = qd; g.C = h->cnull + (size_t)l * D; g.ldc = D;
        g.M = 1; g.N = D; g.K = qd; g.epi = EPI_STORE;
        if ((rc = hgemm(h, g, s))) return rc;
    }
    h->uniform_from = first_row;
    return 0;
}

int acehip_dit_forward(acehip_dit *h, const void *xt, const void *ctx, int Bx, const float *t,
                       const float *t_r, int t_stride, int Bc, int T, int dtype, void *vt_out, void *stream) {
    if (!h || !xt || !ctx || !t || !t_r || !vt_out) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized || !h->have_cond) return fail(ACEHIP_E_STATE, "forward before finalize/set_condition");
    if (Bc != h->cond_Bc) return fail(ACEHIP_E_ARG, "forward: Bc differs from set_condition");
    if (dtype != (h->f32 ? ACEHIP_F32 : ACEHIP_BF16))
        return fail(ACEHIP_E_ARG, h->f32 ? "forward: this handle is the fp32 parity mode (dtype ACEHIP_F32)"
                                         : "forward: this handle is bf16 (dtype ACEHIP_BF16); create with fp32=1 "
                                           "for the fp32 parity mode");
    const int S = (T + 1) / 2;
    if (T <= 0 || S > h->cfg.max_S || Bx <= 0 || Bc % Bx) return fail(ACEHIP_E_ARG, "forward: T/Bx out of range");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    if (h->f32)
        return forward_f32(h, (const float *)xt, (const float *)ctx, Bx, t, t_r, t_stride, Bc, T, (float *)vt_out, s);
    return forward_bf16(h, xt, ctx, Bx, t, t_r, t_stride, -1, Bc, T, vt_out, s);
}

int acehip_dit_set_graph(acehip_dit *h, int enable) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    h->graph_on = enable != 0 && !h->f32;
    return 0;
}

int acehip_dit_set_timesteps(acehip_dit *h, const float *t, const float *t_r, int n_steps, void *stream) {
    if (!h || !t || !t_r) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized) return fail(ACEHIP_E_STATE, "set_timesteps before finalize");
    if (h->f32) return fail(ACEHIP_E_STATE, "set_timesteps: bf16 handles only (the fp32 parity mode runs per step)");
    if (n_steps <= 0 || n_steps > 4096) return fail(ACEHIP_E_ARG, "set_timesteps: n_steps in [1, 4096]");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const int D = h->D;
    if (n_steps > h->ts_cap) {                 // only schedules longer than kTsCap steps
        HIP_TRY(hipStreamSynchronize(s));
        int rc = alloc_timesteps(h, n_steps);
        if (rc) return rc;
    }
    const size_t cap = h->ts_cap;
    bf16_t *emb[2] = {h->ts_scratch, h->ts_scratch + cap * 256};
    bf16_t *h1 = h->ts_scratch + cap * 512;
    bf16_t *temb_e[2] = {h1 + cap * D, h1 + cap * 2 * D};
    bf16_t *proj_e[2] = {h1 + cap * 3 * D, h1 + cap * 9 * D};
    int rc;
    // one sinusoid row per step (t[i], t_r[i]), then the MLPs over all steps: the MLP weights
    // are read once per schedule instead of once per step
    for (int e = 0; e < 2; ++e)
        if ((rc = timestep_sinusoid(t, t_r, 1, e, n_steps, h->freqs, emb[e], s))) return rc;
    if ((rc = timestep_mlps(h, emb, n_steps, h1, temb_e, proj_e, h->ts_temb, h->ts_proj, s))) return rc;
    h->ts_n = n_steps;
    return 0;
}

int acehip_dit_forward_step(acehip_dit *h, const void *xt, const void *ctx, int Bx, int step, int Bc, int T,
                            int dtype, void *vt_out, void *stream) {
    if (!h || !xt || !ctx || !vt_out) return fail(ACEHIP_E_ARG, "null argument");
    if (!h->finalized || !h->have_cond) return fail(ACEHIP_E_STATE, "forward_step before finalize/set_condition");
    if (h->f32 || dtype != ACEHIP_BF16) return fail(ACEHIP_E_ARG, "forward_step: bf16 handles only");
    if (step < 0 || step >= h->ts_n) return fail(ACEHIP_E_STATE, "forward_step: step outside the set_timesteps schedule");
    if (Bc != h->cond_Bc) return fail(ACEHIP_E_ARG, "forward_step: Bc differs from set_condition");
    const int S = (T + 1) / 2;
    if (T <= 0 || S > h->cfg.max_S || Bx <= 0 || Bc % Bx) return fail(ACEHIP_E_ARG, "forward_step: T/Bx out of range");
    HIP_TRY(hipSetDevice(h->device));
    return forward_bf16(h, xt, ctx, Bx, nullptr, nullptr, 0, step, Bc, T, vt_out, (hipStream_t)stream);
}

}  // extern "C"

// Everything of one forward between the input packing and proj_out: reads only handle
// buffers (emb, Xin, weights, K/V cache), so it can be captured once and replayed.
// bf16 forward; step >= 0 takes the timestep MLP outputs from the set_timesteps cache
static int forward_bf16(acehip_dit *h, const void *xt, const void *ctx, int Bx, const float *t, const float *t_r,
                        int t_stride, int step, int Bc, int T, void *vt_out, hipStream_t s) {
    const int S = (T + 1) / 2;
    const int M = Bc * S;
    int rc;
#define RUN(x) do { if ((rc = (x))) return rc; } while (0)
    // the only reads of t / xt / ctx: sinusoid embeddings and patch packing (base:1340-1358);
    // step >= 0: the schedule's precomputed timestep MLP row (acehip_dit_set_timesteps)
    const bool ts_cached = step >= 0;
    if (ts_cached) {
        RUN(bcast_rows(h->ts_temb + (size_t)step * h->D, h->D, h->temb, Bc, s));
        RUN(bcast_rows(h->ts_proj + (size_t)step * 6 * h->D, 6 * h->D, h->proj, Bc, s));
    } else {
        for (int e = 0; e < 2; ++e) RUN(timestep_sinusoid(t, t_r, t_stride, e, Bc, h->freqs, h->emb[e], s));
    }
    RUN(pack_patches((const bf16_t *)xt, (const bf16_t *)ctx, Bx, Bc, T, S, h->Xin, s));
    // CFG: every batch row reads xt/ctx row 0 (Bx = 1) at one broadcast t, so the rows are
    // identical until the first cross-attention — proj_in and layer 0's self-attention
    // block run on row 0 only and are copied (ACEHIP_DIT_DEDUP=0 disables, for A/B)
    const bool dup = Bx == 1 && Bc > 1 && (ts_cached || t_stride == 0) && knobs().dit_dedup;
    if (!h->graph_on || h->prof) {
        RUN(forward_body(h, Bc, S, dup, ts_cached, s));
    } else {
        const int key[6] = {Bc, S, h->cond_Lenc, std::min(h->uniform_from, Bc), (dup ? 1 : 0) | (ts_cached ? 2 : 0),
                            (int)knobs().gen};   // a knob reload re-captures
        if (!h->gexec || memcmp(key, h->gkey, sizeof(key))) {
            if (h->gexec) { HIP_TRY(hipGraphExecDestroy(h->gexec)); h->gexec = nullptr; }
            if (!h->cap_stream) HIP_TRY(hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
            HIP_TRY(hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeRelaxed));
            const int brc = forward_body(h, Bc, S, dup, ts_cached, h->cap_stream);
            hipGraph_t g = nullptr;
            const hipError_t ec = hipStreamEndCapture(h->cap_stream, &g);
            if (brc) { if (g) (void)hipGraphDestroy(g); return brc; }
            if (ec != hipSuccess || !g) return fail(ACEHIP_E_HIP, "forward: graph capture failed");
            const hipError_t ei = hipGraphInstantiate(&h->gexec, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (ei != hipSuccess) { h->gexec = nullptr; return fail(ACEHIP_E_HIP, "forward: graph instantiate failed"); }
            memcpy(h->gkey, key, sizeof(key));
        }
        HIP_TRY(hipGraphLaunch(h->gexec, s));
    }
    // proj_out (base:1491-1501) on the normed output XN
    GemmArgs po{};
    po.A = h->XN; po.lda = h->D; po.W = h->wout; po.ldw = h->D;
    po.C = (T % 2 == 0) ? (bf16_t *)vt_out : h->O2; po.ldc = 128;
    po.M = M; po.N = 128; po.K = h->D; po.epi = EPI_STORE; po.bias = h->bout;
    RUN(hgemm(h, po, s));
    if (T % 2) RUN(crop_rows(h->O2, Bc, 2 * S, T, 64, (bf16_t *)vt_out, s));
#undef RUN
    return 0;
}


#define RUN(x) do { if ((rc = (x))) return rc; } while (0)
// timestep embeddings: temb = temb_t + temb_r, proj = proj_t + proj_r (base:1340-1344) for
// `rows` rows of sinusoid embeddings, in chunks of 16 rows (gemv_small computes every row
// with the same instruction sequence whatever the row count, so a row's result does not
// depend on how many rows share the launch)
static int timestep_mlps(acehip_dit *h, const bf16_t *const emb[2], int rows, bf16_t *h1, bf16_t *const temb_e[2],
                         bf16_t *const proj_e[2], bf16_t *temb, bf16_t *proj, hipStream_t s) {
    const int D = h->D;
    int rc;
    for (int r0 = 0; r0 < rows; r0 += 16) {
        const int n = std::min(16, rows - r0);
        for (int e = 0; e < 2; ++e) {
            RUN(gemv_small(emb[e] + (size_t)r0 * 256, 256, h->te_l1[e], h->te_b1[e], h1 + (size_t)r0 * D, D, n, D,
                           256, 0, s));
            RUN(gemv_small(h1 + (size_t)r0 * D, D, h->te_l2[e], h->te_b2[e], temb_e[e] + (size_t)r0 * D, D, n, D, D,
                           1, s, h->gemv_act));
            RUN(gemv_small(temb_e[e] + (size_t)r0 * D, D, h->te_tp[e], h->te_btp[e], proj_e[e] + (size_t)r0 * 6 * D,
                           6 * D, n, 6 * D, D, 1, s, h->gemv_act));
        }
    }
    RUN(add_bf16(temb_e[0], temb_e[1], temb, (int64_t)rows * D, s));
    RUN(add_bf16(proj_e[0], proj_e[1], proj, (int64_t)rows * 6 * D, s));
    return 0;
}

static int forward_body(acehip_dit *h, int Bc, int S, bool dup, bool ts_cached, hipStream_t s) {
    const int D = h->D, F = h->F, qd = h->qd, kvd = h->kvd, L = h->L, M = Bc * S;
    const int H = h->cfg.heads, KV = h->cfg.kv_heads, Le = h->cond_Lenc;
    const float eps = h->cfg.eps, scale = 1.0f / sqrtf((float)h->cfg.head_dim);
    int rc;
    // timestep MLPs (temb, proj), unless acehip_dit_forward_step already broadcast the
    // schedule's precomputed row into h->temb / h->proj
    if (!ts_cached) RUN(timestep_mlps(h, h->emb, Bc, h->h1, h->temb_e, h->proj_e, h->temb, h->proj, s));
    RUN(modulation(h->tables, L, 6, h->proj, Bc, D, h->mod, s));
    RUN(modulation(h->sst_out, 1, 2, h->temb, Bc, D, h->mod_out, s));

    // proj_in (base:1347-1358) over the packed patches Xin
    GemmArgs g{};
    g.A = h->Xin; g.lda = 384; g.W = h->win; g.ldw = 384; g.C = h->X; g.ldc = D;
    g.M = dup ? S : M; g.N = D; g.K = 384; g.epi = EPI_STORE; g.bias = h->bin;
    RUN(hgemm(h, g, s));

    const bool fuse_rowadd = knobs().fuse_rowadd != 0;
    const size_t cper = (size_t)Bc * kvd * Le;
    const int Bq = std::min(h->uniform_from, Bc), Mq = Bq * S;   // rows with a real cross-attention
    // small-M grids take gemm's split-K path; the residual epilogue of such a GEMM (O, cross-O,
    // down) is then deferred into the next norm, which reads the rows anyway: `pend` carries
    // it (gemm sets pend.part only when it deferred).  Deferral needs that norm to cover every
    // row the GEMM wrote, and no X copy in between (the layer-0 CFG dedup).
    RowAdd pend{};
    for (int l = 0; l < L; ++l) {
        const auto &ly = h->layers[l];
        const bf16_t *md = h->mod + (size_t)l * Bc * 6 * D;
        const int64_t mbs = 6 * D;
        // --- self-attention with AdaLN-Zero (base:499-511); layer 0 of identical CFG rows: row 0
        const int Bs = (dup && l == 0) ? 1 : Bc, Ms = Bs * S;
        RUN(rmsnorm_mod(h->X, ly.n_sa, md + 0 * D, md + 1 * D, mbs, S, h->XN, Ms, D, eps, s, pend));
        pend = RowAdd{};
        // QKV projection with q/k RMSNorm + RoPE + head-major scatter fused in the epilogue
        GemmArgs q{};
        q.A = h->XN; q.lda = D; q.W = ly.wqkv; q.ldw = D;
        q.M = Ms; q.N = qd + 2 * kvd; q.K = D; q.epi = EPI_HEADPOST;
        q.hp.B = Bs; q.hp.S = S; q.hp.nq = H; q.hp.nk = KV; q.hp.nv = KV; q.hp.qw = ly.qn; q.hp.kw = ly.kn;
        q.hp.cos = h->rope_cos; q.hp.sin = h->rope_sin;
        q.hp.q = h->Qh; q.hp.k = h->Kh; q.hp.v = h->Vh; q.hp.S_dst = S; q.hp.eps = eps;
        RUN(timed(h, 2, s, [&] { return hgemm(h, q, s); }));
        RUN(timed(h, h->sliding[l] ? 5 : 4, s, [&] {
            return attention(h->Qh, h->Kh, h->Vh, h->AO, Bs, H, KV, S, S, h->sliding[l] ? h->cfg.window : -1,
                             scale, qd, h->attn_ws, s);
        }));
        GemmArgs o{};
        o.A = h->AO; o.lda = qd; o.W = ly.wo; o.ldw = qd; o.C = h->X; o.ldc = D;
        o.M = Ms; o.N = D; o.K = qd; o.epi = EPI_GATED_RES; o.res = h->X; o.ldr = D;
        o.gate = md + 2 * D; o.gate_bstride = mbs; o.rows_per_batch = S;
        const bool defer_o = fuse_rowadd && Bs == Bc && (Mq == M || Mq == 0);
        RUN(timed(h, 3, s, [&] { return hgemm(h, o, s, defer_o ? &pend : nullptr); }));
        for (int b = Bs; b < Bc; ++b)
            HIP_TRY(hipMemcpyAsync(h->X + (size_t)b * S * D, h->X, (size_t)S * D * 2, hipMemcpyDeviceToDevice, s));
        // --- cross-attention, plain residual (base:513-526); rows >= uniform_from (CFG null
        // rows, base:1907) get their constant cross-O output cnull[l] (set_uniform_rows)
        if (Mq > 0) {
            RUN(rmsnorm_mod(h->X, ly.n_ca, nullptr, nullptr, 0, S, h->XN, Mq, D, eps, s, pend));
            pend = RowAdd{};
            GemmArgs cq{};
            cq.A = h->XN; cq.lda = D; cq.W = ly.wcq; cq.ldw = D;
            cq.M = Mq; cq.N = qd; cq.K = D; cq.epi = EPI_HEADPOST;
            cq.hp.B = Bq; cq.hp.S = S; cq.hp.nq = H; cq.hp.qw = ly.cqn; cq.hp.q = h->Qh; cq.hp.S_dst = S;
            cq.hp.eps = eps;
            RUN(hgemm(h, cq, s));
            RUN(timed(h, 6, s, [&] {
                return attention(h->Qh, h->Kc + l * cper, h->Vc + l * cper, h->AO, Bq, H, KV, S, Le, -1, scale, qd,
                                 h->attn_ws, s);
            }));
            GemmArgs co{};
            co.A = h->AO; co.lda = qd; co.W = ly.wco; co.ldw = qd; co.C = h->X; co.ldc = D;
            co.M = Mq; co.N = D; co.K = qd; co.epi = EPI_RES; co.res = h->X; co.ldr = D;
            RUN(timed(h, 3, s, [&] { return hgemm(h, co, s, fuse_rowadd ? &pend : nullptr); }));
        }
        // --- SwiGLU MLP with AdaLN-Zero (base:528-533); the null rows' constant cross-O output
        // is added inside the norm pass (ACEHIP_FUSE_ROWADD=0: separate add_row_bcast, A/B)
        RowAdd ra = pend;   // rows < ra.prows: the deferred cross-O (or O) epilogue, applied first
        pend = RowAdd{};
        if (Mq < M) {
            if (fuse_rowadd) {
                ra.xw = h->X;
                ra.v = h->cnull + (size_t)l * D;
                ra.from = Mq;
            } else {
                RUN(add_row_bcast(h->X + (size_t)Mq * D, h->cnull + (size_t)l * D, M - Mq, D, s));
            }
        }
        RUN(rmsnorm_mod(h->X, ly.n_mlp, md + 3 * D, md + 4 * D, mbs, S, h->XN, M, D, eps, s, ra));
        GemmArgs gu{};
        gu.A = h->XN; gu.lda = D; gu.W = ly.wgu; gu.ldw = D; gu.C = h->Hb; gu.ldc = F;
        gu.M = M; gu.N = 2 * F; gu.K = D; gu.epi = EPI_SWIGLU;
        RUN(timed(h, 0, s, [&] { return hgemm(h, gu, s); }));
        GemmArgs dn{};
        dn.A = h->Hb; dn.lda = F; dn.W = ly.wdown; dn.ldw = F; dn.C = h->X; dn.ldc = D;
        dn.M = M; dn.N = D; dn.K = F; dn.epi = EPI_GATED_RES; dn.res = h->X; dn.ldr = D;
        dn.gate = md + 5 * D; dn.gate_bstride = mbs; dn.rows_per_batch = S;
        RUN(timed(h, 1, s, [&] { return hgemm(h, dn, s, fuse_rowadd ? &pend : nullptr); }));
    }
    // norm_out AdaLN (base:1491-1497); proj_out runs after the body
    RUN(rmsnorm_mod(h->X, h->norm_out, h->mod_out, h->mod_out + D, 2 * D, S, h->XN, M, D, eps, s, pend));
#undef RUN
    return 0;
}

extern "C" {

int acehip_dit_profile(acehip_dit *h, int enable) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    HIP_TRY(hipSetDevice(h->device));
    if (enable && h->ev.empty()) {
        h->ev.resize(2 * acehip_dit::NPAIR);
        h->ev_kind.resize(acehip_dit::NPAIR);
        for (auto &e : h->ev) HIP_TRY(hipEventCreate(&e));
    }
    h->prof = enable != 0;
    h->ev_used = 0;
    return 0;
}

int acehip_dit_profile_kinds(acehip_dit *h, unsigned mask) {
    if (!h) return fail(ACEHIP_E_ARG, "null handle");
    h->prof_mask = mask;
    return 0;
}

int acehip_dit_profile_read(acehip_dit *h, int kind, int *launches, float *total_ms) {
    if (!h || !launches || !total_ms) return fail(ACEHIP_E_ARG, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    int n = 0;
    float tot = 0.f;
    for (int i = 0; i < h->ev_used; ++i) {
        if (h->ev_kind[i] != kind) continue;
        float ms = 0.f;
        HIP_TRY(hipEventSynchronize(h->ev[2 * i + 1]));
        HIP_TRY(hipEventElapsedTime(&ms, h->ev[2 * i], h->ev[2 * i + 1]));
        tot += ms;
        ++n;
    }
    *launches = n;
    *total_ms = tot;
    return 0;
}

int acehip_dit_destroy(acehip_dit *h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    for (auto &e : h->ev) (void)hipEventDestroy(e);
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
    for (void *p : h->allocs) (void)hipFree(p);
    for (bf16_t *p : {h->ts_temb, h->ts_proj, h->ts_scratch})
        if (p) (void)hipFree(p);
    delete h;
    return 0;
}

static int sampler_dtype(int dtype, bool *f32) {
    if (dtype != ACEHIP_BF16 && dtype != ACEHIP_F32) return fail(ACEHIP_E_ARG, "sampler: dtype");
    *f32 = dtype == ACEHIP_F32;
    return 0;
}

int acehip_sampler_apg_euler(const void *vt, void *xt, void *ra, int B, int T, int C, float guidance,
                             float dt, int apply_cfg, int first_step, int out_mode, int dtype, void *stream) {
    if (!vt || !xt || (apply_cfg > 0 && !ra)) return fail(ACEHIP_E_ARG, "null argument");
    bool f32;
    if (int rc = sampler_dtype(dtype, &f32)) return rc;
    return apg_euler(vt, xt, ra, B, T, C, guidance, dt, apply_cfg, first_step, out_mode, f32, (hipStream_t)stream);
}

int acehip_sampler_adg_euler(const void *vt, void *xt, int B, int T, int C, float guidance, float sigma,
                             float dt, int out_mode, int dtype, void *stream) {
    if (!vt || !xt) return fail(ACEHIP_E_ARG, "null argument");
    bool f32;
    if (int rc = sampler_dtype(dtype, &f32)) return rc;
    return adg_euler(vt, xt, B, T, C, guidance, sigma, dt, out_mode, f32, (hipStream_t)stream);
}

int acehip_sampler_axpy(const void *vt, void *xt, int64_t n, float s, int dtype, void *stream) {
    if (!vt || !xt) return fail(ACEHIP_E_ARG, "null argument");
    bool f32;
    if (int rc = sampler_dtype(dtype, &f32)) return rc;
    return axpy(vt, xt, n, s, f32, (hipStream_t)stream);
}

int acehip_gemm_bf16(const void *A, int lda, const void *W, int ldw, void *C, int ldc, int M, int N,
                     int K, const void *bias, void *stream) {
    GemmArgs g{};
    g.A = (const bf16_t *)A; g.lda = lda; g.W = (const bf16_t *)W; g.ldw = ldw;
    g.C = (bf16_t *)C; g.ldc = ldc; g.M = M; g.N = N; g.K = K; g.epi = EPI_STORE;
    g.bias = (const bf16_t *)bias;
    return gemm(g, (hipStream_t)stream);
}

// lazily allocated split-K workspace of the standalone kernel entry points (one per device)
static std::mutex g_abi_ws_mu;
static void *abi_gemm_ws() {
    static std::map<int, void *> by_dev;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_abi_ws_mu);
    void *&ws = by_dev[dev];
    if (!ws && hipMalloc(&ws, GEMM_WS_BYTES) != hipSuccess) ws = nullptr;
    return ws;
}

int acehip_gemm_bf16_ex(const void *A, int lda, const void *W, int ldw, void *C, int ldc, int M, int N,
                        int K, const void *bias, int epi, int variant, void *stream) {
    GemmArgs g{};
    g.A = (const bf16_t *)A; g.lda = lda; g.W = (const bf16_t *)W; g.ldw = ldw;
    g.C = (bf16_t *)C; g.ldc = ldc; g.M = M; g.N = N; g.K = K;
    g.bias = (const bf16_t *)bias;
    if (epi == 2) { g.epi = EPI_RES; g.res = (const bf16_t *)C; g.ldr = ldc; }
    else if (epi == 3) g.epi = EPI_SWIGLU;   // W rows packed [32 gate; 32 up] per 64-row panel, C[M][N/2]
    else if (epi == 0) g.epi = EPI_STORE;
    else return fail(ACEHIP_E_ARG, "gemm_ex: epilogue");
    if (M <= 0 || N % 128 || K % 64) return fail(ACEHIP_E_ARG, "gemm_ex: shape");
    if (variant < 0) {   // production dispatch (split-K for small grids)
        g.ws = abi_gemm_ws();
        g.ws_bytes = g.ws ? GEMM_WS_BYTES : 0;
        return gemm(g, (hipStream_t)stream);
    }
    return gemm_variant(g, variant, (hipStream_t)stream);
}

int acehip_rmsnorm_bf16(const void *x, const void *w, const void *shift, const void *scale,
                        int64_t mod_bstride, int rows_per_batch, void *out, int M, int D, float eps,
                        int rows_per_wave, void *stream) {
    if (!x || !w || !out) return fail(ACEHIP_E_ARG, "null argument");
    if (rows_per_wave == 3 || rows_per_wave > 4 || (rows_per_wave < 0 && rows_per_wave != -2 && rows_per_wave != -4))
        return fail(ACEHIP_E_ARG, "rows_per_wave");
    return rmsnorm_mod((const bf16_t *)x, (const bf16_t *)w, (const bf16_t *)shift, (const bf16_t *)scale,
                       mod_bstride, rows_per_batch, (bf16_t *)out, M, D, eps, (hipStream_t)stream, RowAdd{},
                       rows_per_wave);
}

int acehip_gemm_headpost_bf16(const void *A, int lda, const void *W, int K, int B, int S, int nq, int nk,
                              int nv, const void *qw, const void *kw, const void *cos, const void *sin,
                              float eps, void *q, void *k, void *v, void *stream) {
    if (!A || !W) return fail(ACEHIP_E_ARG, "null argument");
    if ((nq && !q) || (nk && !k) || (nv && !v)) return fail(ACEHIP_E_ARG, "missing head output");
    GemmArgs g{};
    g.A = (const bf16_t *)A; g.lda = lda; g.W = (const bf16_t *)W; g.ldw = K;
    g.M = B * S; g.N = (nq + nk + nv) * 128; g.K = K; g.epi = EPI_HEADPOST;
    if (g.M <= 0 || K % 64 || K <= 0) return fail(ACEHIP_E_ARG, "gemm_headpost: shape");
    g.hp.B = B; g.hp.S = S; g.hp.nq = nq; g.hp.nk = nk; g.hp.nv = nv;
    g.hp.qw = (const bf16_t *)qw; g.hp.kw = (const bf16_t *)kw;
    g.hp.cos = (const bf16_t *)cos; g.hp.sin = (const bf16_t *)sin;
    g.hp.q = (bf16_t *)q; g.hp.k = (bf16_t *)k; g.hp.v = (bf16_t *)v; g.hp.S_dst = S; g.hp.eps = eps;
    g.ws = abi_gemm_ws();
    g.ws_bytes = g.ws ? GEMM_WS_BYTES : 0;
    return gemm(g, (hipStream_t)stream);
}

int acehip_attention_bf16(const void *q, const void *k, const void *v, void *o, int B, int H, int KV,
                          int Sq, int Sk, int window, float scale, void *stream) {
    return acehip_attention_masked_bf16(q, k, v, o, B, H, KV, Sq, Sk, window, scale, nullptr, stream);
}

int acehip_attention_masked_bf16(const void *q, const void *k, const void *v, void *o, int B, int H, int KV,
                                 int Sq, int Sk, int window, float scale, const uint8_t *kmask, void *stream) {
    // standalone entry (tests / micro-bench): one lazily allocated tail-split workspace
    // per device (the DiT runtime owns its own, allocated at create)
    static std::map<int, void *> ws_by_dev;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    void *&ws = ws_by_dev[dev];
    if (!ws) {
        const size_t wb = attention_ws_bytes();
        if (hipMalloc(&ws, wb) != hipSuccess) return fail(ACEHIP_E_OOM, "attention workspace");
        HIP_TRY(hipMemset(ws, 0, wb));
    }
    return attention((const bf16_t *)q, (const bf16_t *)k, (const bf16_t *)v, (bf16_t *)o, B, H, KV, Sq,
                     Sk, window, scale, (int64_t)H * 128, ws, (hipStream_t)stream, kmask);
}

}  // extern "C"

// ===================================================================== fp32 ====
// The fp32 parity mode (acehip_dit_cfg.fp32 = 1): the reference's
// fp32 forward (what it runs on a non-cuda device, init_service_orchestrator.py:51)
// with fp32 weights and activations throughout, on the kernels of f32.hip.  No
// algebraic shortcuts (no CFG-row dedup, no closed-form null rows, no graphs).

static float *falloc(acehip_dit *h, size_t elems) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(elems, 1) * 4) != hipSuccess) return nullptr;
    h->allocs.push_back(p);
    return (float *)p;
}

static void add_slot_f32(acehip_dit *h, const std::string &name, float *dst, std::vector<int64_t> shape,
                         PackKind kind = P_F32) {
    Slot s;
    s.dst_f32 = dst;
    s.shape = std::move(shape);
    s.kind = kind;
    h->slots[name] = s;
}

static int create_f32(acehip_dit *h) {
    const int D = h->D, F = h->F, qd = h->qd, kvd = h->kvd, L = h->L;
    bool ok = true;
    auto A = [&](size_t n) { float *p = falloc(h, n); ok = ok && p; return p; };
    auto &f = h->f;
    f.tables = A((size_t)L * 6 * D);
    f.layers.resize(L);
    for (int i = 0; i < L && ok; ++i) {
        auto &ly = f.layers[i];
        ly.n_sa = A(D); ly.n_ca = A(D); ly.n_mlp = A(D);
        ly.wqkv = A((size_t)(qd + 2 * kvd) * D); ly.wo = A((size_t)D * qd);
        ly.qn = A(128); ly.kn = A(128); ly.cqn = A(128); ly.ckn = A(128);
        ly.wcq = A((size_t)qd * D); ly.wckv = A((size_t)2 * kvd * D); ly.wco = A((size_t)D * qd);
        ly.wg = A((size_t)F * D); ly.wu = A((size_t)F * D); ly.wdown = A((size_t)D * F);
        if (!ok) break;
        const std::string p = "layers." + std::to_string(i);
        add_slot_f32(h, p + ".scale_shift_table", f.tables + (size_t)i * 6 * D, {1, 6, D});
        add_slot_f32(h, p + ".self_attn_norm.weight", ly.n_sa, {D});
        add_slot_f32(h, p + ".cross_attn_norm.weight", ly.n_ca, {D});
        add_slot_f32(h, p + ".mlp_norm.weight", ly.n_mlp, {D});
        add_slot_f32(h, p + ".self_attn.q_proj.weight", ly.wqkv, {qd, D});
        add_slot_f32(h, p + ".self_attn.k_proj.weight", ly.wqkv + (size_t)qd * D, {kvd, D});
        add_slot_f32(h, p + ".self_attn.v_proj.weight", ly.wqkv + (size_t)(qd + kvd) * D, {kvd, D});
        add_slot_f32(h, p + ".self_attn.o_proj.weight", ly.wo, {D, qd});
        add_slot_f32(h, p + ".self_attn.q_norm.weight", ly.qn, {128});
        add_slot_f32(h, p + ".self_attn.k_norm.weight", ly.kn, {128});
        add_slot_f32(h, p + ".cross_attn.q_proj.weight", ly.wcq, {qd, D});
        add_slot_f32(h, p + ".cross_attn.k_proj.weight", ly.wckv, {kvd, D});
        add_slot_f32(h, p + ".cross_attn.v_proj.weight", ly.wckv + (size_t)kvd * D, {kvd, D});
        add_slot_f32(h, p + ".cross_attn.o_proj.weight", ly.wco, {D, qd});
        add_slot_f32(h, p + ".cross_attn.q_norm.weight", ly.cqn, {128});
        add_slot_f32(h, p + ".cross_attn.k_norm.weight", ly.ckn, {128});
        add_slot_f32(h, p + ".mlp.gate_proj.weight", ly.wg, {F, D});
        add_slot_f32(h, p + ".mlp.up_proj.weight", ly.wu, {F, D});
        add_slot_f32(h, p + ".mlp.down_proj.weight", ly.wdown, {D, F});
    }
    f.sst_out = A(2 * D); f.win = A((size_t)D * 384); f.bin = A(D);
    f.wce = A((size_t)D * D); f.bce = A(D); f.norm_out = A(D);
    f.wout = A((size_t)128 * D); f.bout = A(128);
    const char *te_names[2] = {"time_embed", "time_embed_r"};
    for (int e = 0; e < 2 && ok; ++e) {
        f.te_l1[e] = A((size_t)D * 256); f.te_b1[e] = A(D);
        f.te_l2[e] = A((size_t)D * D); f.te_b2[e] = A(D);
        f.te_tp[e] = A((size_t)6 * D * D); f.te_btp[e] = A(6 * D);
        if (!ok) break;
        const std::string p = te_names[e];
        add_slot_f32(h, p + ".linear_1.weight", f.te_l1[e], {D, 256});
        add_slot_f32(h, p + ".linear_1.bias", f.te_b1[e], {D});
        add_slot_f32(h, p + ".linear_2.weight", f.te_l2[e], {D, D});
        add_slot_f32(h, p + ".linear_2.bias", f.te_b2[e], {D});
        add_slot_f32(h, p + ".time_proj.weight", f.te_tp[e], {6 * D, D});
        add_slot_f32(h, p + ".time_proj.bias", f.te_btp[e], {6 * D});
    }
    if (ok) {
        add_slot_f32(h, "scale_shift_table", f.sst_out, {1, 2, D});
        add_slot_f32(h, "proj_in.1.weight", f.win, {D, 192, 2}, P_F32_PROJ_IN);
        add_slot_f32(h, "proj_in.1.bias", f.bin, {D});
        add_slot_f32(h, "condition_embedder.weight", f.wce, {D, D});
        add_slot_f32(h, "condition_embedder.bias", f.bce, {D});
        add_slot_f32(h, "norm_out.weight", f.norm_out, {D});
        add_slot_f32(h, "proj_out.1.weight", f.wout, {D, 64, 2}, P_F32_PROJ_OUT_W);
        add_slot_f32(h, "proj_out.1.bias", f.bout, {64}, P_F32_PROJ_OUT_B);
    }
    const size_t S = h->cfg.max_S, Bc = h->cfg.max_Bc, M = S * Bc, Le = h->cfg.max_Lenc;
    f.X = A(M * D); f.XN = A(M * D); f.QKV = A(M * (qd + 2 * kvd));
    f.Qh = A(M * qd); f.Kh = A(M * kvd); f.Vh = A(M * kvd); f.AO = A(M * qd);
    f.G = A(M * F); f.U = A(M * F); f.Hb = A(M * F); f.Xin = A(M * 384); f.O2 = A(M * 128);
    for (int e = 0; e < 2; ++e) { f.emb[e] = A(Bc * 256); f.temb_e[e] = A(Bc * D); f.proj_e[e] = A(Bc * 6 * D); }
    f.h1 = A(Bc * D); f.temb = A(Bc * D); f.proj = A(Bc * 6 * D);
    f.mod = A((size_t)L * Bc * 6 * D); f.mod_out = A(Bc * 2 * D);
    f.Kc = A((size_t)L * Bc * kvd * Le); f.Vc = A((size_t)L * Bc * kvd * Le);
    f.E = A(Bc * Le * D); f.KVtmp = A(Bc * Le * 2 * kvd);
    f.rope_cos = A(S * 128); f.rope_sin = A(S * 128);
    h->freqs = A(128);
    if (!ok) return fail(ACEHIP_E_OOM, "dit_create (fp32): device allocation failed");
    float fr[128];
    for (int i = 0; i < 128; ++i) fr[i] = expf((-9.210340371976184f * (float)i) / 128.0f);
    HIP_TRY(hipMemcpy(h->freqs, fr, sizeof(fr), hipMemcpyHostToDevice));
    return 0;
}

// every fp32 weight goes through the host (parity mode: load time is not a concern)
static int set_weight_f32(acehip_dit *h, Slot &s, const void *ptr, int dtype, int64_t n, int on_device) {
    std::vector<float> v(n);
    if (dtype == ACEHIP_F32) {
        HIP_TRY(hipMemcpy(v.data(), ptr, n * 4, on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
    } else {
        std::vector<bf16_t> b(n);
        HIP_TRY(hipMemcpy(b.data(), ptr, n * 2, on_device ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
        for (int64_t i = 0; i < n; ++i) v[i] = bf2f(b[i]);
    }
    std::vector<float> out;
    const std::vector<float> *src = &v;
    if (s.kind == P_F32_PROJ_IN) {            // [D][192][2] → [D][k·192 + c]
        const int64_t D = s.shape[0];
        out.resize(n);
        for (int64_t o = 0; o < D; ++o)
            for (int c = 0; c < 192; ++c)
                for (int k = 0; k < 2; ++k) out[o * 384 + k * 192 + c] = v[(o * 192 + c) * 2 + k];
        src = &out;
    } else if (s.kind == P_F32_PROJ_OUT_W) {  // [D][64][2] → [k·64 + o][D]
        const int64_t D = s.shape[0];
        out.resize(n);
        for (int64_t c = 0; c < D; ++c)
            for (int o = 0; o < 64; ++o)
                for (int k = 0; k < 2; ++k) out[(k * 64 + o) * D + c] = v[(c * 64 + o) * 2 + k];
        src = &out;
    } else if (s.kind == P_F32_PROJ_OUT_B) {  // [64] → [k·64 + o]
        out.resize(128);
        for (int k = 0; k < 2; ++k)
            for (int o = 0; o < 64; ++o) out[k * 64 + o] = v[o];
        src = &out;
    } else if (s.kind != P_F32) {
        return fail(ACEHIP_E_ARG, "dit_set_weight (fp32): unexpected slot");
    }
    HIP_TRY(hipMemcpy(s.dst_f32, src->data(), src->size() * 4, hipMemcpyHostToDevice));
    s.set = true;
    return 0;
}

// Qwen3RotaryEmbedding in fp32: inv_freq stays fp32 (no .to(bf16) in an fp32 model),
// angle = fp32(pos · inv_freq), cos/sin of it
static int build_rope_f32(acehip_dit *h) {
    const int hd = h->cfg.head_dim, S = h->cfg.max_S;
    std::vector<float> inv(hd / 2);
    for (int i = 0; i < hd / 2; ++i)
        inv[i] = !h->inv_freq_override.empty() ? h->inv_freq_override[i]
                                               : 1.0f / powf(h->cfg.rope_theta, (float)(2 * i) / (float)hd);
    std::vector<float> c((size_t)S * hd), sn((size_t)S * hd);
    for (int p = 0; p < S; ++p)
        for (int i = 0; i < hd; ++i) {
            const float a = (float)p * inv[i % (hd / 2)];
            c[(size_t)p * hd + i] = (float)cos((double)a);
            sn[(size_t)p * hd + i] = (float)sin((double)a);
        }
    HIP_TRY(hipMemcpy(h->f.rope_cos, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->f.rope_sin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
    return 0;
}

static int set_condition_f32(acehip_dit *h, const float *enc, int Bc, int Lenc, hipStream_t s) {
    auto &f = h->f;
    const int D = h->D, kvd = h->kvd, M = Bc * Lenc;
    int rc;
    GemmF32Args g{};
    g.A = enc; g.lda = D; g.W = f.wce; g.ldw = D; g.C = f.E; g.ldc = D; g.M = M; g.N = D; g.K = D;
    g.epi = EPI_STORE; g.bias = f.bce;
    if ((rc = gemm_f32(g, s))) return rc;
    const size_t per = (size_t)Bc * kvd * Lenc;
    for (int l = 0; l < h->L; ++l) {
        GemmF32Args k{};
        k.A = f.E; k.lda = D; k.W = f.layers[l].wckv; k.ldw = D; k.C = f.KVtmp; k.ldc = 2 * kvd;
        k.M = M; k.N = 2 * kvd; k.K = D; k.epi = EPI_STORE;
        if ((rc = gemm_f32(k, s))) return rc;
        HeadPostF32Args p{};
        p.src = f.KVtmp; p.ld_src = 2 * kvd; p.B = Bc; p.S = Lenc; p.nq = 0;
        p.nk = h->cfg.kv_heads; p.nv = h->cfg.kv_heads; p.kw = f.layers[l].ckn;
        p.k = f.Kc + l * per; p.v = f.Vc + l * per; p.S_dst = Lenc; p.eps = h->cfg.eps;
        if ((rc = head_post_f32(p, s))) return rc;
    }
    h->have_cond = true;
    h->cond_Bc = Bc;
    h->cond_Lenc = Lenc;
    h->uniform_from = 1 << 30;
    return 0;
}

static int forward_f32(acehip_dit *h, const float *xt, const float *ctx, int Bx, const float *t, const float *t_r,
                       int t_stride, int Bc, int T, float *vt_out, hipStream_t s) {
    auto &f = h->f;
    const int D = h->D, F = h->F, qd = h->qd, kvd = h->kvd, L = h->L, S = (T + 1) / 2, M = Bc * S;
    const int H = h->cfg.heads, KV = h->cfg.kv_heads, Le = h->cond_Lenc;
    const float eps = h->cfg.eps, scale = 1.0f / sqrtf((float)h->cfg.head_dim);
    const int64_t mbs = 6 * D;
    const size_t cper = (size_t)Bc * kvd * Le;
    int rc;
#define RUN(x) do { if ((rc = (x))) return rc; } while (0)
    auto gemm = [&](const float *A, int lda, const float *W, float *C, int ldc, int m, int n, int k, const float *bias,
                    int epi, const float *gate = nullptr) {
        GemmF32Args g{};
        g.A = A; g.lda = lda; g.W = W; g.ldw = k; g.C = C; g.ldc = ldc; g.M = m; g.N = n; g.K = k; g.bias = bias;
        g.epi = epi; g.res = C; g.ldr = ldc; g.gate = gate; g.gate_bstride = mbs; g.rows_per_batch = S;
        return gemm_f32(g, s);
    };
    // timestep embeddings (base:225-254, :1340-1344)
    for (int e = 0; e < 2; ++e) {
        RUN(timestep_sinusoid_f32(t, t_r, t_stride, e, Bc, h->freqs, f.emb[e], s));
        RUN(gemv_f32(f.emb[e], 256, f.te_l1[e], f.te_b1[e], f.h1, D, Bc, D, 256, 0, s));
        RUN(gemv_f32(f.h1, D, f.te_l2[e], f.te_b2[e], f.temb_e[e], D, Bc, D, D, 1, s));
        RUN(gemv_f32(f.temb_e[e], D, f.te_tp[e], f.te_btp[e], f.proj_e[e], 6 * D, Bc, 6 * D, D, 1, s));
    }
    RUN(add_f32(f.temb_e[0], f.temb_e[1], f.temb, (int64_t)Bc * D, s));
    RUN(add_f32(f.proj_e[0], f.proj_e[1], f.proj, (int64_t)Bc * 6 * D, s));
    RUN(modulation_f32(f.tables, L, 6, f.proj, Bc, D, f.mod, s));
    RUN(modulation_f32(f.sst_out, 1, 2, f.temb, Bc, D, f.mod_out, s));
    // concat + pad + proj_in (base:1347-1358)
    RUN(pack_patches_f32(xt, ctx, Bx, Bc, T, S, f.Xin, s));
    RUN(gemm(f.Xin, 384, f.win, f.X, D, M, D, 384, f.bin, EPI_STORE));
    for (int l = 0; l < L; ++l) {
        const auto &ly = f.layers[l];
        const float *md = f.mod + (size_t)l * Bc * 6 * D;
        // self-attention, AdaLN-Zero (base:499-511)
        RUN(rmsnorm_f32(f.X, ly.n_sa, md + 0 * D, md + 1 * D, mbs, S, f.XN, M, D, eps, s));
        RUN(gemm(f.XN, D, ly.wqkv, f.QKV, qd + 2 * kvd, M, qd + 2 * kvd, D, nullptr, EPI_STORE));
        HeadPostF32Args p{};
        p.src = f.QKV; p.ld_src = qd + 2 * kvd; p.B = Bc; p.S = S; p.nq = H; p.nk = KV; p.nv = KV;
        p.qw = ly.qn; p.kw = ly.kn; p.cos = f.rope_cos; p.sin = f.rope_sin;
        p.q = f.Qh; p.k = f.Kh; p.v = f.Vh; p.S_dst = S; p.eps = eps;
        RUN(head_post_f32(p, s));
        AttnF32Args at{};
        at.q = f.Qh; at.k = f.Kh; at.v = f.Vh; at.o = f.AO; at.o_ld = qd; at.B = Bc; at.H = H; at.KV = KV;
        at.Sq = S; at.Sk = S; at.window = h->sliding[l] ? h->cfg.window : -1; at.scale = scale;
        RUN(attention_f32(at, s));
        RUN(gemm(f.AO, qd, ly.wo, f.X, D, M, D, qd, nullptr, EPI_GATED_RES, md + 2 * D));
        // cross-attention, plain residual (base:513-526)
        RUN(rmsnorm_f32(f.X, ly.n_ca, nullptr, nullptr, 0, S, f.XN, M, D, eps, s));
        RUN(gemm(f.XN, D, ly.wcq, f.QKV, qd, M, qd, D, nullptr, EPI_STORE));
        HeadPostF32Args cq{};
        cq.src = f.QKV; cq.ld_src = qd; cq.B = Bc; cq.S = S; cq.nq = H; cq.qw = ly.cqn; cq.q = f.Qh;
        cq.S_dst = S; cq.eps = eps;
        RUN(head_post_f32(cq, s));
        AttnF32Args ca{};
        ca.q = f.Qh; ca.k = f.Kc + l * cper; ca.v = f.Vc + l * cper; ca.o = f.AO; ca.o_ld = qd; ca.B = Bc;
        ca.H = H; ca.KV = KV; ca.Sq = S; ca.Sk = Le; ca.window = -1; ca.scale = scale;
        RUN(attention_f32(ca, s));
        RUN(gemm(f.AO, qd, ly.wco, f.X, D, M, D, qd, nullptr, EPI_RES));
        // SwiGLU MLP, AdaLN-Zero (base:528-533)
        RUN(rmsnorm_f32(f.X, ly.n_mlp, md + 3 * D, md + 4 * D, mbs, S, f.XN, M, D, eps, s));
        RUN(gemm(f.XN, D, ly.wg, f.G, F, M, F, D, nullptr, EPI_STORE));
        RUN(gemm(f.XN, D, ly.wu, f.U, F, M, F, D, nullptr, EPI_STORE));
        RUN(swiglu_f32(f.G, f.U, f.Hb, (int64_t)M * F, s));
        RUN(gemm(f.Hb, F, ly.wdown, f.X, D, M, D, F, nullptr, EPI_GATED_RES, md + 5 * D));
    }
    // norm_out AdaLN + proj_out + crop (base:1491-1501)
    RUN(rmsnorm_f32(f.X, f.norm_out, f.mod_out, f.mod_out + D, 2 * D, S, f.XN, M, D, eps, s));
    RUN(gemm(f.XN, D, f.wout, T % 2 == 0 ? vt_out : f.O2, 128, M, 128, D, f.bout, EPI_STORE));
    if (T % 2) RUN(crop_rows_f32(f.O2, Bc, 2 * S, T, 64, vt_out, s));
#undef RUN
    return 0;
}
