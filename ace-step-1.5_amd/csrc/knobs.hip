// knobs.hip — the library's A/B switches, read from the environment ONCE (first use, or
// acehip_reload_knobs) instead of a getenv on every launch.  Defaults are the production
// choice; DESIGN.md's appendix lists what each alternative measured.
#include <atomic>
#include <cstdlib>
#include <mutex>

#include "kernels.h"
#include "../../include/acehip.h"

namespace acehip {
namespace {

int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}

Knobs read_env() {
    Knobs k;
    k.gemm_tailsplit = env_int("ACEHIP_GEMM_TAILSPLIT", 1);
    k.gemm_tail = env_int("ACEHIP_GEMM_TAIL", 1);
    k.gemm_helpers = env_int("ACEHIP_GEMM_HELPERS", 1);
    k.gemm_w4s = env_int("ACEHIP_GEMM_W4S", 1);
    k.gemm_hp128 = env_int("ACEHIP_GEMM_HP128", 1);
    k.splitk_fuse = env_int("ACEHIP_SPLITK_FUSE", 1);
    k.splitk_bn = env_int("ACEHIP_SPLITK_BN", 0);
    k.smallm_wholek = env_int("ACEHIP_SMALLM_WHOLEK", 2);
    k.attn_pw = env_int("ACEHIP_ATTN_PW", 2);
    k.attn_persist = env_int("ACEHIP_ATTN_PERSIST", 1);
    k.attn_pw_split = env_int("ACEHIP_ATTN_PW_SPLIT", 24);
    k.attn_short_tpp = env_int("ACEHIP_ATTN_SHORT_TPP", 3);
    k.attn_small = env_int("ACEHIP_ATTN_SMALL", 1);
    k.attn_small_mask = env_int("ACEHIP_ATTN_SMALL_MASK", 1);
    k.attn_small_causal = env_int("ACEHIP_ATTN_SMALL_CAUSAL", 1);
    if (k.attn_short_tpp <= 0) k.attn_short_tpp = 3;
    k.attn_cus = env_int("ACEHIP_ATTN_CUS", 0);
    k.attn_streamk = env_int("ACEHIP_ATTN_STREAMK", 1);
    k.fuse_rowadd = env_int("ACEHIP_FUSE_ROWADD", 1);
    k.dit_dedup = env_int("ACEHIP_DIT_DEDUP", 1);
    k.dit_graph = env_int("ACEHIP_DIT_GRAPH", 0);
    k.conv7 = env_int("ACEHIP_CONV7", 2);
    k.convt = env_int("ACEHIP_CONVT", 1);
    k.gemm_tailfuse = env_int("ACEHIP_GEMM_TAILFUSE", 1);
    k.gemm_hp_tail = env_int("ACEHIP_GEMM_HPTAIL", 1);
    k.gemm_pp128 = env_int("ACEHIP_GEMM_PP128", 1);
    k.attn_prio = env_int("ACEHIP_ATTN_PRIO", 0);
    k.convp = env_int("ACEHIP_CONVP", 3);
    k.conv_bm128 = env_int("ACEHIP_CONV_BM128", 2);
    k.ru7 = env_int("ACEHIP_RU7", 2);
    k.kv_group_kib = env_int("ACEHIP_KV_GROUP_KIB", 262144);
    k.vae_snake_in = env_int("ACEHIP_VAE_SNAKE_IN", 1);
    if (k.kv_group_kib <= 0) k.kv_group_kib = 262144;
    return k;
}

std::mutex g_mu;
Knobs g_knobs;
std::atomic<bool> g_loaded{false};

}  // namespace

const Knobs &knobs() {
    if (!g_loaded.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_loaded.load(std::memory_order_relaxed)) {
            g_knobs = read_env();
            g_loaded.store(true, std::memory_order_release);
        }
    }
    return g_knobs;
}

}  // namespace acehip

extern "C" int acehip_reload_knobs(void) {
    std::lock_guard<std::mutex> lk(acehip::g_mu);
    const unsigned gen = acehip::g_knobs.gen + 1;
    acehip::g_knobs = acehip::read_env();
    acehip::g_knobs.gen = gen;
    acehip::g_loaded.store(true, std::memory_order_release);
    return 0;
}
