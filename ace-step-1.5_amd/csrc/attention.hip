// attention.hip — flash attention forward for the DiT (head_dim 128, GQA).
//
// Covers all three attention flavours of the decoder (reference
// AceStepAttention.forward base:289-371 via SDPA):
//   * full bidirectional self-attention (odd layers),
//   * bidirectional band |i−j| ≤ window (even "sliding" layers; only the
//     KV tiles that intersect the band are visited — the reference's SDPA
//     path computes the full S×S and masks it),
//   * unmasked cross-attention over the cached encoder K/V (base:1384-1428:
//     the decoder never masks encoder padding);
//   * key-padding-masked self-attention for the condition encoders
//     (AceStepEncoderLayer base:401-440 with create_4d_mask base:56-135):
//     kmask[b][j] = 0 excludes key j.  The reference's additive mask is the
//     finite finfo.min, so a query row with NO admissible key softmaxes
//     uniformly over all Sk keys (band-excluded ones included); the masked
//     mode therefore visits every KV tile and gives excluded keys a common
//     finite score (NEG) while keys past Sk get a far lower one (PAST),
//     which reproduces exactly that.
//
// Layout: q [B][H][Sq][128], k/v [B][KV][Sk][128] (head-major, written by
// head_post), o token-major [B][Sq][o_ld] at column h·128.
//
// Structure: workgroup = the NREP query heads of one KV head (GQA sharing)
// × 4 waves × 32 queries; KV tiles of 64 keys in a 3-deep LDS ring, the next
// tile's LDS-DMA (global_load_lds, swizzle applied on the source) in flight
// during the current tile's MFMAs, one barrier per tile; the
// second head's waves run P·V one tile late so SIMD partners alternate
// softmax and MFMA work; tiles are stored as rows of 256 B, 16-B chunks XOR-swizzled so that the
// K row reads (ds_read_b128) and the V transposed reads (ds_read_b64_tr_b16)
// are bank-conflict free).  Per wave, v_mfma_f32_32x32x16_bf16 computes the
// swapped score tile Sᵀ = K·Qᵀ, so each lane owns one query row: the row
// max/sum is 32 in-register values plus one cross-half exchange.  Sᵀ's
// accumulator registers, converted to bf16, are directly the B operand of
// Oᵀ = Vᵀ·Pᵀ (no LDS round trip for P).  Online softmax in the exp2 domain;
// masked scores use a finite power-of-two sentinel (a row whose first tiles are
// fully masked accumulates garbage that the first real tile's rescale zeroes).
//
// attn_pw_kernel (band layers by default, ACEHIP_ATTN_PW): the same math with 64 query
// rows per wave at one wave per SIMD, O / Q / K in asm-owned AGPRs and the softmax VALU
// hand-placed between the MFMAs (its header below has the schedule and the A/B numbers).
#include <atomic>
#include <type_traits>
#include "kernels.h"

namespace acehip {
namespace {

#ifndef ATT_XCD
#define ATT_XCD 1          // XCD-aware block → work-unit remap
#endif
#ifndef ATT_DEFER
#define ATT_DEFER 0        // SIMD partners out of phase: waves 4-7 run each tile's P·V one tile late
#endif                     // (3-slot ring) — A/B switch: measured 171 → 191 µs (r02), off
#ifndef ATT_SPLIT_HEADS
#define ATT_SPLIT_HEADS 1  // GQA pair split into two 4-wave workgroups for short KV loops
#endif
// timing experiments only (wrong results; tools/bench_attn.py against the production build):
// attn_fwd_kernel without the QKᵀ MFMAs, the softmax VALU, the P·V MFMAs, the K/V LDS reads or the
// per-tile barrier's wait
#ifndef AF_X_NOQK
#define AF_X_NOQK 0
#endif
#ifndef AF_X_NOSM
#define AF_X_NOSM 0
#endif
#ifndef AF_X_NOPV
#define AF_X_NOPV 0
#endif
#ifndef AF_X_NOREAD
#define AF_X_NOREAD 0
#endif
#ifndef AF_X_NOBAR
#define AF_X_NOBAR 0
#endif
#ifndef ATT_TAU
#define ATT_TAU 8.0f       // lazy-rescale threshold (0: rescale on every new max)
#endif

constexpr int QB = 128;    // queries per workgroup
constexpr int KT = 64;     // keys per tile
// Sentinels are powers of two so that NEG·sl2 is exact: the exp2 argument
// fmaf(NEG, sl2, −m) of a row whose max IS the sentinel is then exactly 0
// (an all-masked row weighs its keys uniformly, and a row's all-masked first
// tiles add finite garbage that the first real tile's rescale zeroes).  With a
// non-power-of-two sentinel the fma's unrounded product differs from the
// rounded max by up to half an ulp of 1e29 — exp2 of that is 0 or inf.
constexpr float NEG = -0x1p100f;
constexpr float PAST = -0x1p126f;   // masked mode: keys past Sk (never weighted, even in an all-masked row)

// tail balancing: units [0, full) run whole; each later unit runs as nsplit
// KV-range parts whose partial (O, m, l) meet in ws, merged by the last part
struct SplitArgs {
    int nq, full, nsplit;
    float *ws;     // ≥ (units − full)·nsplit·8·66·64 floats
    int *cnt;      // ≥ units − full ints, zero between launches
    int units = 0; // attn_pw_kernel: > 0 = persistent over units [0, units) (no splits)
    // attn_fwd_kernel stream-K mode (sk_total > 0): the units' KV tiles form one sequence of
    // sk_total = units · sk_nt tiles (unit-major); workgroup c runs tiles
    // [c·total/grid, (c+1)·total/grid) as pieces of at most a few units.  A split unit's pieces
    // meet through a last-arriver ticket (cnt[first workgroup], self-resetting) and slabs in ws
    // (2·grid slots); no workgroup waits for another, so residency of the grid is not assumed.
    int sk_total = 0, sk_nt = 0;
    int prio = 0;           // attn_fwd_kernel<2>: static s_setprio 1 for waves 4-7 (ACEHIP_ATTN_PRIO)
};

// ds_read_b64_tr_b16 by inline asm (see pv() for why not the builtin)
__device__ __forceinline__ s16x4 ds_read_tr16(const char *lds_ptr) {
    s16x4 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)lds_ptr;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

__device__ __forceinline__ bf16x8 ds_read_b128(const char *lds_ptr) {
    bf16x8 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)lds_ptr;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}
// LDS reads at (per-lane offset VGPR + compile-time immediate): the per-lane parts
// (swizzled chunk offsets) are 8 VGPRs for K and 8 for V; the ring slot and the row
// block are the instruction's 16-bit offset field (the tile loop is unrolled by the
// two ring slots so both are constants) — no address VALU per read, and no hoisted
// VGPR address per (slot, fragment), which had cost ~50 VGPRs and spills.
__device__ __forceinline__ s16x4 opaque_s16x4() {
    s16x4 r;
    asm volatile("" : "=v"(r));
    return r;
}
template <int OFF>
__device__ __forceinline__ bf16x8 ds_read_b128_imm(uint32_t lane_off) {
    static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
    bf16x8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(lane_off), "n"(OFF));
    return r;
}
template <int OFF>
__device__ __forceinline__ s16x4 ds_read_tr16_imm(uint32_t lane_off) {
    static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lane_off), "n"(OFF));
    return r;
}
template <int V>
using IC = std::integral_constant<int, V>;
// s_waitcnt lgkmcnt(0) that the listed fragments depend on (nothing using them can be
// scheduled above it)
__device__ __forceinline__ void lgkm_wait8(bf16x8 (&f)[8]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]),
                 "+v"(f[6]), "+v"(f[7]));
}

__device__ __forceinline__ int kvoff(int row, int ch) {
    return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// Tail-split / short-split hand-off of one wave's (or pw sub-block's) partial (O, m, l):
// 16 KB of O as sixteen 1-KB lane-contiguous chunks (chunk k = O[k / 4][4(k % 4) .. +3] of
// every lane) + (m, l) per lane, published by write-through (sc1) 16-B stores and read back
// by the last arriver with sc1 16-B loads: with the relaxed agent-scope ticket in between this
// is a complete cross-XCD hand-off without a fence (cdna_hip_programming.md §5 "Projection GEMM
// at M = 256" item 2).  Each is ONE asm statement — all loads in flight before the single
// wait, and no register copy of a load's destination can sit between a load and its wait.
__device__ __forceinline__ f32x4 sub4(const f32x16 &v, int q) {
    return f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}
__device__ __forceinline__ void slab_store(float *slab, const f32x16 (&o)[4], float m, float l, int lane) {
    float *b0 = slab + lane * 4, *b1 = b0 + 4 * 256, *b2 = b0 + 8 * 256, *b3 = b0 + 12 * 256;
    float *bm = slab + 16 * 256 + lane * 2;
    const f32x2 ml = {m, l};
    asm volatile(
        "global_store_dwordx4 %0, %5, off sc1\n\t"
        "global_store_dwordx4 %0, %6, off offset:1024 sc1\n\t"
        "global_store_dwordx4 %0, %7, off offset:2048 sc1\n\t"
        "global_store_dwordx4 %0, %8, off offset:3072 sc1\n\t"
        "global_store_dwordx4 %1, %9, off sc1\n\t"
        "global_store_dwordx4 %1, %10, off offset:1024 sc1\n\t"
        "global_store_dwordx4 %1, %11, off offset:2048 sc1\n\t"
        "global_store_dwordx4 %1, %12, off offset:3072 sc1\n\t"
        "global_store_dwordx4 %2, %13, off sc1\n\t"
        "global_store_dwordx4 %2, %14, off offset:1024 sc1\n\t"
        "global_store_dwordx4 %2, %15, off offset:2048 sc1\n\t"
        "global_store_dwordx4 %2, %16, off offset:3072 sc1\n\t"
        "global_store_dwordx4 %3, %17, off sc1\n\t"
        "global_store_dwordx4 %3, %18, off offset:1024 sc1\n\t"
        "global_store_dwordx4 %3, %19, off offset:2048 sc1\n\t"
        "global_store_dwordx4 %3, %20, off offset:3072 sc1\n\t"
        "global_store_dwordx2 %4, %21, off sc1\n\t"
        "s_nop 1"
        :: "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(bm),
           "v"(sub4(o[0], 0)), "v"(sub4(o[0], 1)), "v"(sub4(o[0], 2)), "v"(sub4(o[0], 3)),
           "v"(sub4(o[1], 0)), "v"(sub4(o[1], 1)), "v"(sub4(o[1], 2)), "v"(sub4(o[1], 3)),
           "v"(sub4(o[2], 0)), "v"(sub4(o[2], 1)), "v"(sub4(o[2], 2)), "v"(sub4(o[2], 3)),
           "v"(sub4(o[3], 0)), "v"(sub4(o[3], 1)), "v"(sub4(o[3], 2)), "v"(sub4(o[3], 3)), "v"(ml)
        : "memory");
}
__device__ __forceinline__ void slab_load(const float *slab, f32x16 (&o)[4], float &m, float &l, int lane) {
    const float *b0 = slab + lane * 4, *b1 = b0 + 4 * 256, *b2 = b0 + 8 * 256, *b3 = b0 + 12 * 256;
    const float *bm = slab + 16 * 256 + lane * 2;
    f32x4 v[16];
    f32x2 ml;
    asm volatile(
        "global_load_dwordx4 %0, %17, off sc1\n\t"
        "global_load_dwordx4 %1, %17, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %17, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %17, off offset:3072 sc1\n\t"
        "global_load_dwordx4 %4, %18, off sc1\n\t"
        "global_load_dwordx4 %5, %18, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %6, %18, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %7, %18, off offset:3072 sc1\n\t"
        "global_load_dwordx4 %8, %19, off sc1\n\t"
        "global_load_dwordx4 %9, %19, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %10, %19, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %11, %19, off offset:3072 sc1\n\t"
        "global_load_dwordx4 %12, %20, off sc1\n\t"
        "global_load_dwordx4 %13, %20, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %14, %20, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %15, %20, off offset:3072 sc1\n\t"
        "global_load_dwordx2 %16, %21, off sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
          "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]),
          "=&v"(v[14]), "=&v"(v[15]), "=&v"(ml)
        : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(bm)
        : "memory");
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) o[k >> 2][4 * (k & 3) + e] = v[k][e];
    m = ml[0];
    l = ml[1];
}
// fold part (o2, m2, l2) into the running merge (o, m, l) — the same expression for every
// part whether it was loaded or is the last arriver's own, so the result does not depend on
// which part arrived last (bit-reproducible)
__device__ __forceinline__ void slab_fold(f32x16 (&o)[4], float &m, float &l, const f32x16 (&o2)[4], float m2,
                                          float l2, bool first) {
    if (first) {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = o2[i];
        m = m2;
        l = l2;
        return;
    }
    const float mn = fmaxf(m, m2);
    const float a1 = __builtin_amdgcn_exp2f(m - mn), a2 = __builtin_amdgcn_exp2f(m2 - mn);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) o[i][j] = o[i][j] * a1 + o2[i][j] * a2;
    l = l * a1 + l2 * a2;
    m = mn;
}

// NREP = query heads per KV head handled by one workgroup (GQA sharing:
// each K/V tile is staged once for all NREP heads).  4 waves × 32 queries
// per head → QB = 128 queries per head per workgroup.
template <int NREP>
__global__ __launch_bounds__(256 * NREP, 3 - NREP) void attn_fwd_kernel(const bf16_t *__restrict__ q,
                                                                  const bf16_t *__restrict__ k,
                                                                  const bf16_t *__restrict__ v,
                                                                  bf16_t *__restrict__ o, int H, int KV,
                                                                  int Sq, int Sk, int window, float sl2,
                                                                  int64_t o_ld, SplitArgs sp,
                                                                  const uint8_t *__restrict__ kmask) {
    constexpr int NT = 256 * NREP;
    constexpr int TILE = KT * 256;                 // one K or V tile: 64 rows × 256 B
    // K/V ring: tile j+1 is staged while tile j is computed; 3 slots when the deferred half
    // still reads V(j−1) during tile j (deeper rings with more tiles in flight measured
    // slower on every layer kind, r02: band 53.7 µs at depth 2 vs 56.3 / 56.2 at 3 / 4)
    constexpr bool DEFER = ATT_DEFER && NREP == 2;
    constexpr int NBUF = DEFER ? 3 : 2;
    // [K slot 0 .. NBUF−1 | V slot 0 .. NBUF−1]: the K and the V fragment reads each
    // address their region from their own lane-offset base, so every slot offset fits
    // the 16-bit ds offset field (3 slots of K|V interleaved would reach 96 KiB)
    __shared__ __attribute__((aligned(16))) char lds[NBUF * 2 * TILE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    // work unit u = (b, kvh, q-block), q-block fastest; blocks past sp.full are the
    // KV-range parts of the tail units (tail balancing, see attention())
    // XCD-aware: the blocks one XCD receives (bid ≡ x mod 8) take a contiguous unit range,
    // so the q-blocks of one (b, kv head) share that XCD's L2 copy of its K/V tiles
    // (whole units only: the tail-split parts must stay the grid's last blocks)
    const bool streamk = sp.sk_total > 0;
    int64_t g0 = 0, g1 = 0;                 // stream-K: this workgroup's global tile range
    // stream-K logical workgroup: the blocks of one XCD (bid ≡ x mod 8) take a contiguous range
    // of the tile sequence, so the units they walk share few K/V heads in that XCD's L2 (with
    // blockIdx.x itself, neighbouring ranges went to different XCDs: L2 hit rate 48 %,
    // profiles/r05v_pmc_tcc.json); slabs and tickets are indexed by the logical number
    const int cw = (streamk && ATT_XCD) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    if (streamk) {
        g0 = (int64_t)cw * sp.sk_total / gridDim.x;
        g1 = ((int64_t)cw + 1) * sp.sk_total / gridDim.x;
        if (g0 >= g1) return;
    }
    for (;;) {                              // pieces (one unless stream-K)
    int u = blockIdx.x, part = 0, nsplit = 1;
    int pt0 = 0, pt1 = 0;                   // stream-K: this piece's tiles [pt0, pt1) of unit u
    if (streamk) {
        u = (int)(g0 / sp.sk_nt);
        pt0 = (int)(g0 % sp.sk_nt);
        pt1 = (int)min<int64_t>(sp.sk_nt, pt0 + (g1 - g0));
    } else {
        if (ATT_XCD && u < sp.full) u = xcd_remap(u, sp.full);
        if (u >= sp.full) {
            const int j = u - sp.full;
            u = sp.full + j / sp.nsplit;
            part = j % sp.nsplit;
            nsplit = sp.nsplit;
        }
    }
    // head group hg of NREP query heads; hpw head groups share one KV head
    const int hpw = H / (KV * NREP);
    const int qb = u % sp.nq, hg = (u / sp.nq) % (KV * hpw), b = u / (sp.nq * KV * hpw);
    const int kvh = hg / hpw;
    const int hq = hg * NREP + (wave >> 2);
    const int qblk = qb * QB;
    const int q0 = qblk + (wave & 3) * 32;
    const int qi = q0 + r;
    // the younger half of the SIMD partners (waves 4-7) gets static priority
    // (MI355X_MICROARCH.md "Two waves per SIMD", item 4)
    if (sp.prio && NREP == 2 && __builtin_amdgcn_readfirstlane(wave) >= 4) __builtin_amdgcn_s_setprio(1);

    // Q fragments (B operand of Sᵀ = K·Qᵀ): lane holds Q[qi][16s + 8hh .. +8]
    const bf16_t *qp = q + (((int64_t)b * H + hq) * Sq + min(qi, Sq - 1)) * 128;
    bf16x8 qf[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *(const bf16x8 *)(qp + 16 * s + 8 * hh);
    // retire the Q loads with a waitcnt the compiler SEES (builtin, not asm: vmcnt(0)
    // expcnt(7) lgkmcnt(15)); otherwise its waitcnt pass, which cannot tell the loop's
    // LDS-DMAs from these register loads, re-waits vmcnt(0) at the first use of qf in
    // every tile — draining the K/V ring (cdna_hip_programming.md §5 trap (b))
    __builtin_amdgcn_s_waitcnt(0x0F70);

    const bf16_t *kp = k + ((int64_t)b * KV + kvh) * (int64_t)Sk * 128;
    const bf16_t *vp = v + ((int64_t)b * KV + kvh) * (int64_t)Sk * 128;
    int kv_lo = 0, kv_hi = Sk;
    const uint8_t *km = kmask ? kmask + (int64_t)b * Sk : nullptr;
    const bool causal = window == ATTN_CAUSAL;   // kernel-uniform: keys j <= i only
    if (window >= 0 && !km) {
        kv_lo = max(0, qblk - window);
        kv_hi = min(Sk, qblk + QB + window);
    }
    if (causal) kv_hi = min(Sk, qblk + QB);
    const int wlim = window >= 0 ? window : 0x7fffffff;
    int t_first = kv_lo / KT;
    int ntiles = (kv_hi + KT - 1) / KT - t_first;
    if (nsplit > 1) {                              // this part's contiguous tile range
        const int per = (ntiles + nsplit - 1) / nsplit;
        const int t0 = min(ntiles, part * per), t1 = min(ntiles, t0 + per);
        t_first += t0;
        ntiles = t1 - t0;
    }
    if (streamk) {                                 // unmasked full / cross: every unit has sk_nt tiles
        t_first += pt0;
        ntiles = pt1 - pt0;
    }

    // LDS-DMA staging of one K/V tile (32 KiB = 32 wave-instructions of 1 KiB, 4 per
    // wave): instruction c covers image rows 4c..4c+3 of K (c < 16) or V; lane L
    // writes the 16-B slot (row 4c + L/16, physical chunk L%16), so it fetches the
    // logical chunk that kvoff() places there (the XOR is an involution).  Rows
    // past Sk are clamped to a real row: those keys are masked (K) or meet P = 0 (V).
    auto stage_tile = [&](int kv0, int buf) {
#pragma unroll
        for (int i = 0; i < 32 / (NT / 64); ++i) {
            const int c = wave * (32 / (NT / 64)) + i;
            const int isv = c >> 4, row = (c & 15) * 4 + (lane >> 4), pc = lane & 15;
            const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
            const int key = min(kv0 + row, Sk - 1);
            glds16((isv ? vp : kp) + (int64_t)key * 128 + ch * 8,
                   lds + (isv * NBUF + buf) * TILE + (c & 15) * 1024);
        }
    };

    float m = NEG, l = 0.f;
    f32x16 oacc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) oacc[i][j] = 0.f;

    const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    // LDS byte address of the ring (uniform) and the per-lane swizzled offsets:
    // K fragment (row r [+32], logical chunk 2s+hh) — the swizzle depends on row & 15 only;
    // Vᵀ fragment (d-block dt, row 4(g>>1)+qq [+8]) — rows +16s, +32t are uniform offsets
    const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    uint32_t koff[8], voff[4][2];
#pragma unroll
    for (int s = 0; s < 8; ++s) koff[s] = lds_base + kvoff(r, 2 * s + hh);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int h8 = 0; h8 < 2; ++h8)
            voff[dt][h8] = lds_base + NBUF * TILE +
                           kvoff(4 * (g >> 1) + qq + 8 * h8, 4 * dt + 2 * (g & 1) + (pp >> 1)) + 8 * (pp & 1);
    // Oᵀ[d][q] += Vᵀ·Pᵀ; Vᵀ fragments by transposed LDS reads.  The reads are issued by
    // inline asm: hipcc's waitcnt pass treats its own ds_read_tr builtin as an LDS read
    // that may alias the in-flight LDS-DMA refills and waits vmcnt(0) before it (every
    // tile, draining the ring); the asm reads are waited explicitly (lgkmcnt(0) bound to
    // their results, so no MFMA can move above the wait)
    // VB: the V half of the ring slot (compile-time); key rows +32t +16s are immediates too
    auto pv_reads = [&](auto VBC, int dt, s16x4 (&rd)[2][2][2]) {
        constexpr int VB = decltype(VBC)::value;
        if (AF_X_NOREAD) {
            for (int a0 = 0; a0 < 2; ++a0)
                for (int a1 = 0; a1 < 2; ++a1)
                    for (int a2 = 0; a2 < 2; ++a2) rd[a0][a1][a2] = opaque_s16x4();
            return;
        }
        rd[0][0][0] = ds_read_tr16_imm<VB>(voff[dt][0]);
        rd[0][0][1] = ds_read_tr16_imm<VB>(voff[dt][1]);
        rd[0][1][0] = ds_read_tr16_imm<VB + 16 * 256>(voff[dt][0]);
        rd[0][1][1] = ds_read_tr16_imm<VB + 16 * 256>(voff[dt][1]);
        rd[1][0][0] = ds_read_tr16_imm<VB + 32 * 256>(voff[dt][0]);
        rd[1][0][1] = ds_read_tr16_imm<VB + 32 * 256>(voff[dt][1]);
        rd[1][1][0] = ds_read_tr16_imm<VB + 48 * 256>(voff[dt][0]);
        rd[1][1][1] = ds_read_tr16_imm<VB + 48 * 256>(voff[dt][1]);
    };
    auto pv_wait = [](s16x4 (&rd)[2][2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(rd[0][0][0]), "+v"(rd[0][0][1]), "+v"(rd[0][1][0]), "+v"(rd[0][1][1]),
                       "+v"(rd[1][0][0]), "+v"(rd[1][0][1]), "+v"(rd[1][1][0]), "+v"(rd[1][1][1]));
    };
    auto pv_mfma = [&](int dt, const s16x4 (&rd)[2][2][2], const bf16x8 (&pf)[2][2]) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                // whole-vector reinterpretation (per-element bit_cast<__bf16> insertion
                // is miscompiled by ROCm 7.2 hipcc: it keeps only the first dword)
                const s16x8 cat = __builtin_shufflevector(rd[t][s][0], rd[t][s][1], 0, 1, 2, 3, 4, 5, 6, 7);
                const bf16x8 vf = __builtin_bit_cast(bf16x8, cat);
                if (!AF_X_NOPV) oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[t][s], oacc[dt], 0, 0, 0);
                else oacc[dt][0] += (float)vf[0] + (float)pf[t][s][1];
            }
    };
    // P·V: the reads of d-block dt+1 are in flight during the MFMAs of dt
    auto pv = [&](auto VBC, const bf16x8 (&pf)[2][2]) {
        s16x4 ra[2][2][2], rb[2][2][2];
        pv_reads(VBC, 0, ra);
        pv_wait(ra);
        pv_reads(VBC, 1, rb);
        pv_mfma(0, ra, pf);
        pv_wait(rb);
        pv_reads(VBC, 2, ra);
        pv_mfma(1, rb, pf);
        pv_wait(ra);
        pv_reads(VBC, 3, rb);
        pv_mfma(2, ra, pf);
        pv_wait(rb);
        pv_mfma(3, rb, pf);
    };

    // end-of-tile wait: own DMAs of the next tile landed, own LDS reads retired; then the
    // barrier publishes the tile to every wave and retires the current tile's reads (WAR
    // for the refill of its slot) — a raw s_barrier: __syncthreads() would add a full
    // vmcnt(0) drain
    auto tile_barrier = [&] {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (!AF_X_NOBAR) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    bf16x8 pf[2][2];          // P of the current tile (bf16), B operand of P·V

    // SIMD partners (wave w and w+4 share a SIMD) are put out of phase: the younger half
    // defers each tile's P·V into the next tile's interval, so within one barrier interval
    // wave w runs [QKᵀ(j) | softmax(j) | P·V(j)] while wave w+4 runs [P·V(j−1) | QKᵀ(j) |
    // softmax(j)]: two of the three segments pair MFMAs with the partner's softmax VALU
    // instead of both waves issuing the same kind (MI355X_MICROARCH "Two waves per SIMD").
    // P·V(j−1) precedes softmax(j)'s O rescale, so O is at tile j−1's max when it lands.
    const bool defer = DEFER && __builtin_amdgcn_readfirstlane(wave) >= 4;
    bool pending = false;          // deferred half: P of the last computed tile awaits P·V
    int pend_slot = 0;
    auto pv_slot = [&](int slot, const bf16x8 (&pfv)[2][2]) {
        if (slot == 0) pv(IC<0>{}, pfv);
        else if (slot == 1) pv(IC<TILE>{}, pfv);
        else pv(IC<2 * TILE>{}, pfv);
    };
    // one tile; SLOT (compile-time: the loop is unrolled by the ring slots) is the ring
    // slot holding tile it, so every LDS address offset is an immediate
    auto tile = [&](int it, auto SLOTC) {
        constexpr int SLOT = decltype(SLOTC)::value;
        constexpr int KB = SLOT * TILE, VB = SLOT * TILE;    // K from koff, V from voff (region-biased)
        constexpr int PREV = (SLOT + NBUF - 1) % NBUF;
        const int kv0 = (t_first + it) * KT;
        // refill: tile it+1 into the slot of tile it+1−NBUF, read by nobody now (with 3
        // slots that is tile it−2, whose deferred P·V ran in iteration it−1)
        if (it + 1 < ntiles) stage_tile(kv0 + KT, (SLOT + 1) % NBUF);
        if (DEFER && pending) {                     // wave-uniform: the deferred half only
            pv(IC<PREV * TILE>{}, pf);
            pending = false;
        }
        // band layers: a tile entirely outside this wave's |i−j| ≤ window band is
        // skipped (the wave still joins the barrier); one entirely inside needs no mask
        const bool outside = (window >= 0 && !km && (kv0 > q0 + 31 + window || kv0 + KT - 1 < q0 - window)) ||
                             (causal && kv0 > q0 + 31);
        const bool interior = !km && kv0 + KT <= Sk &&
                              (causal ? kv0 + KT - 1 <= q0
                                      : (window < 0 || (kv0 >= q0 + 31 - window && kv0 + KT - 1 <= q0 + window)));
        if (outside) {
            tile_barrier();
            return;
        }

        // Sᵀ tiles: keys 32t..32t+31 × this wave's 32 queries
        // K fragments by asm reads (see pv()); the reads of key half t=1 are in flight
        // during the MFMAs of t=0
        f32x16 st[2];
        {
            bf16x8 k0[8], k1[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) k0[s] = AF_X_NOREAD ? qf[s] : ds_read_b128_imm<KB>(koff[s]);
            lgkm_wait8(k0);
#pragma unroll
            for (int s = 0; s < 8; ++s) k1[s] = AF_X_NOREAD ? qf[s] : ds_read_b128_imm<KB + 32 * 256>(koff[s]);
#pragma unroll
            for (int j = 0; j < 16; ++j) { st[0][j] = 0.f; st[1][j] = 0.f; }
            if (!AF_X_NOQK) {
#pragma unroll
                for (int s = 0; s < 8; ++s) st[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0[s], qf[s], st[0], 0, 0, 0);
            }
            lgkm_wait8(k1);
            if (!AF_X_NOQK) {
#pragma unroll
                for (int s = 0; s < 8; ++s) st[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1[s], qf[s], st[1], 0, 0, 0);
            } else {
#pragma unroll
                for (int s = 0; s < 8; ++s) {       // keep the reads alive
                    st[0][s] += (float)k0[s][0];
                    st[1][s] += (float)k1[s][0];
                }
            }
        }
        // running max on raw scores (scale folded into the exp2 FMA below);
        // interior tiles of full / cross attention need no mask
        float mx = NEG;
        if (AF_X_NOSM) {
            mx = m;
        } else if (interior) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int j = 0; j < 16; ++j) mx = fmaxf(mx, st[t][j]);
        } else {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int kj = kv0 + 32 * t + (j & 3) + 8 * (j >> 2) + 4 * hh;
                    // branch-free: window < 0 ⇒ wlim = INT_MAX
                    const bool inr = kj < Sk;
                    bool ok = inr & (abs(qi - kj) <= wlim) & (!causal | (kj <= qi));
                    float bad = NEG;
                    if (km) {   // key-padding mode (uniform over branches: km is kernel-uniform)
                        ok = ok && km[inr ? kj : 0] != 0;
                        bad = inr ? NEG : PAST;
                    }
                    const float sv = ok ? st[t][j] : bad;
                    st[t][j] = sv;
                    mx = fmaxf(mx, sv);
                }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
        // lazy rescale: the running reference max moves only when a score exceeds it by more
        // than ATT_TAU (log2 units), so P = 2^(s − m) ≤ 2^TAU and after the first tiles the
        // O/l rescale (64 VALU per lane) is skipped almost always; O/l is the same softmax
        const float mn = mx > m + ATT_TAU ? mx : m;
        const float alpha = __builtin_amdgcn_exp2f(m - mn);   // raw v_exp_f32 (no denormal range fix-up)
        m = mn;
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float p = AF_X_NOSM ? st[t][j] : __builtin_amdgcn_exp2f(fmaf(st[t][j], sl2, -mn));
                st[t][j] = p;
                rs += p;
            }
        rs += __shfl_xor(rs, 32, 64);
        l = l * alpha + rs;
        if (__any(alpha != 1.0f)) {                  // skip the O rescale when no row's max grew
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 16; ++j) oacc[i][j] *= alpha;
        }

        // P (bf16) as the B operand: tile t, k-step s ← registers 8s..8s+7
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[t][s][j] = (__bf16)st[t][8 * s + j];
        if (DEFER && defer) {
            pending = true;
            pend_slot = SLOT;
        } else {
            pv(IC<VB>{}, pf);
        }
        tile_barrier();
    };
    if (ntiles > 0) stage_tile(t_first * KT, 0);
    tile_barrier();
    int it = 0;
    if constexpr (NBUF == 3) {
        for (; it + 2 < ntiles; it += 3) {
            tile(it, IC<0>{});
            tile(it + 1, IC<1>{});
            tile(it + 2, IC<2>{});
        }
        if (it < ntiles) tile(it, IC<0>{});
        if (it + 1 < ntiles) tile(it + 1, IC<1>{});
    } else {
        for (; it + 1 < ntiles; it += 2) {
            tile(it, IC<0>{});
            tile(it + 1, IC<1>{});
        }
        if (it < ntiles) tile(it, IC<0>{});
    }
    if (DEFER && pending) pv_slot(pend_slot, pf);

    if (nsplit > 1) {
        // publish this part's (O, m, l) (slab_store: write-through 16-B stores), then take a
        // ticket; the last part merges every part in part order, its own from registers — no
        // spinning, no fence (a __threadfence() would write back and invalidate the whole L2
        // and evict every co-resident workgroup's K/V tiles)
        const int64_t wsz = 66 * 64;                   // floats per wave: 64 O + m + l per lane
        float *const ws_u = sp.ws + (int64_t)(u - sp.full) * nsplit * 8 * wsz;
        slab_store(ws_u + ((int64_t)part * 8 + wave) * wsz, oacc, m, l, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        __shared__ int s_ticket;
        if (tid == 0) s_ticket = atomicAdd(sp.cnt + (u - sp.full), 1);
        __syncthreads();
        if (s_ticket != nsplit - 1) return;
        // every part, this one's too, from its slab (fp32 store / load is exact): no register
        // copy of the own partial held across the loop (that copy had spilled ~140 VGPRs)
        slab_load(ws_u + wave * wsz, oacc, m, l, lane);
        for (int p2 = 1; p2 < nsplit; ++p2) {
            f32x16 o2[4];
            float m2, l2;
            slab_load(ws_u + ((int64_t)p2 * 8 + wave) * wsz, o2, m2, l2, lane);
            slab_fold(oacc, m, l, o2, m2, l2, false);
        }
        if (tid == 0) sp.cnt[u - sp.full] = 0;         // self-resetting for the next launch
    }

    bool write_o = true;
    if (streamk && !(pt0 == 0 && pt1 == sp.sk_nt)) {
        // unit u is split over the pieces of workgroups c0 .. c1 (c0 holds tile 0).  No workgroup
        // waits for another (nothing assumes the whole grid is resident: two ranks sharing a
        // GPU, or a planned CU count above the device's, only delay pieces).  Ticket cnt[c0]:
        // every later piece publishes its slab (slot c) and adds 1; the tile-0 piece adds BIG —
        // if it sees all n later pieces already counted it folds at once from registers, else it
        // publishes its own slab (slot grid + c0) and adds 1 more.  Whoever makes the count
        // BIG + n + 1 (or the tile-0 piece seeing n) folds pieces c0, c0+1, …, c1 in that order
        // with one expression (slab_fold), so O is the same bits whoever folds.
        constexpr int BIG = 1 << 16;
        const int64_t wsz = 66 * 64;                   // floats per wave: 64 O + m + l per lane
        const int G = (int)gridDim.x;
        auto owner = [&](int64_t t) {                  // workgroup whose tile range holds tile t
            int c = (int)(t * G / sp.sk_total);
            while (c + 1 < G && ((int64_t)c + 1) * sp.sk_total / G <= t) ++c;
            while (c > 0 && (int64_t)c * sp.sk_total / G > t) --c;
            return c;
        };
        const int64_t ub = (int64_t)u * sp.sk_nt;
        const int c0 = pt0 == 0 ? cw : owner(ub), c1 = owner(ub + sp.sk_nt - 1);
        const int n = c1 - c0;
        auto slot = [&](int c) { return sp.ws + ((int64_t)(c == c0 ? G + c0 : c) * 8 + wave) * wsz; };
        __shared__ int s_fold;
        if (pt0 > 0) {
            slab_store(slot(cw), oacc, m, l, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) s_fold = atomicAdd(sp.cnt + c0, 1) == BIG + n;
            __syncthreads();
        } else {
            if (tid == 0) s_fold = atomicAdd(sp.cnt + c0, BIG) == n;
            __syncthreads();
            if (!s_fold) {
                slab_store(slot(cw), oacc, m, l, lane);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) s_fold = atomicAdd(sp.cnt + c0, 1) == BIG + n;
                __syncthreads();
            }
        }
        if (s_fold) {
            // the fold starts from piece c0: the tile-0 piece's own registers when it folds (the
            // usual case), else its slab; a later piece that folds reads its own partial back from
            // the slab it published (exact) — no register copy held across the loop
            if (cw != c0) slab_load(slot(c0), oacc, m, l, lane);
            for (int c2 = c0 + 1; c2 <= c1; ++c2) {
                f32x16 o2[4];
                float m2, l2;
                slab_load(slot(c2), o2, m2, l2, lane);
                slab_fold(oacc, m, l, o2, m2, l2, false);
            }
            if (tid == 0) sp.cnt[c0] = 0;              // self-resetting for the next launch
        } else {
            write_o = false;
        }
        __syncthreads();                               // s_fold is reused by the next piece
    }

    if (write_o && qi < Sq) {                 // both lanes of a row pair (lane, lane ^ 32) agree
    const float inv = 1.0f / l;
    bf16_t *op = o + ((int64_t)b * Sq + qi) * o_ld + hq * 128;
    // lane (r, hh) holds columns 32dt + 8gg + 4hh .. +3 of its row; the two half-waves swap one
    // 4-column group per pair (gg, gg+1) so each lane stores 8 contiguous columns as one 16-B
    // store (the store tail is issue-bound: MI355X_MICROARCH "attention epilogue store tail")
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int gp = 0; gp < 2; ++gp) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a0 = oacc[dt][8 * gp + j] * inv, a1 = oacc[dt][8 * gp + 4 + j] * inv;
                const float got = __shfl_xor(hh ? a0 : a1, 32, 64);
                v[j] = hh ? got : a0;
                v[4 + j] = hh ? a1 : got;
            }
            *(uint4 *)(op + 32 * dt + 16 * gp + 8 * hh) = pack8(v);
        }
    }
    if (!streamk) break;
    g0 += ntiles;
    if (g0 >= g1) break;
    }   // pieces
}

// ---------------------------------------------------------------------------
// attn_pw_kernel helpers.  The kernel owns AGPRs a[0:255] by number (the compiler allocates
// none: its arch-VGPR demand stays < 256 and it issues no MFMA itself):
//   a[0:127]    O of sub-blocks A (a0-63) and B (a64-127), d-block dt at +16·dt
//   a[128:191]  Q of A (a128-159) and B (a160-191), k-step s at +4·s
//   a[192:255]  K fragments of the current tile (keys 0-31 at a192 + 4s, 32-63 at a224 + 4s)
// Everything that touches them is inline asm, so hipcc neither counts those LDS / global
// loads (explicit waits) nor pads their hazards (explicit s_nop, noted where used).
constexpr int PW_O = 0, PW_Q = 128, PW_K = 192;
// timing experiments only (wrong results): drop the mid-tile barrier / the ring refill /
// the exponentials / the row max
#ifndef PW_PV_NOP
#define PW_PV_NOP 0        // s_nop 1 before every P·V MFMA (else one pf_fence per sub-block)
#endif
#ifndef PW_X_NOBAR
#define PW_X_NOBAR 0
#endif
#ifndef PW_X_NODMA
#define PW_X_NODMA 0
#endif
#ifndef PW_X_NOEXP
#define PW_X_NOEXP 0
#endif
#ifndef PW_X_NOMAX
#define PW_X_NOMAX 0
#endif
#ifndef PW_X_NOPV
#define PW_X_NOPV 0
#endif
#ifndef PW_X_NOQK
#define PW_X_NOQK 0
#endif
#ifndef PW_X_NOVREAD
#define PW_X_NOVREAD 0
#endif
#ifndef PW_X_NOKREAD
#define PW_X_NOKREAD 0
#endif
#ifndef PW_X_NOMASK
#define PW_X_NOMASK 0      // band tiles that straddle the band edge processed unmasked
#endif

// compile-time loop: f(IC<I>{}) for I in [I0, I1)
template <int I0, int I1, typename F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (I0 < I1) {
        f(std::integral_constant<int, I0>{});
        sfor<I0 + 1, I1>(f);
    }
}
// opaque redefinition: nothing reading x is scheduled above this point
template <typename T>
__device__ __forceinline__ void pin(T &x) { asm volatile("" : "+v"(x)); }
// single-instruction VALU (no SLP packing into v_pk_* beside the MFMAs, no canonicalising v_max)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vadd(float a, float b) {
    float r;
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vfma(float a, float b, float c) {
    float r;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// max / sum of a value over the lane pair (l, l ^ 32) by v_permlane32_swap: the two
// results hold v[l % 32] and v[32 + l % 32], identical on both lanes of the pair.  asm with
// a leading s_nop 1: the input may come from an asm VALU whose write hipcc does not see
// (VALU write → v_permlane read hazard)
__device__ __forceinline__ f32x2 pair32(float x) {
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return f32x2{a, b};
}
__device__ __forceinline__ float pair_max(float x) { const f32x2 p = pair32(x); return vmax(p[0], p[1]); }
__device__ __forceinline__ float pair_sum(float x) { const f32x2 p = pair32(x); return vadd(p[0], p[1]); }
// two softmax weights p = 2^(s·c − mn) summed into rs, as one hazard-safe stream: each
// transcendental result is read one instruction after it is written (trans → VALU read)
// (two partial sums: no add waits on the previous add)
__device__ __forceinline__ void exp2_pair(float &s0, float &s1, float c, float nmn, float &r0, float &r1) {
    asm volatile("v_fma_f32 %0, %0, %4, %5\n\t"
                 "v_fma_f32 %1, %1, %4, %5\n\t"
                 "v_exp_f32 %0, %0\n\t"
                 "v_exp_f32 %1, %1\n\t"
                 "v_add_f32 %2, %2, %0\n\t"
                 "v_add_f32 %3, %3, %1"
                 : "+v"(s0), "+v"(s1), "+v"(r0), "+v"(r1) : "v"(c), "v"(nmn));
}

// k-step S of Sᵀ = K·Qᵀ into st (VGPRs): K at AGPR KA, Q at AGPR QA; S = 0 starts with C = 0.
// st is not VALU-readable until the XDL write hazard has passed (callers place readers
// ≥ 2 MFMAs later or behind xdl_pad)
template <int S, int KA, int QA>
__device__ __forceinline__ void pw_qk(f32x16 &st) {
#if PW_X_NOQK
    if constexpr (S == 0) asm volatile("" : "=v"(st));
    return;
#endif
    if constexpr (S == 0)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], 0"
                     : "=v"(st) : "n"(KA), "n"(KA + 3), "n"(QA), "n"(QA + 3));
    else
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], %0"
                     : "+v"(st) : "n"(KA), "n"(KA + 3), "n"(QA), "n"(QA + 3));
}
// O (AGPR OA..OA+15) += Vᵀ·Pᵀ; s_nop 1 first: P (and V after a register copy) are VALU
// results the asm cannot see
template <int OA>
__device__ __forceinline__ void pw_pv(const bf16x8 &vf, const bf16x8 &pf) {
#if PW_X_NOPV
    asm volatile("" :: "v"(vf), "v"(pf));
    return;
#endif
#if PW_PV_NOP
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                 :: "n"(OA), "n"(OA + 15), "v"(vf), "v"(pf));
#else
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]" :: "n"(OA), "n"(OA + 15), "v"(vf), "v"(pf));
#endif
}
// P of one sub-block complete (all its bf16 converts above this point) and past the VALU
// write → MFMA read hazard before its P·V starts
__device__ __forceinline__ void pf_fence(bf16x8 (&pf)[2][2]) {
    asm volatile("s_nop 1" : "+v"(pf[0][0]), "+v"(pf[0][1]), "+v"(pf[1][0]), "+v"(pf[1][1]));
}
template <int KA, int OFF>
__device__ __forceinline__ void pw_kread(uint32_t lane_off) {
    static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
#if PW_X_NOKREAD
    return;
#endif
    asm volatile("ds_read_b128 a[%c0:%c1], %2 offset:%c3" :: "n"(KA), "n"(KA + 3), "v"(lane_off), "n"(OFF));
}
// XDL (8 passes) → VALU read of its result: 12 wait states
__device__ __forceinline__ void xdl_pad(f32x16 &a, f32x16 &b) { asm volatile("s_nop 7\n\ts_nop 4" : "+v"(a), "+v"(b)); }
__device__ __forceinline__ const void *pw_uniform(const void *p) {   // pointer known wave-uniform → SGPRs
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const void *)(((uint64_t)hi << 32) | lo);
}
// LDS-DMA of one 1 KiB piece, saddr form (SGPR base, per-lane 32-bit offset); M0 (the LDS
// destination) is written in the same statement
__device__ __forceinline__ void pw_dma(const char *base, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr), "v"(voff),
                 "s"(base) : "memory");
}
template <int A>
__device__ __forceinline__ void pw_qload(const bf16_t *p) {
    asm volatile("global_load_dwordx4 a[%c0:%c1], %2, off" :: "n"(A), "n"(A + 3), "v"(p) : "memory");
}
template <int R>
__device__ __forceinline__ float pw_oread() {
    float x;
    asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "n"(R));
    return x;
}
// O block of one sub-block (64 AGPRs) *= a; ends with the v_accvgpr_write → MFMA C-read pad
template <int R>
__device__ __forceinline__ void pw_scale1(float a) {
    float t;
    asm volatile("v_accvgpr_read_b32 %0, a%c1\n\tv_mul_f32 %0, %0, %2\n\tv_accvgpr_write_b32 a%c1, %0"
                 : "=&v"(t) : "n"(R), "v"(a));
}
template <int OA>
__device__ __forceinline__ void pw_oscale(float a) {
    asm volatile("s_nop 1");                       // a may be a fresh transcendental result
    sfor<0, 64>([&](auto I) __attribute__((always_inline)) { pw_scale1<OA + decltype(I)::value>(a); });
    asm volatile("s_nop 2");
}

// ---------------------------------------------------------------------------
// 64 query rows per wave, one wave per SIMD (full / band / cross of the DiT; GQA pair):
// workgroup = 4 waves = the two query heads of one KV head × 128 queries (waves 0-1 head
// 2·kvh, waves 2-3 head 2·kvh + 1), each wave two 32-row sub-blocks A, B that share every
// K and Vᵀ fragment read (half the LDS read traffic per MFMA of attn_fwd_kernel).  One
// instruction stream interleaves the two sub-blocks: the softmax VALU of one runs in the
// gaps of the other's MFMAs (MI355X_MICROARCH "one wave per SIMD": a few single-issue
// fillers hide per MFMA gap) — attn_fwd_kernel's two waves per SIMD instead run the same
// phase between barriers.  Same work units, tail split, LDS image, swapped Sᵀ = K·Qᵀ
// layout and lazy rescale as attn_fwd_kernel.
__global__ __launch_bounds__(256, 1) void attn_pw_kernel(const bf16_t *__restrict__ q, const bf16_t *__restrict__ k,
                                                         const bf16_t *__restrict__ v, bf16_t *__restrict__ o,
                                                         int H, int KV, int Sq, int Sk, int window, float sl2,
                                                         int64_t o_ld, SplitArgs sp) {
    constexpr int NBUF = 2, TILE = KT * 256;
    __shared__ __attribute__((aligned(16))) char lds[NBUF * 2 * TILE];
    // wave index provably uniform (readfirstlane), so every per-wave tile decision below is a
    // scalar branch (a divergent-looking one makes hipcc structurize both tile variants into
    // one exec-masked sequence with both register sets live)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    // persistent mode (sp.units > 0, band layers with more units than CUs): this workgroup runs
    // units blockIdx.x, blockIdx.x + gridDim.x, ... as ONE stream of KV tiles — the next unit's
    // first two tiles are staged during the current unit's last two, its Q is loaded behind the
    // last tile's barrier and its first K reads ride in the last P·V phase, so a unit boundary
    // costs the O write-out instead of a launch round's prologue (cost model, tools/attn_cost.py:
    // ≈ 9 µs per round of units + ≈ 2 µs per tile)
    const bool persist = sp.units > 0;
    int u = blockIdx.x, part = 0, nsplit = 1;
    if (!persist) {
        if (ATT_XCD && u < sp.full) u = xcd_remap(u, sp.full);
        if (u >= sp.full) {
            const int j = u - sp.full;
            u = sp.full + j / sp.nsplit;
            part = j % sp.nsplit;
            nsplit = sp.nsplit;
        }
    }
    // geometry of unit uu (wave-uniform)
    struct UnitG {
        int b, kvh, hq, q0, t_first, ntiles;
    };
    auto geom = [&](int uu, int pt, int ns) __attribute__((always_inline)) {
        UnitG g;
        const int qb = uu % sp.nq;
        g.kvh = (uu / sp.nq) % KV;
        g.b = uu / (sp.nq * KV);
        g.hq = 2 * g.kvh + (wave >> 1);
        const int qblk = qb * QB;
        g.q0 = qblk + (wave & 1) * 64;     // this wave's 64 rows: sub-block sb = rows q0 + 32·sb + r
        int kv_lo = 0, kv_hi = Sk;
        if (window >= 0) {
            kv_lo = max(0, qblk - window);
            kv_hi = min(Sk, qblk + QB + window);
        }
        g.t_first = kv_lo / KT;
        g.ntiles = (kv_hi + KT - 1) / KT - g.t_first;
        if (ns > 1) {
            const int per = (g.ntiles + ns - 1) / ns;
            const int t0 = min(g.ntiles, pt * per), t1 = min(g.ntiles, t0 + per);
            g.t_first += t0;
            g.ntiles = t1 - t0;
        }
        return g;
    };
    // this wave's LDS-DMA source (waves 0-1 stage K, 2-3 V) of unit g's KV head, as SGPRs
    auto kv_base = [&](const UnitG &g) __attribute__((always_inline)) {
        const bf16_t *base = (wave < 2 ? k : v) + ((int64_t)g.b * KV + g.kvh) * (int64_t)Sk * 128;
        return (const char *)pw_uniform(base);
    };
    // Q of unit g → AGPRs a[128:191]
    auto load_q = [&](const UnitG &g) __attribute__((always_inline)) {
        sfor<0, 2>([&](auto SB) __attribute__((always_inline)) {
            constexpr int sb = decltype(SB)::value;
            const bf16_t *qp = q + (((int64_t)g.b * H + g.hq) * Sq + min(g.q0 + 32 * sb + r, Sq - 1)) * 128 + 8 * hh;
            sfor<0, 8>([&](auto S) __attribute__((always_inline)) {
                pw_qload<PW_Q + 32 * sb + 4 * decltype(S)::value>(qp + 16 * decltype(S)::value);
            });
        });
    };
    // the loop carries only what the tile loop reads (t_first, ntiles, q0 of this unit; t_first,
    // ntiles of the next): the rest is recomputed from the unit index where it is used — the
    // whole-struct copy cost SGPR spills
    int c_tf, c_nt, c_q0;
    {
        const UnitG g = geom(u, part, nsplit);
        c_tf = g.t_first;
        c_nt = g.ntiles;
        c_q0 = g.q0;
    }
    int qi[2] = {c_q0 + r, c_q0 + 32 + r};

    // O = 0 and Q → AGPRs (the clobber of a0 / a255 makes the kernel descriptor allocate all 256)
    sfor<0, 128>([&](auto I) __attribute__((always_inline)) {
        asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "n"(PW_O + decltype(I)::value));
    });
    asm volatile("s_nop 0" ::: "a0", "a255");
    load_q(geom(u, 0, 1));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // 32 KiB tile = 32 LDS-DMA wave-instructions, 8 per wave
    // Whole tiles (kv0 + 64 ≤ Sk) go by the saddr form: SGPR base = K or V + the piece's first
    // key row (uniform: waves 0-1 stage K, 2-3 V), VGPR = the lane's swizzled 16-B slot, one of
    // four per-lane offsets (the swizzle of row 4(c & 3) + lane / 16) — no per-piece address
    // VALU.  The last, partial tile clamps rows past Sk to a real row (per-lane addresses).
    uint32_t dma_off[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = 4 * j + (lane >> 4);
        dma_off[j] = (uint32_t)((lane >> 4) * 256 + (((lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4));
    }
    const char *kv_src = kv_base(geom(u, 0, 1));
    const uint32_t lds_u = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    // tile at key kv0 of the KV head whose K (waves 0-1) or V (waves 2-3) base is src → ring slot buf
    auto stage_tile = [&](const char *src, int kv0, int buf) __attribute__((always_inline)) {
        if (kv0 + KT <= Sk) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int c = wave * 8 + i;
                pw_dma(src + (int64_t)(kv0 + (c & 15) * 4) * 256, dma_off[i & 3],
                       lds_u + ((c >> 4) * NBUF + buf) * TILE + (c & 15) * 1024);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = wave * 8 + i;
            const int isv = c >> 4, row = (c & 15) * 4 + (lane >> 4), pc = lane & 15;
            const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
            const int key = min(kv0 + row, Sk - 1);
            glds16((const bf16_t *)src + (int64_t)key * 128 + ch * 8, lds + (isv * NBUF + buf) * TILE + (c & 15) * 1024);
        }
    };
    // the unit after this one (persistent mode)
    bool has_next = false;
    int un = 0, n_tf = 0, n_nt = 0;
    const char *nx_src = kv_src;

    const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    uint32_t koff[8], voff[4][2];
#pragma unroll
    for (int s = 0; s < 8; ++s) koff[s] = lds_base + kvoff(r, 2 * s + hh);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int h8 = 0; h8 < 2; ++h8)
            voff[dt][h8] = lds_base + NBUF * TILE +
                           kvoff(4 * (g >> 1) + qq + 8 * h8, 4 * dt + 2 * (g & 1) + (pp >> 1)) + 8 * (pp & 1);

    float m[2] = {NEG, NEG}, l[2] = {0.f, 0.f};
    // K read i (0..15) of ring slot SLOT into the K AGPRs
    auto k_read = [&](auto SLOTC, auto IC_) __attribute__((always_inline)) {
        constexpr int KB = decltype(SLOTC)::value * TILE, i = decltype(IC_)::value;
        pw_kread<PW_K + 4 * i, KB + (i >> 3) * 32 * 256>(koff[i & 7]);
    };
    auto tile_barrier = [&] __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // Per tile it (ring slot SLOT; K(it) already read into a[192:255], DMA(it+1) in flight):
    //   1  QKᵀ of A (16 MFMAs)       ∥ the tile's 32 Vᵀ reads, A's max over key half 0
    //   2  QKᵀ of B (16 MFMAs)       ∥ A's max over key half 1, A's exponentials
    //   3  A's last exponentials, P_A, O_A rescale (rare), B's max
    //      ── own DMA landed + own reads retired, barrier: tile it+1 visible, slot SLOT free;
    //         DMA(it+2) into slot SLOT
    //   4  P·V of A (16 MFMAs)       ∥ B's exponentials
    //   5  P_B, O_B rescale (rare); P·V of B (16 MFMAs) ∥ K(it+1) reads
    // A wave whose 64 rows have no key of the tile in their band skips the compute (barrier,
    // DMA and the next K reads stay).
    auto tile = [&](int it, auto SLOTC, auto MASKC, bool outside) __attribute__((always_inline)) {
        constexpr int SLOT = decltype(SLOTC)::value;
        constexpr int NSLOT = (SLOT + 1) % NBUF;
        const int kv0 = (c_tf + it) * KT;
        s16x4 rv[4][2][2][2];         // Vᵀ fragments of the current tile, per d-block
        f32x16 st[2][2];              // scores per sub-block and key half
        bf16x8 pf[2][2][2];           // P (bf16) per sub-block, B operand of P·V
        float mx[2], mx2[2], mn[2], alpha[2], rs[2], rs2[2];

        // Vᵀ read i (0..31) of ring slot SLOT
        auto v_read = [&](auto SLOTC, auto IC_) __attribute__((always_inline)) {
            constexpr int VB = decltype(SLOTC)::value * TILE, i = decltype(IC_)::value;
            constexpr int dt = i >> 3, t = (i >> 2) & 1, s = (i >> 1) & 1, h8 = i & 1;
#if PW_X_NOVREAD
            rv[dt][t][s][h8] = opaque_s16x4();
#else
            rv[dt][t][s][h8] = ds_read_tr16_imm<VB + (32 * t + 16 * s) * 256>(voff[dt][h8]);
#endif
        };
        auto v_wait = [&] __attribute__((always_inline)) {
    #pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(rv[dt][0][0][0]), "+v"(rv[dt][0][0][1]), "+v"(rv[dt][0][1][0]), "+v"(rv[dt][0][1][1]),
                               "+v"(rv[dt][1][0][0]), "+v"(rv[dt][1][0][1]), "+v"(rv[dt][1][1][0]), "+v"(rv[dt][1][1][1]));
        };
        // MFMA gg (0..15) of the Sᵀ products of sub-block SB: key half gg / 8, k-step gg % 8
        auto qk_mfma = [&](auto SBC, auto GC) __attribute__((always_inline)) {
            constexpr int sb = decltype(SBC)::value, gg = decltype(GC)::value;
            constexpr int t = gg >> 3, s = gg & 7;
            pw_qk<s, PW_K + 32 * t + 4 * s, PW_Q + 32 * sb + 4 * s>(st[sb][t]);
        };
        // MFMA gg (0..15) of P·V of sub-block SB: d-block gg / 4, (key half, k-step) gg % 4
        auto pv_mfma = [&](auto SBC, auto GC) __attribute__((always_inline)) {
            constexpr int sb = decltype(SBC)::value, gg = decltype(GC)::value;
            constexpr int dt = gg >> 2, t = (gg >> 1) & 1, s = gg & 1;
            const s16x8 cat = __builtin_shufflevector(rv[dt][t][s][0], rv[dt][t][s][1], 0, 1, 2, 3, 4, 5, 6, 7);
            pw_pv<PW_O + 64 * sb + 16 * dt>(__builtin_bit_cast(bf16x8, cat), pf[sb][t][s]);
        };
        // Softmax pieces.  Each opens with pin() of what it reads: an opaque redefinition after
        // the MFMA issued just before it, so hipcc cannot hoist the piece above that MFMA (it
        // would otherwise gather all VALU ahead of the MFMA stream); its running result feeds the
        // next piece's pin, so it cannot sink far either.
        // max over scores j0 .. j0+7 of key half T (the band / Sk mask first when MASK)
        auto max_piece = [&](auto SBC, auto TC, auto J0C, auto MASKC, int kv0) __attribute__((always_inline)) {
            constexpr int sb = decltype(SBC)::value, t = decltype(TC)::value, j0 = decltype(J0C)::value;
            pin(mx[sb]);
            pin(mx2[sb]);
            if constexpr (decltype(MASKC)::value && !PW_X_NOMASK) {
                // key kv0 + c (c = 32t + (j&3) + 8(j>>2) + 4hh) is admissible iff c ∈ [lo, hi]
                const int lo = (window >= 0 ? qi[sb] - window : -0x40000000) - kv0 - 4 * hh;
                const int hi = min(window >= 0 ? qi[sb] + window : 0x3fffffff, Sk - 1) - kv0 - 4 * hh;
                const uint32_t span = hi >= lo ? (uint32_t)(hi - lo) : 0u;
                const bool none = hi < lo;
    #pragma unroll
                for (int j = j0; j < j0 + 8; ++j) {
                    const int c = 32 * t + (j & 3) + 8 * (j >> 2);
                    const bool ok = !none & ((uint32_t)(c - lo) <= span);
                    st[sb][t][j] = ok ? st[sb][t][j] : NEG;
                }
            }
    #pragma unroll
            for (int j = j0; j < j0 + 8; j += 4) {
#if !PW_X_NOMAX
            mx[sb] = vmax3(mx[sb], st[sb][t][j], st[sb][t][j + 1]);
            mx2[sb] = vmax3(mx2[sb], st[sb][t][j + 2], st[sb][t][j + 3]);
#endif
        }
        };
        // row max over the lane pair, the lazy-rescale reference max and its factor
        auto max_finish = [&](auto SBC) __attribute__((always_inline)) {
            constexpr int sb = decltype(SBC)::value;
            pin(mx[sb]);
            pin(mx2[sb]);
            const float x = pair_max(vmax(mx[sb], mx2[sb])) * sl2;
            mn[sb] = x > m[sb] + ATT_TAU ? x : m[sb];
            alpha[sb] = __builtin_amdgcn_exp2f(m[sb] - mn[sb]);
            m[sb] = mn[sb];
            rs[sb] = 0.f;
            rs2[sb] = 0.f;
        };
        // P = 2^(s·sl2 − mn) of scores j0, j0+1 of key half T, summed into rs
        auto exp_piece = [&](auto SBC, auto TC, auto J0C) __attribute__((always_inline)) {
            constexpr int sb = decltype(SBC)::value, t = decltype(TC)::value, j0 = decltype(J0C)::value;
            pin(rs[sb]);
            pin(rs2[sb]);
            float s0 = st[sb][t][j0], s1 = st[sb][t][j0 + 1];
#if !PW_X_NOEXP
            exp2_pair(s0, s1, sl2, -mn[sb], rs[sb], rs2[sb]);
#endif
            st[sb][t][j0] = s0;
            st[sb][t][j0 + 1] = s1;
        };
        // row sum over the lane pair, l, P → bf16, and the (rare) O rescale
        auto exp_finish = [&](auto SBC) __attribute__((always_inline)) {
            constexpr int sb = decltype(SBC)::value;
            pin(rs[sb]);
            pin(rs2[sb]);
            l[sb] = l[sb] * alpha[sb] + pair_sum(vadd(rs[sb], rs2[sb]));
    #pragma unroll
            for (int t = 0; t < 2; ++t)
    #pragma unroll
                for (int s = 0; s < 2; ++s)
    #pragma unroll
                    for (int j = 0; j < 8; ++j) pf[sb][t][s][j] = (__bf16)st[sb][t][8 * s + j];
            if (__any(alpha[sb] != 1.0f)) pw_oscale<PW_O + 64 * sb>(alpha[sb]);
        };
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // K(it) in a[192:255]
        if (!outside) {
            mx[0] = mx[1] = mx2[0] = mx2[1] = NEG;
            sfor<0, 16>([&](auto G) __attribute__((always_inline)) {     // phase 1
                constexpr int gg = decltype(G)::value;
                qk_mfma(IC<0>{}, G);
                v_read(SLOTC, IC<2 * gg>{});
                v_read(SLOTC, IC<2 * gg + 1>{});
                if constexpr (gg >= 10 && gg < 12) max_piece(IC<0>{}, IC<0>{}, IC<8 * (gg - 10)>{}, MASKC, kv0);
            });
            sfor<0, 16>([&](auto G) __attribute__((always_inline)) {     // phase 2
                constexpr int gg = decltype(G)::value;
                qk_mfma(IC<1>{}, G);
                if constexpr (gg >= 2 && gg < 4) max_piece(IC<0>{}, IC<1>{}, IC<8 * (gg - 2)>{}, MASKC, kv0);
                if constexpr (gg == 4) max_finish(IC<0>{});
                if constexpr (gg >= 5) exp_piece(IC<0>{}, IC<((gg - 5) >> 3)>{}, IC<(2 * ((gg - 5) & 7))>{});
            });
            // phase 3: A's exponentials of key half 1, j = 6..15
            sfor<0, 5>([&](auto G) __attribute__((always_inline)) {
                exp_piece(IC<0>{}, IC<1>{}, IC<(6 + 2 * decltype(G)::value)>{});
            });
            exp_finish(IC<0>{});
            xdl_pad(st[1][0], st[1][1]);           // B's QKᵀ chain just ended
            max_piece(IC<1>{}, IC<0>{}, IC<0>{}, MASKC, kv0);
            max_piece(IC<1>{}, IC<0>{}, IC<8>{}, MASKC, kv0);
            max_piece(IC<1>{}, IC<1>{}, IC<0>{}, MASKC, kv0);
            max_piece(IC<1>{}, IC<1>{}, IC<8>{}, MASKC, kv0);
            max_finish(IC<1>{});
            v_wait();
        }
#if !PW_X_NOBAR
        tile_barrier();
#endif
        if (has_next && it == c_nt - 1) {
            // the next unit's Q, behind the barrier that follows this unit's last QKᵀ MFMAs
            // (s_nop: their AGPR reads before the loads' writes); it lands during this tile's
            // P·V and the O write-out, waited for before the first QKᵀ of that unit
            asm volatile("s_nop 7" ::: "memory");
            load_q(geom(un, 0, 1));
        }
#if !PW_X_NODMA
        if (it + 2 < c_nt) stage_tile(kv_src, kv0 + 2 * KT, SLOT);
        else if (has_next && it + 2 - c_nt < n_nt) stage_tile(nx_src, (n_tf + it + 2 - c_nt) * KT, SLOT);
#endif
        const bool more = it + 1 < c_nt || has_next;
        if (!outside) {
            pf_fence(pf[0]);
            sfor<0, 16>([&](auto G) __attribute__((always_inline)) {     // phase 4
                constexpr int gg = decltype(G)::value;
                pv_mfma(IC<0>{}, G);
                exp_piece(IC<1>{}, IC<(gg >> 3)>{}, IC<(2 * (gg & 7))>{});
            });
            exp_finish(IC<1>{});
            pf_fence(pf[1]);
            if (more) {
                sfor<0, 16>([&](auto G) __attribute__((always_inline)) {  // phase 5
                    pv_mfma(IC<1>{}, G);
                    k_read(IC<NSLOT>{}, G);
                });
            } else {
                sfor<0, 16>([&](auto G) __attribute__((always_inline)) { pv_mfma(IC<1>{}, G); });
            }
        } else if (more) {
            sfor<0, 16>([&](auto G) __attribute__((always_inline)) { k_read(IC<NSLOT>{}, G); });
        }
    };
    // band: tiles outside the band of all 64 rows skipped; tiles inside it for all 64 mask-free
    auto run_tile = [&](int it, auto SLOTC) __attribute__((always_inline)) {
        const int kv0 = (c_tf + it) * KT, q0 = c_q0;
        const bool outside = window >= 0 && (kv0 > q0 + 63 + window || kv0 + KT - 1 < q0 - window);
        const bool interior = kv0 + KT <= Sk && (window < 0 || (kv0 >= q0 + 63 - window && kv0 + KT - 1 <= q0 + window));
        if (interior) tile(it, SLOTC, IC<0>{}, outside);
        else tile(it, SLOTC, IC<1>{}, outside);
    };
    // prologue: tile 0 staged and visible, tile 1 in flight, K(0) read
    if (c_nt > 0) stage_tile(kv_src, c_tf * KT, 0);
    tile_barrier();
    if (c_nt > 1) stage_tile(kv_src, (c_tf + 1) * KT, 1);
    if (c_nt > 0) sfor<0, 16>([&](auto G) __attribute__((always_inline)) { k_read(IC<0>{}, G); });
    int gpos = 0;   // position of the current tile in the workgroup's tile stream: ring slot gpos & 1
    for (;;) {
    un = u + (int)gridDim.x;
    has_next = persist && un < sp.units;
    if (has_next) {
        const UnitG g = geom(un, 0, 1);
        n_tf = g.t_first;
        n_nt = g.ntiles;
        nx_src = kv_base(g);
    }
    for (int it = 0; it < c_nt; ++it, ++gpos) {
        if (gpos & 1) run_tile(it, IC<1>{});
        else run_tile(it, IC<0>{});
    }

    // O out of the AGPRs (the last MFMAs wrote them just before: XDL → read pad)
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
    f32x16 oacc[2][4];
    sfor<0, 128>([&](auto I) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        oacc[i >> 6][(i >> 4) & 3][i & 15] = pw_oread<PW_O + i>();
    });

    if (nsplit > 1) {
        // tail-split hand-off as in attn_fwd_kernel's first version (4-B agent-scope relaxed
        // atomics; pw runs split only off the production path): the 16-B slab form's register
        // footprint beside both sub-blocks' O pushes hipcc past 256 arch VGPRs into AGPR
        // spills, which this kernel's asm-owned AGPRs cannot take.  "sub-wave" index 2·wave + sb
        const int64_t wsz = 66 * 64;
        auto st_c = [](float *p, float x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        auto ld_c = [](const float *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
            float *mine = sp.ws + (((int64_t)(u - sp.full) * nsplit + part) * 8 + 2 * wave + sb) * wsz;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 16; ++j) st_c(mine + (16 * i + j) * 64 + lane, oacc[sb][i][j]);
            st_c(mine + 64 * 64 + lane, m[sb]);
            st_c(mine + 65 * 64 + lane, l[sb]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        __shared__ int s_ticket;
        if (tid == 0) s_ticket = atomicAdd(sp.cnt + (u - sp.full), 1);
        __syncthreads();
        if (s_ticket != nsplit - 1) return;
        for (int p2 = 0; p2 < nsplit; ++p2) {          // all parts in part order (reproducible)
#pragma unroll
            for (int sb = 0; sb < 2; ++sb) {
                const float *oth = sp.ws + (((int64_t)(u - sp.full) * nsplit + p2) * 8 + 2 * wave + sb) * wsz;
                const float m2 = ld_c(oth + 64 * 64 + lane), l2 = ld_c(oth + 65 * 64 + lane);
                if (p2 == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 16; ++j) oacc[sb][i][j] = ld_c(oth + (16 * i + j) * 64 + lane);
                    l[sb] = l2;
                    m[sb] = m2;
                    continue;
                }
                const float mm = fmaxf(m[sb], m2);
                const float a1 = __builtin_amdgcn_exp2f(m[sb] - mm), a2 = __builtin_amdgcn_exp2f(m2 - mm);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 16; ++j)
                        oacc[sb][i][j] = oacc[sb][i][j] * a1 + ld_c(oth + (16 * i + j) * 64 + lane) * a2;
                l[sb] = l[sb] * a1 + l2 * a2;
                m[sb] = mm;
            }
        }
        if (tid == 0) sp.cnt[u - sp.full] = 0;
    }

    if (has_next) {
        // the next unit's Q (16 loads) landed; only its tile-1 LDS-DMA (8 pieces, issued after
        // the Q loads) may still be in flight — before any store joins the vmcnt queue
        if (n_nt >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
        if (qi[sb] >= Sq) continue;            // both lanes of a row pair leave together
        const float inv = 1.0f / l[sb];
        const int ub = u / (sp.nq * KV), uhq = 2 * ((u / sp.nq) % KV) + (wave >> 1);
        bf16_t *op = o + ((int64_t)ub * Sq + qi[sb]) * o_ld + uhq * 128;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int gp = 0; gp < 2; ++gp) {
                float vv[8];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float a0 = oacc[sb][dt][8 * gp + j] * inv, a1 = oacc[sb][dt][8 * gp + 4 + j] * inv;
                    const float got = __shfl_xor(hh ? a0 : a1, 32, 64);
                    vv[j] = hh ? got : a0;
                    vv[4 + j] = hh ? a1 : got;
                }
                *(uint4 *)(op + 32 * dt + 16 * gp + 8 * hh) = pack8(vv);
            }
    }
    if (!has_next) break;
    // next unit: O = 0 (its first P·V is a whole tile away), fresh softmax state
    sfor<0, 128>([&](auto I) __attribute__((always_inline)) {
        asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "n"(PW_O + decltype(I)::value));
    });
    m[0] = m[1] = NEG;
    l[0] = l[1] = 0.f;
    u = un;
    c_tf = n_tf;
    c_nt = n_nt;
    c_q0 = (u % sp.nq) * QB + (wave & 1) * 64;
    kv_src = nx_src;
    qi[0] = c_q0 + r;
    qi[1] = c_q0 + 32 + r;
    }   // unit loop
}

// one wave's folded partial of attn_small_kernel: 16 values + (m, l) per lane, lane-contiguous
// 1-KB chunks, write-through (sc1) stores / sc1 loads as slab_store / slab_load
__device__ __forceinline__ void small_part_store(float *p, const f32x16 &a, float m, float l, int lane) {
    float *b0 = p + lane * 4, *bm = p + 16 * 64 + lane * 2;
    const f32x2 ml = {m, l};
    asm volatile(
        "global_store_dwordx4 %0, %2, off sc1\n\t"
        "global_store_dwordx4 %0, %3, off offset:1024 sc1\n\t"
        "global_store_dwordx4 %0, %4, off offset:2048 sc1\n\t"
        "global_store_dwordx4 %0, %5, off offset:3072 sc1\n\t"
        "global_store_dwordx2 %1, %6, off sc1"
        :: "v"(b0), "v"(bm), "v"(sub4(a, 0)), "v"(sub4(a, 1)), "v"(sub4(a, 2)), "v"(sub4(a, 3)), "v"(ml)
        : "memory");
}
__device__ __forceinline__ void small_part_load(const float *p, f32x16 &a, float &m, float &l, int lane) {
    const float *b0 = p + lane * 4, *bm = p + 16 * 64 + lane * 2;
    f32x4 v0, v1, v2, v3;
    f32x2 ml;
    asm volatile(
        "global_load_dwordx4 %0, %5, off sc1\n\t"
        "global_load_dwordx4 %1, %5, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %5, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %5, off offset:3072 sc1\n\t"
        "global_load_dwordx2 %4, %6, off sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(ml)
        : "v"(b0), "v"(bm)
        : "memory");
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        a[e] = v0[e];
        a[4 + e] = v1[e];
        a[8 + e] = v2[e];
        a[12 + e] = v3[e];
    }
    m = ml[0];
    l = ml[1];
}

// attn_small_kernel (ACEHIP_ATTN_SMALL): unmasked full / cross attention with few query rows — the
// turbo 10 s song (Sq = 125: 8 GQA-pair units, and 2 KV tiles of self-attention or 11 of cross).
// attn_fwd_kernel runs such a grid on 8 workgroups (self) or 8 units × 4 KV parts handed off
// through global slabs (cross): a few CUs, or a cross-CU merge of 135 KB per part that one CU
// reads back.  Here a workgroup is ONE head × 32 query rows and its four waves (one per SIMD)
// take the KV tiles w, w + 4, w + 8, … each: every wave owns its K fragments (loaded straight into
// registers in the MFMA A-operand layout, the next tile's in flight during the current one) and a
// private two-slot LDS ring for V (LDS-DMA, read transposed), so the tile loop has no barrier;
// the four partial (O, m, l) meet once in LDS and wave w writes head dims 32w … 32w + 31.
// Per-tile math (Sᵀ = K·Qᵀ, exp2-domain online softmax with the lazy rescale, Oᵀ += Vᵀ·Pᵀ) is
// attn_fwd_kernel's.
__global__ __launch_bounds__(256, 1) void attn_small_kernel(const bf16_t *__restrict__ q, const bf16_t *__restrict__ k,
                                                           const bf16_t *__restrict__ v, bf16_t *__restrict__ o, int H,
                                                           int KV, int Sq, int Sk, float sl2, int64_t o_ld, int nparts,
                                                           float *__restrict__ ws, int *__restrict__ cnt,
                                                           const uint8_t *__restrict__ kmask, int causal) {
    constexpr int VT = KT * 256;                 // one V tile: 64 keys × 256 B
    __shared__ __attribute__((aligned(16))) char lds[4 * 2 * VT];   // 128 KB: per wave two V slots
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int nq = (Sq + 31) / 32;
    const int unit = blockIdx.x / nparts, part = blockIdx.x % nparts;
    const int qb = unit % nq, hq = (unit / nq) % H, b = unit / (nq * H);
    const int kvh = hq / (H / KV);
    const int qi = qb * 32 + r;
    bf16x8 qf[8];
    {
        const bf16_t *qp = q + (((int64_t)b * H + hq) * Sq + min(qi, Sq - 1)) * 128;
#pragma unroll
        for (int s = 0; s < 8; ++s) qf[s] = *(const bf16x8 *)(qp + 16 * s + 8 * hh);
    }
    const bf16_t *kp = k + ((int64_t)b * KV + kvh) * (int64_t)Sk * 128;
    const bf16_t *vp = v + ((int64_t)b * KV + kvh) * (int64_t)Sk * 128;
    // key-padding mode (the condition encoders): excluded keys score NEG, keys past Sk PAST, as
    // attn_fwd_kernel's masked mode — an all-excluded row softmaxes uniformly over its Sk keys
    const uint8_t *km = kmask ? kmask + (int64_t)b * Sk : nullptr;
    // KV part `part` of nparts: tiles [t0, t1); wave w takes t0 + w, t0 + w + 4, …
    // causal (the text encoder, no key mask): the unit's keys end at its last row's diagonal
    const int klast = causal ? min(Sk, min(Sq, qb * 32 + 32)) : Sk;
    const int ntall = (klast + KT - 1) / KT, per = (ntall + nparts - 1) / nparts;
    const int t0 = min(ntall, part * per), ntiles = min(ntall, t0 + per) - t0;
    const int nmine = ntiles > wave ? (ntiles - wave + 3) / 4 : 0;
    char *const vl = lds + wave * 2 * VT;
    auto stage_v = [&](int kv0, int buf) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const int row = c * 4 + (lane >> 4), pc = lane & 15;
            const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
            glds16(vp + (int64_t)min(kv0 + row, Sk - 1) * 128 + ch * 8, vl + buf * VT + c * 1024);
        }
    };
    // K fragments of keys kv0 + r (kk[0..7]) and kv0 + 32 + r (kk[8..15]): dims 16s + 8hh … +8
    auto load_k = [&](int kv0, bf16x8 (&kk)[16]) {
        const bf16_t *p0 = kp + (int64_t)min(kv0 + r, Sk - 1) * 128 + 8 * hh;
        const bf16_t *p1 = kp + (int64_t)min(kv0 + 32 + r, Sk - 1) * 128 + 8 * hh;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            kk[s] = *(const bf16x8 *)(p0 + 16 * s);
            kk[8 + s] = *(const bf16x8 *)(p1 + 16 * s);
        }
    };
    const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    const uint32_t vbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)vl;
    uint32_t voff[4][2];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int h8 = 0; h8 < 2; ++h8)
            voff[dt][h8] = vbase + kvoff(4 * (g >> 1) + qq + 8 * h8, 4 * dt + 2 * (g & 1) + (pp >> 1)) + 8 * (pp & 1);

    float m = NEG, l = 0.f;
    f32x16 oacc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) oacc[i][j] = 0.f;

    auto tile = [&](int j, auto SLOTC, bf16x8 (&kc)[16], bf16x8 (&kn)[16]) {
        constexpr int VB = decltype(SLOTC)::value * VT;
        const int kv0 = (t0 + wave + 4 * j) * KT;
        // this tile's K registers and V slot landed (issued one tile ago); the next tile's are
        // issued now, into the other slot, whose last reads retired inside the previous tile
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (j + 1 < nmine) {
            load_k(kv0 + 4 * KT, kn);
            stage_v(kv0 + 4 * KT, decltype(SLOTC)::value ^ 1);
        }
        f32x16 st[2];
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) { st[0][jj] = 0.f; st[1][jj] = 0.f; }
#pragma unroll
        for (int s = 0; s < 8; ++s) st[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc[s], qf[s], st[0], 0, 0, 0);
#pragma unroll
        for (int s = 0; s < 8; ++s) st[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc[8 + s], qf[s], st[1], 0, 0, 0);
        float mx = NEG;
        if (!km && kv0 + KT <= Sk && (!causal || kv0 + KT - 1 <= qb * 32)) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) mx = fmaxf(mx, st[t][jj]);
        } else {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) {
                    const int kj = kv0 + 32 * t + (jj & 3) + 8 * (jj >> 2) + 4 * hh;
                    // keys past the diagonal score NEG like keys past Sk: a wave whose tile is
                    // wholly past a row's diagonal adds finite garbage that the fold's weight
                    // 2^(m_w − m) = 0 removes (every row has key 0)
                    const bool inr = kj < Sk && (!causal || kj <= qi);
                    float sv = inr ? st[t][jj] : NEG;
                    if (km) sv = inr ? (km[kj] != 0 ? sv : NEG) : PAST;   // km is kernel-uniform
                    st[t][jj] = sv;
                    mx = fmaxf(mx, sv);
                }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
        const float mn = mx > m + ATT_TAU ? mx : m;
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        m = mn;
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const float pv = __builtin_amdgcn_exp2f(fmaf(st[t][jj], sl2, -mn));
                st[t][jj] = pv;
                rs += pv;
            }
        rs += __shfl_xor(rs, 32, 64);
        l = l * alpha + rs;
        if (__any(alpha != 1.0f)) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) oacc[i][jj] *= alpha;
        }
        bf16x8 pf[2][2];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) pf[t][s2][jj] = (__bf16)st[t][8 * s2 + jj];
        // Oᵀ += Vᵀ·Pᵀ: the Vᵀ reads of block dt + 1 in flight during the MFMAs of dt
        s16x4 rd[2][2][2][2];
        auto reads = [&](int dt, s16x4 (&x)[2][2][2]) {
            x[0][0][0] = ds_read_tr16_imm<VB>(voff[dt][0]);
            x[0][0][1] = ds_read_tr16_imm<VB>(voff[dt][1]);
            x[0][1][0] = ds_read_tr16_imm<VB + 16 * 256>(voff[dt][0]);
            x[0][1][1] = ds_read_tr16_imm<VB + 16 * 256>(voff[dt][1]);
            x[1][0][0] = ds_read_tr16_imm<VB + 32 * 256>(voff[dt][0]);
            x[1][0][1] = ds_read_tr16_imm<VB + 32 * 256>(voff[dt][1]);
            x[1][1][0] = ds_read_tr16_imm<VB + 48 * 256>(voff[dt][0]);
            x[1][1][1] = ds_read_tr16_imm<VB + 48 * 256>(voff[dt][1]);
        };
        auto wait = [](s16x4 (&x)[2][2][2]) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(x[0][0][0]), "+v"(x[0][0][1]), "+v"(x[0][1][0]), "+v"(x[0][1][1]),
                           "+v"(x[1][0][0]), "+v"(x[1][0][1]), "+v"(x[1][1][0]), "+v"(x[1][1][1]));
        };
        auto mfmas = [&](int dt, const s16x4 (&x)[2][2][2]) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const s16x8 cat = __builtin_shufflevector(x[t][s2][0], x[t][s2][1], 0, 1, 2, 3, 4, 5, 6, 7);
                    oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, cat), pf[t][s2],
                                                                       oacc[dt], 0, 0, 0);
                }
        };
        reads(0, rd[0]);
        wait(rd[0]);
        reads(1, rd[1]);
        mfmas(0, rd[0]);
        wait(rd[1]);
        reads(2, rd[0]);
        mfmas(1, rd[1]);
        wait(rd[0]);
        reads(3, rd[1]);
        mfmas(2, rd[0]);
        wait(rd[1]);
        mfmas(3, rd[1]);
    };
    bf16x8 ka[16], kb[16];
    if (nmine > 0) {
        load_k((t0 + wave) * KT, ka);
        stage_v((t0 + wave) * KT, 0);
    }
    int j = 0;
    for (; j + 1 < nmine; j += 2) {
        tile(j, IC<0>{}, ka, kb);
        tile(j + 1, IC<1>{}, kb, ka);
    }
    if (j < nmine) tile(j, IC<0>{}, ka, kb);

    // the four waves' partial (O, m, l) → LDS (the V rings are dead after the barrier), then wave w
    // folds head dims 32w … 32w + 31 in wave order
    __syncthreads();
    float *const po = (float *)lds;                 // [wave][64 values][64 lanes]
    float *const pml = (float *)(lds + 4 * 64 * 64 * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) po[(wave * 64 + i * 16 + jj) * 64 + lane] = oacc[i][jj];
    pml[wave * 128 + lane] = m;
    pml[wave * 128 + 64 + lane] = l;
    __syncthreads();
    float mw[4], lw[4], mt = NEG;
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) {
        mw[w2] = pml[w2 * 128 + lane];
        lw[w2] = pml[w2 * 128 + 64 + lane];
        mt = fmaxf(mt, mw[w2]);
    }
    float lt = 0.f;
    f32x16 acc;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) acc[jj] = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) {
        const float a = __builtin_amdgcn_exp2f(mw[w2] - mt);   // a wave without tiles: l = 0, O = 0
        lt = fmaf(lw[w2], a, lt);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) acc[jj] = fmaf(po[(w2 * 64 + wave * 16 + jj) * 64 + lane], a, acc[jj]);
    }
    if (nparts > 1) {
        // KV parts of one unit meet in ws: each publishes its folded (O rows × dims 32w …, m, l)
        // by write-through stores, the last arriver of the ticket folds them in part order
        // (bit-reproducible) — 16.5 KB per part, against 135 KB per part of attn_fwd_kernel's
        // 8-wave slabs
        float *const wsu = ws + (int64_t)unit * nparts * (4 * 18 * 64);
        small_part_store(wsu + ((int64_t)part * 4 + wave) * 18 * 64, acc, mt, lt, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        __shared__ int s_ticket;
        if (tid == 0) s_ticket = atomicAdd(cnt + unit, 1);
        __syncthreads();
        if (s_ticket != nparts - 1) return;
        const f32x16 own = acc;
        const float m_own = mt, l_own = lt;
        for (int p2 = 0; p2 < nparts; ++p2) {
            f32x16 a2 = own;
            float m2 = m_own, l2 = l_own;
            if (p2 != part) small_part_load(wsu + ((int64_t)p2 * 4 + wave) * 18 * 64, a2, m2, l2, lane);
            if (p2 == 0) {
                acc = a2;
                mt = m2;
                lt = l2;
            } else {
                const float mn = fmaxf(mt, m2);
                const float a1 = __builtin_amdgcn_exp2f(mt - mn), b2 = __builtin_amdgcn_exp2f(m2 - mn);
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) acc[jj] = acc[jj] * a1 + a2[jj] * b2;
                lt = lt * a1 + l2 * b2;
                mt = mn;
            }
        }
        if (tid == 0) cnt[unit] = 0;
    }
    if (qi < Sq) {                                  // both lanes of a row pair agree
        const float inv = 1.0f / lt;
        bf16_t *op = o + ((int64_t)b * Sq + qi) * o_ld + hq * 128 + 32 * wave;
#pragma unroll
        for (int gp = 0; gp < 2; ++gp) {
            float vv[8];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const float a0 = acc[8 * gp + jj] * inv, a1 = acc[8 * gp + 4 + jj] * inv;
                const float got = __shfl_xor(hh ? a0 : a1, 32, 64);
                vv[jj] = hh ? got : a0;
                vv[4 + jj] = hh ? a1 : got;
            }
            *(uint4 *)(op + 16 * gp + 8 * hh) = pack8(vv);
        }
    }
}

}  // namespace

static int num_cus_attn() {
    // ACEHIP_ATTN_CUS overrides the CU count the tail split plans for (tests use it
    // to exercise 3- and 4-way splits on small shapes)
    if (knobs().attn_cus > 0) return knobs().attn_cus;
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

// short-sequence KV split (a grid of a few units, e.g. the 10 s song's cross-attention: 8
// units): KV tiles per part.  ACEHIP_ATTN_SHORT_TPP (A/B).  Turbo 10 s cross
// (11 tiles, 8 units; tools/gpu_r03z.sh, one process): 1 tile per part 28.5 µs, 2: 22.7, 3: 20.3
// (DiT song 27.7 / 27.1 / 26.8 ms) — fewer, longer parts pay fewer hand-offs; 4 and 6 tiles
// (after the slab hand-off, tools/gpu_r03m2.sh): 19.6 / 21.9 vs 19.7 µs, song 25.7 / 26.1 vs 25.6
// ms; default 3
static int short_tpp() { return knobs().attn_short_tpp; }

size_t attention_ws_bytes() {
    const size_t cus = std::max<size_t>(1024, (size_t)num_cus_attn());
    // [tickets: cus ints][slabs: cus · 8 waves · 66·64 floats]; stream-K uses 2 slabs per workgroup
    return cus * 8 * 66 * 64 * sizeof(float) + cus * sizeof(int);   // ≤ cus split parts in flight
}

int attention(const bf16_t *q, const bf16_t *k, const bf16_t *v, bf16_t *o, int B, int H, int KV,
              int Sq, int Sk, int window, float scale, int64_t o_ld, void *ws, hipStream_t s,
              const uint8_t *kmask) {
    if (B <= 0 || Sq <= 0) return 0;
    if (Sk <= 0 || KV <= 0 || H % KV) return fail(-1, "attention: bad heads/lengths");
    if (o_ld % 8) return fail(-1, "attention: o_ld must be a multiple of 8");
    // a band wider than the sequence (|i − j| ≤ max(Sq, Sk) − 1 ≤ window: every pair admitted)
    // is full attention — the 10 s songs' sliding layers (S = 125, window 128) then run the full
    // kernel without per-tile band classification and masks
    if (window >= 0 && !kmask && std::max(Sq, Sk) - 1 <= window) window = -1;
    const int grp = H / KV;
    const float sl2 = scale * 1.4426950408889634f;
    const int nq = (Sq + QB - 1) / QB;
    const int cus = num_cus_attn();
    const int unit_tiles = (window >= 0 && !kmask) ? (QB + 2 * window) / KT + 1 : (Sk + KT - 1) / KT;
    // heads per workgroup: the GQA pair shares one 8-wave workgroup (K/V staged once per
    // tile for both heads), or each head gets its own 4-wave workgroup, two per CU, whose
    // SIMD partners run out of phase. Measured (r02, one box): band −3 %, cross −9 %,
    // full (47 tiles: the doubled K/V staging dominates) +7 %, cross with fewer pair units
    // than CUs (B = 1) +11 %, short split-KV cross slower.
    // 64-row-per-wave kernel for the DiT's unmasked GQA-pair layers: ACEHIP_ATTN_PW = bit mask of
    // the layer kinds that use it (1 full, 2 band, 4 cross = window < 0 with Sk != Sq).  r02 A/B
    // (tools/bench_attn.py, one process, three boxes): band 46.4-48.4 vs 47.6-48.8 µs (kept),
    // full 166-189 vs 161-179 and B = 1 cross 30.5-31.8 vs 29.6-30.6 (stay on attn_fwd_kernel)
    const Knobs &kn = knobs();
    const int pw_mask = kn.attn_pw;
    const int kind_bit = window >= 0 ? 2 : (Sk == Sq ? 1 : 4);
    // attn_small_kernel where its grid is at most 1.5 rounds of one-head × 32-row units (measured,
    // tools/bench_attn.py, one process, profiles/r05an_attn_small_vs_fwd.log: B = 2 full / cross at
    // S = 125 8.6 / 13.5 vs 15.6 / 26.7 µs, S = 375 (384 units) 21.6 / 29.1 vs 24.6 / 30.6; at
    // S = 750 (768 units) 45.1 / 43.0 vs 34.8 / 34.0 — attn_fwd_kernel's 128-row GQA-pair units
    // read K / V once per pair and tile, and win once the grid fills the chip)
    const int64_t small_units = (int64_t)((Sq + 31) / 32) * H * B;
    const bool small_causal = window == ATTN_CAUSAL && !kmask && kn.attn_small_causal;
    if (kn.attn_small && window < 0 && (window != ATTN_CAUSAL || small_causal) && small_units <= cus + cus / 2 &&
        (!kmask || kn.attn_small_mask)) {
        const int64_t units = small_units;
        // KV parts per unit: about one tile per wave while the grid stays within one round
        // (ACEHIP_ATTN_SMALL=2: no parts)
        int parts = 1;
        const int ntall = (Sk + KT - 1) / KT;
        if (ws && kn.attn_small == 1 && units <= std::max(1024, cus))
            parts = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)(ntall + 3) / 4, cus / units, 16}));
        attn_small_kernel<<<(unsigned)(units * parts), 256, 0, s>>>(
            q, k, v, o, H, KV, Sq, Sk, sl2, o_ld, parts,
            parts > 1 ? (float *)((char *)ws + (size_t)std::max(1024, cus) * sizeof(int)) : nullptr,
            parts > 1 ? (int *)ws : nullptr, kmask, small_causal ? 1 : 0);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    if (grp == 2 && !kmask && window != ATTN_CAUSAL && (pw_mask & kind_bit)) {
        const int units = nq * KV * B;
        SplitArgs sp{nq, units, 1, nullptr, nullptr};
        const int tail = units % cus;
        const int split_min = kn.attn_pw_split;   // shortest KV loop (tiles) whose tail units are split
        if (ws && unit_tiles >= split_min && units > cus && tail > 0 && tail <= cus / 2) {
            sp.full = units - tail;
            sp.nsplit = min(4, cus / tail);
        } else if (ws && window < 0 && units * 2 <= cus && unit_tiles >= 4) {
            sp.full = 0;
            sp.nsplit = min(min(cus / units, (unit_tiles + short_tpp() - 1) / short_tpp()), 16);
        }
        if (sp.nsplit > 1) {
            sp.cnt = (int *)ws;
            sp.ws = (float *)((char *)ws + (size_t)std::max(1024, cus) * sizeof(int));
        }
        int grid = sp.full + (units - sp.full) * sp.nsplit;
        // band layers with more units than CUs: one persistent workgroup per CU walking units
        // blockIdx.x + k·grid as one KV-tile stream (every unit then has ≥ 2 tiles: window ≥ KT,
        // Sq = Sk > 2·KT).  ACEHIP_ATTN_PERSIST=0 restores one workgroup per unit (A/B)
        if (kn.attn_persist && sp.nsplit == 1 && window >= KT && Sq == Sk && Sq > 2 * KT && units > cus) {
            sp.units = units;
            grid = cus;
        }
        attn_pw_kernel<<<grid, 256, 0, s>>>(q, k, v, o, H, KV, Sq, Sk, window, sl2, o_ld, sp);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    const bool short_split = window < 0 && nq * KV * B * 2 <= cus && unit_tiles >= 4;
    const bool split_heads = ATT_SPLIT_HEADS && grp == 2 && window != ATTN_CAUSAL &&
                             unit_tiles < 24 && !short_split && nq * KV * B > cus;
    const int nrep = split_heads ? 1 : grp;
    const int units = nq * KV * (grp / nrep) * B;
    SplitArgs sp{nq, units, 1, nullptr, nullptr};
    // one workgroup per CU: a partial last round of whole units is replaced by
    // tail units split over ⌊CUs / tail⌋ KV ranges (1.5 rounds instead of 2 at
    // 384 units on 256 CUs)
    const int tail = units % cus;
    // only long KV loops pay for the partial write + merge (measured: full attention
    // at S = 3000, 47 tiles, −27 %; band (≈7 tiles) and cross (11 tiles) lose)
    if (window == ATTN_CAUSAL) {
        // causal (text encoder): whole units only — a KV-range part past the diagonal
        // would hold no valid key
    } else if (ws && nrep == 2 && unit_tiles >= 24 && units > cus && tail > 0 && tail <= cus / 2) {
        sp.full = units - tail;
        sp.nsplit = min(4, cus / tail);
        sp.cnt = (int *)ws;
        sp.ws = (float *)((char *)ws + (size_t)std::max(1024, cus) * sizeof(int));
    } else if (ws && nrep == 2 && short_split) {
        // short sequences (a few query blocks): every unit split over KV ranges so the
        // grid reaches the CUs (cross-attention of a 10 s song: 8 units → 40 parts)
        sp.full = 0;
        sp.nsplit = min(min(cus / units, (unit_tiles + short_tpp() - 1) / short_tpp()), 16);
        sp.cnt = (int *)ws;
        sp.ws = (float *)((char *)ws + (size_t)std::max(1024, cus) * sizeof(int));
    }
    int grid = sp.full + (units - sp.full) * sp.nsplit;
    // stream-K (ACEHIP_ATTN_STREAMK): unmasked full layers whose units do not divide into whole
    // rounds run as ONE round of `cus` workgroups over the units' concatenated KV tiles, instead
    // of a whole round + tail-split parts (a second round's fixed cost).  240 s full attention
    // (384 units × 47 tiles on 256 CUs) 186.1 → 175.8 µs in one process; the one-round cross grid
    // (192 units × 11 tiles) loses, 34.8 → 45.8 (its pieces' restart + merge ≥ the 2.75 tiles
    // saved), so only grids of more units than CUs and long loops take it
    // (two slab slots per workgroup: 2·cus ≤ the workspace's 1024 slots)
    if (kn.attn_streamk && ws && nrep == 2 && window < 0 && !kmask && units > cus && units % cus != 0 &&
        unit_tiles >= 24 && 2 * (size_t)cus <= (size_t)std::max(1024, cus)) {
        const size_t wcus = (size_t)std::max(1024, cus);
        sp = SplitArgs{nq, units, 1, nullptr, nullptr};
        sp.sk_nt = unit_tiles;
        sp.sk_total = units * unit_tiles;
        sp.cnt = (int *)ws;
        sp.ws = (float *)((char *)ws + wcus * sizeof(int));
        grid = cus;
    }
    sp.prio = kn.attn_prio;
    if (nrep == 2) {
        attn_fwd_kernel<2><<<grid, 512, 0, s>>>(q, k, v, o, H, KV, Sq, Sk, window, sl2, o_ld, sp, kmask);
    } else if (nrep == 1) {
        attn_fwd_kernel<1><<<grid, 256, 0, s>>>(q, k, v, o, H, KV, Sq, Sk, window, sl2, o_ld, sp, kmask);
    } else {
        return fail(-1, "attention: heads/kv_heads must be 1 or 2");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace acehip
