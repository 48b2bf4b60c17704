// GEMM v6 (bf16 MFMA, gfx950) for the dense linear layers without a residual epilogue (the transformer's QKV / Q /
// KV projections and linear1 + GELU): B straight from L2.  Round-5 experiment, off by default (slower than gemm5 so
// far: numbers at gemm6_enabled below).
//
// gemm5 stages both operands of its 256 x 256 x 64 tile through LDS by LDS-DMA, 64 KB per K-tile, and its K-loop is
// bound by that staging stream (round-3 ablation: without the in-loop staging it ran at 1174 TFLOP/s).  The weights
// (<= 2 MB) are L2-resident, so here only A goes through LDS and every wave loads its own B fragments from L2 into
// VGPRs:
//   - tile 256 rows x 256 columns, 8 waves; wave w owns columns 32 w .. 32 w + 31 of all 256 rows (16 x 2 accumulator
//     tiles of 16 x 16: 128 registers); no B fragment is shared between waves, so none needs LDS;
//   - A: 32-KB K-tiles by LDS-DMA into a 4-deep ring (gemm3's swizzled image), three K-tiles ahead;
//   - B: 16-B fragments by global_load_dwordx4 in inline asm, three K-steps ahead, waited for by explicit counts (with
//     VGPR-returning loads and LDS-DMA both in flight the compiler's wait insertion drains the whole VM counter before
//     every use; rowln.hip); the A fragments are read by ds_read_b128 in inline asm for the same reason, four in flight;
//   - persistent: the resident workgroups walk the tiles; the next tile's first three A K-tiles and its first B
//     fragments are issued before the current tile's epilogue (gemm_epi.h), so their latency hides under it.
#include <cstdlib>

#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

namespace athd {

namespace {

constexpr int G6_BM = 256, G6_BN = 256, G6_NW = 8, G6_NT = 64 * G6_NW;
constexpr int G6_TM = G6_BM / 16, G6_TN = G6_BN / G6_NW / 16;     // 16 x 2 tiles per wave
constexpr int G6_STAGE = G6_BM * 128;                           // 32 KB: 256 rows x 64 bf16
constexpr int G6_NS = 4;                                        // A ring depth
constexpr int G6_AQ = G6_BM / 8 / G6_NW;                        // A DMA pieces per wave per K-tile (4)
typedef __attribute__((address_space(3))) void g6_lds_void;
typedef __attribute__((address_space(1))) void g6_gbl_void;

ATHD_DEV int g6_xcd_remap(int i, int n) {
    const int q = n / 8, r = n % 8, x = i % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
}

}  // namespace

template <unsigned F>
__global__ __launch_bounds__(G6_NT, 2) void gemm6_kernel(const GemmDesc d) {
    constexpr int TM = G6_TM, TN = G6_TN;
    __shared__ __attribute__((aligned(1024))) char ring[G6_NS * G6_STAGE];
    __shared__ double st_lds[2 * EPI_MAXG];
    __shared__ __attribute__((aligned(1024))) char sink[1024];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l15 = lane & 15, l4 = lane >> 4;
    const uint32_t M = (uint32_t)d.nb * d.H_out;
    const int ntm = (int)((M + G6_BM - 1) / G6_BM), ntn = d.N / G6_BN;
    const int ntiles = ntm * ntn;
    const int KT = d.K / 64;
    const int wn0 = 32 * wave;
    const uint32_t a_lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)ring;
    const int lrow = lane >> 3, chunk = (lane & 7) ^ lrow;

    // tiles in (m tile, n tile) order, each XCD a contiguous range: the n tiles of an m tile share its A rows in L2
    int tile = (int)blockIdx.x;
    if (tile >= ntiles) return;
    // addressing: wave-uniform 64-bit bases (SGPRs) + 32-bit per-lane byte offsets (gemm5's LIN form); rows past M
    // read row M - 1 (their results are never stored)
    uint32_t m0 = 0;
    int n0 = 0;
    uint32_t aoff[G6_AQ];
    const char* bbase[TN];
    const char* const abase = (const char*)d.A;
    const uint32_t boff = (uint32_t)(l15 * d.Kp + 8 * l4) * 2;
    auto setup = [&](int t) {
        const int L = g6_xcd_remap(t, ntiles);
        m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)((L / ntn) * G6_BM));
        n0 = __builtin_amdgcn_readfirstlane((L % ntn) * G6_BN);
#pragma unroll
        for (int j = 0; j < TN; ++j) bbase[j] = (const char*)d.Wp + (int64_t)(n0 + wn0 + 16 * j) * d.Kp * 2;
#pragma unroll
        for (int q = 0; q < G6_AQ; ++q) {
            uint32_t m = m0 + 8 * (wave + G6_NW * q) + lrow;
            m = m < M ? m : M - 1;
            aoff[q] = (m * (uint32_t)d.a_ld + 8 * chunk) * 2;
        }
    };
    // K-tile kt of A into ring slot kt % 4; past the last K-tile the same pieces re-read K-tile 0 into a 1-KB sink, so that every K-step issues the same operations and the wait counts are constants
    auto dma_a = [&](int kt) {
        const bool real = kt < KT;                   // (wave-uniform)
        char* dst = real ? ring + (kt % G6_NS) * G6_STAGE : sink;
        const char* ab = abase + (int64_t)(real ? kt : 0) * 128;
#pragma unroll
        for (int q = 0; q < G6_AQ; ++q)
            __builtin_amdgcn_global_load_lds((g6_gbl_void*)(ab + aoff[q]),
                                             (g6_lds_void*)(real ? dst + (wave + G6_NW * q) * 1024 : dst), 16, 0, 0);
    };
    // B fragments G6_BD K-steps ahead in a ring of G6_BD + 1 register sets: the A DMA of K-tile kt + 3, issued
    // after B(2 kt + 3), then stays in flight until the wait for B(2 kt + 4), two K-tiles later (one vmcnt orders both
    // streams: waiting for a B load also waits for every older A piece)
    constexpr int BD = 3;
    bf16x8_t bq[BD + 1][TN];                     // [K-step % 4][column tile]
    // (the base of column tile j at K-step ks is wave-uniform: an SGPR pair; the lane's part is boff)
    // (the tile's column-tile bases are wave-uniform SGPR pairs, set by setup; a K-step past the last re-reads K-step
    // 0 into the free register set, so that every K-step issues the same operations)
#define G6_LOAD_B(KS_, BUF)                                                                                        \
    do {                                                                                                           \
        const uint32_t vo_ = boff + (uint32_t)((KS_) < 2 * KT ? (KS_) : 0) * 64;                                   \
        for (int j_ = 0; j_ < TN; ++j_)                                                                            \
            asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(bq[BUF][j_]) : "v"(vo_), "s"(bbase[j_]));       \
    } while (0)
    // B of K-step ks landed: with the constant issue pattern, 14 younger operations may be in flight from K-step 2
    // on, 10 at K-steps 0 and 1 (the prologue's three B loads came after its A pieces); simulated over the issue
    // order for KT = 4, 8, 32, including that A(kt + 1) has landed in every wave before the barrier ending K-tile kt
#define G6_WAIT_B(KS_, BUF)                                                                                        \
    do {                                                                                                           \
        if ((KS_) < 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");                                         \
        else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");                                                    \
        for (int j_ = 0; j_ < TN; ++j_) asm volatile("" : "+v"(bq[BUF][j_]));                                    \
    } while (0)

    float4 bias4[TN];
    // A(0 .. 2), then B(K-steps 0 .. 2) of the current tile: the A pieces go first so that the waits for B(0) / B(1)
    // also land them (A(0) before K-tile 0, A(1) before the barrier that ends it)
    auto prologue = [&]() {
#pragma unroll
        for (int k = 0; k < G6_NS - 1; ++k) dma_a(k);
        asm volatile("" ::: "memory");
        G6_LOAD_B(0, 0);
        G6_LOAD_B(1, 1);
        G6_LOAD_B(2, 2);
        asm volatile("" ::: "memory");
    };
    setup(tile);
    prologue();
    if (d.stats && tid < 2 * EPI_MAXG) st_lds[tid] = 0.0;

    f32x4_t acc[TM][TN];
    for (;;) {
        load_bias4<TN>(d, n0, wn0, lane, bias4);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // K-step ks = 2 kt + s: issue B(ks + 3) and (s = 0) A(kt + 3) (dummies past the end); wait for B(ks).  At the
        // first K-step of K-tile kt - 1 that wait also landed A(kt) (issued before B(2 kt - 5)), in every wave, and
        // the barrier that ends K-tile kt - 1 published it
#define G6_KSTEP(KS_, BUF)                                                                                         \
        {                                                                                                          \
            const int ks = (KS_), kt = ks / 2, s = ks % 2;                                                         \
            G6_LOAD_B(ks + BD, ((BUF) + BD) % (BD + 1));                                                           \
            asm volatile("" ::: "memory");                                                                         \
            if (s == 0) dma_a(kt + 3);                                                                             \
            asm volatile("" ::: "memory");                                                                         \
            G6_WAIT_B(ks, BUF);                                                                                    \
            if (ks == 0) __builtin_amdgcn_s_barrier();    /* A(0) of every wave */                                \
            const uint32_t ab = a_lds + (uint32_t)((kt % G6_NS) * G6_STAGE) + (uint32_t)(l15 * 128) +             \
                                (uint32_t)(((4 * s + l4) ^ (l15 & 7)) * 16);                                       \
            /* the 16 row fragments in 4 groups of 4, the next group's reads in flight over the MFMAs */           \
            bf16x8_t af[2][4];                                                                                     \
            for (int u = 0; u < 4; ++u)                                                                            \
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[0][u]) : "v"(ab), "i"(u * 2048));           \
            for (int gi = 0; gi < 4; ++gi) {                                                                       \
                if (gi + 1 < 4) {                                                                                  \
                    for (int u = 0; u < 4; ++u)                                                                    \
                        asm volatile("ds_read_b128 %0, %1 offset:%2"                                               \
                                     : "=v"(af[(gi + 1) & 1][u]) : "v"(ab), "i"(((gi + 1) * 4 + u) * 2048));      \
                    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");                                            \
                } else {                                                                                           \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                            \
                }                                                                                                  \
                for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(af[gi & 1][u]));                               \
                for (int u = 0; u < 4; ++u)                                                                        \
                    for (int j = 0; j < TN; ++j)                                                                   \
                        acc[4 * gi + u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                              \
                            bq[BUF][j], af[gi & 1][u], acc[4 * gi + u][j], 0, 0, 0);                               \
            }                                                                                                      \
            if (s == 1) __builtin_amdgcn_s_barrier();   /* slot kt % 4 read by every wave: A(kt + 4) refills */    \
        }
#pragma unroll 1
        for (int ks4 = 0; ks4 < 2 * KT; ks4 += 4) {   // (four K-steps per iteration: the B ring index is a constant)
            G6_KSTEP(ks4, 0)
            G6_KSTEP(ks4 + 1, 1)
            G6_KSTEP(ks4 + 2, 2)
            G6_KSTEP(ks4 + 3, 3)
        }
#undef G6_KSTEP
        // the next tile's B(0) and A(0 .. 2) before this tile's epilogue (the ring is free: the barrier above)
        const uint32_t m0_done = m0;
        const int n0_done = n0;
        const int next = tile + (int)gridDim.x;
#ifndef ATHD_G6_LATE
        if (next < ntiles) {
            setup(next);
            prologue();
        }
#endif
        gemm_epilogue<TM, TN, F, true>(d, acc, m0_done, n0_done, 0, wn0, lane, st_lds, G6_BM, bias4);
#ifdef ATHD_G6_LATE
        if (next < ntiles) {
            setup(next);
            prologue();
        }
#endif
        // (the dummy A pieces of the last K-steps land in the sink: they must finish before the workgroup's LDS is
        // released; the next prologue's B loads write the registers of the dummy B loads after them, in order)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the epilogue's stores and the prologue's loads)
        if (next >= ntiles) break;
        tile = next;
        __builtin_amdgcn_s_barrier();
    }
#undef G6_LOAD_B
#undef G6_WAIT_B
}

// dense bf16 linear rows (one tap, A row m at m * a_ld), K a multiple of 128 (the K-loop takes 4 K-steps per
// iteration) with K == Kp, N a multiple of 256, an
// epilogue without residual or statistics
bool gemm6_supported(const GemmDesc& d) {
    const unsigned f = epi_flags(d);
    return (f == F_CBF16 || f == (F_GELU | F_CBF16)) && d.a_bf16 && d.ntaps == 1 && d.W == 1 && d.in_stride == 1 &&
           d.in_off == 0 && d.H_out == d.H_in && d.a_hs < 0 && d.a_bs < 0 && d.C_in == d.K && d.K == d.Kp &&
           d.K % 128 == 0 && d.K >= 256 && d.K <= 4096 && d.a_ld % 8 == 0 && d.a_cs == 1 && !d.a_norm && d.N % G6_BN == 0 &&
           !d.col_split && d.ldo == d.N && (int64_t)d.nb * d.H_in * d.a_ld * 2 < (1LL << 31) &&
           (int64_t)d.N * d.Kp * 2 < (1LL << 31);
}

// Measured (round 5, serialised events per forward, one box): linear1 2.93 -> 3.48 ms, QKV 1.16 -> 1.36, KV 0.58 ->
// 0.69, Q 0.34 -> 0.41 against gemm5; SQ: 4.3 VALU and 3.1 SALU instructions per MFMA (gemm5: ~2), MFMA busy 0.24 vs
// 0.29, waits 0.35.  Not the product path: ATHD_G6=1 selects it (the next round's starting point).
static bool gemm6_enabled() {
    static int v = -1;
    if (v < 0) { const char* e = std::getenv("ATHD_G6"); v = (e && e[0] == '1') ? 1 : 0; }
    return v == 1;
}

template <unsigned F>
static void launch6f(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out;
    const int64_t tiles = ((M + G6_BM - 1) / G6_BM) * (d.N / G6_BN);
    int64_t grid = (int64_t)device_cus() / 8 * 8;            // one 128-KB-LDS workgroup per CU, whole XCD rounds
    if (grid < 8) grid = 8;
    if (grid > tiles) grid = tiles;
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin(klabel("gemm6_kernel<%u>", F), fl, by);
    }
    hipLaunchKernelGGL((gemm6_kernel<F>), dim3((unsigned)grid), dim3(G6_NT), 0, s, with_fastdiv(d));
}

int gemm6_launch(const GemmDesc& d, hipStream_t s) {
    if (!gemm6_enabled() || !gemm6_supported(d)) return -2;
    if (epi_flags(d) == F_CBF16) launch6f<F_CBF16>(d, s);
    else launch6f<F_GELU | F_CBF16>(d, s);
    return (int)hipGetLastError();
}

}  // namespace athd
