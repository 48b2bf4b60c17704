// GEMM v5 (bf16 MFMA, gfx950): gemm4's 256 x 256 x 64 tile, slots and epilogues with a staggered two-group K-loop
// (cdna_hip_programming.md §5 "The 256² 8-phase template"; MI355X_MICROARCH.md §Two waves per SIMD).
//
// The 8 waves are two groups of 4, G0 = waves 0-3 (tile rows 0-127) and G1 = waves 4-7 (rows 128-255): a SIMD holds
// one wave of each.  A K-tile is 4 phases, one 64 x 32 accumulator quadrant each (16 v_mfma_f32_16x16x32_bf16):
//   p0 (A0, B0)   p1 (A0, B1)   p2 (A1, B1)   p3 (A1, B0)        fragment reads: p0 A0 + B0, p1 B1, p2 A1, p3 none
// and a group spends a phase in two SECTIONS separated by workgroup barriers: a load section (its fragment reads and
// its share of the LDS-DMA staging) and an MFMA section (s_waitcnt lgkmcnt(0), s_setprio 1, the 16 MFMAs).  G1 runs
// one section behind G0 (one extra barrier before its first section), so in every section one group's MFMAs share
// each SIMD with the other group's LDS reads and DMA issue: matrix beside memory.
//
// Staging: every half-tile slot of K-tile u + 2 is restaged in the first section its WAR allows (a slot's last
// fragment reads retire at the reader's next lgkmcnt(0), one section later, before that section's barrier), each
// wave issuing gemm4's 2 pieces of 1 KB per half-tile.  Sections s = 0..7 of K-tile u, G0 loading in even s, G1 in
// odd s:
//   s0 G0: A1(u+1)   s1 G1: -   s2 G0: -   s3 G1: A0 B0(u+2)   s4 G0: A0 B0(u+2)   s5 G1: B1(u+2)   s6 G0: B1(u+2)
//   s7 G1: A1(u+2)
// RAW: at each load section a wave waits (counted vmcnt) until only the pieces of its previous 4 load sections are in
// flight: a piece issued in section x is retired by section x + 10 and published by that section's barrier; every
// slot is first read >= 12 sections after its pieces were issued.  That keeps ~1 K-tile (64 KB) per CU in flight.
// kbench (one box, random operands; tools/kbench.py g5var): M = 132608, N = 1536 / 512, K = 512: +5 / +14 % over
// gemm4; K = 2048: equal.  The start-up sleep gemm4 uses to desynchronise epilogue store bursts cost 4096^3 a third
// of its time in isolation, so gemm5 has none.
// Persistent grid (epilogues without residual or statistics, as gemm4): the resident blocks walk their tiles and
// issue the next tile's first K-tiles before the current tile's epilogue.
#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

#include <algorithm>
#include <climits>
#include <type_traits>

namespace athd {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

constexpr int G5_SLOT = 16384;     // one half-tile slot: 128 rows x 64 bf16
// The K-loop's VM-counter bookkeeping: every issueA / issueB issues exactly G5_PIECES LDS-DMA pieces,
// each group makes G5_ISSUES_KTILE issue calls per K-tile (4 load sections), and the K-loop has no other global
// loads or stores.  The steady-state wait keeps the pieces of the previous 4 load sections in flight: vmcnt of
// G5_STEADY_VM.  Any change to the piece map or the staging schedule must keep these in step (the ATHD_G5_CHECK
// debug build compares the counted history with the constant on every steady K-step).
constexpr int G5_PIECES = 2;
constexpr int G5_ISSUES_KTILE = 4;
constexpr int G5_STEADY_VM = G5_PIECES * G5_ISSUES_KTILE;
static_assert(G5_STEADY_VM == 8, "the steady-state s_waitcnt below is written as vmcnt(8)");

ATHD_DEV void vm_wait_n(int n) {   // n = 0, 2, 4, 6, 8 (wave-uniform)
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

ATHD_DEV void section_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// persistent grid: epilogues without residual or statistics (as gemm4); ATHD_G5_PRES=1 adds the residual-stream
// epilogue with statistics (F_RES | F_STATS, not F_RGN: that one stages its affine through a ring slot)
#ifndef ATHD_G5_PRES
#define ATHD_G5_PRES 0
#endif
ATHD_HD constexpr bool g5_persist(unsigned F) {
    return (F & (F_RES | F_STATS)) == 0 || (ATHD_G5_PRES && (F & F_RGN) == 0 && (F & ~(F_RES | F_STATS)) == 0);
}

ATHD_DEV int xcd_remap5(int i, int n) {
    const int q = n / 8, r = n % 8, x = i % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
}

}  // namespace

__device__ __attribute__((aligned(64))) uint4 g_zero_page5[4];

// PROBE (tools/kbench ablations only; the product instantiates 0): 1 = no LDS-DMA staging in the K-loop, 2 = no
// fragment reads in the K-loop, 3 = no MFMAs, 4 = no section barriers in the K-loop (results are garbage).
// LIN: dense single-tap rows (linear / 1x1 layers: A row of output row m at m * a_ld, K == Kp == C_in).  Each lane's A
// source is then a 32-bit byte offset fixed per tile, and a K-tile's address is a wave-uniform base + that offset
// (global_load_lds with an SGPR base: no per-issue VALU), instead of the implicit-GEMM row / tap / bounds arithmetic
// (~170 VALU instructions per K-tile and wave in the general form, against 64 MFMAs).  In both forms the
// steady-state K-steps (u + 2 < nk) wait with a constant vmcnt(8) (every window of 4 consecutive load sections issues
// 8 pieces) instead of the counted-history branch chain; the last two K-steps keep the history.
template <unsigned F, int PROBE = 0, bool LIN = false>
__global__ __launch_bounds__(512) void gemm5_kernel(const GemmDesc d) {
    constexpr bool PERSIST = g5_persist(F);
    constexpr int TM = 8, TN = 4;
    constexpr int NW = 8;
    // one LDS array (cdna_hip_programming.md §5 item 4(a)): 8 staging slots | GroupNorm statistics | bias of the
    // current and the next tile (the bias stays out of the K-loop's registers)
    __shared__ __attribute__((aligned(16))) char smem[8 * G5_SLOT + 2 * EPI_MAXG * 8 + 2 * 256 * 4];
    double* st_lds = reinterpret_cast<double*>(smem + 8 * G5_SLOT);
    float* bias_lds = reinterpret_cast<float*>(smem + 8 * G5_SLOT + 2 * EPI_MAXG * 8);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;          // wr = the wave's group
    const int wm0 = wr * 128, wn0 = wc * 64;
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int ntn = (d.N + 255) / 256;
    const int ntiles = (int)((M + 255) / 256) * ntn;
    const int64_t a_bs = d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld;
    const int64_t rowpitch = d.a_hs >= 0 ? d.a_hs : (int64_t)d.W * d.a_ld;
    const int lrow = lane >> 3;
    const int chunk = (lane & 7) ^ lrow;       // global 16-B chunk this lane fetches (LDS slot = chunk ^ row&7)
    const char* zero = reinterpret_cast<const char*>(g_zero_page5);

    int tile = blockIdx.x;
    int64_t m0 = 0;
    int n0 = 0;
    // split-K tail (non-persistent launches, GemmDesc::sk_ws): blocks >= sk_full are K pieces of the last partial
    // round's tiles; piece q covers K-tiles [kb0, kb0 + nk) of tile sk_full + q / sk_S and leaves its f32 partial tile
    // in the scratch (gemm5_sk_reduce_kernel adds the pieces in order and runs the epilogue)
    int kb0 = 0, nk = d.Kp / 64, sk_piece = -1;
    // this lane's slot rows: sr = 8 (wave + 8 q) + lrow, q = 0, 1 (gemm4's piece map)
    uint32_t a_base[2][2];
    int a_h0[2][2];
    uint32_t b_off[2];
    const uint32_t a_ld2 = (uint32_t)d.a_ld * 2u;
    auto setup = [&](int t) {
        int id;
        if (!PERSIST && d.sk_ws && t >= d.sk_full) {
            const int q = t - d.sk_full, j = q / d.sk_S, p = q - j * d.sk_S, nkt = d.Kp / 64;
            id = d.sk_full + j;
            kb0 = p * nkt / d.sk_S;
            nk = (p + 1) * nkt / d.sk_S - kb0;
            sk_piece = q;
        } else {
            id = xcd_remap5(t, !PERSIST && d.sk_ws ? d.sk_full : ntiles);
        }
        m0 = (int64_t)(id / ntn) * 256;
        n0 = (id % ntn) * 256;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int sr = 8 * (wave + NW * q) + lrow;
                const int r = (sr >> 6) * 128 + 64 * h + (sr & 63);
                const uint32_t m = (uint32_t)(m0 + r);
                const bool ok = m < (uint32_t)M;
                if constexpr (LIN) {      // rows past M re-read row M - 1 (their outputs are never stored)
                    a_base[h][q] = (ok ? m : (uint32_t)M - 1u) * a_ld2 + 16u * (uint32_t)chunk;
                    if (h == 0) b_off[q] = (uint32_t)(((int64_t)(n0 + (sr >> 5) * 64 + (sr & 31)) * d.Kp + 8 * chunk) * 2);
                    continue;
                }
                const uint32_t mm = ok ? m : 0u;
                const uint32_t t2 = fdiv(mm, d.fd_w);
                const uint32_t w = mm - t2 * (uint32_t)d.W;
                const uint32_t b = fdiv(t2, d.fd_h);
                const uint32_t ho = t2 - b * (uint32_t)d.H_out;
                a_base[h][q] = (uint32_t)(b * a_bs + (int64_t)w * d.a_ld);
                a_h0[h][q] = ok ? (int)ho * d.in_stride + d.in_off : (INT_MIN / 2);
                if (h == 0) b_off[q] = (uint32_t)(((int64_t)(n0 + (sr >> 5) * 64 + (sr & 31)) * d.Kp + 8 * chunk) * 2);
            }
    };
    const uint32_t b_h1 = (uint32_t)(32 * d.Kp * 2);     // slot B1 rows are 32 columns further

    auto issueA = [&](int kt, int h) {
        if (PROBE == 1 && kt > 1) return;
        char* dst = smem + ((kt & 1) * 4 + h) * G5_SLOT;
        if constexpr (LIN) {
            const char* base = (const char*)d.A + (int64_t)(kb0 + kt) * 128;      // wave-uniform
#pragma unroll
            for (int q = 0; q < G5_PIECES; ++q)
                __builtin_amdgcn_global_load_lds((gbl_void*)(base + a_base[h][q]), (lds_void*)(dst + (wave + NW * q) * 1024),
                                                 16, 0, 0);
            return;
        }
        const int k = (kb0 + kt) * 64 + 8 * chunk;
        const bool kok = k < d.K;
        const int tap = k / d.C_in, ci = k - tap * d.C_in;
#pragma unroll
        for (int q = 0; q < G5_PIECES; ++q) {
            const int row = a_h0[h][q] + tap * d.dil;
            const bool ok = kok && row >= 0 && row < d.H_in;
            const char* src = ok ? (const char*)d.A + ((int64_t)a_base[h][q] + (int64_t)row * rowpitch + ci) * 2 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + (wave + NW * q) * 1024), 16, 0, 0);
        }
    };
    auto issueB = [&](int kt, int h) {
        if (PROBE == 1 && kt > 1) return;
        char* dst = smem + ((kt & 1) * 4 + 2 + h) * G5_SLOT;
        const char* wb = (const char*)d.Wp + (int64_t)(kb0 + kt) * 128 + (h ? b_h1 : 0u);
#pragma unroll
        for (int q = 0; q < G5_PIECES; ++q)
            __builtin_amdgcn_global_load_lds((gbl_void*)(wb + b_off[q]), (lds_void*)(dst + (wave + NW * q) * 1024), 16, 0, 0);
    };

    const int fr = lane & 15, g = lane >> 4;
    auto readA = [&](int buf, int mh, bf16v8 (&af)[4][2]) {
        if (PROBE == 2) return;
        const char* base = smem + (buf * 4 + mh) * G5_SLOT + (wr * 64 + fr) * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                af[i][ks] = *reinterpret_cast<const bf16v8*>(base + i * 16 * 128 + ((4 * ks + g) ^ (fr & 7)) * 16);
    };
    auto readB = [&](int buf, int nh, bf16v8 (&bf)[2][2]) {
        if (PROBE == 2) return;
        const char* base = smem + (buf * 4 + 2 + nh) * G5_SLOT + (wc * 32 + fr) * 128;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                bf[j][ks] = *reinterpret_cast<const bf16v8*>(base + j * 16 * 128 + ((4 * ks + g) ^ (fr & 7)) * 16);
    };

    f32x4_t acc[TM][TN];
    auto quad = [&](int mh, int nh, const bf16v8 (&af)[4][2], const bf16v8 (&bf)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (PROBE == 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i][0]), "v"(af[i][1]));
#pragma unroll
            for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(bf[j][0]), "v"(bf[j][1]));
            __builtin_amdgcn_s_setprio(0);
            return;
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[4 * mh + i][2 * nh + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], acc[4 * mh + i][2 * nh + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    // pieces this wave issued in each of its previous load sections (hist[0] = most recent), for the counted waits
    int hist[4] = {0, 0, 0, 0};
    auto load_wait = [&]() { vm_wait_n(hist[0] + hist[1] + hist[2] + hist[3]); };
    auto push = [&](int pieces) {
        hist[3] = hist[2];
        hist[2] = hist[1];
        hist[1] = hist[0];
        hist[0] = pieces;
    };
    // prologue of a tile: K-tile 0 whole, then what the sections of K-tile -1 would have staged: A0(1), B0(1), B1(1)
    // (both groups) and A1(1) (G1; G0 stages its pieces in section 0); afterwards the pieces of K-tile 1 are the
    // in-flight history
    // (nk is per block: a split-K piece covers a K range of its own)
    auto prologue = [&]() {
        issueA(0, 0);
        issueB(0, 0);
        issueB(0, 1);
        issueA(0, 1);
        hist[0] = hist[1] = hist[2] = hist[3] = 0;
        if (nk > 1) {
            issueA(1, 0);
            issueB(1, 0);
            issueB(1, 1);
            if (wr == 1) issueA(1, 1);
            if (wr == 0) { hist[0] = G5_PIECES; hist[1] = 2 * G5_PIECES; }                 // u=-1: p3 B1, p2 A0 + B0
            else { hist[0] = G5_PIECES; hist[1] = G5_PIECES; hist[2] = 2 * G5_PIECES; }   // u=-1: p3 A1, p2 B1, p1 A0 + B0
        }
    };
    if (d.stats && tid < 2 * EPI_MAXG) st_lds[tid] = 0.0;
    setup(tile);
    // the tile's 256 bias values, one per thread of waves 0-3 (0 past N or without bias)
    auto bias_load = [&]() -> float {
        return (tid < 256 && d.bias && n0 + tid < d.N) ? d.bias[n0 + tid] : 0.f;
    };
    int bsel = 0;
    {
        const float bv = bias_load();
        if (tid < 256) bias_lds[tid] = bv;
    }
    prologue();
    load_wait();                                  // K-tile 0 retired (K-tile 1's pieces stay in flight) ...
    section_barrier();                            // ... and published (the bias too)

    bf16v8 af[4][2], bf0[2][2], bf1[2][2];
    if (PROBE == 2) {
        const bf16v8 z = {};
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i][0] = af[i][1] = z;
#pragma unroll
        for (int j = 0; j < 2; ++j) bf0[j][0] = bf0[j][1] = bf1[j][0] = bf1[j][1] = z;
    }
    auto sbar = [&]() {
        if (PROBE != 4) section_barrier();
    };
    for (;;) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (wr == 1) section_barrier();           // the stagger: G1 runs one section behind G0
        // one K-tile u; STEADY (u + 2 < nk): n1 = n2 = true and the load waits are the constant vmcnt(8)
        auto kstep = [&](int u, auto steady) {
            constexpr bool ST = decltype(steady)::value;
            const int buf = u & 1;
            const bool n1 = ST || u + 1 < nk, n2 = ST || u + 2 < nk;
            auto lw = [&]() {
                if constexpr (ST) {
#ifdef ATHD_G5_CHECK
                    if (hist[0] + hist[1] + hist[2] + hist[3] != G5_STEADY_VM && lane == 0)
                        printf("gemm5: steady vmcnt %d != %d\n", hist[0] + hist[1] + hist[2] + hist[3], G5_STEADY_VM);
#endif
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // G5_STEADY_VM
                } else {
                    load_wait();
                }
            };
            // ---- phase 0: (A0, B0)
            lw();
            if (wr == 0 && n1) issueA(u + 1, 1);
            push(wr == 0 && n1 ? G5_PIECES : 0);
            readB(buf, 0, bf0);
            readA(buf, 0, af);
            sbar();
            quad(0, 0, af, bf0);
            sbar();
            // ---- phase 1: (A0, B1)
            lw();
            if (wr == 1 && n2) {
                issueA(u + 2, 0);
                issueB(u + 2, 0);
            }
            push(wr == 1 && n2 ? 2 * G5_PIECES : 0);
            readB(buf, 1, bf1);
            sbar();
            quad(0, 1, af, bf1);
            sbar();
            // ---- phase 2: (A1, B1)
            lw();
            if (n2) {
                if (wr == 0) {
                    issueA(u + 2, 0);
                    issueB(u + 2, 0);
                } else {
                    issueB(u + 2, 1);
                }
            }
            push(n2 ? (wr == 0 ? 2 : 1) * G5_PIECES : 0);
            readA(buf, 1, af);
            sbar();
            quad(1, 1, af, bf1);
            sbar();
            // ---- phase 3: (A1, B0)
            lw();
            if (n2) {
                if (wr == 0) issueB(u + 2, 1);
                else issueA(u + 2, 1);
            }
            push(n2 ? G5_PIECES : 0);
            sbar();
            quad(1, 0, af, bf0);
            sbar();
        };
        int u = 0;
        if constexpr (PROBE == 0) {
            for (; u + 2 < nk; ++u) kstep(u, std::true_type{});
        }
        for (; u < nk; ++u) kstep(u, std::false_type{});
        if (wr == 0) section_barrier();           // G0 waits out G1's last MFMA section: equal barrier counts
        // every slot's last fragment reads have retired (lgkmcnt(0) before the barriers above)
        const int next = tile + (int)gridDim.x;
        const int64_t m0_done = m0;
        const int n0_done = n0;
        float bnext = 0.f;
        if (PERSIST && next < ntiles) {
            setup(next);
            bnext = bias_load();                  // (before the DMA: its wait then needs no glds retired)
            prologue();                           // the next tile's loads overlap this tile's epilogue
        } else {
            vm_wait_n(0);
        }
        if (sk_piece >= 0) {                      // split-K piece: the raw partial tile, row-major [256][256] f32
            float* slab = d.sk_ws + (size_t)sk_piece * 65536;
            const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    *reinterpret_cast<float4*>(slab + (wm0 + 16 * i + fr) * 256 + wn0 + 16 * j + 4 * fg) =
                        make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
            break;
        }
        float4 bias4[TN];
        {
            const float* bl = bias_lds + 256 * bsel + wn0 + 4 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < TN; ++j) bias4[j] = *reinterpret_cast<const float4*>(bl + 16 * j);
        }
        bool fast = false;
        if constexpr ((F & F_RES) != 0 && (F & ~(F_RES | F_STATS | F_RGN)) == 0) {
            if (epi_res_fast_ok(d)) {
                float* gn_lds = nullptr;
                if constexpr ((F & F_RGN) != 0) {
                    // the residual GroupNorm affine of the tile's 256 columns -> staging slot 0 (free: not persistent, so
                    // no next-tile prologue; every wave's last fragment reads retired before the loop's last barrier)
                    static_assert(!PERSIST, "F_RGN stages through a ring slot");
                    gn_lds = reinterpret_cast<float*>(smem);
                    if (tid < 256) {
                        const int n = n0_done + tid < d.N ? n0_done + tid : d.N - 1;
                        gn_lds[tid] = d.res_gn_w[n];
                        gn_lds[256 + tid] = d.res_gn_b[n];
                        gn_lds[512 + tid] = d.res_scale ? d.res_scale[n] : 1.f;
                    }
                    __syncthreads();
                }
                gemm_epilogue_res<TM, TN, F>(d, acc, m0_done, n0_done, wm0, wn0, lane, st_lds, 256, bias4, gn_lds);
                fast = true;
            }
        }
        if constexpr (F == (F_GN | F_GLU | F_RES | F_CBF16) && TN % 2 == 0) {
            if (epi_glures_ok(d)) {
                gemm_epilogue_glures<TM, TN>(d, acc, m0_done, n0_done, wm0, wn0, lane, bias4);
                fast = true;
            }
        }
        if (!fast) gemm_epilogue<TM, TN, F, true>(d, acc, m0_done, n0_done, wm0, wn0, lane, st_lds, 256, bias4);
        if (!PERSIST || next >= ntiles) break;
        tile = next;
        // the epilogue's stores sit behind the staged K-tiles on the VM counter: drain all (K-tile 1 included);
        // stage the next bias; publish K-tile 0 and the bias
        vm_wait_n(0);
        hist[0] = hist[1] = hist[2] = hist[3] = 0;
        bsel ^= 1;
        if (tid < 256) bias_lds[256 * bsel + tid] = bnext;
        section_barrier();
    }
}

// Split-K tail reduce (GemmDesc::sk_ws): block = 4 rows of one tail tile (one per wave), lane = 4 columns.  The S f32
// partial tiles of the tile are loaded together (all S pieces in flight) and added in piece order (deterministic),
// then the residual-stream epilogue of gemm_epilogue_res: out = res + res_scale * (acc + bias), f32, and the per-batch
// {sum, sumsq} statistics.  (Round 6: 16 rows per block with the pieces loaded row after row took 18 us per launch.)
constexpr int SK_MAX_S = 16;
__global__ __launch_bounds__(256) void gemm5_sk_reduce_kernel(const GemmDesc d) {
    __shared__ double red[4][4][2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j = blockIdx.x >> 6, r = (blockIdx.x & 63) * 4 + w;
    const int ntn = (d.N + 255) / 256;
    const int id = d.sk_full + j;
    const int64_t m0 = (int64_t)(id / ntn) * 256;
    const int n0 = (id % ntn) * 256;
    const uint32_t M = (uint32_t)d.nb * d.H_out * d.W;
    const int c = 4 * lane, n = n0 + c;
    const uint32_t m = (uint32_t)(m0 + r);
    const float* slab = d.sk_ws + (size_t)j * d.sk_S * 65536;
    const uint32_t mb = (uint32_t)(m0 + (blockIdx.x & 63) * 4);
    const uint32_t g0 = fdiv(mb < M ? mb : M - 1, d.fd_hw);
    double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};
    if (m < M && n < d.N) {
        float4 part[SK_MAX_S];
#pragma unroll
        for (int p = 0; p < SK_MAX_S; ++p)
            if (p < d.sk_S) part[p] = *reinterpret_cast<const float4*>(slab + (size_t)p * 65536 + r * 256 + c);
        const int64_t off = (int64_t)m * d.ldo + d.col_off + n;
        const float4 rc = *reinterpret_cast<const float4*>((const float*)d.res + off);
        const float4 bias = d.bias ? *reinterpret_cast<const float4*>(d.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 sc = d.res_scale ? *reinterpret_cast<const float4*>(d.res_scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
        float4 a = part[0];
#pragma unroll
        for (int p = 1; p < SK_MAX_S; ++p)
            if (p < d.sk_S) { a.x += part[p].x; a.y += part[p].y; a.z += part[p].z; a.w += part[p].w; }
        const float4 o = make_float4(rc.x + sc.x * (a.x + bias.x), rc.y + sc.y * (a.y + bias.y), rc.z + sc.z * (a.z + bias.z),
                                     rc.w + sc.w * (a.w + bias.w));
        *reinterpret_cast<float4*>((float*)d.C + off) = o;
        const int gi = fdiv(m, d.fd_hw) != g0 ? 1 : 0;     // 4 rows span at most two batches (H_out * W >= 4)
        s1[gi] = (double)((o.x + o.y) + (o.z + o.w));
        s2[gi] = (double)((o.x * o.x + o.y * o.y) + (o.z * o.z + o.w * o.w));
    }
    if (!d.stats) return;
#pragma unroll
    for (int gi = 0; gi < 2; ++gi) {
        const double t1 = wave_sum_d(s1[gi]), t2 = wave_sum_d(s2[gi]);
        if (lane == 0) { red[w][gi][0] = t1; red[w][gi][1] = t2; }
    }
    __syncthreads();
    if (tid < 4) {
        const int gi = tid >> 1, q = tid & 1;
        const double v = (red[0][gi][q] + red[1][gi][q]) + (red[2][gi][q] + red[3][gi][q]);
        if (v != 0.0) atomicAdd(&d.stats[2 * (g0 + gi) + q], v);
    }
}

bool gemm5_supported(const GemmDesc& d) {
    const int64_t a_elems = (d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld) * d.nb;
    // N % 64 == 0: the packed weights hold roundup(N, 256) rows (ctx.h up_gemm), the epilogue skips columns >= N
    return d.a_bf16 && !d.a_norm && d.C_in % 8 == 0 && d.a_ld % 8 == 0 && d.a_cs == 1 && d.Kp % 64 == 0 &&
           d.N % 64 == 0 && (int64_t)(d.N + 255) * d.Kp * 2 < (1LL << 31) && a_elems < (1LL << 31) &&
           d.col_split % 4 == 0 && (d.act != ACT_GLU || d.N % 32 == 0);
}

template <unsigned F, int PROBE = 0, bool LIN = false>
static void launch5f(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int64_t tiles = ((M + 255) / 256) * ((d.N + 255) / 256);
    int64_t grid = tiles;
    if constexpr (g5_persist(F)) {   // persistent: the resident blocks (one per CU), a multiple of 8
        static int per_cu = 0;   // a property of the kernel; the CU count is the current device's
        if (per_cu == 0) {
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm5_kernel<F, PROBE, LIN>, 512, 0);
            if (per_cu <= 0) per_cu = -1;
        }
        const int resident = per_cu > 0 ? per_cu * device_cus() / 8 * 8 : -1;
        if (resident >= 8 && resident < tiles) grid = resident;
    }
    GemmDesc e = with_fastdiv(d);
    int sk_tail = 0;
    if constexpr (!g5_persist(F) && LIN && (F == (F_RES | F_STATS) || F == F_RES)) {
        // split-K tail: a grid of `tiles` one-tile blocks at one block per CU runs ceil(tiles / R) rounds; the last
        // round's `tail` tiles (e.g. linear2: 1036 = 4 x 256 + 12) leave the other CUs idle for a whole tile time.
        // Those tiles are cut into S K pieces each (>= 4 K-tiles), computed as extra blocks of the same launch, and
        // added up by gemm5_sk_reduce_kernel, which also runs their epilogue.
        static int per_cu = 0;
        if (per_cu == 0) {
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm5_kernel<F, PROBE, LIN>, 512, 0);
            if (per_cu <= 0) per_cu = -1;
        }
        const int64_t R = per_cu > 0 ? (int64_t)per_cu * device_cus() : 0;
        const int nkt = d.Kp / 64;
        const int64_t tail = R > 0 ? tiles % R : 0;
        if (d.sk_ws && epi_res_fast_ok(d) && tiles > R && tail > 0 && 2 * tail <= R && nkt >= 8) {
            int S = (int)std::min<int64_t>(std::min<int64_t>(R / tail, nkt / 4), SK_MAX_S);
            S = std::min<int64_t>(S, SK_MAX_PIECES / tail);
            if (S >= 2) {
                e.sk_full = (int)(tiles - tail);
                e.sk_S = S;
                grid = e.sk_full + tail * S;
                sk_tail = (int)tail;
            }
        }
    }
    if (!sk_tail) e.sk_ws = nullptr;
    {
        KScope ks(s);
        if (ks.on()) {
            double fl, by;
            gemm_work(d, 1, fl, by);
            ks.begin(klabel("gemm5_kernel<%u,%d,%s>", F, PROBE, LIN ? "true" : "false"), fl, by);
        }
        hipLaunchKernelGGL((gemm5_kernel<F, PROBE, LIN>), dim3((unsigned)grid), dim3(512), 0, s, e);
    }
    if (sk_tail) {
        KScope ks(s);
        if (ks.on()) ks.begin("gemm5_sk_reduce_kernel", 0.0, (double)sk_tail * 65536 * 4 * (e.sk_S + 2));
        hipLaunchKernelGGL(gemm5_sk_reduce_kernel, dim3((unsigned)sk_tail * 64), dim3(256), 0, s, e);
    }
}

// dense single-tap rows: the LIN fast path of gemm5_kernel applies
static bool gemm5_lin(const GemmDesc& d) {
    return d.ntaps == 1 && d.in_stride == 1 && d.in_off == 0 && d.H_out == d.H_in && d.a_hs < 0 &&
           (d.a_bs < 0 || d.a_bs == (int64_t)d.H_in * d.W * d.a_ld) && d.C_in == d.K && d.K == d.Kp &&
           d.a_cs == 1 && !d.k_blk && (int64_t)d.nb * d.H_in * d.W * d.a_ld * 2 < (1LL << 32);
}

#ifndef ATHD_G5_LIN
#define ATHD_G5_LIN 1       // (0: every launch takes the general implicit-GEMM addressing; kbench A/B builds)
#endif

int gemm5_launch(const GemmDesc& d, hipStream_t s) {
    const bool lin = ATHD_G5_LIN && gemm5_lin(d);
    switch (epi_flags(d)) {
#define ATHD_CASE(FL) \
    case (FL): lin ? launch5f<(FL), 0, true>(d, s) : launch5f<(FL)>(d, s); break;
        ATHD_EPI_LIST(ATHD_CASE)
#undef ATHD_CASE
        default: launch5f<F_ALL>(d, s); break;
    }
    return (int)hipGetLastError();
}

#ifdef ATHD_KBENCH
int gemm5_probe_launch(const GemmDesc& d, hipStream_t s, int probe) {
    if (epi_flags(d) != F_CBF16) return -1;
    if (probe == 1) launch5f<F_CBF16, 1>(d, s);
    else if (probe == 2) launch5f<F_CBF16, 2>(d, s);
    else if (probe == 3) launch5f<F_CBF16, 3>(d, s);
    else if (probe == 4) launch5f<F_CBF16, 4>(d, s);
    else return -1;
    return (int)hipGetLastError();
}
#endif

}  // namespace athd
