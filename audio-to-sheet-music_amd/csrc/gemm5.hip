// GEMM v5 (bf16 MFMA, gfx950): gemm4's 256 x 256 x 64 tile, slots and epilogues with a staggered two-group K-loop
// (cdna_hip_programming.md §5 "The 256² 8-phase template"; MI355X_MICROARCH.md §Two waves per SIMD).
//
// The 8 waves are two groups of 4, G0 = waves 0-3 (tile rows 0-127) and G1 = waves 4-7 (rows 128-255): a SIMD holds
// one wave of each.  A K-tile is 4 phases, one 64 x 32 accumulator quadrant each (16 v_mfma_f32_16x16x32_bf16):
//   p0 (A0, B0)   p1 (A0, B1)   p2 (A1, B1)   p3 (A1, B0)        fragment reads: p0 A0 + B0, p1 B1, p2 A1, p3 none
// and a group spends a phase in two SECTIONS separated by workgroup barriers: a load section (its fragment reads, one
// half-tile of LDS-DMA staging) and an MFMA section (s_waitcnt lgkmcnt(0), s_setprio 1, the 16 MFMAs).  G1 runs one
// section behind G0 (one extra barrier before its first section), so in every section one group's MFMAs share each
// SIMD with the other group's LDS reads and DMA issue: matrix beside memory.  gemm4 (both waves of a SIMD read, then
// both multiply) issues MFMAs ~53 % of its K-loop cycles.
//
// Sections s = 0..7 of K-tile u (G0 loads in even s, G1 in odd s); the half-tile each group stages (2 pieces of 1 KB
// per wave, gemm4's piece -> wave map, so a half-tile is complete after one G0 and one G1 section):
//   s0 G0: B1(u+1)  s1 G1: A1(u+1)  s2 G0: A1(u+1)  s3 G1: A0(u+2)  s4 G0: A0(u+2)  s5 G1: B0(u+2)  s6 G0: B0(u+2)
//   s7 G1: B1(u+2)
// WAR: each slot is restaged >= 2 sections after its last fragment read (those reads retire at the reader's next
// lgkmcnt(0), one section later, before a barrier).  RAW: at each load section a wave waits until only the pieces of
// its previous 3 load sections are in flight (counted vmcnt), so a piece issued in section x is retired in section
// x + 8 and published by that section's closing barrier; every slot is first read >= 10 sections after its pieces
// were issued.
#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

#include <climits>

namespace athd {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

constexpr int G5_SLOT = 16384;     // one half-tile slot: 128 rows x 64 bf16

ATHD_DEV void vm_wait_n(int n) {   // n = 0, 2, 4, 6 (wave-uniform)
    if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

ATHD_DEV void section_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

ATHD_DEV int xcd_remap5(int i, int n) {
    const int q = n / 8, r = n % 8, x = i % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
}

}  // namespace

__device__ __attribute__((aligned(64))) uint4 g_zero_page5[4];

template <unsigned F>
__global__ __launch_bounds__(512) void gemm5_kernel(const GemmDesc d) {
    constexpr int TM = 8, TN = 4;
    constexpr int NW = 8;
    __shared__ __attribute__((aligned(16))) char smem[8 * G5_SLOT + 2 * EPI_MAXG * 8];
    double* st_lds = reinterpret_cast<double*>(smem + 8 * G5_SLOT);

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

    const int id = xcd_remap5(blockIdx.x, ntiles);
    const int64_t m0 = (int64_t)(id / ntn) * 256;
    const int n0 = (id % ntn) * 256;
    // this lane's slot rows: sr = 8 (wave + 8 q) + lrow, q = 0, 1 (gemm4's piece map)
    uint32_t a_base[2][2];
    int a_h0[2][2];
    uint32_t b_off[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int sr = 8 * (wave + NW * q) + lrow;
            const int r = (sr >> 6) * 128 + 64 * h + (sr & 63);
            const uint32_t m = (uint32_t)(m0 + r);
            const bool ok = m < (uint32_t)M;
            const uint32_t mm = ok ? m : 0u;
            const uint32_t t2 = fdiv(mm, d.fd_w);
            const uint32_t w = mm - t2 * (uint32_t)d.W;
            const uint32_t b = fdiv(t2, d.fd_h);
            const uint32_t ho = t2 - b * (uint32_t)d.H_out;
            a_base[h][q] = (uint32_t)(b * a_bs + (int64_t)w * d.a_ld);
            a_h0[h][q] = ok ? (int)ho * d.in_stride + d.in_off : (INT_MIN / 2);
            if (h == 0) b_off[q] = (uint32_t)(((int64_t)(n0 + (sr >> 5) * 64 + (sr & 31)) * d.Kp + 8 * chunk) * 2);
        }
    const uint32_t b_h1 = (uint32_t)(32 * d.Kp * 2);     // slot B1 rows are 32 columns further
    const int nk = d.Kp / 64;

    auto issueA = [&](int kt, int h) {
        char* dst = smem + ((kt & 1) * 4 + h) * G5_SLOT;
        const int k = kt * 64 + 8 * chunk;
        const bool kok = k < d.K;
        const int tap = k / d.C_in, ci = k - tap * d.C_in;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int row = a_h0[h][q] + tap * d.dil;
            const bool ok = kok && row >= 0 && row < d.H_in;
            const char* src = ok ? (const char*)d.A + ((int64_t)a_base[h][q] + (int64_t)row * rowpitch + ci) * 2 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + (wave + NW * q) * 1024), 16, 0, 0);
        }
    };
    auto issueB = [&](int kt, int h) {
        char* dst = smem + ((kt & 1) * 4 + 2 + h) * G5_SLOT;
        const char* wb = (const char*)d.Wp + (int64_t)kt * 128 + (h ? b_h1 : 0u);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            __builtin_amdgcn_global_load_lds((gbl_void*)(wb + b_off[q]), (lds_void*)(dst + (wave + NW * q) * 1024), 16, 0, 0);
    };

    const int fr = lane & 15, g = lane >> 4;
    auto readA = [&](int buf, int mh, bf16v8 (&af)[4][2]) {
        const char* base = smem + (buf * 4 + mh) * G5_SLOT + (wr * 64 + fr) * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                af[i][ks] = *reinterpret_cast<const bf16v8*>(base + i * 16 * 128 + ((4 * ks + g) ^ (fr & 7)) * 16);
    };
    auto readB = [&](int buf, int nh, bf16v8 (&bf)[2][2]) {
        const char* base = smem + (buf * 4 + 2 + nh) * G5_SLOT + (wc * 32 + fr) * 128;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                bf[j][ks] = *reinterpret_cast<const bf16v8*>(base + j * 16 * 128 + ((4 * ks + g) ^ (fr & 7)) * 16);
    };

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    auto quad = [&](int mh, int nh, const bf16v8 (&af)[4][2], const bf16v8 (&bf)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
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
    if (d.stats && tid < 2 * EPI_MAXG) st_lds[tid] = 0.0;
    float4 bias4[TN];                             // loaded now: retired long before the epilogue needs it
    load_bias4<TN>(d, n0, wn0, lane, bias4);
    // Desynchronise the first wave of workgroups (one per CU) as gemm4 does: their epilogue store bursts then
    // overlap other CUs' K-loops
    if (blockIdx.x < 256) {
        const int q = (int)(blockIdx.x >> 3) & 3;
        const int n = q * (nk + 5) / 8;
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
    }

    // prologue: K-tile 0 whole, then what the steady state would have staged in the sections of K-tile -1:
    // A0(1), B0(1) (both groups), B1(1) (G1 only; G0 stages its pieces in section 0)
    issueA(0, 0);
    issueB(0, 0);
    issueB(0, 1);
    issueA(0, 1);
    const bool two = nk > 1;
    if (two) {
        issueA(1, 0);
        issueB(1, 0);
        if (wr == 1) issueB(1, 1);
    }
    // retire K-tile 0 (this wave's pieces of tile 1 stay in flight) and publish it
    if (!two) vm_wait_n(0);
    else if (wr == 0) vm_wait_n(4);
    else vm_wait_n(6);
    section_barrier();
    // issue history of this wave's previous three load sections (for the counted waits); the prologue's tile-1
    // pieces stand for the K-tile -1 sections that would have issued them
    bool h1 = two, h2 = two, h3 = two && wr == 1;
    auto load_wait = [&]() { vm_wait_n(2 * ((int)h1 + (int)h2 + (int)h3)); };
    auto push = [&](bool issued) {
        h3 = h2;
        h2 = h1;
        h1 = issued;
    };
    if (wr == 1) section_barrier();               // the stagger: G1 runs one section behind G0

    bf16v8 af[4][2], bf0[2][2], bf1[2][2];
    for (int u = 0; u < nk; ++u) {
        const int buf = u & 1;
        const bool n1 = u + 1 < nk, n2 = u + 2 < nk;
        // ---- phase 0: (A0, B0)
        load_wait();
        if (wr == 0) {
            if (n1) issueB(u + 1, 1);
            push(n1);
        } else {
            if (n1) issueA(u + 1, 1);
            push(n1);
        }
        readB(buf, 0, bf0);
        readA(buf, 0, af);
        section_barrier();
        quad(0, 0, af, bf0);
        section_barrier();
        // ---- phase 1: (A0, B1)
        load_wait();
        if (wr == 0) {
            if (n1) issueA(u + 1, 1);
            push(n1);
        } else {
            if (n2) issueA(u + 2, 0);
            push(n2);
        }
        readB(buf, 1, bf1);
        section_barrier();
        quad(0, 1, af, bf1);
        section_barrier();
        // ---- phase 2: (A1, B1)
        load_wait();
        if (wr == 0) {
            if (n2) issueA(u + 2, 0);
        } else {
            if (n2) issueB(u + 2, 0);
        }
        push(n2);
        readA(buf, 1, af);
        section_barrier();
        quad(1, 1, af, bf1);
        section_barrier();
        // ---- phase 3: (A1, B0)
        load_wait();
        if (wr == 0) {
            if (n2) issueB(u + 2, 0);
        } else {
            if (n2) issueB(u + 2, 1);
        }
        push(n2);
        section_barrier();
        quad(1, 0, af, bf0);
        section_barrier();
    }
    if (wr == 0) section_barrier();               // G0 waits out G1's last MFMA section: equal barrier counts
    vm_wait_n(0);

    // consume the bias registers once, unconditionally (gemm4)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bias4[j].x), "v"(bias4[j].y), "v"(bias4[j].z), "v"(bias4[j].w));
    bool fast = false;
    if constexpr ((F & F_RES) != 0 && (F & ~(F_RES | F_STATS)) == 0) {
        if (epi_res_fast_ok(d)) {
            gemm_epilogue_res<TM, TN, F>(d, acc, m0, n0, wm0, wn0, lane, st_lds, 256, bias4);
            fast = true;
        }
    }
    if (!fast) gemm_epilogue<TM, TN, F, true>(d, acc, m0, n0, wm0, wn0, lane, st_lds, 256, bias4);
}

template <unsigned F>
static void launch5f(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int64_t tiles = ((M + 255) / 256) * ((d.N + 255) / 256);
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin(klabel("gemm5_kernel<%u>", F), fl, by);
    }
    hipLaunchKernelGGL((gemm5_kernel<F>), dim3((unsigned)tiles), dim3(512), 0, s, with_fastdiv(d));
}

int gemm5_launch(const GemmDesc& d, hipStream_t s) {
    switch (epi_flags(d)) {
#define ATHD_CASE(FL) \
    case (FL): launch5f<(FL)>(d, s); break;
        ATHD_EPI_LIST(ATHD_CASE)
#undef ATHD_CASE
        default: launch5f<F_ALL>(d, s); break;
    }
    return (int)hipGetLastError();
}

}  // namespace athd
