// GEMM v4 (bf16 MFMA, gfx950) for the wide layers (N a multiple of 256 or close to it): 256 x 256 x 64 tiles,
// 8 waves as 2 (M) x 4 (N), each wave 128 x 64 outputs = 8 x 4 accumulator tiles of v_mfma_f32_16x16x32_bf16.
//
// Staging (cdna_hip_programming.md §5 "Pipelining across barriers", "The 256² 8-phase template"): two K-tile
// buffers of four 16 KB half-tile slots, filled by global_load_lds_dwordx4 (lane-linear LDS image, XOR swizzle
// on the source chunk as in gemm2/gemm3):
//   A0 = tile rows {0..63, 128..191}, A1 = rows {64..127, 192..255}   (slot row sr <-> (sr/64)*128 + 64h + sr%64)
//   B0 = tile cols {64w + 0..31},     B1 = cols {64w + 32..63}        (slot row sr <-> (sr/32)*64 + 32h + sr%32)
// so that wave quadrant (mh, nh) of a K-tile reads exactly slots A_mh and B_nh.  A K-tile is computed in four
// phases, quadrant order (0,0) (0,1) (1,1) (1,0); the B0 fragments stay in registers from the first phase to the
// last, so each slot is read once, in one phase:
//   phase 0: read A0, B0        | phase 1: read B1, restage A0, B0 of tile t+2
//   phase 2: read A1, restage B1 | phase 3: restage A1
// Every phase starts with [counted vmcnt] + s_barrier: the barrier both publishes the slots the phase reads
// (their LDS-DMA retired by each issuing wave's vmcnt before it) and retires the previous phase's reads before a
// slot is restaged.  In steady state two whole K-tiles of loads are in flight (12 glds per wave), so the barrier
// never drains the load queue (a __syncthreads() would: it waits vmcnt(0)).
// Same descriptor, implicit-conv A addressing and epilogue (C^T tiles, gemm_epi.h) as the other GEMM kernels.
#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

namespace athd {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

constexpr int G4_SLOT = 16384;     // one half-tile slot: 128 rows x 64 bf16

template <int N>
ATHD_DEV void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// all of this wave's LDS reads retired, then the workgroup barrier (no vmcnt: LDS-DMA stays in flight)
ATHD_DEV void phase_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

ATHD_DEV int xcd_remap4(int i, int n) {
    const int q = n / 8, r = n % 8, x = i % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
}

}  // namespace

__device__ __attribute__((aligned(64))) uint4 g_zero_page4[4];

template <unsigned F>
__global__ __launch_bounds__(512) void gemm4_kernel(const GemmDesc d) {
    constexpr int TM = 8, TN = 4;
    __shared__ __attribute__((aligned(16))) char smem[8 * G4_SLOT + 2 * EPI_MAXG * 8];
    double* st_lds = reinterpret_cast<double*>(smem + 8 * G4_SLOT);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int wm0 = wr * 128, wn0 = wc * 64;
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int ntn = (d.N + 255) / 256;
    // XCD-aware order (T1): the N tiles of one M tile are consecutive ids on one XCD, sharing its A rows in L2
    const int id = xcd_remap4(blockIdx.x, gridDim.x);
    const int64_t m0 = (int64_t)(id / ntn) * 256;
    const int n0 = (id % ntn) * 256;
    const int64_t a_bs = d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld;
    const int64_t rowpitch = d.a_hs >= 0 ? d.a_hs : (int64_t)d.W * d.a_ld;
    const int lrow = lane >> 3;
    const int chunk = (lane & 7) ^ lrow;       // global 16-B chunk this lane fetches (LDS slot = chunk ^ row&7)
    const char* zero = reinterpret_cast<const char*>(g_zero_page4);

    // this lane's slot rows: sr = 8 (wave + 8 q) + lrow, q = 0, 1 (both slot halves h use the same sr)
    int64_t a_base[2][2];
    int a_h0[2][2];
    bool a_ok[2][2];
    const char* bptr[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int sr = 8 * (wave + 8 * q) + lrow;
            const int r = (sr >> 6) * 128 + 64 * h + (sr & 63);
            const uint32_t m = (uint32_t)(m0 + r);
            a_ok[h][q] = m < (uint32_t)M;
            const uint32_t mm = a_ok[h][q] ? m : 0u;
            const uint32_t w = mm % (uint32_t)d.W;
            const uint32_t t = mm / (uint32_t)d.W;
            const uint32_t ho = t % (uint32_t)d.H_out;
            const uint32_t b = t / (uint32_t)d.H_out;
            a_base[h][q] = (int64_t)b * a_bs + (int64_t)w * d.a_ld;
            a_h0[h][q] = (int)ho * d.in_stride + d.in_off;
            const int c = (sr >> 5) * 64 + 32 * h + (sr & 31);
            const int n = n0 + c;
            bptr[h][q] = n < d.N ? (const char*)d.Wp + ((int64_t)n * d.Kp + 8 * chunk) * 2 : nullptr;
        }
    const int nk = d.Kp / 64;

    auto issueA = [&](int kt, int h) {
        char* dst = smem + ((kt & 1) * 4 + h) * G4_SLOT;
        const int k = kt * 64 + 8 * chunk;
        const bool kok = k < d.K;
        const int tap = k / d.C_in, ci = k - tap * d.C_in;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int row = a_h0[h][q] + tap * d.dil;
            const bool ok = a_ok[h][q] && kok && row >= 0 && row < d.H_in;
            const char* src = ok ? (const char*)d.A + (a_base[h][q] + (int64_t)row * rowpitch + ci) * 2 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + (wave + 8 * q) * 1024), 16, 0, 0);
        }
    };
    auto issueB = [&](int kt, int h) {
        char* dst = smem + ((kt & 1) * 4 + 2 + h) * G4_SLOT;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const char* src = bptr[h][q] ? bptr[h][q] + (int64_t)kt * 128 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + (wave + 8 * q) * 1024), 16, 0, 0);
        }
    };

    const int fr = lane & 15, g = lane >> 4;
    // fragments of slot A_mh: rows wr*64 + 16 i + fr; of slot B_nh: rows wc*32 + 16 j + fr
    auto readA = [&](int buf, int mh, bf16v8 (&af)[4][2]) {
        const char* base = smem + (buf * 4 + mh) * G4_SLOT + (wr * 64 + fr) * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                af[i][ks] = *reinterpret_cast<const bf16v8*>(base + i * 16 * 128 + ((4 * ks + g) ^ (fr & 7)) * 16);
    };
    auto readB = [&](int buf, int nh, bf16v8 (&bf)[2][2]) {
        const char* base = smem + (buf * 4 + 2 + nh) * G4_SLOT + (wc * 32 + fr) * 128;
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
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[4 * mh + i][2 * nh + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], acc[4 * mh + i][2 * nh + j], 0, 0, 0);
    };
    if (d.stats && tid < 2 * EPI_MAXG) st_lds[tid] = 0.0;

    // prologue: tiles 0 and 1 in the steady-state issue order (A0 B0 | B1 | A1)
#pragma unroll
    for (int t = 0; t < 2; ++t)
        if (t < nk) {
            issueA(t, 0);
            issueB(t, 0);
            issueB(t, 1);
            issueA(t, 1);
        }

    bf16v8 af[4][2], bf0[2][2], bf1[2][2];
    for (int t = 0; t < nk; ++t) {
        const int buf = t & 1;
        const bool has_next = t + 1 < nk;       // tile t+1's 8 glds were issued before tile t's phases
        const bool issue2 = t + 2 < nk;         // tile t+2 is restaged during tile t
        // phase 0: A0, B0 of tile t (issued after them: B1, A1 of tile t [4] + tile t+1 [8])
        if (has_next) vm_wait<12>();
        else vm_wait<4>();
        phase_barrier();
        readA(buf, 0, af);
        readB(buf, 0, bf0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        quad(0, 0, af, bf0);
        // phase 1: B1 of tile t (after it: A1 of tile t [2] + tile t+1 [8]); restage A0, B0 with tile t+2
        if (has_next) vm_wait<10>();
        else vm_wait<2>();
        phase_barrier();
        if (issue2) {
            issueA(t + 2, 0);
            issueB(t + 2, 0);
        }
        readB(buf, 1, bf1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        quad(0, 1, af, bf1);
        // phase 2: A1 of tile t (after it: tile t+1 [8] + A0, B0 of tile t+2 [4]); restage B1
        if (issue2) vm_wait<12>();
        else if (has_next) vm_wait<8>();
        else vm_wait<0>();
        phase_barrier();
        if (issue2) issueB(t + 2, 1);
        readA(buf, 1, af);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        quad(1, 1, af, bf1);
        // phase 3: restage A1 (every wave's phase-2 reads retired by the barrier); B0 still in registers
        phase_barrier();
        if (issue2) issueA(t + 2, 1);
        quad(1, 0, af, bf0);
    }
    gemm_epilogue<TM, TN, F, true>(d, acc, m0, n0, wm0, wn0, lane, st_lds, 256);
}

bool gemm4_supported(const GemmDesc& d) {
    return d.a_bf16 && !d.a_norm && d.C_in % 8 == 0 && d.a_ld % 8 == 0 && d.a_cs == 1 && d.Kp % 64 == 0 &&
           d.N >= 256 && d.col_split % 4 == 0 && (d.act != ACT_GLU || d.N % 32 == 0);
}

template <unsigned F>
static void launch4f(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int64_t tiles = ((M + 255) / 256) * ((d.N + 255) / 256);
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin(klabel("gemm4_kernel<%u>", F), fl, by);
    }
    hipLaunchKernelGGL((gemm4_kernel<F>), dim3((unsigned)tiles), dim3(512), 0, s, d);
}

int gemm4_launch(const GemmDesc& d, hipStream_t s) {
    switch (epi_flags(d)) {
#define ATHD_CASE(FL) \
    case (FL): launch4f<(FL)>(d, s); break;
        ATHD_EPI_LIST(ATHD_CASE)
#undef ATHD_CASE
        default: launch4f<F_ALL>(d, s); break;
    }
    return (int)hipGetLastError();
}

}  // namespace athd
