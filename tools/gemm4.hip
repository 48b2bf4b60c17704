// GEMM v4 (bf16 MFMA, gfx950) for the wide layers (N a multiple of 256): 256 x 256 x 64 tiles, 8 waves as 2 (M) x
// 4 (N), each wave 128 x 64 outputs = 8 x 4 accumulator tiles of v_mfma_f32_16x16x32_bf16.
//
// Staging (cdna_hip_programming.md §5 "Pipelining across barriers"): two K-tile buffers of four 16 KB half-tile
// slots, filled by global_load_lds_dwordx4 (lane-linear LDS image, XOR swizzle on the source chunk as in
// gemm2/gemm3):
//   A0 = tile rows {0..63, 128..191}, A1 = rows {64..127, 192..255}   (slot row sr <-> (sr/64)*128 + 64h + sr%64)
//   B0 = tile cols {64w + 0..31},     B1 = cols {64w + 32..63}        (slot row sr <-> (sr/32)*64 + 32h + sr%32)
// so that a wave's rows 0..63 / 64..127 read exactly slot A0 / A1.  A K-tile is two phases (A0 against both B
// halves, then A1): each phase starts with [counted vmcnt] + s_barrier, which both publishes the slots the phase
// reads (their LDS-DMA retired by each issuing wave's vmcnt before it) and retires the previous phase's reads, so
// the slots read there can be restaged right after it.  About 1.5 K-tiles of loads stay in flight across every
// barrier (a __syncthreads() would drain them: it waits vmcnt(0)).  Register budget (2 waves per SIMD): 128
// accumulators + 64 fragment registers + compact 32-bit addressing, no spills.
// Same descriptor, implicit-conv A addressing and epilogue (C^T tiles, gemm_epi.h) as the other GEMM kernels.
#include "../audio-to-sheet-music_amd/csrc/common.h"
#include "../audio-to-sheet-music_amd/csrc/prof.h"
#include "../audio-to-sheet-music_amd/csrc/gemm.h"
#ifdef ATHD_G4_STAMP
namespace athd {
__device__ uint64_t* g4_stamp = nullptr;
constexpr int G4_NSTAMP = 24;
}
#define ATHD_EPI_MARK(i)                                                                                       \
    do {                                                                                                       \
        if (athd::g4_stamp && threadIdx.x == 0)                                                                \
            athd::g4_stamp[(int64_t)blockIdx.x * athd::G4_NSTAMP + (i)] = __builtin_amdgcn_s_memtime();        \
    } while (0)
#endif
#include "../audio-to-sheet-music_amd/csrc/gemm_epi.h"

#include <climits>
#include <cstdlib>

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
// ATHD_G4_STAMP (tools/kbench build only): wave 0 lane 0 of each block records s_memtime at the phase points
// (kernel start, prologue issued, phase 0 of K-tiles 0, 1 and the last, epilogue start / end) into g4_stamp.

// ATHD_G4_PRIO (tools/kbench build only, A/B measurement): s_setprio(1) around each phase's MFMA cluster
// (cdna_hip_programming.md T5: keeps hipcc from moving the MFMAs across the raw s_barriers)
#ifdef ATHD_G4_PRIO
#define G4_PRIO(x) __builtin_amdgcn_s_setprio(x)
#else
#define G4_PRIO(x)
#endif

template <unsigned F>
__global__ __launch_bounds__(512) void gemm4_kernel(const GemmDesc d) {
    constexpr int TM = 8, TN = 4;
    constexpr int NW = 8;
    __shared__ __attribute__((aligned(16))) char smem[8 * G4_SLOT + 2 * EPI_MAXG * 8];
    double* st_lds = reinterpret_cast<double*>(smem + 8 * G4_SLOT);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int wm0 = wr * 128, wn0 = wc * 64;
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int ntn = (d.N + 255) / 256;
#ifdef ATHD_G4_STAMP
    uint64_t* stamp = g4_stamp && tid == 0 ? g4_stamp + (int64_t)blockIdx.x * G4_NSTAMP : nullptr;
    int nst = 0;
    auto mark = [&]() {
        if (stamp && nst < G4_NSTAMP) stamp[nst] = __builtin_amdgcn_s_memtime();
        ++nst;
    };
#else
    auto mark = [&]() {};
#endif
    mark();
    // Tiles: XCD-aware order (T1): the N tiles of one M tile are consecutive ids on one XCD, sharing its A rows in L2.
    // PERSIST (epilogues without residual or statistics): the launch sizes the grid to the resident blocks (a
    // multiple of 8, so tiles t, t + gridDim.x, ... of a block stay on its XCD) and each block walks its tiles, staging
    // the next tile's first 1.5 K-tiles BEFORE this tile's epilogue so their load latency hides under the epilogue's
    // VALU work and stores (gemm3's tile loop).  The residual / statistics epilogues keep one tile per block: around
    // them the loop spills.
    constexpr bool PERSIST = (F & (F_RES | F_STATS)) == 0;
    const int ntiles = (int)((M + 255) / 256) * ntn;
    const int64_t a_bs = d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld;
    const int64_t rowpitch = d.a_hs >= 0 ? d.a_hs : (int64_t)d.W * d.a_ld;
    const int lrow = lane >> 3;
    const int chunk = (lane & 7) ^ lrow;       // global 16-B chunk this lane fetches (LDS slot = chunk ^ row&7)
    const char* zero = reinterpret_cast<const char*>(g_zero_page4);

    // this lane's slot rows: sr = 8 (wave + 8 q) + lrow, q = 0, 1 (both slot halves h use the same sr).
    // 32-bit element offsets (gemm4_supported: A < 2^31 elements; the weights hold whole 256-row tiles); a row past M
    // gets a_h0 = INT_MIN / 2, which fails the row >= 0 test for every tap.
    int tile = blockIdx.x;
    int64_t m0 = 0;
    int n0 = 0;
    uint32_t a_base[2][2];
    int a_h0[2][2];
    uint32_t b_off[2];
    auto setup = [&](int t) {
        const int id = xcd_remap4(t, ntiles);
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
    const int nk = d.Kp / 64;

    auto issueA = [&](int kt, int h) {
        char* dst = smem + ((kt & 1) * 4 + h) * G4_SLOT;
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
        char* dst = smem + ((kt & 1) * 4 + 2 + h) * G4_SLOT;
        const char* wb = (const char*)d.Wp + (int64_t)kt * 128 + (h ? b_h1 : 0u);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            __builtin_amdgcn_global_load_lds((gbl_void*)(wb + b_off[q]), (lds_void*)(dst + (wave + NW * q) * 1024), 16, 0, 0);
    };
    // prologue of a tile: A0 B0 B1 (0), A1 (0), A0 B0 B1 (1)
    auto prologue = [&]() {
        issueA(0, 0);
        issueB(0, 0);
        issueB(0, 1);
        issueA(0, 1);
        if (nk > 1) {
            issueA(1, 0);
            issueB(1, 0);
            issueB(1, 1);
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
    setup(tile);
    float4 bias4[TN];                             // loaded now: retired long before the epilogue needs it
    load_bias4<TN>(d, n0, wn0, lane, bias4);
    // Desynchronise the first wave of workgroups (one per CU): with equal tiles everywhere every CU would reach its
    // epilogue at the same moment, and the C stores of all CUs share the HBM write bandwidth (~7 B/clk/CU when all
    // store at once) while the matrix cores idle.  Offsetting the CUs by quarter tiles lets one CU's store burst
    // overlap the others' K-loops; later workgroups inherit the offsets.
    if (blockIdx.x < 256) {
        const int q = (int)(blockIdx.x >> 3) & 3;
        const int n = q * (nk + 5) / 8;
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
    }

    // Two phases per K-tile (2 glds per slot and wave):
    //   phase A(t): publish A0, B0, B1 (t); restage A1 <- t+1 (its last reads were phase B(t-1)); read A0, B0, B1;
    //               MFMA (A0, B0), (A0, B1)
    //   phase B(t): publish A1(t); restage A0, B0, B1 <- t+2 (last read in phase A(t)); read A1; MFMA (A1, B1),
    //               (A1, B0)
    // Issue order: ... A0B0B1(t) | A1(t) | A0B0B1(t+1) | A1(t+1) | ...  (each load gets ~1.5 K-tiles to land)
    prologue();
    mark();
    for (;;) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        bf16v8 af[4][2], bf0[2][2], bf1[2][2];
        for (int t = 0; t < nk; ++t) {
            const int buf = t & 1;
            const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
            // phase A: after A0B0B1(t): A1(t) [2] + A0B0B1(t+1) [6]
            if (has1) vm_wait<8>();
            else vm_wait<2>();
            phase_barrier();
            if (t < 2 || t == nk - 1) mark();
            if (has1) issueA(t + 1, 1);
            readA(buf, 0, af);
            readB(buf, 0, bf0);
            readB(buf, 1, bf1);
            G4_PRIO(1);
            quad(0, 0, af, bf0);
            quad(0, 1, af, bf1);
            G4_PRIO(0);
            // phase B: after A1(t): A0B0B1(t+1) [6] + A1(t+1) [2]
            if (has1) vm_wait<8>();
            else vm_wait<0>();
            phase_barrier();
            if (has2) {
                issueA(t + 2, 0);
                issueB(t + 2, 0);
                issueB(t + 2, 1);
            }
            readA(buf, 1, af);
            G4_PRIO(1);
            quad(1, 1, af, bf1);
            quad(1, 0, af, bf0);
            G4_PRIO(0);
        }
        mark();
        const int next = tile + (int)gridDim.x;
        const int64_t m0_done = m0;
        const int n0_done = n0;
        if (PERSIST && next < ntiles) {
            phase_barrier();                      // every wave's fragment reads of the last K-tile retired
            setup(next);
            prologue();
        }
        // consume the bias registers once, unconditionally: the compiler places their (now free) vmcnt wait here
        // instead of before every branch-guarded use
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bias4[j].x), "v"(bias4[j].y), "v"(bias4[j].z), "v"(bias4[j].w));
        bool fast = false;
        if constexpr ((F & F_RES) != 0 && (F & ~(F_RES | F_STATS)) == 0) {
            if (epi_res_fast_ok(d)) {
                gemm_epilogue_res<TM, TN, F>(d, acc, m0_done, n0_done, wm0, wn0, lane, st_lds, 256, bias4);
                fast = true;
            }
        }
        if (!fast) gemm_epilogue<TM, TN, F, true>(d, acc, m0_done, n0_done, wm0, wn0, lane, st_lds, 256, bias4);
        if (!PERSIST || next >= ntiles) break;
        tile = next;
        // the epilogue's stores sit behind the staged K-tiles on the VM counter: drain all, then the next tile's bias
        vm_wait<0>();
        load_bias4<TN>(d, n0, wn0, lane, bias4);
    }
#ifdef ATHD_G4_STAMP
    if (stamp) {
        mark();                                  // epilogue issued
        __builtin_amdgcn_s_waitcnt(0);
        mark();                                  // its stores retired
        stamp[G4_NSTAMP - 3] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: CU / SH / SE
        stamp[G4_NSTAMP - 2] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
        stamp[G4_NSTAMP - 1] = nst;
    }
#endif
}

bool gemm4_supported(const GemmDesc& d) {
    const int64_t a_elems = (d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld) * d.nb;
    // N % 64 == 0: the packed weights hold roundup(N, 256) rows (ctx.h up_gemm), the epilogue skips columns >= N
    return d.a_bf16 && !d.a_norm && d.C_in % 8 == 0 && d.a_ld % 8 == 0 && d.a_cs == 1 && d.Kp % 64 == 0 &&
           d.N % 64 == 0 && (int64_t)(d.N + 255) * d.Kp * 2 < (1LL << 31) && a_elems < (1LL << 31) &&
           d.col_split % 4 == 0 && (d.act != ACT_GLU || d.N % 32 == 0);
}

template <unsigned F>
static void launch4f(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int64_t tiles = ((M + 255) / 256) * ((d.N + 255) / 256);
    int64_t grid = tiles;
    if constexpr ((F & (F_RES | F_STATS)) == 0) {   // persistent: the resident blocks (one per CU), a multiple of 8
        static int resident = 0;
        if (resident == 0) {
            int per_cu = 0, cus = 0, dev = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm4_kernel<F>, 512, 0);
            resident = per_cu > 0 && cus > 0 ? per_cu * cus / 8 * 8 : -1;
        }
        if (resident >= 8 && resident < tiles) grid = resident;
    }
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin(klabel("gemm4_kernel<%u>", F), fl, by);
    }
    hipLaunchKernelGGL((gemm4_kernel<F>), dim3((unsigned)grid), dim3(512), 0, s, with_fastdiv(d));
}

#ifdef ATHD_G4_STAMP
extern "C" int athd_g4_stamp_set(uint64_t* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g4_stamp), &p, sizeof(p));
}
#endif

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
