// GEMM v3 (bf16 MFMA, gfx950), for bf16 activations: BM x BN x 64 tiles, WM x WN waves, a STAGES-deep LDS ring
// filled by global_load_lds_dwordx4 with a COUNTED vmcnt and raw s_barrier, so STAGES-2 tiles stay in flight
// across every barrier (a __syncthreads() would drain them: cdna_hip_programming.md §5 "Pipelining across
// barriers").  LDS image and swizzle as in gemm2.hip (per-lane source chunk (L%8)^(L/8), slot = chunk ^ (row&7)).
// Same descriptor and epilogue (C^T tiles) as the other GEMM kernels.
#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

namespace athd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

static __device__ __attribute__((aligned(64))) uint4 g_zero_page3[4];

template <int N>
ATHD_DEV void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// XCD-aware tile order (cdna_hip_programming.md T1): workgroup i runs on XCD i % 8, so hand each XCD a contiguous
// range of M tiles (bijective for any tile count) - neighbouring tiles share input rows (conv taps) in that L2.
ATHD_DEV int xcd_remap(int i, int n) {
    const int q = n / 8, r = n % 8, x = i % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
}

// F_LN epilogue (the text cross-attention's mlp2 + norm_out, ATHTDemucs_v2.py:47-49): BN == N, so a tile holds whole
// output rows.  v = acc + pbias[batch] (+ bias) + residual (batch / res_div, f32), then LayerNorm over the row: the
// row's partial sums over each wave's BN / WN columns meet in LDS (red: [2][BM][WN] floats), mean first, then the
// sum of squared deviations (layernorm_kernel's two-pass form), and the normalised row leaves as bf16.
template <int BM, int BN, int WM, int WN, int TM, int TN>
ATHD_DEV void gemm3_epilogue_ln(const GemmDesc& d, f32x4_t (&acc)[TM][TN], int64_t m0, int wm0, int wn0, int lane,
                                int wcol, float* red, const float4 (&bj)[TN]) {
    const int fr = lane & 15, fg = lane >> 4;
    const uint32_t M = (uint32_t)d.nb * d.H_out * d.W;
    float rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
        const uint32_t mm = m < M ? m : M - 1;
        const uint32_t b = fdiv(mm, d.fd_hw);
        const int64_t inb = (int64_t)(mm - b * (uint32_t)d.H_out * (uint32_t)d.W) * d.ldo;
        const int64_t rbase = (d.res_div > 1 ? (int64_t)(b / d.res_div) * d.res_bs : (int64_t)b * d.H_out * d.W * d.ldo) + inb;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = wn0 + 16 * j + 4 * fg;
            float4 pb = make_float4(0.f, 0.f, 0.f, 0.f);
            if (d.pbias) pb = *reinterpret_cast<const float4*>(d.pbias + (int64_t)b * d.N + n);
            float4 rr = make_float4(0.f, 0.f, 0.f, 0.f);
            if (d.res) rr = *reinterpret_cast<const float4*>((const float*)d.res + rbase + n);
            acc[i][j][0] = rr.x + (acc[i][j][0] + bj[j].x + pb.x);
            acc[i][j][1] = rr.y + (acc[i][j][1] + bj[j].y + pb.y);
            acc[i][j][2] = rr.z + (acc[i][j][2] + bj[j].z + pb.z);
            acc[i][j][3] = rr.w + (acc[i][j][3] + bj[j].w + pb.w);
            s += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
        }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        rs[i] = s;
    }
    if (fg == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) red[(wm0 + 16 * i + fr) * WN + wcol] = rs[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    float mean[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        float t = 0.f;
#pragma unroll
        for (int c = 0; c < WN; ++c) t += red[(wm0 + 16 * i + fr) * WN + c];
        mean[i] = t * (1.f / (float)BN);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float dv = acc[i][j][e] - mean[i];
                q += dv * dv;
            }
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        rs[i] = q;
    }
    float* red2 = red + BM * WN;
    if (fg == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) red2[(wm0 + 16 * i + fr) * WN + wcol] = rs[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
        float t = 0.f;
#pragma unroll
        for (int c = 0; c < WN; ++c) t += red2[(wm0 + 16 * i + fr) * WN + c];
        const float rstd = 1.f / sqrtf(t * (1.f / (float)BN) + 1e-5f);
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = wn0 + 16 * j + 4 * fg;
            const float4 lw = *reinterpret_cast<const float4*>(d.ln_w + n), lb = *reinterpret_cast<const float4*>(d.ln_b + n);
            const float y0 = (acc[i][j][0] - mean[i]) * rstd * lw.x + lb.x;
            const float y1 = (acc[i][j][1] - mean[i]) * rstd * lw.y + lb.y;
            const float y2 = (acc[i][j][2] - mean[i]) * rstd * lw.z + lb.z;
            const float y3 = (acc[i][j][3] - mean[i]) * rstd * lw.w + lb.w;
            *reinterpret_cast<uint2*>((bf16_t*)d.C + (int64_t)m * d.ldo + n) = make_uint2(pack2bf(y0, y1), pack2bf(y2, y3));
        }
    }
}

template <int BM, int BN, int WM, int WN, int STAGES, unsigned F>
__global__ __launch_bounds__(WM * WN * 64) void gemm3_kernel(const GemmDesc d) {
    constexpr int NW = WM * WN;
    constexpr int ROWB = 128;
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
    constexpr int AQ = BM / 8 / NW, BQ = BN / 8 / NW;
    static_assert(AQ * 8 * NW == BM && BQ * 8 * NW == BN, "tile / wave count");
    constexpr int LPT = AQ + BQ;                 // LDS-DMA instructions per wave per tile
    __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE + 2 * EPI_MAXG * 8];
    double* st_lds = reinterpret_cast<double*>(smem + STAGES * STAGE);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm0 = (wave / WN) * (BM / WM), wn0 = (wave % WN) * (BN / WN);
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int ntm = (int)((M + BM - 1) / BM);
    const int n0 = blockIdx.y * BN;
    if ((int)blockIdx.x >= ntm) return;           // (the launch never sizes gridDim.x above ntm)
    const int64_t a_bs = d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld;
    const int64_t rowpitch = d.a_hs >= 0 ? d.a_hs : (int64_t)d.W * d.a_ld;
    const int lrow = lane >> 3;
    const int chunk = (lane & 7) ^ lrow;

    // Tile loop: block x takes M tiles x, x + gridDim.x, ... (one tile when gridDim.x == ntm; persistent when the
    // launch sizes the grid to the resident blocks, gridDim.x % 8 == 0 so every tile of a block maps to its XCD's
    // contiguous range).  The next tile's first STAGES-1 K-tiles are issued BEFORE this tile's epilogue, so their
    // load latency hides under the epilogue's VALU work and stores.
    int tile = blockIdx.x;
    int64_t m0 = 0;
    int64_t a_base[AQ];
    int a_h0[AQ];
    bool a_ok[AQ];
    int k_cur = 0, tap = 0, ci = 0;
    auto setup = [&](int t) {
        m0 = (int64_t)xcd_remap(t, ntm) * BM;
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
            const uint32_t m = (uint32_t)(m0 + 8 * (wave + NW * q) + lrow);
            a_ok[q] = m < (uint32_t)M;
            const uint32_t mm = a_ok[q] ? m : 0u;
            const uint32_t tt = fdiv(mm, d.fd_w);
            const uint32_t w = mm - tt * (uint32_t)d.W;
            const uint32_t bb = fdiv(tt, d.fd_h);
            const uint32_t ho = tt - bb * (uint32_t)d.H_out;
            a_base[q] = (int64_t)bb * a_bs + (int64_t)w * d.a_ld;
            a_h0[q] = (int)ho * d.in_stride + d.in_off;
        }
        k_cur = 8 * chunk;
        tap = k_cur / d.C_in;
        ci = k_cur - tap * d.C_in;
    };
    const char* bptr[BQ];
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
        const int n = n0 + 8 * (wave + NW * q) + lrow;
        bptr[q] = n < d.N ? (const char*)d.Wp + ((int64_t)n * d.Kp + 8 * chunk) * 2 : nullptr;
    }
    const char* zero = reinterpret_cast<const char*>(g_zero_page3);
    const int nk = d.Kp / 64;

    auto issue = [&](int kt, int st) {
        char* sA = smem + st * STAGE;
        char* sB = sA + BM * ROWB;
        const bool kok = k_cur < d.K;
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
            const int row = a_h0[q] + tap * d.dil;
            const bool ok = a_ok[q] && kok && row >= 0 && row < d.H_in;
            const char* src = ok ? (const char*)d.A + (a_base[q] + (int64_t)row * rowpitch + ci) * 2 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sA + (wave + NW * q) * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < BQ; ++q) {
            const char* src = bptr[q] ? bptr[q] + (int64_t)kt * 128 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sB + (wave + NW * q) * 1024), 16, 0, 0);
        }
        k_cur += 64;
        ci += 64;
        while (ci >= d.C_in) { ci -= d.C_in; ++tap; }
    };

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (d.stats && tid < 2 * EPI_MAXG) st_lds[tid] = 0.0;
    float4 bias4[TN];                             // loaded before the main loop (gemm_epi.h: load_bias4)
    load_bias4<TN>(d, n0, wn0, lane, bias4);

    // K sub-steps (32 wide) this wave multiplies: the zero K padding beyond K is skipped everywhere, and with k_blk
    // the residue groups' zero blocks (the wave's BN/WN columns lie in one residue pair; wave-uniform branch)
    int s_lo = 0, s_hi = (d.K + 31) / 32;
    if (d.k_blk > 0) {
        const int ga = (n0 + wn0) / d.col_split, gb = (n0 + wn0 + BN / WN - 1) / d.col_split;
        if (gb < 2) s_hi = min(s_hi, 2 * d.k_blk / 32);
        else if (ga >= 2) s_lo = d.k_blk / 32;
    }
    const int fr = lane & 15, g = lane >> 4;

    // prologue of the first tile: STAGES-1 K-tiles in flight, wait for K-tile 0
    setup(tile);
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) issue(s, s);
    if (nk >= STAGES - 1) wait_vm<(STAGES - 2) * LPT>();
    else wait_vm<0>();
    for (;;) {
        __builtin_amdgcn_s_barrier();
        int cur = 0;
        for (int kt = 0; kt < nk; ++kt) {
            const int nxt = kt + STAGES - 1;
            if (nxt < nk) issue(nxt, nxt % STAGES);
            const char* sA = smem + cur * STAGE;
            const char* sB = sA + BM * ROWB;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                if (2 * kt + ks < s_lo || 2 * kt + ks >= s_hi) continue;
                const int slot = ((4 * ks + g) ^ (fr & 7)) * 16;
                bf16v8 af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16v8*>(sA + (wm0 + 16 * i + fr) * ROWB + slot);
#pragma unroll
                for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16v8*>(sB + (wn0 + 16 * j + fr) * ROWB + slot);
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
            }
            // K-tile kt+1 must have landed before the next iteration; K-tiles issued after it may stay in flight
            if (nxt < nk) wait_vm<(STAGES - 2) * LPT>();
            else wait_vm<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            cur = cur + 1 == STAGES ? 0 : cur + 1;
        }
        // every wave's LDS reads of this tile retired (barrier above): stage the next tile's first K-tiles now
        const int64_t m0_done = m0;
        const int next = tile + (int)gridDim.x;
        if (next < ntm) {
            setup(next);
#pragma unroll
            for (int s = 0; s < STAGES - 1; ++s)
                if (s < nk) issue(s, s);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bias4[j].x), "v"(bias4[j].y), "v"(bias4[j].z), "v"(bias4[j].w));
        if constexpr ((F & F_LN) != 0) {
            // the last ring stage is free here (the next tile's prologue filled stages 0 .. STAGES-2)
            gemm3_epilogue_ln<BM, BN, WM, WN, TM, TN>(d, acc, m0_done, wm0, wn0, lane, wave % WN,
                                                      reinterpret_cast<float*>(smem + (STAGES - 1) * STAGE), bias4);
        } else if constexpr (F == (F_GN | F_GLU | F_RES | F_CBF16) && TN % 2 == 0) {
            if (epi_glures_ok(d)) gemm_epilogue_glures<TM, TN>(d, acc, m0_done, n0, wm0, wn0, lane, bias4);
            else gemm_epilogue<TM, TN, F, true>(d, acc, m0_done, n0, wm0, wn0, lane, st_lds, BM, bias4);
        } else {
            gemm_epilogue<TM, TN, F, true>(d, acc, m0_done, n0, wm0, wn0, lane, st_lds, BM, bias4);
        }
        if (next >= ntm) break;
        tile = next;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // the epilogue's stores sit behind the staged K-tiles on the VM counter: drain all before the barrier
        wait_vm<0>();
    }
}

bool gemm3_supported(const GemmDesc& d) {
    return (d.k_blk == 0 || (d.k_blk % 32 == 0 && d.col_split > 0)) && d.a_bf16 && !d.a_norm && d.C_in % 8 == 0 && d.a_ld % 8 == 0 && d.a_cs == 1 && d.Kp % 64 == 0 && d.N >= 96 && d.col_split % 4 == 0 &&
           (d.act != ACT_GLU || d.N % 32 == 0);
}

// Persistent grid: resident blocks per CU (occupancy API, once per instantiation) x CUs, split over the N tiles,
// rounded down to a multiple of 8 (XCD count) and capped at the M tile count.
template <int BM, int BN, int WM, int WN, int ST, unsigned F>
static unsigned resident_grid_x(int ntm, int ntn) {
    static int per_cu = 0;       // a property of the kernel; the CU count is the current device's
    if (per_cu == 0) {
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm3_kernel<BM, BN, WM, WN, ST, F>, WM * WN * 64, 0);
        if (per_cu <= 0) per_cu = -1;
    }
    const int resident = per_cu > 0 ? per_cu * device_cus() : -1;
    if (resident < 0) return (unsigned)ntm;
    int gx = resident / ntn / 8 * 8;
    if (gx < 8) gx = 8;
    return (unsigned)(gx < ntm ? gx : ntm);
}

template <int BM, int BN, int WM, int WN, int ST, unsigned F>
static void launch3f(const GemmDesc& d, hipStream_t s, bool persist) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int ntm = (int)((M + BM - 1) / BM), ntn = (d.N + BN - 1) / BN;
    dim3 grid(persist ? resident_grid_x<BM, BN, WM, WN, ST, F>(ntm, ntn) : (unsigned)ntm, (unsigned)ntn);
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin(klabel("gemm3_kernel<%d,%d,%d,%d,%d,%u>", BM, BN, WM, WN, ST, F), fl, by);
    }
    hipLaunchKernelGGL((gemm3_kernel<BM, BN, WM, WN, ST, F>), grid, dim3(WM * WN * 64), 0, s, with_fastdiv(d));
}

template <int BM, int BN, int WM, int WN, int ST>
static void launch3(const GemmDesc& d, hipStream_t s, bool persist) {
    switch (epi_flags(d)) {
#define ATHD_CASE(FL) \
    case (FL): launch3f<BM, BN, WM, WN, ST, (FL)>(d, s, persist); return;
        ATHD_EPI_LIST(ATHD_CASE)
#undef ATHD_CASE
        default: launch3f<BM, BN, WM, WN, ST, F_ALL>(d, s, persist); return;
    }
}

// the row-LayerNorm epilogue exists only here (gemm3_ln_launch): BN == N
static constexpr unsigned F_TEXT_LN = F_RES | F_PB | F_LN | F_CBF16;

// variant: 0 = auto, 1 = 256x128 (8 waves, 3 stages), 2 = 128x128 (4 waves, 3 stages), 3 = 256x192 (8 waves, 2 st),
// 4 = 128x192 (4 waves, 2 stages: 80 KB LDS, 2 blocks/CU), 5 = 128x192 (4 waves, 3 stages), 6 = 128x96 (4 waves, 3 st),
// 7 = 192x192 (8 waves, 3 stages: 144 KB LDS), 8 = 128x192 (8 waves, 2 stages: 80 KB, 2 blocks/CU); + 100: persistent
// grid (resident blocks walk the M tiles)
int gemm3_ln_launch(const GemmDesc& d, hipStream_t s) {
    if (epi_flags(d) != F_TEXT_LN || d.N != 384 || !gemm3_supported(d) || d.ldo != 384 || d.res_bf16 || d.col_off != 0)
        return -2;
    launch3f<128, 384, 2, 4, 2, F_TEXT_LN>(d, s, true);
    return (int)hipGetLastError();
}

int gemm3_launch(const GemmDesc& d, hipStream_t s, int variant) {
    const bool persist = variant >= 100;
    if (persist) variant -= 100;
    if (variant == 0) variant = (d.N % 192 == 0 && d.N % 128 != 0) ? 3 : 1;
    if (variant == 1) launch3<256, 128, 4, 2, 3>(d, s, persist);
    else if (variant == 2) launch3<128, 128, 2, 2, 3>(d, s, persist);
    else if (variant == 4) launch3<128, 192, 2, 2, 2>(d, s, persist);
    else if (variant == 5) launch3<128, 192, 2, 2, 3>(d, s, persist);
    else if (variant == 6) launch3<128, 96, 2, 2, 3>(d, s, persist);
    else if (variant == 7) launch3<192, 192, 4, 2, 3>(d, s, persist);
    else if (variant == 8) launch3<128, 192, 4, 2, 2>(d, s, persist);     // 8 waves, 80 KB: 2 blocks per CU
    else launch3<256, 192, 4, 2, 2>(d, s, persist);
    return (int)hipGetLastError();
}

}  // namespace athd
