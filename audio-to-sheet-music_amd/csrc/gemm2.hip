// GEMM v2 (bf16 MFMA, gfx950): BM x BN x 64 tiles, 4 waves (2 x 2), both operands streamed global -> LDS.
//
// LDS image per stage: [rows][64 bf16] = 128 B per row, eight 16-B chunks stored XOR-swizzled
// (slot = chunk ^ (row & 7)) so that the 16x16x32 fragment reads (16 rows x one chunk per lane group) are
// conflict-free for ds_read_b128.  A wave instruction fills 8 rows x 128 B = 1 KiB; lane L lands at
// base + 16 L, i.e. row L/8, slot L%8, so it fetches global chunk (L%8) ^ (L/8): the swizzle lives in the
// per-lane SOURCE address (the LDS-DMA destination is lane-linear).
//   * bf16 operands (weights, and A when the activation is stored bf16): global_load_lds_dwordx4 straight
//     into LDS; out-of-range taps / rows / k read a 16-B zero page.
//   * fp32 A (residual streams kept in fp32): the same lane -> (row, chunk) map, loaded to registers,
//     converted to bf16 and written with ds_write_b128 after the MFMAs of the current tile.
// Two LDS stages: tile t+1 is issued before the MFMAs of tile t; one drain + barrier per k-tile.
#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

namespace athd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __attribute__((aligned(64))) uint4 g_zero_page[4];

template <int BM, int BN, bool A_BF16, unsigned F>
__global__ __launch_bounds__(256) void gemm2_kernel(const GemmDesc d) {
    constexpr int ROWB = 128;                                  // bytes per LDS row (64 bf16)
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int TM = BM / 2 / 16, TN = BN / 2 / 16;
    constexpr int AQ = BM / 32;                                // A instructions (8 rows each) per wave
    constexpr int BQ = BN / 32;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2 * EPI_MAXG * 8];
    double* st_lds = reinterpret_cast<double*>(smem + 2 * STAGE);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave >> 1) * (BM / 2), wn0 = (wave & 1) * (BN / 2);
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    // 1-D grid, column tile fastest and each XCD a contiguous id range (workgroup i runs on XCD i % 8): the N / BN
    // column tiles of a row block run together on one XCD and read its A rows from HBM once (a 2-D grid ran every
    // row block's column tiles ntm blocks apart: the downsampler's fp32 A was read 2.2x, PMC)
    const int ntm2 = (int)(((int64_t)d.nb * d.H_out * d.W + BM - 1) / BM), ntn2 = (d.N + BN - 1) / BN;
    int id2;
    {
        const int n = ntm2 * ntn2, q = n / 8, r = n % 8, x = (int)blockIdx.x % 8;
        id2 = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (int)blockIdx.x / 8;
    }
    const int64_t m0 = (int64_t)(id2 / ntn2) * BM;
    const int n0 = (id2 % ntn2) * BN;
    const int64_t a_bs = d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld;
    const int64_t rowpitch = d.a_hs >= 0 ? d.a_hs : (int64_t)d.W * d.a_ld;
    const int lrow = lane >> 3;                                // row within an 8-row instruction
    const int chunk = (lane & 7) ^ lrow;                       // global 16-B chunk this lane fetches

    // per-lane A rows: row = 8 (wave + 4 q) + lrow
    int64_t a_base[AQ];
    int a_h0[AQ], a_b[AQ];
    bool a_ok[AQ];
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
        const int64_t m = m0 + 8 * (wave + 4 * q) + lrow;
        a_ok[q] = m < M;
        const int64_t mm = a_ok[q] ? m : 0;
        const int w = (int)(mm % d.W);
        const int64_t t = mm / d.W;
        const int ho = (int)(t % d.H_out);
        const int b = (int)(t / d.H_out);
        a_b[q] = b;
        a_base[q] = (int64_t)b * a_bs + (int64_t)w * d.a_ld;
        a_h0[q] = ho * d.in_stride + d.in_off;
    }
    const char* bptr[BQ];
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
        const int n = n0 + 8 * (wave + 4 * q) + lrow;
        bptr[q] = n < d.N ? (const char*)d.Wp + ((int64_t)n * d.Kp + 8 * chunk) * 2 : nullptr;
    }
    // k -> (tap, ci) for this lane's chunk, advanced incrementally by 64 per tile
    int k_cur = 8 * chunk, tap = k_cur / d.C_in, ci = k_cur - tap * d.C_in;
    const char* zero = reinterpret_cast<const char*>(g_zero_page);
    const int nk = d.Kp / 64;

    const bool flat = d.C_in < 8;                             // (gemm2_supported: fp32 A, a_hs == C_in, dil 1)
    float4 ra[AQ][2];   // fp32-A staging
    unsigned rv[AQ];    // per-element in-bounds mask (normalisation applies to in-bounds values only; padding stays 0)
    int ra_ci = 0;      // channel of the staged chunk (A GroupNorm)
    float agm[AQ], agr[AQ];                                   // A GroupNorm mean / rstd of each staged row's batch
    (void)ra;
    (void)rv;
    (void)ra_ci;
    if constexpr (!A_BF16) {
        if (d.a_gn_stats) {
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                const double m = d.a_gn_stats[2 * a_b[q]] / (double)d.a_gn_count;
                double var = d.a_gn_stats[2 * a_b[q] + 1] / (double)d.a_gn_count - m * m;
                if (var < 0) var = 0;
                agm[q] = (float)m;
                agr[q] = (float)(1.0 / sqrt(var + 1e-5));
            }
        }
    }

    auto issue = [&](int kt, int st) {
        char* sA = smem + st * STAGE;
        char* sB = sA + BM * ROWB;
        const bool kok = k_cur < d.K;
        ra_ci = ci;
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
            const int row = a_h0[q] + tap * d.dil;
            const bool ok = a_ok[q] && kok && row >= 0 && row < d.H_in;
            const int64_t off = a_base[q] + (int64_t)row * rowpitch + ci;
            if constexpr (A_BF16) {
                const char* src = ok ? (const char*)d.A + off * 2 : zero;
                __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sA + (wave + 4 * q) * 1024), 16, 0, 0);
            } else if (flat) {
                // flat K (C_in < 8, taps contiguous): the 8 elements span taps tap .. tap + (ci + 7) / C_in
                const int row_l = row + (ci + 7) / d.C_in * d.dil;
                const bool ok_l = a_ok[q] && kok && row_l >= 0 && row_l < d.H_in;
                if (ok && ok_l && k_cur + 8 <= d.K) {
                    rv[q] = 0xFFu;
                    const float4* p = reinterpret_cast<const float4*>((const float*)d.A + off);
                    ra[q][0] = p[0];
                    ra[q][1] = p[1];
                } else {
                    float v[8];
                    unsigned m = 0u;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int rj = row + (ci + j) / d.C_in * d.dil;
                        const bool okj = a_ok[q] && k_cur + j < d.K && rj >= 0 && rj < d.H_in;
                        v[j] = okj ? ((const float*)d.A)[off + j] : 0.f;
                        m |= okj ? (1u << j) : 0u;
                    }
                    rv[q] = m;
                    ra[q][0] = make_float4(v[0], v[1], v[2], v[3]);
                    ra[q][1] = make_float4(v[4], v[5], v[6], v[7]);
                }
            } else {
                rv[q] = ok ? 0xFFu : 0u;
                if (ok) {
                    const float4* p = reinterpret_cast<const float4*>((const float*)d.A + off);
                    ra[q][0] = p[0];
                    ra[q][1] = p[1];
                } else {
                    ra[q][0] = make_float4(0.f, 0.f, 0.f, 0.f);
                    ra[q][1] = ra[q][0];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < BQ; ++q) {
            const char* src = bptr[q] ? bptr[q] + (int64_t)kt * 128 : zero;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sB + (wave + 4 * q) * 1024), 16, 0, 0);
        }
        // advance this lane's k by 64
        k_cur += 64;
        ci += 64;
        while (ci >= d.C_in) { ci -= d.C_in; ++tap; }
    };
    auto write_a = [&](int st) {
        if constexpr (!A_BF16) {
            char* sA = smem + st * STAGE;
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                float v[8] = {ra[q][0].x, ra[q][0].y, ra[q][0].z, ra[q][0].w, ra[q][1].x, ra[q][1].y, ra[q][1].z, ra[q][1].w};
                if (d.a_norm && rv[q]) {
                    const float sub = d.a_norm[2 * a_b[q]], dv = d.a_norm[2 * a_b[q] + 1];
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = ((rv[q] >> j) & 1u) ? (v[j] - sub) / dv : 0.f;
                }
                if (d.a_gn_stats && rv[q]) {           // (ntaps == 1: the chunk is channels ra_ci .. + 7)
                    const float4 w0 = *reinterpret_cast<const float4*>(d.a_gn_w + ra_ci);
                    const float4 w1 = *reinterpret_cast<const float4*>(d.a_gn_w + ra_ci + 4);
                    const float4 c0 = *reinterpret_cast<const float4*>(d.a_gn_b + ra_ci);
                    const float4 c1 = *reinterpret_cast<const float4*>(d.a_gn_b + ra_ci + 4);
                    const float gw[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
                    const float gb[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = ((rv[q] >> j) & 1u) ? (v[j] - agm[q]) * agr[q] * gw[j] + gb[j] : 0.f;
                }
                bf16_t h[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) h[j] = f2bf(v[j]);
                *reinterpret_cast<uint4*>(sA + (wave + 4 * q) * 1024 + lane * 16) = *reinterpret_cast<uint4*>(h);
            }
        }
    };

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (d.stats && tid < 2 * EPI_MAXG) st_lds[tid] = 0.0;
    float4 bias4[TN];                             // loaded before the main loop (gemm_epi.h: load_bias4)
    load_bias4<TN>(d, n0, wn0, lane, bias4);

    issue(0, 0);
    write_a(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int fr = lane & 15, g = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
        const char* sA = smem + cur * STAGE;
        const char* sB = sA + BM * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
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
        if (kt + 1 < nk) write_a(cur ^ 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bias4[j].x), "v"(bias4[j].y), "v"(bias4[j].z), "v"(bias4[j].w));
    gemm_epilogue<TM, TN, F, true>(d, acc, m0, n0, wm0, wn0, lane, st_lds, BM, bias4);
}

bool gemm2_supported(const GemmDesc& d) {
    const bool flat = d.C_in < 8 && 8 % d.C_in == 0 && !d.a_bf16 && d.a_hs == d.C_in && d.dil == 1;
    const bool narrow = d.N <= 32 && d.N % 4 == 0 && d.a_bf16 && epi_flags(d) == F_STATS;   // launch2f<256, 32>
    if ((d.C_in % 8 != 0 && !flat) || d.a_ld % (flat ? d.C_in : 8) != 0 || d.a_cs != 1 || d.Kp % 64 != 0 ||
        (d.N < 48 && !narrow))
        return false;
    if (flat && (d.a_bs % 4 != 0 || d.a_ld % 4 != 0)) return false;      // 16-B aligned chunk starts
    if (d.a_bf16 && d.a_norm) return false;
    if (d.a_gn_stats && (d.a_bf16 || d.ntaps != 1 || d.C_in % 8 != 0 || flat)) return false;
    if (d.act == ACT_GLU && d.N % 32 != 0) return false;
    return true;
}

template <int BM, int BN, unsigned F>
static void launch2f(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    dim3 grid((unsigned)(((M + BM - 1) / BM) * ((d.N + BN - 1) / BN)));
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin(klabel("gemm2_kernel<%d,%d,%s,%u>", BM, BN, d.a_bf16 ? "true" : "false", F), fl, by);
    }
    if (d.a_bf16) hipLaunchKernelGGL((gemm2_kernel<BM, BN, true, F>), grid, dim3(256), 0, s, with_fastdiv(d));
    else hipLaunchKernelGGL((gemm2_kernel<BM, BN, false, F>), grid, dim3(256), 0, s, with_fastdiv(d));
}

template <int BM, int BN>
static void launch2(const GemmDesc& d, hipStream_t s) {
    const unsigned f = epi_flags(d);
    switch (f) {
#define ATHD_CASE(FL) \
    case (FL): launch2f<BM, BN, (FL)>(d, s); return;
        ATHD_EPI_LIST(ATHD_CASE)
#undef ATHD_CASE
        default: launch2f<BM, BN, F_ALL>(d, s); return;
    }
}

int gemm2_launch(const GemmDesc& d, hipStream_t s) {
    // N <= 32 (the wide DConv levels' conv3, C -> C/8 = 24, with the GroupNorm statistics of h): 256 x 32 tiles,
    // instantiated for that epilogue only (round 2 ran it on the v1 kernel at 1.4 TB/s)
    if (d.N <= 32 && d.a_bf16 && epi_flags(d) == F_STATS) launch2f<256, 32, F_STATS>(d, s);
    else if (d.N <= 64) launch2<128, 64>(d, s);
    else launch2<128, 128>(d, s);
    return (int)hipGetLastError();
}

}  // namespace athd
