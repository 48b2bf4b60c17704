// Implicit-GEMM conv / linear kernel on MFMA for gfx950.  See gemm.h for the descriptor.
//
// Block tile BM x BN x 32, 256 threads = 4 waves laid out WM x WN, each wave (BM/WM) x (BN/WN) built from
// 16x16 MFMA tiles.  Both operands are staged in LDS as [row][32 k] (+pad) in the compute dtype so that every
// lane reads its 8 consecutive k of one row with one 16-B (bf16) or two 16-B (f32) LDS reads:
//   bf16: one v_mfma_f32_16x16x32_bf16 per tile per k-step (lane l: row l&15, k = 8(l>>4)..+7)
//   f32 : eight v_mfma_f32_16x16x4_f32 per tile; instruction s takes k = 8(l>>4)+s from each lane group, a
//         permutation of the 32 k that A and B share, so the result is the exact f32 fmaf chain per k-order.
// Global->LDS is register staged and double buffered: tile t+1 is loaded into registers before the MFMAs of
// tile t and written to the other LDS buffer after them; one barrier per k-step.
#include <cstdlib>

#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "gemm_epi.h"

namespace athd {

constexpr int BK = 32;

template <int MODE> struct CT;
template <> struct CT<0> { typedef float T; };
template <> struct CT<1> { typedef bf16_t T; };

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;

template <typename T> struct Vec8 { T v[8]; };

template <int MODE, int BM, int BN, int WM, int WN, bool VEC8>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmDesc d) {
    using T = typename CT<MODE>::T;
    constexpr int PAD = (MODE == 1) ? 8 : 4;
    constexpr int LD = BK + PAD;
    constexpr int TM = BM / WM / 16;
    constexpr int TN = BN / WN / 16;
    constexpr int AROWS = BM / 64;                 // A rows loaded per thread (8 k each)
    constexpr int BGROUPS = (BN * 4 + 255) / 256;  // B groups per thread
    __shared__ __attribute__((aligned(16))) T lds[2][(BM + BN) * LD];
    __shared__ double st_lds[2 * EPI_MAXG];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave / WN, wc = wave % WN;
    const int wm0 = wr * (BM / WM), wn0 = wc * (BN / WN);

    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int64_t a_bs = d.a_bs >= 0 ? d.a_bs : (int64_t)d.H_in * d.W * d.a_ld;
    const int64_t rowpitch = d.a_hs >= 0 ? d.a_hs : (int64_t)d.W * d.a_ld;

    // ---- per-thread A rows (fixed across k) ----
    const int kg = tid & 3;
    int64_t a_base[AROWS];
    int a_h0[AROWS];
    int a_b[AROWS];
    bool a_ok[AROWS];
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
        int64_t m = m0 + (tid >> 2) + 64 * i;
        a_ok[i] = m < M;
        int64_t mm = a_ok[i] ? m : 0;
        int w = (int)(mm % d.W);
        int64_t t = mm / d.W;
        int ho = (int)(t % d.H_out);
        int b = (int)(t / d.H_out);
        a_b[i] = b;
        a_base[i] = (int64_t)b * a_bs + (int64_t)w * d.a_ld;
        a_h0[i] = ho * d.in_stride + d.in_off;
    }

    Vec8<T> ra[AROWS];
    Vec8<T> rb[BGROUPS];
    const int nk = d.Kp / BK;

    auto load_tile = [&](int kt) {
        const int k = kt * BK + 8 * kg;
#pragma unroll
        for (int i = 0; i < AROWS; ++i) {
            float v[8];
            if constexpr (VEC8) {
                const int tap = k / d.C_in;
                const int ci = k - tap * d.C_in;
                const int row = a_h0[i] + tap * d.dil;
                const bool ok = a_ok[i] && k < d.K && row >= 0 && row < d.H_in;
                if (ok) {
                    const int64_t off = a_base[i] + (int64_t)row * rowpitch + ci;
                    if (d.a_bf16) {
                        uint4 q = *reinterpret_cast<const uint4*>((const bf16_t*)d.A + off);
                        const bf16_t* h = reinterpret_cast<const bf16_t*>(&q);
#pragma unroll
                        for (int j = 0; j < 8; ++j) v[j] = bf2f(h[j]);
                    } else {
                        const float4* p = reinterpret_cast<const float4*>((const float*)d.A + off);
                        float4 x0 = p[0], x1 = p[1];
                        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
                        v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
                    }
                    if (d.a_norm) {
                        const float sub = d.a_norm[2 * a_b[i]], dv = d.a_norm[2 * a_b[i] + 1];
#pragma unroll
                        for (int j = 0; j < 8; ++j) v[j] = (v[j] - sub) / dv;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = 0.f;
                }
            } else if (d.ntaps == 1) {
                const int row = a_h0[i];
                const bool rok = a_ok[i] && row >= 0 && row < d.H_in;
                const int64_t rb = a_base[i] + (int64_t)row * rowpitch;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int kk = k + j;
                    float x = 0.f;
                    if (rok && kk < d.K) {
                        const int64_t off = rb + (int64_t)kk * d.a_cs;
                        x = d.a_bf16 ? bf2f(((const bf16_t*)d.A)[off]) : ((const float*)d.A)[off];
                        if (d.a_norm) x = (x - d.a_norm[2 * a_b[i]]) / d.a_norm[2 * a_b[i] + 1];
                    }
                    v[j] = x;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int kk = k + j;
                    const int tap = kk / d.C_in;
                    const int ci = kk - tap * d.C_in;
                    const int row = a_h0[i] + tap * d.dil;
                    const bool ok = a_ok[i] && kk < d.K && row >= 0 && row < d.H_in;
                    float x = 0.f;
                    if (ok) {
                        const int64_t off = a_base[i] + (int64_t)row * rowpitch + (int64_t)ci * d.a_cs;
                        x = d.a_bf16 ? bf2f(((const bf16_t*)d.A)[off]) : ((const float*)d.A)[off];
                        if (d.a_norm) x = (x - d.a_norm[2 * a_b[i]]) / d.a_norm[2 * a_b[i] + 1];
                    }
                    v[j] = x;
                }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if constexpr (MODE == 1) ra[i].v[j] = f2bf(v[j]);
                else ra[i].v[j] = v[j];
            }
        }
#pragma unroll
        for (int g = 0; g < BGROUPS; ++g) {
            const int gi = tid + 256 * g;
            const int n = gi >> 2;
            const int kb = kt * BK + 8 * (gi & 3);
            if (gi < BN * 4 && n0 + n < d.N) {
                const T* p = (const T*)d.Wp + (int64_t)(n0 + n) * d.Kp + kb;
                if constexpr (MODE == 1) {
                    *reinterpret_cast<uint4*>(&rb[g]) = *reinterpret_cast<const uint4*>(p);
                } else {
                    reinterpret_cast<float4*>(&rb[g])[0] = reinterpret_cast<const float4*>(p)[0];
                    reinterpret_cast<float4*>(&rb[g])[1] = reinterpret_cast<const float4*>(p)[1];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) rb[g].v[j] = (T)0;
            }
        }
    };

    auto store_tile = [&](int st) {
        T* L = lds[st];
#pragma unroll
        for (int i = 0; i < AROWS; ++i) {
            T* dst = L + ((tid >> 2) + 64 * i) * LD + 8 * kg;
            if constexpr (MODE == 1) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(&ra[i]);
            else {
                reinterpret_cast<float4*>(dst)[0] = reinterpret_cast<const float4*>(&ra[i])[0];
                reinterpret_cast<float4*>(dst)[1] = reinterpret_cast<const float4*>(&ra[i])[1];
            }
        }
#pragma unroll
        for (int g = 0; g < BGROUPS; ++g) {
            const int gi = tid + 256 * g;
            if (gi < BN * 4) {
                T* dst = L + (BM + (gi >> 2)) * LD + 8 * (gi & 3);
                if constexpr (MODE == 1) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(&rb[g]);
                else {
                    reinterpret_cast<float4*>(dst)[0] = reinterpret_cast<const float4*>(&rb[g])[0];
                    reinterpret_cast<float4*>(dst)[1] = reinterpret_cast<const float4*>(&rb[g])[1];
                }
            }
        }
    };

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    if (d.stats && threadIdx.x < 2 * EPI_MAXG) st_lds[threadIdx.x] = 0.0;
    float4 bias4[TN];                             // loaded before the main loop (gemm_epi.h: load_bias4)
    load_bias4<TN>(d, n0, wn0, lane, bias4);
    load_tile(0);
    store_tile(0);
    __syncthreads();

    const int fr = lane & 15, fk = 8 * (lane >> 4);
    for (int kt = 0; kt < nk; ++kt) {
        const int st = kt & 1;
        if (kt + 1 < nk) load_tile(kt + 1);
        const T* L = lds[st];
        if constexpr (MODE == 1) {
            bf16v8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *reinterpret_cast<const bf16v8*>(L + (wm0 + 16 * i + fr) * LD + fk);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfr[j] = *reinterpret_cast<const bf16v8*>(L + (BM + wn0 + 16 * j + fr) * LD + fk);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        } else {
            float af[TM][8], bfr[TN][8];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float4* p = reinterpret_cast<const float4*>(L + (wm0 + 16 * i + fr) * LD + fk);
                float4 x0 = p[0], x1 = p[1];
                af[i][0] = x0.x; af[i][1] = x0.y; af[i][2] = x0.z; af[i][3] = x0.w;
                af[i][4] = x1.x; af[i][5] = x1.y; af[i][6] = x1.z; af[i][7] = x1.w;
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const float4* p = reinterpret_cast<const float4*>(L + (BM + wn0 + 16 * j + fr) * LD + fk);
                float4 x0 = p[0], x1 = p[1];
                bfr[j][0] = x0.x; bfr[j][1] = x0.y; bfr[j][2] = x0.z; bfr[j][3] = x0.w;
                bfr[j][4] = x1.x; bfr[j][5] = x1.y; bfr[j][6] = x1.z; bfr[j][7] = x1.w;
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[j][s], af[i][s], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store_tile(st ^ 1);
        __syncthreads();
    }

#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bias4[j].x), "v"(bias4[j].y), "v"(bias4[j].z), "v"(bias4[j].w));
    gemm_epilogue<TM, TN, F_ALL, MODE == 1>(d, acc, m0, n0, wm0, wn0, lane, st_lds, BM, bias4);
}

template <int MODE, int BM, int BN, int WM, int WN>
static void launch_cfg(const GemmDesc& d, hipStream_t s) {
    const int64_t M = (int64_t)d.nb * d.H_out * d.W;
    dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((d.N + BN - 1) / BN));
    const bool vec8 = (d.C_in % 8 == 0) && (d.a_ld % 8 == 0) && d.a_cs == 1;
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, MODE, fl, by);
        ks.begin(klabel("gemm_kernel<%d,%d,%d,%d,%d,%s>", MODE, BM, BN, WM, WN, vec8 ? "true" : "false"), fl, by);
    }
    if (vec8) hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, true>), grid, dim3(256), 0, s, with_fastdiv(d));
    else hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, false>), grid, dim3(256), 0, s, with_fastdiv(d));
}

template <int MODE>
static void launch_mode(const GemmDesc& d, hipStream_t s) {
    if (d.N <= 16 && d.act != ACT_GLU) launch_cfg<MODE, 256, 16, 4, 1>(d, s);
    else if (d.N <= 32) launch_cfg<MODE, 256, 32, 4, 1>(d, s);
    else if (d.N <= 64) launch_cfg<MODE, 128, 64, 2, 2>(d, s);
    else launch_cfg<MODE, 128, 128, 2, 2>(d, s);
}

bool gemm2_supported(const GemmDesc& d);
int gemm2_launch(const GemmDesc& d, hipStream_t s);
bool gemm3_supported(const GemmDesc& d);
int gemm3_launch(const GemmDesc& d, hipStream_t s, int variant);
int gemm3_ln_launch(const GemmDesc& d, hipStream_t s);
bool gemm5_supported(const GemmDesc& d);
int gemm5_launch(const GemmDesc& d, hipStream_t s);

bool rowln_supported(const GemmDesc& d);
int rowln_launch(const GemmDesc& d, hipStream_t s);
bool rowln_text_enabled();
int rowln_text_launch(const GemmDesc& d, hipStream_t s);
#ifdef ATHD_KBENCH
int gemm6_launch(const GemmDesc& d, hipStream_t s);
#endif

int gemm_launch(const GemmDesc& d0, int mode, hipStream_t s) {
    if (d0.Kp % BK != 0 || d0.Kp < d0.K || d0.C_in <= 0 || d0.N <= 0) return -2;
    const GemmDesc d = with_fastdiv(d0);
    if (d.act == ACT_GLU && (d.N % 32 != 0)) return -2;
    // residual projection + the next LayerNorm (rowln.hip), bf16 mode only
    if (d.ln_out) return mode == 1 && rowln_supported(d) ? rowln_launch(d, s) : -2;
    // row-LayerNorm epilogue (the text mlp2): rowln.hip's text form, else gemm3
    if (d.ln_w) {
        if (mode != 1) return -2;
        if (rowln_text_enabled()) {
            const int rc = rowln_text_launch(d, s);
            if (rc != -2) return rc;
        }
        return gemm3_ln_launch(d, s);
    }
    // the GroupNorm folded into the A load (a_gn_*, the transformer's last pending GroupNorm): gemm2 only; refuse
    // rather than silently skip it on another kernel
    if (d.a_gn_stats) return mode == 1 && gemm2_supported(d) ? gemm2_launch(d, s) : -2;
    // the residual's GroupNorm (res_gn_*): gemm5's residual epilogue only
    if (d.res_gn_stats && !(mode == 1 && gemm5_supported(d) && d.N % 256 == 0 && epi_res_fast_ok(d))) return -2;
    // bf16 activations, N a multiple of 256: 256x256 tile, staggered two-group K-loop (gemm5.hip; it replaced round
    // 2's gemm4.hip, which tools/kbench still builds as the A/B baseline: kbench +6..16 % on the transformer shapes,
    // equal at K = 2048).  (Measured on N = 192 / 384: slower than gemm3's 256x192 tiles, which waste no columns.)
#ifdef ATHD_KBENCH
    // dense linear rows without a residual epilogue, B from L2 (gemm6.hip, round-5 experiment, measured slower than
    // gemm5: built into tools/libkbench.so only, with ATHD_G6=1; -2 otherwise or when the shape is not its)
    if (mode == 1) {
        const int rc = gemm6_launch(d, s);
        if (rc != -2) return rc;
    }
#endif
    if (mode == 1 && gemm5_supported(d) && d.N % 256 == 0) return gemm5_launch(d, s);
    // other N >= 192: 256x192 or 192x192 tile, 8 waves (gemm3.hip)
    // (K >= 384: 192x192 tiles with a 3-stage ring, two K-tiles in flight across each barrier; measured per call
    // site 2-20 % faster there.  Shorter K, e.g. the K=288 four-residue ConvT, keeps 256x192 x 2 stages.)
    if (mode == 1 && gemm3_supported(d) && d.N >= 192) {
        const int v = d.K >= 384 ? 7 : 3;
        return gemm3_launch(d, s, 100 + v);               // persistent grid
    }
    if (mode == 1 && gemm2_supported(d)) return gemm2_launch(d, s);
    if (mode == 1) launch_mode<1>(d, s);
    else launch_mode<0>(d, s);
    return (int)hipGetLastError();
}

}  // namespace athd
