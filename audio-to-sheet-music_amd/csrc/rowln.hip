// Residual-stream projection with the next LayerNorm in its epilogue (bf16 mode; the transformer's out_proj + norm2,
// demucs transformer.py MyTransformerEncoderLayer / CrossTransformerEncoderLayer with norm_first: x = x + gamma_1 *
// out_proj(attn); the FFN then reads norm2(x)).
//
//   X[m][:]  = res'[m][:] + res_scale * (A[m][:] @ W^T + bias)      (res' = X with its pending GroupNorm, if any)
//   H[m][:]  = LayerNorm(X[m][:]) * ln_w + ln_b                      (bf16)
//
// The unfused pair (gemm5 out_proj, then layernorm_rows_kernel) reads the f32 rows of X twice: 271 MB more per freq
// layer than this pass, which needs whole rows in one workgroup (N = 512).  Tile = BM rows x 512 columns, K = 512,
// NW waves; wave w owns 512 / NW columns of all BM rows (TM x TN accumulator tiles of 16 x 16, 144 registers at
// BM = 144).  One workgroup per CU (8 waves at 2 per SIMD, 246 VGPRs each), so a workgroup's
// K-loop (matrix cores, B from L2) and its epilogue (HBM: 10 bytes per output element) alternate.  Measured forms
// (serialised events for the 10 launches of a forward, one box each): 128 x 512 tiles 2.08 ms; 64 x 512 tiles of 4
// waves, two workgroups per CU so one's epilogue runs beside the other's K-loop, 2.34 ms (the B fragments, re-read
// from L2 for every 64 rows, then need ~39 TB/s of L2 bandwidth); out_proj + LayerNorm unfused 2.03 ms.  Whole step
// neutral in A/B (ATHD_ROWLN=0, 4 alternating pairs: 1822 vs 1821 segments/s); kept for the 10 fewer launches and
// 2.7 GB less HBM traffic per forward.  144-row tiles (round 5; 18 A pieces per K-tile, 3 per wave, the 6 surplus
// ones from the zero page into a sink): the freq / time launches take 4 / 2 rounds of tiles instead of 5 / 3, 2.13 ->
// 1.84 ms, whole step 1837 -> 1855 segments/s (3 alternating runs each, driver protocol).
//   - A (the attention output, bf16) is shared by all waves: 16-KB K-tiles by LDS-DMA into a 3-deep ring (gemm3's
//     swizzled image and counted waits).
//   - B (the weights, 512 KB of bf16: resident in every XCD's L2) goes global -> VGPR as MFMA fragments, one K-step
//     ahead.  Each wave's 64 columns are its own, so nothing of B is shared and no LDS holds it: a 512-column B
//     K-tile would be 64 KB per stage.
//   - epilogue: residual rows streamed two fragments ahead (f32, with the pending GroupNorm and the layer scale),
//     X stored, the row's sum and then its squared deviations reduced across the 8 waves in LDS (layernorm_kernel's
//     two-pass form), H stored as bf16.  Per-column parameters (bias, scale, GroupNorm and LayerNorm affines) come
//     from LDS: 16 columns x 6 parameters in registers would not fit beside the 128 accumulators.
#include "common.h"
#include "prof.h"
#include "gemm.h"

namespace athd {

namespace {

constexpr int RL_N = 512, RL_K = 512;           // the out_proj shape
constexpr int RT_N = 384, RT_K = 384;           // the text cross-attention's mlp2 shape (TEXT)
constexpr int RL_NS = 3;                         // A ring depth
typedef __attribute__((address_space(3))) void rl_lds_void;
typedef __attribute__((address_space(1))) void rl_gbl_void;
__device__ __attribute__((aligned(64))) uint4 g_zero_rl[4];

template <int N>
ATHD_DEV void rl_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// The VM issue schedule of the K-loop, for the counted waits (every count is the number of VM operations issued AFTER
// the one waited for).  Prologue: B(0) (TN loads), A(0), A(1) (AQ DMAs each).  K-step ks: B(ks + 1), then at even ks
// A(ks / 2 + 2).
template <int KS, int TN, int AQ>
struct RlSched {
    static constexpr int KT = KS / 2;
    static constexpr int step(int ks) { return (ks + 1 < KS ? TN : 0) + ((ks % 2 == 0 && ks / 2 + 2 < KT) ? AQ : 0); }
    static constexpr int through(int ks) {       // issued by the end of step ks's issue block
        int n = TN + 2 * AQ;
        for (int k = 0; k <= ks; ++k) n += step(k);
        return n;
    }
    static constexpr int pos_b(int k) {          // position of B(k)'s last load
        if (k == 0) return TN;
        return through(k - 2) + TN;              // B(k) opens step k - 1 (through(-1) = the prologue)
    }
    static constexpr int pos_a(int t) {          // position of A(t)'s last DMA
        if (t < 2) return TN + (t + 1) * AQ;
        return through(2 * (t - 2) - 1) + TN + AQ;
    }
    static constexpr int wait_b(int ks) { return through(ks) - pos_b(ks); }
    static constexpr int wait_a(int ks) { return through(ks) - pos_a(ks / 2 + 1); }   // at the end of odd ks
};

}  // namespace

#ifndef ATHD_RL_RD
#define ATHD_RL_RD 2
#endif
#ifndef ATHD_RL_PROBE
#define ATHD_RL_PROBE 0      // ablations for A/B builds only (outputs garbage): 1 = K-loop only (no epilogue), 2 = no MFMAs
#endif

// TEXT: the text cross-attention's mlp2 + norm_out (ATHTDemucs_v2.py:47-49; gemm3_epilogue_ln's epilogue, N = K = 384):
// v = res[item / res_div][row] + (acc + bias + pbias[item]), LayerNorm over the row, bf16 to C; nothing else stored.
// Per-column parameter slots in LDS: 0 bias, 1 / 2 res_scale / res_gn_w (out_proj) or the pbias rows of the tile's
// two items (TEXT), 3 res_gn_b, 4 / 5 ln_w / ln_b.
template <int BM, int NW, int N, int K, bool TEXT>
__global__ __launch_bounds__(64 * NW, 2) void rowln_kernel(const GemmDesc d) {
    constexpr int NT = 64 * NW;
    constexpr int RL_N = N, RL_K = K;
    constexpr int RL_KT = K / 64, RL_KS = K / 32;
    constexpr int RL_PAR = 6 * N;
    constexpr int TM = BM / 16, TN = RL_N / NW / 16;
    constexpr int STAGE = BM * 128;
    constexpr int AP = BM / 8;                   // 1-KB A pieces (8 rows) per K-tile
    constexpr int AQ = (AP + NW - 1) / NW;       // A DMAs per wave per K-tile (surplus pieces: zero page -> sink)
    static_assert(AP * 8 == BM && BM % 16 == 0 && TN * 16 * NW == RL_N && K % 64 == 0, "tile shape");
    static_assert(RL_KS == 16 || RL_KS == 12, "K-steps below");
    using S = RlSched<RL_KS, TN, AQ>;
    __shared__ __attribute__((aligned(1024))) char ring[RL_NS * STAGE];
    __shared__ __attribute__((aligned(16))) float par[RL_PAR];
    __shared__ __attribute__((aligned(16))) float red[2][BM][NW];
    __shared__ __attribute__((aligned(1024))) char sink[AQ * NW > AP ? 1024 : 16];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l15 = lane & 15, l4 = lane >> 4;
    const uint32_t M = (uint32_t)d.nb * d.H_out;
    const uint32_t rpb = (uint32_t)d.H_out;      // rows per batch (item)
    const int ntm = (int)((M + BM - 1) / BM);
    // XCD-aware: workgroup i runs on XCD i % 8; each XCD takes a contiguous range of row tiles
    int tile;
    {
        const int n = (int)gridDim.x, q = n / 8, r = n % 8, x = (int)blockIdx.x % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (int)blockIdx.x / 8;
    }
    if (tile >= ntm) return;
    // (TEXT, measured: per-item tiles with the res_div prompts of a segment's rows adjacent, so that one XCD's L2
    // serves the shared residual rows: the kernel 0.49 -> 0.47 ms, the whole step 1.9 % slower, 3 alternating pairs)
    const uint32_t m0 = (uint32_t)tile * BM, Mend = M;      // the tile's rows [m0, Mend)
    const int n0 = TN * 16 * wave;               // this wave's columns

    // ---- per-column parameters -> LDS (published by the K-loop's first barrier) ----
    const uint32_t b0 = m0 / rpb;
    const uint32_t b1 = (b0 + 1) * rpb < M ? b0 + 1 : b0;   // the tile's second batch (H_out >= BM: at most two)
    for (int i = tid; i < RL_PAR; i += NT) {
        const int k = i / RL_N, n = i % RL_N;
        if constexpr (TEXT) {
            const float* src = k == 0 ? d.bias : k == 1 ? (d.pbias ? d.pbias + (int64_t)b0 * RL_N : nullptr)
                             : k == 2 ? (d.pbias ? d.pbias + (int64_t)b1 * RL_N : nullptr) : k == 3 ? nullptr
                             : k == 4 ? d.ln_w : d.ln_b;
            par[i] = src ? src[n] : 0.f;
        } else {
            const float* src = k == 0 ? d.bias : k == 1 ? d.res_scale : k == 2 ? d.res_gn_w : k == 3 ? d.res_gn_b
                                                                         : k == 4 ? d.ln_w : d.ln_b;
            par[i] = src ? src[n] : (k == 1 ? 1.f : 0.f);
        }
    }

    // ---- operand streams ----
    const int lrow = lane >> 3, chunk = (lane & 7) ^ lrow;
    const char* zero = reinterpret_cast<const char*>(g_zero_rl);
    const char* arow[AQ];
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
        const uint32_t m = m0 + 8 * (wave + NW * q) + lrow;
        arow[q] = m < Mend && wave + NW * q < AP ? (const char*)d.A + ((int64_t)m * RL_K + 8 * chunk) * 2 : nullptr;
    }
    auto dma_a = [&](int kt) {
        char* dst = ring + (kt % RL_NS) * STAGE;
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
            const char* src = arow[q] ? arow[q] + kt * 128 : zero;
            char* to = dst + (wave + NW * q) * 1024;
            if (AQ * NW > AP && wave + NW * q >= AP) to = sink;      // (wave-uniform)
            __builtin_amdgcn_global_load_lds((rl_gbl_void*)src, (rl_lds_void*)to, 16, 0, 0);
        }
    };
    // B fragments by global_load_dwordx4 in inline asm, waited for by explicit counts: with VGPR-returning loads and
    // LDS-DMA both in flight the compiler's wait insertion treats the VM counter as out of order and drains it
    // (vmcnt(0) before every MFMA group whose fragments were loaded); the asm loads are invisible to it.  The lane's
    // row pointer per fragment column.
    const bf16_t* wrow[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) wrow[j] = (const bf16_t*)d.Wp + (int64_t)(n0 + 16 * j + l15) * d.Kp + 8 * l4;
    bf16x8_t bq[2][TN];
#define load_b(KS)                                                                                                 \
    for (int j = 0; j < TN; ++j)                                                                                   \
        asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(bq[(KS) & 1][j]) : "v"(wrow[j]), "i"(64 * (KS)))

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const uint32_t a_lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)ring;

    load_b(0);
    asm volatile("" ::: "memory");
    dma_a(0);
    dma_a(1);
    rl_wait_vm<AQ>();                            // B(0), A(0) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // K-step ks (the body is a macro so that ks is a literal in every copy: the wait counts and LDS offsets fold)
#define RL_KSTEP(ks)                                                                                               \
    {                                                                                                              \
        constexpr int kt = (ks) / 2, s = (ks) % 2;                                                                \
        if constexpr ((ks) + 1 < RL_KS) load_b((ks) + 1);                                                          \
        asm volatile("" ::: "memory");                                                                             \
        if constexpr (s == 0 && kt + 2 < RL_KT) dma_a(kt + 2);                                                     \
        asm volatile("" ::: "memory");                                                                             \
        rl_wait_vm<S::wait_b(ks)>();             /* B(ks) landed */                                                \
        for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bq[(ks) & 1][j]));                                   \
        /* the A fragments by ds_read in inline asm: read through a pointer, the compiler cannot separate the ring */ \
        /* slot being read from the slots the DMAs in flight write, and puts a vmcnt(0) before the reads.  The    */ \
        /* counted wait at the end of the previous K-tile covers the slot.                                         */ \
        const uint32_t ab = a_lds + (uint32_t)(l15 * 128 + ((4 * s + l4) ^ (l15 & 7)) * 16);                     \
        bf16x8_t af[TM];                                                                                           \
        for (int i = 0; i < TM; ++i)                                                                               \
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[i]) : "v"(ab), "i"((kt % RL_NS) * STAGE + i * 2048)); \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                         \
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));                                              \
        for (int i = 0; i < TM; ++i)                                                                               \
            for (int j = 0; j < TN; ++j)                                                                           \
                if constexpr (ATHD_RL_PROBE != 2)                                                                  \
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[(ks) & 1][j], af[i], acc[i][j], 0, 0, 0);   \
        if constexpr (s == 1 && kt + 1 < RL_KT) {                                                                  \
            rl_wait_vm<S::wait_a(ks)>();         /* A(kt + 1) landed (this wave's pieces) ...                  */  \
            __builtin_amdgcn_s_barrier();        /* ... and every wave's; slot kt % 3 is free for A(kt + 3)     */  \
        }                                                                                                          \
    }
    RL_KSTEP(0) RL_KSTEP(1) RL_KSTEP(2) RL_KSTEP(3) RL_KSTEP(4) RL_KSTEP(5) RL_KSTEP(6) RL_KSTEP(7)
    RL_KSTEP(8) RL_KSTEP(9) RL_KSTEP(10) RL_KSTEP(11)
    if constexpr (RL_KS == 16) {
        RL_KSTEP(12) RL_KSTEP(13) RL_KSTEP(14) RL_KSTEP(15)
    }
#undef RL_KSTEP
#undef load_b
    rl_wait_vm<0>();                             // (nothing the compiler does not know of stays in flight)
    if constexpr (ATHD_RL_PROBE == 1) {          // keep the accumulators live, store nothing
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) t += acc[i][j][0] + acc[i][j][3];
        if (t == 1234.5f) ((float*)d.res)[m0] = t;
        return;
    }

    // ---- epilogue 1: X = res' + scale * (acc + bias), stored; acc keeps X ----
    // the pending GroupNorm's (mean, rstd) of the tile's first batch and the next (a tile spans at most two batches:
    // H_out >= BM rows per batch, rowln_supported)
    float gm0 = 0.f, gr0 = 1.f, gm1 = 0.f, gr1 = 1.f;
    const bool rgn = !TEXT && d.res_gn_stats != nullptr;
    if (rgn) {
        const uint32_t blast = (M - 1) / rpb;
        gn_params(d.res_gn_stats, b0, d.res_gn_count, gm0, gr0);
        gn_params(d.res_gn_stats, b0 + 1 <= blast ? b0 + 1 : blast, d.res_gn_count, gm1, gr1);
    }
    float* X = (float*)d.C;
    const float* R = (const float*)d.res;
    const int cl = n0 + 4 * l4;                  // + 16 j: this lane's 4 columns of fragment column j
    int64_t rb[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const uint32_t m = m0 + 16 * i + l15;
        const uint32_t mm = m < Mend ? m : Mend - 1;
        if constexpr (TEXT) {                    // the segment's residual row, shared by its res_div prompts
            const uint32_t b = mm / rpb;
            rb[i] = (d.res_div > 1 ? (int64_t)(b / (uint32_t)d.res_div) * d.res_bs : (int64_t)b * rpb * RL_N) +
                    (int64_t)(mm - b * rpb) * RL_N + cl;
        } else {
            rb[i] = (int64_t)mm * RL_N + cl;
        }
    }
    // residual pieces of 4 (3) fragment columns (16 rows x 64 (48) columns of the wave), RD pieces in flight ahead of
    // the one being used: a whole row tile ahead (TN float4s per lane twice) spilled accumulators
    constexpr int PC = TN % 4 == 0 ? 4 : TN % 3 == 0 ? 3 : 1, NPC = TN / PC, NP = TM * NPC, RD = ATHD_RL_RD;
    static_assert(TN % PC == 0, "residual pieces");
    float4 rr[RD + 1][PC];
    auto load_piece = [&](int p, float4 (&dst)[PC]) {
        const int i = p / NPC, j0 = (p % NPC) * PC;
#pragma unroll
        for (int jj = 0; jj < PC; ++jj) dst[jj] = *reinterpret_cast<const float4*>(R + rb[i] + 16 * (j0 + jj));
    };
#pragma unroll
    for (int p = 0; p < RD; ++p) load_piece(p, rr[p]);
    float rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) rs[i] = 0.f;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        if (p + RD < NP) load_piece(p + RD, rr[(p + RD) % (RD + 1)]);
        const int i = p / NPC, j0 = (p % NPC) * PC;
        const uint32_t m = m0 + 16 * i + l15;
        const bool second = m >= (b0 + 1) * rpb;
        const float gm = second ? gm1 : gm0, gr = second ? gr1 : gr0;
        float sum = 0.f;
#pragma unroll
        for (int jj = 0; jj < PC; ++jj) {
            const int j = j0 + jj;
            const int c = cl + 16 * j;
            const float4 bi = *reinterpret_cast<const float4*>(&par[c]);
            float4 r = rr[p % (RD + 1)][jj];
            if constexpr (TEXT) {                // v = res + (acc + bias + pbias), gemm3_epilogue_ln's order
                const float4 pb = *reinterpret_cast<const float4*>(&par[(second ? 2 : 1) * RL_N + c]);
                acc[i][j][0] = r.x + (acc[i][j][0] + bi.x + pb.x);
                acc[i][j][1] = r.y + (acc[i][j][1] + bi.y + pb.y);
                acc[i][j][2] = r.z + (acc[i][j][2] + bi.z + pb.z);
                acc[i][j][3] = r.w + (acc[i][j][3] + bi.w + pb.w);
                sum += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
                continue;
            }
            const float4 sc = *reinterpret_cast<const float4*>(&par[RL_N + c]);
            if (rgn) {
                const float4 gw = *reinterpret_cast<const float4*>(&par[2 * RL_N + c]);
                const float4 gb = *reinterpret_cast<const float4*>(&par[3 * RL_N + c]);
                r.x = (r.x - gm) * gr * gw.x + gb.x;
                r.y = (r.y - gm) * gr * gw.y + gb.y;
                r.z = (r.z - gm) * gr * gw.z + gb.z;
                r.w = (r.w - gm) * gr * gw.w + gb.w;
            }
            acc[i][j][0] = r.x + sc.x * (acc[i][j][0] + bi.x);
            acc[i][j][1] = r.y + sc.y * (acc[i][j][1] + bi.y);
            acc[i][j][2] = r.z + sc.z * (acc[i][j][2] + bi.z);
            acc[i][j][3] = r.w + sc.w * (acc[i][j][3] + bi.w);
            if (m < Mend)
                *reinterpret_cast<float4*>(X + rb[i] + 16 * j) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
            sum += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
        }
        rs[i] += sum;
        __builtin_amdgcn_sched_barrier(0);       // (the next piece's parameter reads are not hoisted above this one)
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        rs[i] += __shfl_xor(rs[i], 16, 64);
        rs[i] += __shfl_xor(rs[i], 32, 64);
    }
    // ---- epilogue 2: the row LayerNorm (mean, then the squared deviations; layernorm_kernel's two-pass form) ----
    auto row_total = [&](int buf, int row) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; w += 4) {
            const float4 a = *reinterpret_cast<const float4*>(&red[buf][row][w]);
            t += (a.x + a.y) + (a.z + a.w);
        }
        return t;
    };
    if (l4 == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) red[0][16 * i + l15][wave] = rs[i];
    }
    __syncthreads();
    float mean[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        mean[i] = row_total(0, 16 * i + l15) * (1.f / RL_N);
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
    if (l4 == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) red[1][16 * i + l15][wave] = rs[i];
    }
    __syncthreads();
    bf16_t* Hout = (bf16_t*)(TEXT ? d.C : d.ln_out);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const float rstd = 1.f / sqrtf(row_total(1, 16 * i + l15) * (1.f / RL_N) + 1e-5f);
        const uint32_t m = m0 + 16 * i + l15;
        if (m >= Mend) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int c = cl + 16 * j;
            const float4 lw = *reinterpret_cast<const float4*>(&par[4 * RL_N + c]);
            const float4 lb = *reinterpret_cast<const float4*>(&par[5 * RL_N + c]);
            const float y0 = (acc[i][j][0] - mean[i]) * rstd * lw.x + lb.x;
            const float y1 = (acc[i][j][1] - mean[i]) * rstd * lw.y + lb.y;
            const float y2 = (acc[i][j][2] - mean[i]) * rstd * lw.z + lb.z;
            const float y3 = (acc[i][j][3] - mean[i]) * rstd * lw.w + lb.w;
            *reinterpret_cast<uint2*>(Hout + (int64_t)m * RL_N + c) = make_uint2(pack2bf(y0, y1), pack2bf(y2, y3));
        }
    }
}

#ifndef ATHD_RL_BM
#define ATHD_RL_BM 144       // (the tile-round count: 921 / 460 row tiles over 256 CUs for M = 132608 / 66176, where
#endif                       // 128-row tiles need 1036 / 517, i.e. 5 and 3 rounds; 2.13 -> 1.84 ms per forward)
#ifndef ATHD_RL_NW
#define ATHD_RL_NW 8
#endif
constexpr int RL_BM = ATHD_RL_BM, RL_NW = ATHD_RL_NW;

// the shapes rowln_kernel handles: bf16 A [M][512] dense, K = 512, N = 512, f32 residual = output (dense rows), a
// LayerNorm output, >= RL_BM rows per batch (a tile spans at most two residual GroupNorm batches)
bool rowln_supported(const GemmDesc& d) {
    return d.ln_out && d.ln_w && d.ln_b && d.a_bf16 && d.N == RL_N && d.K == RL_K && d.Kp >= RL_K && d.Kp % 8 == 0 &&
           d.C_in == RL_K && d.a_ld == RL_K && d.ntaps == 1 && d.W == 1 && d.H_in == d.H_out && d.res && !d.res_bf16 &&
           !d.c_bf16 && d.ldo == RL_N && d.col_off == 0 && d.act == ACT_NONE && !d.stats && !d.gn_stats && !d.pbias &&
           !d.row_add && !d.col_split && d.o_stride == 1 && d.o_off == 0 && d.H_out_total == d.H_out && d.c_bs < 0 &&
           d.H_out >= RL_BM && d.res_div <= 1 && !d.a_norm && !d.a_gn_stats && d.a_bs < 0 && d.a_hs < 0 &&
           (!d.res_gn_stats || (d.res_gn_w && d.res_gn_b && d.res_gn_count > 0));
}

int rowln_launch(const GemmDesc& d, hipStream_t s) {
    if (!rowln_supported(d)) return -2;
    const int64_t M = (int64_t)d.nb * d.H_out;
    const int ntm = (int)((M + RL_BM - 1) / RL_BM);
    KScope ks(s);
    if (ks.on()) {
        // flops: 2 M N K; bytes: A once + weights + residual read + X written + H written
        ks.begin("rowln_kernel", 2.0 * M * RL_N * RL_K,
                 (double)M * RL_K * 2 + (double)RL_N * RL_K * 2 + (double)M * RL_N * (4 + 4 + 2));
    }
    hipLaunchKernelGGL((rowln_kernel<RL_BM, RL_NW, RL_N, RL_K, false>), dim3((unsigned)ntm), dim3(64 * RL_NW), 0, s, d);
    return (int)hipGetLastError();
}

// The text cross-attention's mlp2 + norm_out (gemm_launch's F_LN route; round 6): the gemm3 form (128 x 384 tiles,
// A and B through a 2-stage LDS ring of 64-KB K-tiles) ran at 2 TB/s, 26 % of its HBM floor - each 128-row tile
// streamed all 288 KB of weights through LDS one K-tile ahead.  Here the weights go L2 -> VGPR per wave (48 columns
// each, one K-step ahead) and only A is staged, 3 deep.  ATHD_RLT=0 keeps the gemm3 form (A/B, tested).
bool rowln_text_enabled() {                     // (read at every launch: the tests switch it between forwards)
    const char* e = getenv("ATHD_RLT");
    return !(e && e[0] == '0');
}

bool rowln_text_supported(const GemmDesc& d) {
    return d.ln_w && d.ln_b && !d.ln_out && d.a_bf16 && d.N == RT_N && d.K == RT_K && d.Kp >= RT_K && d.Kp % 8 == 0 &&
           d.C_in == RT_K && d.a_ld == RT_K && d.ntaps == 1 && d.W == 1 && d.H_in == d.H_out && d.res && !d.res_bf16 &&
           d.c_bf16 && d.store && d.ldo == RT_N && d.col_off == 0 && d.act == ACT_NONE && !d.stats && !d.gn_stats &&
           !d.res_scale && !d.res_gn_stats && !d.row_add && !d.col_split && d.o_stride == 1 && d.o_off == 0 &&
           d.H_out_total == d.H_out && d.c_bs < 0 && d.pfold <= 1 && d.H_out >= RL_BM && d.res_div >= 1 &&
           (d.res_div == 1 || d.res_bs >= (int64_t)d.H_out * RT_N) && !d.a_norm && !d.a_gn_stats && d.a_bs < 0 &&
           d.a_hs < 0;
}

int rowln_text_launch(const GemmDesc& d, hipStream_t s) {
    if (!rowln_text_supported(d)) return -2;
    const int64_t M = (int64_t)d.nb * d.H_out;
    const int ntm = (int)((M + RL_BM - 1) / RL_BM);
    KScope ks(s);
    if (ks.on()) {
        double fl, by;
        gemm_work(d, 1, fl, by);
        ks.begin("rowln_kernel<text>", fl, by);
    }
    hipLaunchKernelGGL((rowln_kernel<RL_BM, RL_NW, RT_N, RT_K, true>), dim3((unsigned)ntm), dim3(64 * RL_NW), 0, s, d);
    return (int)hipGetLastError();
}

}  // namespace athd
