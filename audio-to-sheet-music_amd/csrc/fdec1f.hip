// FreqDecoder level 1, GroupNorm statistics as a quadratic form (bf16 mode; ATHTDemucs_v2.py:90-103 for i = 1, the
// re-association of fdec_lr.hip).
//
// fdec_lr.hip writes Z = S @ [W_0 .. W_7] (3.3 GB of bf16 at the bench size) and sweeps it twice: once for the
// GroupNorm(1) {sum, sumsq} of the level-1 ConvT output Y, once to merge.  The merge pass only reads taps 0, 3, 4, 7
// (rows 4d+1, 4d+2), so Z is needed in full only for the statistics - and those need no sweep at all.  Every ConvT
// output row r = 4v + rho involves ONE tap class q = (rho + 2) % 4, i.e. taps {q, q+4}:
//   y_r[w][c] = b_c + c_r . x_q[w][c],   x_q = (Z_q[0..31], Z_{q+4}[0..31], Zs_q[0..7], Zs_{q+4}[0..7])   (80 values)
// with c_r the resize-lerp coefficients of the row (2 per tap, 0.1 on the Zs rows).  Over the Hd rows of a class:
//   sum   y   = Hd W sum_c b_c    + c1_q . u_q                   c1_q = sum_r c_r,      u_q  = sum_wc x_q
//   sum   y^2 = Hd W sum_c b_c^2  + 2 c1_q . ub_q + <Q_q, G_q>   Q_q = sum_r c_r c_r^T, ub_q = sum_wc b_c x_q,
//                                                                                       G_q  = sum_wc x_q x_q^T
// Q_q / c1_q depend only on (Hd, Hs, Hk) (fdec1_gram_q_kernel, double); G_q and the per-channel sums of x_q are a
// Gram matrix over (w, c): matrix-core work on the Z tile while it is in LDS.  So this pass computes Z tile by tile
// (MFMA, into LDS, never to HBM), accumulates the 4 classes' 80 x 80 Gram blocks in MFMA accumulators across the
// tiles of an item, flushes them per item into a partial slot of its own (workgroup, item), fdec1_gram_reduce_kernel
// sums an item's slots in a fixed order (bit-reproducible, round 5: the fp32 atomics of rounds 3-4 made two forwards
// differ at ~121 dB) and fdec1_gram_final_kernel forms {sum, sumsq}.  It
// replaces the 8-tap Z GEMM + fdec_lr_stats3_kernel's sweep (VALU-bound); it also stores the 4-tap Z (taps 0, 3, 4, 7)
// the merge pass reads, from the same LDS tiles.
//
// Tile = (item n, 8 consecutive w columns, channel group of 16), all 32 rows j of S:
//   Z GEMM   rows R = 8 j + wl (256; A = S[n][j][w0 + wl][0..191]), cols t * 16 + c (8 taps x 16 channels, K = 192);
//            wave wv: rows 32 wv .. +31, all 128 columns (v_mfma_f32_16x16x32_bf16, weights as the A operand)
//   LDS      ZT [t * 32 + j][wl * 16 + c] (bf16; the Gram's X rows), Zs [q * 16 + (t >> 2) * 8 + m][wl * 16 + c]
//   Gram     per class q: X row blocks R0..R3 (Z, 16 rows each) and R4 (Zs), K = (wl, c) = 128; blocks (ri <= ci)
//            of X X^T plus X times a one-hot channel matrix (the per-channel sums); wave wv: class wv >> 1, half
//            wv & 1 of the class's 20 blocks (10 each), accumulated across the item's tiles.
// Each persistent workgroup owns one channel group (its 128 weight rows stay in LDS, 48 KB) and walks a contiguous
// run of (item, w block) tiles.  LDS chunks (16 B) of every [row][256 B] array are XOR-swizzled by (row & 15):
// the MFMA-layout stores (ds_write_b64, 32 lanes) and the operand reads (ds_read_b128, 16 rows) both cover the 64
// banks once.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace athd {

namespace {

constexpr int G_CI = 192, G_CO = 96, G_HS = 32, G_HK = 8;
constexpr int G_WB = 8;                       // w columns per tile
constexpr int G_CG = 16;                      // channels per group
constexpr int G_NG = G_CO / G_CG;             // 6 groups
constexpr int G_THREADS = 512;
constexpr int G_B_BYTES = 128 * 384;          // weights [128 cols][192 K]
constexpr int G_ZT_BYTES = 256 * 256;         // ZT [(t, j)][(wl, c)]
constexpr int G_ZS_BYTES = 64 * 256;          // Zs [(q, t >> 2, m)][(wl, c)]
constexpr int G_LDS = G_B_BYTES + G_ZT_BYTES + G_ZS_BYTES;   // 128 KB
constexpr int G_NX = 80;                      // x_q entries
constexpr int G_NB = G_NX + G_CO;             // Gram row: 80 data columns + 96 per-channel sums
constexpr int G_ITEM = 4 * G_NX * G_NB;       // floats per item
constexpr int G_PSLOT = 8 * 10 * 64 * 4;      // floats per partial slot: the 8 waves' 10 Gram blocks as held in registers

// tile range [tb(qi), tb(qi + 1)) of the workgroups with logical index L = NG qi + g (T tiles over Qg ranges)
ATHD_HD int g_tb(int qi, int T, int Qg) { return (int)((int64_t)T * qi / Qg); }

ATHD_DEV int swz(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

ATHD_DEV int g_xcd_remap(int i, int n) {
    const int q = n / 8, r = n % 8, x = i % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
}

// the Gram blocks of a wave (10 each): half 0 of a class takes rows R0 (columns 0..5), R3 (3..5) and R4 (5), half 1
// rows R1 (1..5), R2 (2..5) and R4 (4); column 5 = the one-hot channel matrix
constexpr int G_NBLK = 10;
ATHD_HD constexpr int blk_r(int h, int b) {
    return h == 0 ? (b < 6 ? 0 : b < 9 ? 3 : 4) : (b < 5 ? 1 : b < 9 ? 2 : 4);
}
ATHD_HD constexpr int blk_c(int h, int b) {
    return h == 0 ? (b < 6 ? b : b < 9 ? b - 3 : 5) : (b < 5 ? b + 1 : b < 9 ? b - 3 : 4);
}

// resize-lerp coefficient of x_q entry a in ConvT output row 4v + rho (rho = (q + 2) % 4): the row is
// T_v[rho + 2] + (rho < 2 ? T_{v-1}[rho + 6] : T_{v+1}[rho - 2]) (fdec_lr.hip), T_s = lerp of the Z rows + 0.1 lerp
// of the Zs rows at step s (zero outside 0 <= s < Hd)
ATHD_HD double g_coef(int q, int v, int a, int Hd) {
    const int rho = (q + 2) & 3;
    const int t_main = rho < 2 ? q : q + 4;
    const int v_oth = rho < 2 ? v - 1 : v + 1;
    const bool zs = a >= 64;
    const int idx = zs ? (a - 64) & 7 : a & 31;
    const int tap = zs ? (a < 72 ? q : q + 4) : (a < 32 ? q : q + 4);
    const int s = tap == t_main ? v : v_oth;
    if (s < 0 || s >= Hd) return 0.0;
    const LinIdx li = lin_index(s, zs ? G_HK : G_HS, Hd);
    const double cf = (idx == li.i0 ? 1.0 - (double)li.l1 : 0.0) + (idx == li.i1 ? (double)li.l1 : 0.0);
    return zs ? cf * (double)0.1f : cf;
}

}  // namespace

// Q_q [4][80][80] and c1_q [4][80] (double, per class q: 6400 + 80 entries): one thread per entry
__global__ __launch_bounds__(256) void fdec1_gram_q_kernel(double* gq, int Hd) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int per = G_NX * G_NX + G_NX;
    if (e >= 4 * per) return;
    const int q = e / per, k = e % per;
    double s = 0.0;
    if (k < G_NX * G_NX) {
        const int a = k / G_NX, b = k % G_NX;
        for (int v = 0; v < Hd; ++v) {
            const double ca = g_coef(q, v, a, Hd);
            if (ca != 0.0) s += ca * g_coef(q, v, b, Hd);
        }
    } else {
        const int a = k - G_NX * G_NX;
        for (int v = 0; v < Hd; ++v) s += g_coef(q, v, a, Hd);
    }
    gq[e] = s;
}

#ifdef ATHD_GR_STAMP
// measurement build only (-DATHD_GR_STAMP): per wave, s_memtime cycles summed over its tiles per phase (0 flush + Z
// MFMA + the previous tile's 4-tap stores, 1 first barrier, 2 ZT / Zs stores + second barrier, 3 Zs prefetch, 4 Gram),
// tile count, span ->
// g_gr_stamp[block][wave][8]; read back with athd_gr_stamps
__device__ uint64_t g_gr_stamp[1024 * 8 * 8];
#define GR_MARK(k) do { const uint64_t now_ = __builtin_amdgcn_s_memtime(); ph_[k] += now_ - tp_; tp_ = now_; } while (0)
#else
#define GR_MARK(k) do { } while (0)
#endif

__global__ __launch_bounds__(G_THREADS, 1) void fdec1_gram_kernel(const LowRankDesc d, float* gram, float* part,
                                                                    int kmax) {
    __shared__ __attribute__((aligned(16))) char smem[G_LDS];
    char* const bl = smem;                                    // weights
    char* const zt = smem + G_B_BYTES;                        // ZT
    char* const zsl = zt + G_ZT_BYTES;                        // Zs

    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nblk = (int)gridDim.x;
    const int L = g_xcd_remap((int)blockIdx.x, nblk);
    const int g = L % G_NG, qi = L / G_NG, Qg = (nblk - 1 - g) / G_NG + 1;
    const int c0 = g * G_CG;
    const int W = d.W;
    const int NWB = (W + G_WB - 1) / G_WB;
    const int T = d.NI * NWB;                      // (< 2^31: fdec1_gram_supported)
    const int t_beg = (int)((int64_t)T * qi / Qg), t_end = (int)((int64_t)T * (qi + 1) / Qg);
    const bf16_t* const S = (const bf16_t*)d.S;
    const bf16_t* const Wt = (const bf16_t*)d.Wt;
    const bf16_t* const Zs = (const bf16_t*)d.Zs;
    bf16_t* const z4 = (bf16_t*)d.z4;

    // ---- weights of this channel group -> LDS (column t * 16 + c = weight row t * 96 + c0 + c) ----
    for (int idx = tid; idx < 128 * 24; idx += G_THREADS) {
        const int col = idx / 24, qq = idx % 24;
        const int wrow = (col >> 4) * G_CO + c0 + (col & 15);
        const uint4 v = *reinterpret_cast<const uint4*>(Wt + (int64_t)wrow * d.w_ld + qq * 8);
        *reinterpret_cast<uint4*>(bl + col * 384 + ((qq ^ ((col >> 1) & 7)) << 4)) = v;
    }

    // ---- Z GEMM operands: this wave's tile rows 32 wv .. +31 ----
    bf16x8_t sf[2][6];
    // a tile's first column: the last tile of an item is shifted left to end at W (W >= G_WB), so that every load and
    // store of a tile is in range and unconditional (no per-lane branches: the wait counters stay exact across the
    // loop); its columns the previous tile already covered are masked out of the Gram operands and their Z stored
    // again (the same values)
    auto w_first = [&](int t) { return min((t % NWB) * G_WB, W - G_WB); };
    auto s_row = [&](int t, int i) {              // this lane's S row of row block i of tile t
        const int n = t / NWB, w0 = w_first(t);
        const int R = (2 * wv + i) * 16 + (lane & 15);
        const int j = R >> 3, w = w0 + (R & 7);
        return S + (((int64_t)n * G_HS + j) * W + w) * G_CI + 8 * (lane >> 4);
    };
    // Zs rows of a tile: 1024 pieces of 16 B (t, m, wl, half), two per thread (adjacent halves: the second is the
    // first + 16 B).  Two named registers, not an array: a private array is promoted to LDS by the compiler
    uint4 zsr0, zsr1;
    const int zs_tm = tid >> 3, zs_wl = tid & 7;
    auto load_zs = [&](int t) {
        const int n = t / NWB, w = w_first(t) + zs_wl, seg = n / d.P;
        const int tp = zs_tm >> 3, m = zs_tm & 7;
        const bf16_t* p = Zs + (((int64_t)seg * G_HK + m) * W + w) * (8 * G_CO) + tp * G_CO + c0;
        zsr0 = *reinterpret_cast<const uint4*>(p);
        zsr1 = *reinterpret_cast<const uint4*>(p + 8);
    };

    // ---- Gram roles ----
    const int gq = wv >> 1, gh = wv & 1;
    // one-hot channel matrix as the B operand: lane n = lane & 15 (channel), k = 8 (lane >> 4) + e is channel
    // 8 ((lane >> 4) & 1) + e of the K index (wl, c)
    bf16x8_t onehot;
    {
        const int e = (lane & 15) - 8 * ((lane >> 4) & 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) onehot[i] = (short)(i == e ? 0x3F80 : 0);
    }
    f32x4_t gacc[G_NBLK];
#pragma unroll
    for (int b = 0; b < G_NBLK; ++b) gacc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // the item's partial slot of this workgroup (slot n - first item of the range), the accumulators as they are held
    const int n_first = t_beg / NWB;
    auto flush = [&](int n) {
        f32x4_t* const pb = reinterpret_cast<f32x4_t*>(part + ((int64_t)L * kmax + (n - n_first)) * G_PSLOT) +
                            wv * G_NBLK * 64 + lane;
#pragma unroll
        for (int b = 0; b < G_NBLK; ++b) {
            pb[b * 64] = gacc[b];
            gacc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
    };

    int n_cur = -1;
    if (t_beg < t_end) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const bf16_t* p = s_row(t_beg, i);
#pragma unroll
            for (int ks = 0; ks < 6; ++ks) sf[i][ks] = *reinterpret_cast<const bf16x8_t*>(p + ks * 32);
        }
        load_zs(t_beg);
        // four stores of zeros to a scratch slot after the Gram rows, in the place of the loop's four 4-tap stores:
        // the compiler's wait counts at the loop head are the minimum over its entry and back edge, so without them
        // every tile's first S fragments wait for two of the previous tile's stores to complete
        f32x4_t* const pad = reinterpret_cast<f32x4_t*>(gram + (int64_t)d.NI * G_ITEM) + tid;
#pragma unroll
        for (int k = 0; k < 4; ++k) pad[k * G_THREADS] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();                               // weights visible
#ifdef ATHD_GR_STAMP
    uint64_t ph_[5] = {0, 0, 0, 0, 0};
    const uint64_t t0_ = __builtin_amdgcn_s_memtime();
    uint64_t tp_ = t0_;
#endif

    for (int t = t_beg; t < t_end; ++t) {
        const int n = t / NWB, w0 = w_first(t), skip = (t % NWB) * G_WB - w0;   // skip: columns already covered
        if (n != n_cur) {
            if (n_cur >= 0) flush(n_cur);
            n_cur = n;
        }
        // 1. Z tile (fp32 accumulators).  Each K-step's S fragments are reloaded with the NEXT tile's as soon as its
        //    MFMAs have issued, so those loads have the rest of this tile (barriers, LDS stores, Gram) to arrive
        //    without a second register set (the last tile reloads its own rows: harmless)
        const bf16_t* const pn0 = s_row(t + 1 < t_end ? t + 1 : t, 0);
        const bf16_t* const pn1 = s_row(t + 1 < t_end ? t + 1 : t, 1);
        f32x4_t acc[2][8];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) acc[i][cb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) {
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {
                const int col = cb * 16 + (lane & 15);
                const int qq = ks * 4 + (lane >> 4);
                const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(bl + col * 384 + ((qq ^ ((col >> 1) & 7)) << 4));
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, sf[i][ks], acc[i][cb], 0, 0, 0);
            }
            sf[0][ks] = *reinterpret_cast<const bf16x8_t*>(pn0 + ks * 32);
            sf[1][ks] = *reinterpret_cast<const bf16x8_t*>(pn1 + ks * 32);
        }
        // 2. -> LDS as bf16 (the rounding of the stored Z of the unfused path), once the previous tile's Gram reads
        //    are done
        GR_MARK(0);
        __syncthreads();
        GR_MARK(1);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int R = (2 * wv + i) * 16 + (lane & 15);
            const int j = R >> 3, wl = R & 7;
            const int c = 4 * (lane >> 4);
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {
                uint2 v;
                v.x = pack2bf(acc[i][cb][0], acc[i][cb][1]);
                v.y = pack2bf(acc[i][cb][2], acc[i][cb][3]);
                *reinterpret_cast<uint2*>(zt + swz(cb * 32 + j, wl * 2 + (c >> 3)) + ((c >> 2) & 1) * 8) = v;
            }
        }
        {
            const int tp = zs_tm >> 3, m = zs_tm & 7, row = (tp & 3) * 16 + (tp >> 2) * 8 + m;
            *reinterpret_cast<uint4*>(zsl + swz(row, zs_wl * 2)) = zsr0;
            *reinterpret_cast<uint4*>(zsl + swz(row, zs_wl * 2 + 1)) = zsr1;
        }
        __syncthreads();
        GR_MARK(2);
        load_zs(t + 1 < t_end ? t + 1 : t);
        GR_MARK(3);
        // 3. Gram blocks of class gq over this tile's K = (wl, c): X row block ri = 16 consecutive LDS rows starting
        //    at a multiple of 16, so the swizzle key of its row l & 15 is l & 15
        auto gram_tile = [&](auto H) {             // H: this wave's half of the class blocks (compile time)
            constexpr int h = decltype(H)::value;
            constexpr int nbh = G_NBLK;
#pragma unroll 1
            for (int ks = 0; ks < 4; ++ks) {
                const int chunk = ks * 4 + (lane >> 4), row = lane & 15;
                const bool kill = (chunk >> 1) < skip;            // K = (wl, c): a column the previous tile covered
                bf16x8_t xf[5];
#pragma unroll
                for (int ri = 0; ri < 5; ++ri) {
                    const char* base =
                        ri < 4 ? zt + ((ri < 2 ? gq : gq + 4) * 32 + (ri & 1) * 16) * 256 : zsl + gq * 16 * 256;
                    xf[ri] = *reinterpret_cast<const bf16x8_t*>(base + row * 256 + ((chunk ^ row) << 4));
                    if (kill) xf[ri] = bf16x8_t{};
                }
#pragma unroll
                for (int b = 0; b < nbh; ++b) {
                    const int ri = blk_r(h, b), ci = blk_c(h, b);
                    gacc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[ri], ci < 5 ? xf[ci] : onehot, gacc[b], 0, 0, 0);
                }
            }
        };
        if (gh == 0) gram_tile(std::integral_constant<int, 0>{});
        else gram_tile(std::integral_constant<int, 1>{});
        GR_MARK(4);
        // the merge pass's Z (taps 0, 3, 4, 7) from the tile in LDS as [n][j][w][group][4][16] (128 B per (j, w) of
        // this group, its 8 pieces in one store instruction; each 16-lane LDS read phase takes 16 chunks of one ZT
        // row), after the Gram MFMAs (issued earlier they queue behind the S / Zs prefetch loads and hold the Gram
        // back) and after those loads, so that waiting for them does not wait for these stores: 2048 pieces of 16 B,
        // four per thread
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = tid + k * G_THREADS;
            const int hf = p & 1, wl = (p >> 1) & 7, ti = (p >> 4) & 3, j = p >> 6;   // 16 lanes: one row
            const int tp = (ti >> 1) * 4 + (ti & 1) * 3;                                // taps 0, 3, 4, 7
            const uint4 v = *reinterpret_cast<const uint4*>(zt + swz(tp * 32 + j, wl * 2 + hf));
            *reinterpret_cast<uint4*>(z4 + (((int64_t)n * G_HS + j) * W + w0 + wl) * (4 * G_CO) + g * 64 + ti * 16 +
                                      hf * 8) = v;
        }
    }
    if (n_cur >= 0) flush(n_cur);
#ifdef ATHD_GR_STAMP
    if (lane == 0) {
        uint64_t* o = g_gr_stamp + ((size_t)blockIdx.x * 8 + wv) * 8;
        for (int k = 0; k < 5; ++k) o[k] = ph_[k];
        o[5] = (uint64_t)(t_end - t_beg);
        o[6] = tp_ - t0_;
        o[7] = 1;
    }
#endif
}

// item n's Gram blocks from the partial slots of the workgroups whose tile ranges meet the item, summed in a fixed
// order (channel group, then range): one thread per accumulator register quadruple (wave, block, lane) of a slot.
// The 5 x 5 upper block triangle is summed over all channel groups; the one-hot blocks (per-channel sums) belong to
// one group each.  Every entry fdec1_gram_final_kernel reads is written here.
__global__ __launch_bounds__(256) void fdec1_gram_reduce_kernel(const float* part, float* gram, int kmax, int T, int Qg,
                                                                int NWB) {
    const int n = blockIdx.y;
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= 8 * G_NBLK * 64) return;
    const int wv = p / (G_NBLK * 64), b = (p / 64) % G_NBLK, lane = p % 64;
    const int gq = wv >> 1, gh = wv & 1, ri = blk_r(gh, b), ci = blk_c(gh, b);
    auto owner = [&](int t) {                          // the range holding tile t
        int q = (int)((int64_t)t * Qg / T);
        while (q + 1 < Qg && g_tb(q + 1, T, Qg) <= t) ++q;
        while (q > 0 && g_tb(q, T, Qg) > t) --q;
        return q;
    };
    const int q_lo = owner(n * NWB), q_hi = owner(n * NWB + NWB - 1);
    float* const gb = gram + ((int64_t)n * 4 + gq) * G_NX * G_NB;
    f32x4_t tot = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int g = 0; g < G_NG; ++g) {
        f32x4_t sg = f32x4_t{0.f, 0.f, 0.f, 0.f};
        for (int qi = q_lo; qi <= q_hi; ++qi) {
            const int tb = g_tb(qi, T, Qg);
            if (tb >= g_tb(qi + 1, T, Qg)) continue;   // an empty range flushed nothing
            const int L = qi * G_NG + g, k = n - tb / NWB;
            const f32x4_t v = *(reinterpret_cast<const f32x4_t*>(part + ((int64_t)L * kmax + k) * G_PSLOT) + p);
            sg[0] += v[0]; sg[1] += v[1]; sg[2] += v[2]; sg[3] += v[3];
        }
        if (ci == 5) {                                 // this group's channel columns
            const int col = G_NX + g * G_CG + (lane & 15);
#pragma unroll
            for (int i = 0; i < 4; ++i) gb[(ri * 16 + 4 * (lane >> 4) + i) * G_NB + col] = sg[i];
        } else {
            tot[0] += sg[0]; tot[1] += sg[1]; tot[2] += sg[2]; tot[3] += sg[3];
        }
    }
    if (ci < 5) {
        const int col = ci * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) gb[(ri * 16 + 4 * (lane >> 4) + i) * G_NB + col] = tot[i];
    }
}

// {sum, sumsq} of item n from its Gram blocks: one 256-thread block per item
__global__ __launch_bounds__(256) void fdec1_gram_final_kernel(const float* gram, const double* gq, const float* bias,
                                                               double* stats, int Hd, int W) {
    const int n = blockIdx.x, tid = threadIdx.x;
    const float* const gi = gram + (int64_t)n * G_ITEM;
    const int per = G_NX * G_NX + G_NX;
    double s1 = 0.0, s2 = 0.0;
    // <Q_q, G_q> over the upper block triangle (off-diagonal blocks twice)
    for (int e = tid; e < 4 * G_NX * G_NX; e += 256) {
        const int q = e / (G_NX * G_NX), k = e % (G_NX * G_NX), a = k / G_NX, b = k % G_NX;
        const int ra = a >> 4, rb = b >> 4;
        if (ra <= rb) s2 += (ra == rb ? 1.0 : 2.0) * gq[q * per + k] * (double)gi[(q * G_NX + a) * G_NB + b];
    }
    // c1 . u and 2 c1 . ub from the per-channel sums
    for (int e = tid; e < 4 * G_NX; e += 256) {
        const int q = e / G_NX, a = e % G_NX;
        const float* row = gi + (q * G_NX + a) * G_NB + G_NX;
        double u = 0.0, ub = 0.0;
        for (int c = 0; c < G_CO; ++c) {
            u += (double)row[c];
            ub += (double)bias[c] * (double)row[c];
        }
        const double c1 = gq[q * per + G_NX * G_NX + a];
        s1 += c1 * u;
        s2 += 2.0 * c1 * ub;
    }
    if (tid < G_CO) {
        const double b = bias[tid], rows = 4.0 * Hd * W;
        s1 += rows * b;
        s2 += rows * b * b;
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    __shared__ double sh[2][4];
    if ((tid & 63) == 0) { sh[0][tid >> 6] = s1; sh[1][tid >> 6] = s2; }
    __syncthreads();
    if (tid == 0) {
        stats[2 * n] = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
        stats[2 * n + 1] = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    }
}

#ifdef ATHD_GR_STAMP
extern "C" int athd_gr_stamps(void* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gr_stamp), sizeof(uint64_t) * 1024 * 64, 0, hipMemcpyDeviceToHost);
}
#endif

bool fdec1_gram_supported(const LowRankDesc& d) {
    return d.S && d.Wt && d.w_ld >= G_CI && d.w_ld % 8 == 0 && d.Ci == G_CI && d.Co == G_CO && d.Hs == G_HS &&
           d.Hk == G_HK && d.z_bf16 && d.Zs && d.bias && d.stats && d.W >= 1 && d.P >= 1 && d.NI >= 1 &&
           d.NI % d.P == 0 && d.Hd > G_HS && d.Hd < 65536 && d.W >= G_WB &&
           (int64_t)d.NI * ((d.W + G_WB - 1) / G_WB) < (1LL << 31);
}

int64_t fdec1_gram_q_doubles() { return 4 * (G_NX * G_NX + G_NX); }

static int g_blocks() {
    // one workgroup per CU, a multiple of the 6 channel groups: the six workgroups L = 6q .. 6q + 5 (one XCD) then
    // walk the same tile range together and read each S row from HBM once (with 256 the groups' ranges drifted apart:
    // 1.72x the algorithmic bytes, PMC).  The current device's CU count (device_cus, per device id: ADVICE r04 #5)
    int cus = device_cus();
    if (cus < G_NG) cus = 256;
    return cus / G_NG * G_NG;
}

// partial slots per workgroup: the most items one tile range can meet
static int g_kmax(int64_t NI, int W) {
    const int64_t NWB = (W + G_WB - 1) / G_WB, T = NI * NWB, Qg = g_blocks() / G_NG;
    const int64_t len = (T + Qg - 1) / Qg;
    return (int)((len + NWB - 1) / NWB + 1);
}

// the item Gram rows, the prologue's scratch slot, the partial slots
int64_t fdec1_gram_floats(int64_t NI, int W) {
    return NI * G_ITEM + G_THREADS * 16 + (int64_t)g_blocks() * g_kmax(NI, W) * G_PSLOT;
}

int fdec1_gram_launch(const LowRankDesc& d, float* gram, double* gq, hipStream_t s) {
    if (!fdec1_gram_supported(d) || !gram || !gq || !d.z4 || d.z_taps != 4) return -1;
    const int nblk = g_blocks(), kmax = g_kmax(d.NI, d.W);
    float* const part = gram + (int64_t)d.NI * G_ITEM + G_THREADS * 16;
    {
        KScope ks(s);
        if (ks.on()) ks.begin("fdec1_gram_q_kernel", 0.0, (double)fdec1_gram_q_doubles() * 8.0);
        const int ne = (int)fdec1_gram_q_doubles();
        hipLaunchKernelGGL(fdec1_gram_q_kernel, dim3((ne + 255) / 256), dim3(256), 0, s, gq, d.Hd);
        HIP_CHECK_RET(hipGetLastError());
    }
    {
        KScope ks(s);
        if (ks.on()) {
            // algorithmic: S (read once), Zs (once per segment), the Gram rows (written once per item); flops: the
            // 8-tap Z GEMM + the Gram blocks (20 per class)
            const double rows = (double)d.NI * G_HS * d.W;
            const double by = rows * G_CI * 2.0 + (double)(d.NI / d.P) * G_HK * d.W * 8.0 * G_CO * 2.0 +
                              (double)d.NI * G_ITEM * 4.0 + (d.z4 ? rows * 4.0 * G_CO * 2.0 : 0.0);
            const double fl = 2.0 * rows * G_CI * 8 * G_CO + 2.0 * (double)d.NI * d.W * G_CO * 4 * 20 * 256;
            ks.begin("fdec1_gram_kernel", fl, by);
        }
        hipLaunchKernelGGL(fdec1_gram_kernel, dim3(nblk), dim3(G_THREADS), 0, s, d, gram, part, kmax);
        HIP_CHECK_RET(hipGetLastError());
    }
    {
        KScope ks(s);
        const int NWB = (d.W + G_WB - 1) / G_WB;
        if (ks.on()) ks.begin("fdec1_gram_reduce_kernel", 0.0, (double)nblk * kmax * G_PSLOT * 4.0 + d.NI * G_ITEM * 4.0);
        hipLaunchKernelGGL(fdec1_gram_reduce_kernel, dim3((8 * G_NBLK * 64 + 255) / 256, d.NI), dim3(256), 0, s, part,
                           gram, kmax, d.NI * NWB, nblk / G_NG, NWB);
        HIP_CHECK_RET(hipGetLastError());
    }
    {
        KScope ks(s);
        if (ks.on()) ks.begin("fdec1_gram_final_kernel", 0.0, (double)d.NI * G_ITEM * 4.0);
        hipLaunchKernelGGL(fdec1_gram_final_kernel, dim3(d.NI), dim3(256), 0, s, gram, gq, d.bias, d.stats, d.Hd, d.W);
        HIP_CHECK_RET(hipGetLastError());
    }
    return 0;
}

}  // namespace athd
