// Decoder level-2 ConvTranspose (k8, s4, p2; 96 -> 48 channels) with all four output residues in one pass, bf16
// mode (ATHTDemucs_v2.py:82-104 / 125-139 -> demucs HDecLayer.conv_tr).
//
//   out row 4u+rho of item b = sum over the two input rows u-1, u (rho = 0, 1) or u, u+1 (rho = 2, 3) of
//   x[b][row][w][:] . W_rho[tap], + bias;  GroupNorm(1) statistics over all four residues.
//
// As a GEMM this is M = NI*H*W rows, K = 3 taps x 96 (one third zero per residue pair), N = 4 x 48: five 64-wide
// K-steps per 256-row tile, so the tiled GEMM (gemm3, 2-stage LDS ring, barrier per K-step) spent its time on load
// latency and barriers (MFMA busy 15 %, waits 44 %).  Here:
//   - the weights of both residue pairs ([2][96][192] bf16, 72 KB) are loaded into LDS ONCE per workgroup
//     (XOR-swizzled 16-B chunks: conflict-free ds_read_b128 fragments) and stay there;
//   - activations go global -> VGPR directly as MFMA B fragments (16 B per lane: row m, 8 channels), three taps
//     per row (rows m - W, m, m + W; the tap re-reads hit L2: the XCD's waves work on neighbouring rows);
//   - every wave owns whole 32-row units (2 row fragments x all 192 output columns = 96 accumulators) and walks
//     its units with NO workgroup barrier; the next unit's tap fragments are loaded tap by tap as soon as the
//     current unit has consumed them, so about one unit of loads is in flight per wave across the epilogue.
//   - epilogue: bias, per-lane fp32 statistics per unit folded into fp64 running sums per item (flushed once per
//     item change: wave reduction + one fp64 atomic pair), bf16 8-B stores of the stored residues.
// keep = 1 (freq level 2): only residues 1, 2 are stored, as rows 2t, 2t+1 (the rows a following /4 bilinear
// resize reads); keep = 0 (time level 2): all four, as rows 4t + rho.  Row t = (b, u) = m / W, column w = m % W.
#include <cstdlib>

#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "kernels.h"


namespace athd {

namespace {

constexpr int CT_CI = 96, CT_CO = 48;
constexpr int CT_KP = 2 * CT_CI;           // pair-local K: [lower tap row | upper tap row]
constexpr int CT_WROW = CT_KP * 2;         // 384 B per weight row in LDS

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;

__device__ __attribute__((aligned(64))) uint4 g_zero_ct4[4];
__device__ uint2 g_sink_ct4[64];          // store target of rows past M (branch-free epilogue)

}  // namespace

// RF row fragments (16 rows each) per wave unit, NW waves per workgroup (one workgroup per CU)
template <bool KEEP, int RF, int NW>
__global__ __launch_bounds__(NW * 64) void convt4_kernel(const ConvT4Desc d) {
    constexpr int CT_NW = NW, CT_UNIT = 16 * RF;
    __shared__ __attribute__((aligned(16))) char wl[4 * CT_CO * CT_WROW];   // 73,728 B
    // weights: global [192 rows][24 chunks of 16 B] -> LDS chunk c of row n at (c ^ (n & 7))
    for (int c = threadIdx.x; c < 4 * CT_CO * 24; c += CT_NW * 64) {
        const int n = c / 24, ch = c - 24 * (c / 24);
        const uint4 v = reinterpret_cast<const uint4*>(d.w)[c];
        *reinterpret_cast<uint4*>(wl + n * CT_WROW + ((ch ^ (n & 7)) * 16)) = v;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int fr = lane & 15, g = lane >> 4;
    const uint32_t M = d.M;
    const int nunits = (int)((M + CT_UNIT - 1) / CT_UNIT);
    // XCD-aware split: workgroup i runs on XCD i % 8; each XCD owns a contiguous unit range, its waves walk it in
    // lockstep-free strides of (waves on that XCD), so concurrently running waves touch neighbouring rows
    const int xcd = blockIdx.x & 7;
    const int nbx = (int)(gridDim.x >> 3);
    const int ux0 = (int)((int64_t)nunits * xcd / 8), ux1 = (int)((int64_t)nunits * (xcd + 1) / 8);
    const int wx = (int)(blockIdx.x >> 3) * CT_NW + wave, nwx = nbx * CT_NW;
    int unit = ux0 + wx;
    if (unit >= ux1) return;

    // bias of the lane's 4 columns in each of the 3 column fragments of a residue (co = 16 jj + 4 g + q)
    float4 b4[3];
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) b4[jj] = *reinterpret_cast<const float4*>(d.bias + 16 * jj + 4 * g);

    // LDS fragment addresses: row n = 96 p + 16 jj + fr (n & 7 = fr & 7), chunk 4 s + g -> (4 s + g) ^ (fr & 7)
    //   = 8 (s >> 1) + [(s & 1) ? 4 (1 - (fr >> 2 & 1)) : 4 (fr >> 2 & 1)] + (g ^ (fr & 3))
    const int f7 = fr & 7;
    const uint32_t wb_even = (uint32_t)(fr * CT_WROW + (4 * (f7 >> 2) + (g ^ (f7 & 3))) * 16);
    const uint32_t wb_odd = (uint32_t)(fr * CT_WROW + (4 * (1 - (f7 >> 2)) + (g ^ (f7 & 3))) * 16);
    uint32_t wbe = wb_even, wbo = wb_odd;
    // a group's reads may not be scheduled above the previous group's MFMAs (register pressure: 6 fragments live)
    auto fence = [&]() { asm volatile("" : "+v"(wbe), "+v"(wbo)); };
    auto wfrag = [&](int p, int jj, int s) -> bf16v8 {
        const uint32_t a = ((s & 1) ? wbo : wbe) + (uint32_t)((96 * p + 16 * jj) * CT_WROW + 128 * (s >> 1));
        return *reinterpret_cast<const bf16v8*>(wl + a);
    };

    const char* const xb = reinterpret_cast<const char*>(d.x);
    const char* const zero = reinterpret_cast<const char*>(g_zero_ct4);
    const int64_t rowW = (int64_t)d.W * (CT_CI * 2);      // bytes between input rows u and u+1
    const int H = d.H;
    uint2* const sink = g_sink_ct4 + lane;

    // per-unit row state of this lane: row fragment i holds row m0 + 16 i + fr
    struct Rows {
        int64_t off[RF];     // byte offset of the row in x (clamped to row 0 past M)
        bool ok[RF], lo[RF], hi[RF];
        uint32_t m[RF], w[RF];
    };
    auto setup = [&](int u, bool valid, Rows& r) {
#pragma unroll
        for (int i = 0; i < RF; ++i) {
            const uint32_t m = (uint32_t)u * CT_UNIT + 16 * i + fr;
            const bool ok = valid && m < M;
            const uint32_t mm = ok ? m : 0u;
            const uint32_t t = fdiv(mm, d.fd_w);
            const uint32_t w = mm - t * (uint32_t)d.W;
            const uint32_t b = fdiv(t, d.fd_h);
            const uint32_t hu = t - b * (uint32_t)H;
            r.off[i] = (int64_t)mm * (CT_CI * 2);
            r.ok[i] = ok;
            r.lo[i] = ok && hu >= 1u;
            r.hi[i] = ok && (int)hu <= H - 2;
            r.m[i] = m;
            r.w[i] = w;
        }
    };
    // tap fragments: tap 0 = row u-1, 1 = row u, 2 = row u+1; F[i][s3] = channels 32 s3 + 8 g .. + 7
    auto load_tap = [&](const Rows& r, int tap, bf16v8 (&F)[RF][3]) {
#pragma unroll
        for (int i = 0; i < RF; ++i) {
            const bool ok = tap == 0 ? r.lo[i] : tap == 2 ? r.hi[i] : r.ok[i];
            const char* p = ok ? xb + r.off[i] + (int64_t)(tap - 1) * rowW + 16 * g : zero;
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3)
                F[i][s3] = *reinterpret_cast<const bf16v8*>(ok ? p + 64 * s3 : p);
        }
    };

    f32x4_t acc[RF][6];
    bf16v8 Fl[RF][3], Fc[RF][3], Fh[RF][3];
    Rows rc, rn;
    setup(unit, true, rc);
    load_tap(rc, 0, Fl);
    load_tap(rc, 1, Fc);
    load_tap(rc, 2, Fh);

    // running GroupNorm sums of the item cur_b (per lane, fp64)
    int cur_b = -1;
    double r1 = 0.0, r2 = 0.0;
    auto flush = [&]() {
        if (cur_b >= 0) {
            const double t1 = wave_sum_d(r1), t2 = wave_sum_d(r2);
            if (lane == 0) {
                atomicAdd(&d.stats[2 * cur_b], t1);
                atomicAdd(&d.stats[2 * cur_b + 1], t2);
            }
        }
        r1 = 0.0;
        r2 = 0.0;
    };
    const uint32_t HW = (uint32_t)H * (uint32_t)d.W;
    const f32x4_t z4 = {0.f, 0.f, 0.f, 0.f};
    // acc = W_p[:, 3 h .. 3 h + 2] . F (K sub-steps 3h + s of residue pair p), F = the pair's lower (h = 0) / upper
    // (h = 1) tap
    auto mma = [&](int p, int h, const bf16v8 (&F)[RF][3]) {
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            fence();
#pragma unroll
            for (int jj = 0; jj < 6; ++jj) {
                const bf16v8 wf = wfrag(p, jj, 3 * h + s);
#pragma unroll
                for (int i = 0; i < RF; ++i)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, F[i][s], (h == 0 && s == 0) ? z4 : acc[i][jj], 0, 0, 0);
            }
        }
    };
    float s1a = 0.f, s2a = 0.f, s1b = 0.f, s2b = 0.f;      // this unit's statistics: item bf / item bl rows
    uint32_t split = 0;
    // residue pair p's epilogue: bias, statistics, bf16 stores of its stored residues
    auto epilogue = [&](int p) {
#pragma unroll
        for (int i = 0; i < RF; ++i) {
            const bool ok = rc.ok[i];
            // element offset of (row t, residue rho, column w, channel 0):
            //   keep: rows 2t + rho - 1 -> (2 t W + w) + (rho - 1) W = 2 m - w + (rho - 1) W
            //   all : rows 4t + rho     -> (4 t W + w) + rho W     = 4 m - 3 w + rho W
            const int64_t mrow = KEEP ? (int64_t)2 * rc.m[i] - rc.w[i] : (int64_t)4 * rc.m[i] - 3 * (int64_t)rc.w[i];
            bf16_t* const ob = d.out + mrow * CT_CO + 4 * g;
            float p1 = 0.f, p2 = 0.f;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int rho = 2 * p + j / 3, jj = j - 3 * (j / 3);
                const float4 bb = b4[jj];
                const float v0 = acc[i][j][0] + bb.x, v1 = acc[i][j][1] + bb.y;
                const float v2 = acc[i][j][2] + bb.z, v3 = acc[i][j][3] + bb.w;
                p1 += (v0 + v1) + (v2 + v3);
                p2 += (v0 * v0 + v1 * v1) + (v2 * v2 + v3 * v3);
                if (KEEP ? (rho == 1 || rho == 2) : true) {     // (compile-time) stored residue
                    const int64_t ro = KEEP ? (int64_t)(rho - 1) * d.W : (int64_t)rho * d.W;
                    uint2* dst = ok ? reinterpret_cast<uint2*>(ob + ro * CT_CO + 16 * jj) : sink;   // branch-free
                    *dst = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
                }
            }
            p1 = ok ? p1 : 0.f;
            p2 = ok ? p2 : 0.f;
            const bool inb = rc.m[i] >= split;
            s1a += inb ? 0.f : p1;
            s2a += inb ? 0.f : p2;
            s1b += inb ? p1 : 0.f;
            s2b += inb ? p2 : 0.f;
        }
    };

    for (;;) {
        asm volatile("" : "+v"(wbe), "+v"(wbo));   // (weight fragment reads stay in the loop, not hoisted)
        const int next = unit + nwx;
        const bool has_next = next < ux1;
        setup(next, has_next, rn);     // (past the range: every load of the prefetch reads the zero page)
        const uint32_t m0 = (uint32_t)unit * CT_UNIT;
        const uint32_t mlast = m0 + CT_UNIT - 1 < M ? m0 + CT_UNIT - 1 : M - 1;
        const int bf = (int)fdiv(m0, d.fd_hw), bl = (int)fdiv(mlast, d.fd_hw);
        split = (uint32_t)(bf + 1) * HW;           // rows >= split belong to item bl (when bl > bf)
        s1a = s2a = s1b = s2b = 0.f;
        // residue pair 0 (residues 0, 1): rows u-1, u
        mma(0, 0, Fl);
        load_tap(rn, 0, Fl);
        mma(0, 1, Fc);
        epilogue(0);
        // residue pair 1 (residues 2, 3): rows u, u+1
        mma(1, 0, Fc);
        load_tap(rn, 1, Fc);
        mma(1, 1, Fh);
        load_tap(rn, 2, Fh);
        epilogue(1);
        if (bf != cur_b) {
            flush();
            cur_b = bf;
        }
        r1 += (double)s1a;
        r2 += (double)s2a;
        if (bl != bf) {
            flush();
            cur_b = bl;
            r1 = (double)s1b;
            r2 = (double)s2b;
        }
        if (!has_next) break;
        unit = next;
        rc = rn;
    }
    flush();
}

// ---------------------------------------------------------------------------------------------------------------
// Column walk (W >= 16 RF, the frequency branch: H = W = Tspec; round 5).  The unit kernel above reads every input
// row three times (as tap u-1, u and u+1 of three units 259 rows apart) and relied on L2 for the re-reads; with the
// waves of an XCD drifting apart, PMC showed 1.29x the algorithmic HBM bytes.  Here a wave owns a column block (item
// b, 16 RF consecutive w) and a segment of rows u0 .. u1-1 and walks it row by row: the tap fragments of rows u-1, u,
// u+1 are kept in three register sets that rotate, so each step loads ONE new row (u+2) - every input row is read once
// per column block (+ 2 halo rows per segment).  Rows and columns outside the item read zeros (buffer descriptors);
// columns past W are neither stored nor counted.  One residue at a time (3 x RF accumulators live, each weight
// fragment read from LDS feeds RF MFMAs), and the two stored rows of a step leave through a per-wave LDS stage as
// contiguous 16-B-per-lane segments.  GroupNorm statistics: per lane fp32 per step, fp64 across the segment, one fp64
// atomic pair per segment (a segment lies in one item).
// Measured (freq level 2 per forward, serialised events, one box): unit kernel 2.07 ms; walk, RF = 1, 12 waves 2.02
// (HBM bytes 8.48 -> 5.12 GB per launch, time unchanged: not memory-bound); one residue at a time 1.95; RF = 2 at 8
// waves (2 per SIMD; at 12 waves it spills) 1.94; + staged stores 1.82 (staged stores at RF = 1: 1.95).
#ifndef ATHD_CW_RF
#define ATHD_CW_RF 2
#endif
#ifndef ATHD_CW_SEG
#define ATHD_CW_SEG 14
#endif
#ifndef ATHD_CW_NW
#define ATHD_CW_NW 8
#endif
constexpr int CW_RF = ATHD_CW_RF, CW_NW = ATHD_CW_NW, CW_SEG = ATHD_CW_SEG;  // 32-wide column blocks, 8 waves per workgroup, 14 row segments
template <bool KEEP>
__global__ __launch_bounds__(CW_NW * 64) void convt4_walk_kernel(const ConvT4Desc d) {
    constexpr int RF = CW_RF;
    constexpr int OSB = 16 * RF * CT_CO * 2;      // bytes of one stored output row segment of a wave (16 RF columns)
    __shared__ __attribute__((aligned(16))) char wl[4 * CT_CO * CT_WROW];   // 73,728 B
    // KEEP: per wave the two stored rows of a step ([2][16 RF columns][48] bf16), written to HBM as whole contiguous
    // segments (16 B per lane) instead of 32-B pieces at a 96-B stride (16 per store instruction)
    __shared__ __attribute__((aligned(16))) char ostg[KEEP ? CW_NW : 1][2 * OSB];
    for (int c = threadIdx.x; c < 4 * CT_CO * 24; c += CW_NW * 64) {
        const int n = c / 24, ch = c - 24 * (c / 24);
        const uint4 v = reinterpret_cast<const uint4*>(d.w)[c];
        *reinterpret_cast<uint4*>(wl + n * CT_WROW + ((ch ^ (n & 7)) * 16)) = v;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int fr = lane & 15, g = lane >> 4;
    const int H = d.H, W = d.W;
    const int nwb = (W + 16 * RF - 1) / (16 * RF);
    const int items = d.nb * nwb * CW_SEG;
    // items in (segment, w block, item b) order, each XCD a contiguous range (neighbouring column blocks share the
    // L2 lines of a row: 32 x 192 B = 6 KB of each 50-KB row); waves of the XCD stride through it
    const int xcd = blockIdx.x & 7;
    const int nwx = (int)(gridDim.x >> 3) * CW_NW;
    const int i0 = (int)((int64_t)items * xcd / 8), i1 = (int)((int64_t)items * (xcd + 1) / 8);
    int it = i0 + (int)(blockIdx.x >> 3) * CW_NW + wave;
    if (it >= i1) return;

    float4 b4[3];
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) b4[jj] = *reinterpret_cast<const float4*>(d.bias + 16 * jj + 4 * g);
    const int f7 = fr & 7;
    const uint32_t wb_even = (uint32_t)(fr * CT_WROW + (4 * (f7 >> 2) + (g ^ (f7 & 3))) * 16);
    const uint32_t wb_odd = (uint32_t)(fr * CT_WROW + (4 * (1 - (f7 >> 2)) + (g ^ (f7 & 3))) * 16);
    uint32_t wbe = wb_even, wbo = wb_odd;
    auto fence = [&]() { asm volatile("" : "+v"(wbe), "+v"(wbo)); };
    auto wfrag = [&](int p, int jj, int s) -> bf16v8 {
        const uint32_t a = ((s & 1) ? wbo : wbe) + (uint32_t)((96 * p + 16 * jj) * CT_WROW + 128 * (s >> 1));
        return *reinterpret_cast<const bf16v8*>(wl + a);
    };
    const char* const xb = reinterpret_cast<const char*>(d.x);
    const char* const zero = reinterpret_cast<const char*>(g_zero_ct4);
    const f32x4_t z4 = {0.f, 0.f, 0.f, 0.f};
    // one residue rho at a time (its 3 channel tiles: pair p = rho / 2, pair-local tiles 3 (rho & 1) ..): each weight
    // fragment feeds RF MFMAs, and only 3 x RF accumulators are live
    f32x4_t acc[RF][3];
    auto mma = [&](int rho, int h, const bf16v8 (&F)[RF][3]) {
        const int p = rho >> 1, j0 = 3 * (rho & 1);
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            fence();
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                const bf16v8 wf = wfrag(p, j0 + jj, 3 * h + s);
#pragma unroll
                for (int i = 0; i < RF; ++i)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, F[i][s], (h == 0 && s == 0) ? z4 : acc[i][jj], 0, 0, 0);
            }
        }
    };

    for (;;) {
        const int seg = it / (d.nb * nwb), rem = it - seg * (d.nb * nwb);
        const int wblk = rem / d.nb, b = rem - wblk * d.nb;
        const int u0 = (int)((int64_t)H * seg / CW_SEG), u1 = (int)((int64_t)H * (seg + 1) / CW_SEG);
        // this lane's columns w = 32 wblk + 16 i + fr: per-lane byte offsets (32 bits) from the item's wave-uniform
        // row bases, which carry the row index
        uint32_t cin_off[RF], cout_off[RF];
        bool cok[RF];
#pragma unroll
        for (int i = 0; i < RF; ++i) {
            const int cw = 16 * RF * wblk + 16 * i + fr;
            cok[i] = cw < W;
            cin_off[i] = (uint32_t)(cok[i] ? cw : 0) * (CT_CI * 2) + 16 * g;
            cout_off[i] = (uint32_t)(cok[i] ? cw : 0) * (CT_CO * 2) + 8 * g;
        }
        const char* const xitem = xb + (int64_t)b * H * W * (CT_CI * 2);
        char* const oitem = reinterpret_cast<char*>(d.out) + (int64_t)b * H * (KEEP ? 2 : 4) * W * (CT_CO * 2);
        const int64_t rowB = (int64_t)W * (CT_CI * 2), orowB = (int64_t)W * (CT_CO * 2);
        const int ocol0 = 16 * RF * wblk * (CT_CO * 2);                       // the segment's byte offset in a row
        const int ovalid = min(16 * RF, W - 16 * RF * wblk) * (CT_CO * 2);   // its stored bytes
        // row u through a buffer descriptor of that row (wave-uniform): a row outside the item has zero records and a
        // column past W an out-of-range offset, so those loads return zeros (no per-lane 64-bit address selects)
        uint32_t lofs[RF];
#pragma unroll
        for (int i = 0; i < RF; ++i) lofs[i] = cok[i] ? cin_off[i] : 0x40000000u;
        auto load_row = [&](int u, bf16v8 (&F)[RF][3]) {
            const bool uok = u >= 0 && u < H;                 // (wave-uniform)
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(xitem + (uok ? (int64_t)u * rowB : 0)), (short)0, uok ? (int)rowB : 0, 0x00020000);
#pragma unroll
            for (int i = 0; i < RF; ++i)
#pragma unroll
                for (int s3 = 0; s3 < 3; ++s3)
                    F[i][s3] = __builtin_bit_cast(bf16v8, __builtin_amdgcn_raw_buffer_load_b128(rs, lofs[i] + 64 * s3, 0, 0));
        };
        double r1 = 0.0, r2 = 0.0;
        // one row u with taps (Fa, Fb, Fc) = rows (u-1, u, u+1); Fa is refilled with row u+2 once pair 0 is done
        auto step = [&](int u, bf16v8 (&Fa)[RF][3], bf16v8 (&Fb)[RF][3], bf16v8 (&Fc)[RF][3]) {
            float p1 = 0.f, p2 = 0.f;
            auto epi = [&](int rho) {
#pragma unroll
                for (int i = 0; i < RF; ++i) {
#pragma unroll
                    for (int jj = 0; jj < 3; ++jj) {
                        const float4 bb = b4[jj];
                        const float v0 = acc[i][jj][0] + bb.x, v1 = acc[i][jj][1] + bb.y;
                        const float v2 = acc[i][jj][2] + bb.z, v3 = acc[i][jj][3] + bb.w;
                        const float q1 = (v0 + v1) + (v2 + v3), q2 = (v0 * v0 + v1 * v1) + (v2 * v2 + v3 * v3);
                        p1 += cok[i] ? q1 : 0.f;
                        p2 += cok[i] ? q2 : 0.f;
                        if constexpr (KEEP) {
                            if (rho == 1 || rho == 2)     // staged: row segment rho - 1, column 16 i + fr
                                *reinterpret_cast<uint2*>(ostg[wave] + (rho - 1) * OSB + (16 * i + fr) * (CT_CO * 2) +
                                                          32 * jj + 8 * g) = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
                        } else {
                            // output row 4u + rho of the item: a wave-uniform base
                            const char* ob = oitem + (int64_t)(4 * u + rho) * orowB;
                            if (cok[i])
                                *reinterpret_cast<uint2*>((char*)ob + cout_off[i] + 32 * jj) =
                                    make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
                        }
                    }
                }
            };
            // residues 0, 1 read rows u-1, u (Fa, Fb); 2, 3 read u, u+1 (Fb, Fc).  Fa is free after residue 1.
            mma(0, 0, Fa);
            mma(0, 1, Fb);
            epi(0);
            mma(1, 0, Fa);
            load_row(u + 2, Fa);                  // (row u+2 is the next step's upper tap)
            mma(1, 1, Fb);
            epi(1);
            mma(2, 0, Fb);
            mma(2, 1, Fc);
            epi(2);
            if constexpr (KEEP) {
                // the staged rows 2u, 2u + 1 (this wave's segment): 16 B per lane, columns past W not stored
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int k = 0; k < 2 * OSB / (16 * 64); ++k) {
                    const int c = lane + 64 * k, r = c / (OSB / 16), wb = (c % (OSB / 16)) * 16;
                    const uint4 v = *reinterpret_cast<const uint4*>(ostg[wave] + r * OSB + wb);
                    if (wb < ovalid)
                        *reinterpret_cast<uint4*>(oitem + (int64_t)(2 * u + r) * orowB + ocol0 + wb) = v;
                }
            }
            mma(3, 0, Fb);
            mma(3, 1, Fc);
            epi(3);
            r1 += (double)p1;
            r2 += (double)p2;
        };
        bf16v8 FA[RF][3], FB[RF][3], FC[RF][3];
        load_row(u0 - 1, FA);
        load_row(u0, FB);
        load_row(u0 + 1, FC);
#pragma unroll 1
        for (int u = u0; u < u1; ++u) {
            asm volatile("" : "+v"(wbe), "+v"(wbo));   // (weight fragment reads stay in the loop, not hoisted)
            step(u, FA, FB, FC);                  // (FA now holds row u + 2)
#pragma unroll
            for (int i = 0; i < RF; ++i)          // rotate the taps: (u-1, u, u+1) <- (u, u+1, u+2)
#pragma unroll
                for (int s3 = 0; s3 < 3; ++s3) {
                    const bf16v8 t = FA[i][s3];
                    FA[i][s3] = FB[i][s3];
                    FB[i][s3] = FC[i][s3];
                    FC[i][s3] = t;
                }
        }
        {
            const double t1 = wave_sum_d(r1), t2 = wave_sum_d(r2);
            if (lane == 0) {
                atomicAdd(&d.stats[2 * b], t1);
                atomicAdd(&d.stats[2 * b + 1], t2);
            }
        }
        it += nwx;
        if (it >= i1) break;
    }
}

// A 32-row unit covers at most two items (its statistics split at one item boundary: bf / bl in the loop above), which
// holds when an item has at least 32 rows, H*W >= 32: Tspec >= 6 for the freq branch (H*W = Tspec^2 after the
// 259 -> Tspec resize), L >= 32 for the time branch.  Shorter inputs take the tiled GEMM (forward.cpp conv_t).
bool convt4_supported(int cin, int cout, int64_t nb, int64_t H, int64_t W) {
    const int64_t M = nb * H * W;
    return cin == CT_CI && cout == CT_CO && H * W >= 32 && M > 0 && M < (1LL << 31);
}

template <bool KEEP, int RF, int NW>
static void launch_ct4(const ConvT4Desc& d, int cus, hipStream_t s) {
    const int64_t nunits = ((int64_t)d.M + 16 * RF - 1) / (16 * RF);
    int64_t blocks = (int64_t)cus;                                  // one workgroup (72 KB LDS) per CU
    const int64_t need = (nunits + NW - 1) / NW;
    if (blocks > need) blocks = need;
    blocks = ((blocks + 7) / 8) * 8;                                // whole XCD rounds
    KScope ks(s);
    if (ks.on()) {
        const double M = (double)d.M;
        const double flops = 2.0 * M * (4 * CT_CO) * CT_KP;          // every residue reads 2 taps x 96
        const double bytes = M * CT_CI * 2 + M * (KEEP ? 2 : 4) * CT_CO * 2 + 4.0 * CT_CO * CT_KP * 2;
        ks.begin(klabel("convt4_kernel<%s,%d,%d>", KEEP ? "true" : "false", RF, NW), flops, bytes);
    }
    hipLaunchKernelGGL((convt4_kernel<KEEP, RF, NW>), dim3((unsigned)blocks), dim3(NW * 64), 0, s, d);
}

int convt4_launch(const ConvT4Desc& d0, hipStream_t s) {
    if (!convt4_supported(CT_CI, CT_CO, d0.nb, d0.H, d0.W)) return -1;
    ConvT4Desc d = d0;
    d.fd_w = make_fastdiv((uint32_t)d.W);
    d.fd_h = make_fastdiv((uint32_t)d.H);
    d.fd_hw = make_fastdiv((uint32_t)d.H * (uint32_t)d.W);
    d.M = (uint32_t)((int64_t)d.nb * d.H * d.W);
    const int cus = device_cus();
    if (d.W >= 16 * CW_RF) {
        // column walk: one workgroup (72 KB of weights + the store stages) per CU, a multiple of 8
        const int64_t items = (int64_t)d.nb * ((d.W + 16 * CW_RF - 1) / (16 * CW_RF)) * CW_SEG;
        int64_t blocks = cus;
        if (blocks * CW_NW > items) blocks = (items + CW_NW - 1) / CW_NW;
        blocks = (blocks + 7) / 8 * 8;
        KScope ks(s);
        if (ks.on()) {
            const double M = (double)d.M;
            const double flops = 2.0 * M * (4 * CT_CO) * CT_KP;
            const double bytes = M * CT_CI * 2 + M * (d.keep ? 2 : 4) * CT_CO * 2 + 4.0 * CT_CO * CT_KP * 2;
            ks.begin(d.keep ? "convt4_walk_kernel<true>" : "convt4_walk_kernel<false>", flops, bytes);
        }
        if (d.keep) hipLaunchKernelGGL(convt4_walk_kernel<true>, dim3((unsigned)blocks), dim3(CW_NW * 64), 0, s, d);
        else hipLaunchKernelGGL(convt4_walk_kernel<false>, dim3((unsigned)blocks), dim3(CW_NW * 64), 0, s, d);
        return (int)hipGetLastError();
    }
    // 2 row fragments per unit, 8 waves (2 per SIMD).  (1 fragment at 12 / 16 waves per workgroup measured slower.)
    if (d.keep) launch_ct4<true, 2, 8>(d, cus, s);
    else launch_ct4<false, 2, 8>(d, cus, s);
    return (int)hipGetLastError();
}

}  // namespace athd
