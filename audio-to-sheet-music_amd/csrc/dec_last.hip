// The last decoder level of both branches as ONE pass over its input, with the 1x1 output projection folded in.
//
// FreqDecoder level 3 (ATHTDemucs_v2.py:76-104 with i = 3, then freq_out :294):
//   ConvTranspose2d(48 -> 4, (8,1), (4,1), (2,0)) -> bilinear H-resize 4*Ts -> Ts -> + 0.1 * resize(saved[0][:, :4])
//   -> Conv2d(4, 2, 1).
//   The resize is an exact /4 (scale 4.0, src = 4d + 1.5): output row d = 0.5 * (y[4d+1] + y[4d+2]), with
//   y[4u+1] = W7 x[u-1] + W3 x[u] and y[4u+2] = W4 x[u] + W0 x[u+1] (k8 s4 p2 residue taps).  The projection P
//   is linear, so FO[d] = Am x[d-1] + A0 x[d] + Ap x[d+1] + 0.1 P skip_r[d] + (P b + pb) with the 2 x 48
//   matrices Am = P W7 / 2, A0 = P (W3 + W4) / 2, Ap = P W0 / 2 folded on the host (athd_finalize).
//   The reference materialises the 4-channel ConvT output (4 x the input rows), resizes it and projects it; here
//   the 48-channel input is read once and 2 floats per output position are written.
// TimeDecoder level 3 (ATHTDemucs_v2.py:125-139 with i = 3, then time_out :314):
//   ConvTranspose1d(48 -> 4, 8, 4, 2) -> linear resize 4*Lin -> T -> + 0.1 * resize(saved_t[0][:, :4]) -> Conv1d(4,2,1).
//   With Q_k = P_t W_k (2 x 48, k = 0..7): z[4u+rho] = Q_{k0} x[u+off] + Q_{k1} x[u+off+1] (RES_K0/RES_K1/RES_OFF of
//   ctx.h), then the resize, the skip term and the biases.  Output xt2[item][n][2] = time_out(...) (incl. its bias),
//   consumed by combine_kernel (denorm + branch sum).
#include "common.h"
#include "kernels.h"
#include "prof.h"

#include <algorithm>

namespace athd {

namespace {

constexpr int DL_C = 48;   // decoder input channels of the last level (DEC_CH[3])

template <typename TX>
ATHD_DEV void ld_row48(const TX* p, float* x) {
    if constexpr (sizeof(TX) == 2) {
#pragma unroll
        for (int q = 0; q < DL_C / 8; ++q) {
            const uint4 v = reinterpret_cast<const uint4*>(p)[q];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                x[8 * q + 2 * e] = __uint_as_float(w[e] << 16);
                x[8 * q + 2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < DL_C / 4; ++q) {
            const float4 v = reinterpret_cast<const float4*>(p)[q];
            x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
        }
    }
}

// 4 leading channels of a skip row (bf16 or f32)
ATHD_DEV void ld_skip4(const void* p, int bf, int64_t off, float* s) {
    if (bf) {
        const uint2 q = *reinterpret_cast<const uint2*>((const bf16_t*)p + off);
        s[0] = __uint_as_float(q.x << 16); s[1] = __uint_as_float(q.x & 0xFFFF0000u);
        s[2] = __uint_as_float(q.y << 16); s[3] = __uint_as_float(q.y & 0xFFFF0000u);
    } else {
        const float4 v = *reinterpret_cast<const float4*>((const float*)p + off);
        s[0] = v.x; s[1] = v.y; s[2] = v.z; s[3] = v.w;
    }
}

// 2-channel projection of a 48-vector by a folded [2][48] matrix (uniform address: scalar loads, SGPR operands)
ATHD_DEV void dot2(const float* m, const float* x, float& o0, float& o1) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int c = 0; c < DL_C; ++c) {
        a = fmaf(m[c], x[c], a);
        b = fmaf(m[DL_C + c], x[c], b);
    }
    o0 = a;
    o1 = b;
}

}  // namespace

// ------------------------------------------------------------------------------------------------- freq level 3
// thread = (item, d-chunk, w); lanes run along w (adjacent 96-B / 192-B input rows: coalesced); each thread slides
// down its FL_DC output rows keeping the pending partial sums in registers.  The folded weights are re-read per
// row through the scalar cache (a compiler barrier per row keeps LICM from hoisting all 288 of them into VGPRs).
constexpr int FL_DC = 16;

template <typename TX>
__global__ __launch_bounds__(256) void fdec_last_kernel(const DecLastDesc d) {
    const int64_t item = blockIdx.y;
    const int64_t seg = item / d.P;
    const int H = d.H, W = d.W;
    const int nch = (H + FL_DC - 1) / FL_DC;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nch * W) return;
    const int w = t % W, c = t / W;
    const int d0 = c * FL_DC;
    const int d1 = min(H, d0 + FL_DC);
    const float* F = d.fold;
    const float* Am = F;
    const float* A0 = F + 2 * DL_C;
    const float* Ap = F + 4 * DL_C;
    const float* cst = F + 6 * DL_C;
    const float* S = F + 6 * DL_C + 2;
    const int64_t sk = seg * d.H_skip * W * d.C_skip;
    const TX* x = reinterpret_cast<const TX*>(d.in) + item * (int64_t)H * W * DL_C + (int64_t)w * DL_C;
    float* fo = d.out + (item * W + w) * (int64_t)H * 2;
    float xr[DL_C];
    float cr0 = 0.f, cr1 = 0.f;                // Am x[u-1]: carry into row u
    if (d0 > 0) {
        ld_row48<TX>(x + (int64_t)(d0 - 1) * W * DL_C, xr);
        dot2(Am, xr, cr0, cr1);
    }
    float pe0 = 0.f, pe1 = 0.f;                // pending FO[u-1] without its Ap x[u] term
#pragma unroll 1
    for (int u = d0; u < d1; ++u) {
        asm volatile("" ::: "memory");
        ld_row48<TX>(x + (int64_t)u * W * DL_C, xr);
        // 0.1 P resize_H(skip[:, :4])[u] + (P b + pb)
        const LinIdx lj = lin_index(u, d.H_skip, H);
        float sa[4], sb[4], s4[4];
        ld_skip4(d.skip, d.skip_bf16, sk + ((int64_t)lj.i0 * W + w) * d.C_skip, sa);
        ld_skip4(d.skip, d.skip_bf16, sk + ((int64_t)lj.i1 * W + w) * d.C_skip, sb);
#pragma unroll
        for (int q = 0; q < 4; ++q) s4[q] = lj.l0 * sa[q] + lj.l1 * sb[q];
        float a0, a1, m0, m1, q0, q1;
        dot2(A0, xr, a0, a1);
        dot2(Ap, xr, q0, q1);
        dot2(Am, xr, m0, m1);
        if (u > d0) *reinterpret_cast<float2*>(fo + 2 * (u - 1)) = make_float2(pe0 + q0, pe1 + q1);
        pe0 = cst[0] + (S[0] * s4[0] + S[1] * s4[1] + S[2] * s4[2] + S[3] * s4[3]) + cr0 + a0;
        pe1 = cst[1] + (S[4] * s4[0] + S[5] * s4[1] + S[6] * s4[2] + S[7] * s4[3]) + cr1 + a1;
        cr0 = m0;
        cr1 = m1;
    }
    // last row of the chunk: add Ap x[d1] (x[H] = 0)
    float q0 = 0.f, q1 = 0.f;
    if (d1 < H) {
        ld_row48<TX>(x + (int64_t)d1 * W * DL_C, xr);
        dot2(Ap, xr, q0, q1);
    }
    *reinterpret_cast<float2*>(fo + 2 * (d1 - 1)) = make_float2(pe0 + q0, pe1 + q1);
}

// ------------------------------------------------------------------------------------------------- time level 3
// Exact case 4*Lin == T (the resize is the identity): block = (item, 256 consecutive input rows u: 254 interior
// + 1 halo row each side); each thread forms the 8 tap products Q_k x[u], trades the u-1 / u+1 halves through LDS
// and writes its 4 output samples x 2 channels as 32 contiguous bytes.
constexpr int TL_NT = 256;
constexpr int TL_IN = TL_NT - 2;

template <typename TX>
__global__ __launch_bounds__(TL_NT) void tdec_last_kernel(const DecLastDesc d) {
    __shared__ float4 lo[TL_NT], hi[TL_NT];
    const int64_t item = blockIdx.y;
    const int64_t seg = item / d.P;
    const int tid = threadIdx.x;
    const int Lin = d.H;
    const int u = blockIdx.x * TL_IN - 1 + tid;
    const bool interior = tid > 0 && tid < TL_NT - 1 && u < Lin;
    const float* F = d.fold;
    const float* Q = F;                          // [8][2][48]
    const float* cb = F + 16 * DL_C;             // P b (2), then tb (2), then 0.1 P (8)
    const float* S = cb + 4;
    float xr[DL_C];
    if (u >= 0 && u < Lin) {
        ld_row48<TX>(reinterpret_cast<const TX*>(d.in) + (item * Lin + u) * DL_C, xr);
    } else {
#pragma unroll
        for (int c = 0; c < DL_C; ++c) xr[c] = 0.f;
    }
    float z[8][2];
#pragma unroll
    for (int k = 0; k < 8; ++k) dot2(Q + k * 2 * DL_C, xr, z[k][0], z[k][1]);
    lo[tid] = make_float4(z[6][0], z[6][1], z[7][0], z[7][1]);   // taps of row u feeding rows 4(u+1)+{0,1}
    hi[tid] = make_float4(z[0][0], z[0][1], z[1][0], z[1][1]);   // taps of row u feeding rows 4(u-1)+{2,3}
    __syncthreads();
    if (!interior) return;
    // skip term of the 4 outputs 4u + rho, plus P b + tb
    const float c0 = cb[0] + cb[2], c1 = cb[1] + cb[3];
    float sb[4][2];
    const int64_t sk = seg * d.H_skip * d.C_skip;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const LinIdx lj = lin_index(4 * u + r, d.H_skip, (int)d.T);
        float a[4], b[4], s[4];
        ld_skip4(d.skip, d.skip_bf16, sk + (int64_t)lj.i0 * d.C_skip, a);
        ld_skip4(d.skip, d.skip_bf16, sk + (int64_t)lj.i1 * d.C_skip, b);
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] = lj.l0 * a[q] + lj.l1 * b[q];
        sb[r][0] = c0 + (S[0] * s[0] + S[1] * s[1] + S[2] * s[2] + S[3] * s[3]);
        sb[r][1] = c1 + (S[4] * s[0] + S[5] * s[1] + S[6] * s[2] + S[7] * s[3]);
    }
    const float4 l = lo[tid - 1], h = hi[tid + 1];
    float4 o0, o1;
    o0.x = (z[2][0] + l.x) + sb[0][0];
    o0.y = (z[2][1] + l.y) + sb[0][1];
    o0.z = (z[3][0] + l.z) + sb[1][0];
    o0.w = (z[3][1] + l.w) + sb[1][1];
    o1.x = (z[4][0] + h.x) + sb[2][0];
    o1.y = (z[4][1] + h.y) + sb[2][1];
    o1.z = (z[5][0] + h.z) + sb[3][0];
    o1.w = (z[5][1] + h.w) + sb[3][1];
    float4* o = reinterpret_cast<float4*>(d.out + (item * (int64_t)d.T + 4 * (int64_t)u) * 2);
    o[0] = o0;
    o[1] = o1;
}

// General case 4*Lin != T (ragged window): one thread per output sample, both resize source rows of the ConvT
// output computed from their two input rows each.
template <typename TX>
__global__ __launch_bounds__(256) void tdec_last_generic_kernel(const DecLastDesc d) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t item = blockIdx.y;
    if (n >= d.T) return;
    const int64_t seg = item / d.P;
    const int Lin = d.H;
    const float* F = d.fold;
    const float* Q = F;
    const float* cb = F + 16 * DL_C;
    const float* S = cb + 4;
    const TX* x = reinterpret_cast<const TX*>(d.in) + item * (int64_t)Lin * DL_C;
    constexpr int K0[4] = {6, 7, 4, 5}, K1[4] = {2, 3, 0, 1}, OFF[4] = {-1, -1, 0, 0};
    auto zrow = [&](int o, float& z0, float& z1) {
        const int uu = o >> 2, r = o & 3;
        z0 = cb[0];
        z1 = cb[1];
        float xr[DL_C];
        const int ra = uu + OFF[r], rb = ra + 1;
        if (ra >= 0 && ra < Lin) {
            ld_row48<TX>(x + (int64_t)ra * DL_C, xr);
            float a, b;
            dot2(Q + K0[r] * 2 * DL_C, xr, a, b);
            z0 += a;
            z1 += b;
        }
        if (rb >= 0 && rb < Lin) {
            ld_row48<TX>(x + (int64_t)rb * DL_C, xr);
            float a, b;
            dot2(Q + K1[r] * 2 * DL_C, xr, a, b);
            z0 += a;
            z1 += b;
        }
    };
    const LinIdx li = lin_index((int)n, 4 * Lin, (int)d.T);
    float a0, a1, b0, b1;
    zrow(li.i0, a0, a1);
    zrow(li.i1, b0, b1);
    const LinIdx lj = lin_index((int)n, d.H_skip, (int)d.T);
    float sa[4], sbv[4], s[4];
    const int64_t sk = seg * d.H_skip * d.C_skip;
    ld_skip4(d.skip, d.skip_bf16, sk + (int64_t)lj.i0 * d.C_skip, sa);
    ld_skip4(d.skip, d.skip_bf16, sk + (int64_t)lj.i1 * d.C_skip, sbv);
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] = lj.l0 * sa[q] + lj.l1 * sbv[q];
    // time_out(resize(y) + 0.1 resize(skip)) = resize(P y) + 0.1 P resize(skip) + tb, P y including P b
    float2 o;
    o.x = (li.l0 * a0 + li.l1 * b0) + cb[2] + (S[0] * s[0] + S[1] * s[1] + S[2] * s[2] + S[3] * s[3]);
    o.y = (li.l0 * a1 + li.l1 * b1) + cb[3] + (S[4] * s[0] + S[5] * s[1] + S[6] * s[2] + S[7] * s[3]);
    *reinterpret_cast<float2*>(d.out + (item * (int64_t)d.T + n) * 2) = o;
}

// ------------------------------------------------------------------------------------------ fused level-2 merge
// dec_tail: the level-2 merge of both branches (ATHTDemucs_v2.py:88-103 / :126-138 with i = 2: GroupNorm -> GELU of
// the ConvT output, resize, + 0.1 * resize(skip[:, :48])) computed in front of the folded last level, so the merged
// 48-channel level-2 output never goes to HBM: per output row the kernel reads the ConvT rows the resize touches and
// the skip rows, and writes 2 floats.  Same fp32 expression order as dec_merge_kernel (norm.hip) for each value.

namespace {
// Uniform read-only tables (folded weights, GroupNorm affine) read through the constant address space: the compiler
// cannot prove a generic pointer unclobbered by the kernel's own stores and would otherwise use vector loads and
// hold ~300 weights in VGPRs.
typedef const __attribute__((address_space(4))) float cfloat;
ATHD_DEV cfloat* cview(const float* p) { return (cfloat*)p; }
// a zero the compiler cannot see through: table addresses offset by it cannot be hoisted above the point it is made,
// which bounds how many uniform weights are live in scalar registers at once
ATHD_DEV int opaque_zero() {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}

// 8 channels (bf16 or f32) -> f32
ATHD_DEV void ld8(const void* p, int bf, int64_t off, float* v) {
    if (bf) {
        const uint4 q = *reinterpret_cast<const uint4*>((const bf16_t*)p + off);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[2 * e] = __uint_as_float(w[e] << 16);
            v[2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
        }
    } else {
        const float4 a = *reinterpret_cast<const float4*>((const float*)p + off);
        const float4 b = *reinterpret_cast<const float4*>((const float*)p + off + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
}

template <bool FAST>
ATHD_DEV float gn_act(float y, float mean, float rstd, float w, float b) {
    return gelu<FAST>((y - mean) * rstd * w + b);
}
}  // namespace

// Raw loads of one lane's 12-channel slice (channels 12 cg .. 12 cg + 11) of the four rows an x row needs: the two
// ConvT rows the resize reads and the two level-2 skip rows.
template <bool BF> struct Slice12;
template <> struct Slice12<true> {
    uint2 v[4][3];
    ATHD_DEV void load(int r, const void* p, int64_t off) {
#pragma unroll
        for (int i = 0; i < 3; ++i) v[r][i] = *reinterpret_cast<const uint2*>((const bf16_t*)p + off + 4 * i);
    }
    ATHD_DEV float get(int r, int j) const {
        const uint2 q = v[r][j >> 2];
        const uint32_t w = (j & 2) ? q.y : q.x;
        return (j & 1) ? __uint_as_float(w & 0xFFFF0000u) : __uint_as_float(w << 16);
    }
    ATHD_DEV athd_f2v get2(int r, int sp) const {        // channels 2 sp, 2 sp + 1
        const uint2 q = v[r][sp >> 1];
        const uint32_t w = (sp & 1) ? q.y : q.x;
        return (athd_f2v){__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
    }
};
template <> struct Slice12<false> {
    float4 v[4][3];
    ATHD_DEV void load(int r, const void* p, int64_t off) {
#pragma unroll
        for (int i = 0; i < 3; ++i) v[r][i] = *reinterpret_cast<const float4*>((const float*)p + off + 4 * i);
    }
    ATHD_DEV float get(int r, int j) const {
        const float4 q = v[r][j >> 2];
        return (j & 3) == 0 ? q.x : (j & 3) == 1 ? q.y : (j & 3) == 2 ? q.z : q.w;
    }
};

// freq: one wave = (item, d-chunk of FT_DC rows, 16 consecutive w).  Lane l: position w = 16 wt + (l & 15), channel
// group cg = l >> 4.  Per row u the lane forms x[u] at its 12 channels (0.5 act(y[4u+1]) + 0.5 act(y[4u+2]) + skip,
// dec_merge_kernel's fp32 expression order) and the 6 projections [Am; A0; Ap] x[u] come out of 12 exact-f32
// v_mfma_f32_16x16x4_f32 (A = the folded weights, rows 0..5, K permuted to channel 12 cg + step; B = x): the row
// reduction over channels happens in the matrix core and the weights are 12 per-lane constants.
// Block order (1-D grid, XCD-aware): the P prompts of one segment read the same level-2 skip rows, so the blocks of
// one region (chunk, 64 w) for the P items of a segment are consecutive in one XCD's dispatch order (block i runs on
// XCD i % 8) and share those rows through its L2.  The chunk's FO values (16 w x FT_DC rows x 2) are staged in LDS
// and stored as FT_DC * 8 contiguous bytes per w ([item][w][row][2], the iSTFT's frame-major order) instead of one
// 8-B store per lane and row.
#ifndef ATHD_FT_DC
#define ATHD_FT_DC 32
#endif
constexpr int FT_DC = ATHD_FT_DC;   // rows per wave chunk (A/B builds: -DATHD_FT_DC)

#ifndef ATHD_FT_LB
#define ATHD_FT_LB 4         // the bf16 form at 4 waves per SIMD (A/B: 0 = the compiler's choice, 130 VGPRs, 3 waves)
#endif
template <bool BF>
__global__ __launch_bounds__(256, BF && ATHD_FT_LB > 0 ? ATHD_FT_LB : 1) void fdec_tail_kernel(const DecLastDesc d, int nreg) {
    __shared__ __attribute__((aligned(16))) float2 ost[4][16][FT_DC + 1];
    // 1-D block index -> (segment region g, prompt): XCD x runs regions g = x, x + 8, ... with the P prompts of each
    // back to back
    const int L = blockIdx.x, x8 = L & 7, j = L >> 3;
    const int g = 8 * (j / d.P) + x8, pr = j % d.P;
    if (g >= nreg * (d.NI / d.P)) return;                    // block-uniform
    const int64_t seg = g / nreg;
    const int64_t item = seg * d.P + pr;
    const int H = d.H, W = d.W;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nwt = (W + 15) / 16;
    const int nch = (H + FT_DC - 1) / FT_DC;
    const int wv = (g % nreg) * 4 + wave;
    if (wv >= nch * nwt) return;                       // wave-uniform (no block-level barrier below)
    const int wt = wv % nwt, c = wv / nwt;
    const int p = lane & 15, cg = lane >> 4;
    const int w = wt * 16 + p;
    const int wc = w < W ? w : W - 1;                  // clamped: the spare lanes compute a duplicate, never stored
    const int d0 = c * FT_DC;
    const int d1 = min(H, d0 + FT_DC);
    float mean, rstd;
    gn_params(d.stats, item, d.gn_count, mean, rstd);
    const int ch0 = 12 * cg;
    float wA[12], gw[12], gb[12];
#pragma unroll
    for (int s = 0; s < 12; ++s) {
        wA[s] = p < 6 ? d.fold[p * DL_C + ch0 + s] : 0.f;
        gw[s] = d.gn_w[ch0 + s];
        gb[s] = d.gn_b[ch0 + s];
    }
    // bf16 mode: the GroupNorm affine folded into one FMA (a = rstd w, c = b - mean a) on channel pairs
    athd_f2v ga2[6], gc2[6];
#pragma unroll
    for (int sp = 0; sp < 6; ++sp) {
        ga2[sp] = (athd_f2v){rstd * gw[2 * sp], rstd * gw[2 * sp + 1]};
        gc2[sp] = (athd_f2v){gb[2 * sp], gb[2 * sp + 1]} - (athd_f2v){mean, mean} * ga2[sp];
    }
    const float* F = d.fold;
    const float* cst = F + 6 * DL_C;
    const float* S = F + 6 * DL_C + 2;
    const int64_t g_item = item * (int64_t)(2 * H) * W * DL_C + (int64_t)wc * DL_C + ch0;
    const int64_t sk2 = seg * (int64_t)d.H_skip2 * W * d.C_skip2 + (int64_t)wc * d.C_skip2 + ch0;
    const int64_t sk = seg * d.H_skip * W * d.C_skip;
    float2 (*const os)[FT_DC + 1] = ost[wave];

    auto load = [&](int u, Slice12<BF>& r) {
        const LinIdx lj = lin_index(u, d.H_skip2, H);
        const int64_t o0 = g_item + (int64_t)(2 * u) * W * DL_C;   // kept slots 2u, 2u+1 = rows 4u+1, 4u+2
        r.load(0, d.g, o0);
        r.load(1, d.g, o0 + (int64_t)W * DL_C);
        r.load(2, d.skip2, sk2 + (int64_t)lj.i0 * W * d.C_skip2);
        r.load(3, d.skip2, sk2 + (int64_t)lj.i1 * W * d.C_skip2);
    };
    // [Am0 Am1 A00 A01] x[u] (lanes cg = 0) and [Ap0 Ap1 0 0] x[u] (lanes cg = 1)
    auto proj = [&](int u, const Slice12<BF>& r) {
        const LinIdx li = lin_index(u, 4 * H, H);
        const LinIdx lj = lin_index(u, d.H_skip2, H);
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
        if constexpr (BF) {
            const athd_f2v l0 = {li.l0, li.l0}, l1 = {li.l1, li.l1}, k0 = {lj.l0, lj.l0}, k1 = {lj.l1, lj.l1};
#pragma unroll
            for (int sp = 0; sp < 6; ++sp) {
                const athd_f2v sv = __builtin_elementwise_fma(k0, r.get2(2, sp), k1 * r.get2(3, sp)) *
                                    (athd_f2v){0.1f, 0.1f};
                const athd_f2v x = gelu_fast_wsum_pk(l0, __builtin_elementwise_fma(r.get2(0, sp), ga2[sp], gc2[sp]), l1,
                                                     __builtin_elementwise_fma(r.get2(1, sp), ga2[sp], gc2[sp])) + sv;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[2 * sp], x.x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[2 * sp + 1], x.y, acc, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int s = 0; s < 12; ++s) {
                const float va = gn_act<BF>(r.get(0, s), mean, rstd, gw[s], gb[s]);
                const float vb = gn_act<BF>(r.get(1, s), mean, rstd, gw[s], gb[s]);
                const float sv = (lj.l0 * r.get(2, s) + lj.l1 * r.get(3, s)) * 0.1f;
                const float x = (li.l0 * va + li.l1 * vb) + sv;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[s], x, acc, 0, 0, 0);
            }
        }
        return acc;
    };

    Slice12<BF> cur, nxt;
    float cr0 = 0.f, cr1 = 0.f;                // Am x[u-1]: carry into row u
    if (d0 > 0) {
        load(d0 - 1, cur);
        const f32x4_t a = proj(d0 - 1, cur);
        cr0 = a[0];
        cr1 = a[1];
    }
    load(d0, cur);
    float pe0 = 0.f, pe1 = 0.f;                // pending FO[u-1] without its Ap x[u] term
#pragma unroll 1
    for (int u = d0; u < d1; ++u) {
        if (u + 1 < H) load(u + 1, nxt);       // prefetch (also the halo row d1)
        const f32x4_t a = proj(u, cur);
        const float ap0 = __shfl(a[0], p + 16, 64), ap1 = __shfl(a[1], p + 16, 64);
        if (cg == 0) {
            const LinIdx lj = lin_index(u, d.H_skip, H);
            float sa[4], sb[4], s4[4];
            ld_skip4(d.skip, BF, sk + ((int64_t)lj.i0 * W + wc) * d.C_skip, sa);
            ld_skip4(d.skip, BF, sk + ((int64_t)lj.i1 * W + wc) * d.C_skip, sb);
#pragma unroll
            for (int q = 0; q < 4; ++q) s4[q] = lj.l0 * sa[q] + lj.l1 * sb[q];
            if (u > d0) os[p][u - 1 - d0] = make_float2(pe0 + ap0, pe1 + ap1);
            pe0 = cst[0] + (S[0] * s4[0] + S[1] * s4[1] + S[2] * s4[2] + S[3] * s4[3]) + cr0 + a[2];
            pe1 = cst[1] + (S[4] * s4[0] + S[5] * s4[1] + S[6] * s4[2] + S[7] * s4[3]) + cr1 + a[3];
            cr0 = a[0];
            cr1 = a[1];
        }
        cur = nxt;
    }
    float q0 = 0.f, q1 = 0.f;
    if (d1 < H) {                              // halo: Ap x[d1] (loaded by the last iteration)
        const f32x4_t a = proj(d1, cur);
        q0 = __shfl(a[0], p + 16, 64);
        q1 = __shfl(a[1], p + 16, 64);
    }
    if (cg == 0) os[p][d1 - 1 - d0] = make_float2(pe0 + q0, pe1 + q1);
    __builtin_amdgcn_s_waitcnt(0xc07f);        // lgkmcnt(0): the wave's staged values landed
    __builtin_amdgcn_wave_barrier();
    // store: per w the chunk's rows d0 .. d1 - 1 are contiguous; consecutive lanes take consecutive rows
    const int nrow = d1 - d0;
    for (int i = lane; i < 16 * nrow; i += 64) {
        const int wl = i / nrow, rr = i - wl * nrow;
        const int ww = wt * 16 + wl;
        if (ww < W) *reinterpret_cast<float2*>(d.out + ((item * W + ww) * (int64_t)H + d0 + rr) * 2) = os[wl][rr];
    }
}

// time (4 H == T): block = (item, TL_IN output rows + 1 halo row each side), row r <-> u = TL_IN bx - 1 + r.
//   phase 1: GroupNorm + GELU of the block's span of ConvT rows (<= TT_ROWS) into LDS (fp32);
//   phase 2: wave w, pass k: rows r = 64 k + 16 w + (l & 15); the lane forms x[u] at channels 12 cg .. 12 cg + 11
//            (resize of the LDS rows + 0.1 resize(skip2)) and 12 v_mfma_f32_16x16x4_f32 give the 16 tap products
//            z[u] = [Q_0; ..; Q_7] x[u] (row 2k + j = tap k, channel j) - lane (p, cg) ends with taps 2cg, 2cg + 1;
//   phase 3: z rows through LDS; thread r writes the 4 output samples 4u .. 4u + 3 of its row (x 2 channels).
constexpr int TT_ROWS = 264;
constexpr int TT_LD = 50;        // LDS row pitch in floats (3 blocks per CU)

ATHD_HD int tt_span(int bx, int Lin, int Hg, int& r0) {
    const int ua = bx * TL_IN - 1 < 0 ? 0 : bx * TL_IN - 1;
    const int ub = bx * TL_IN + TL_IN < Lin - 1 ? bx * TL_IN + TL_IN : Lin - 1;
    r0 = lin_index(ua, Hg, Lin).i0;
    return lin_index(ub, Hg, Lin).i1 - r0 + 1;
}

// bf16 mode keeps the activated rows as bf16 in LDS (29.6 KB instead of 52.8: 5 blocks per CU instead of 3); the
// f32 parity mode keeps fp32
constexpr int TT_LDB = 56;       // bf16 row pitch (elements)
template <bool BF> struct TtRow;
template <> struct TtRow<false> {
    static constexpr int BYTES = TT_ROWS * TT_LD * 4;
    ATHD_DEV static void put8(char* g, int row, int c0, const float* v) {
        float2* dst = reinterpret_cast<float2*>((float*)g + row * TT_LD + c0);
#pragma unroll
        for (int j = 0; j < 8; j += 2) dst[j / 2] = make_float2(v[j], v[j + 1]);
    }
    ATHD_DEV static void get12(const char* g, int row, int c0, float* v) {
        const float* src = (const float*)g + row * TT_LD + c0;
#pragma unroll
        for (int s = 0; s < 12; ++s) v[s] = src[s];
    }
};
template <> struct TtRow<true> {
    static constexpr int BYTES = TT_ROWS * TT_LDB * 2;
    ATHD_DEV static void put8(char* g, int row, int c0, const float* v) {
        *reinterpret_cast<uint4*>((bf16_t*)g + row * TT_LDB + c0) =
            make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
    }
    ATHD_DEV static void get12(const char* g, int row, int c0, float* v) {
        const uint2* src = reinterpret_cast<const uint2*>((const bf16_t*)g + row * TT_LDB + c0);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint2 q = src[i];
            v[4 * i + 0] = __uint_as_float(q.x << 16);
            v[4 * i + 1] = __uint_as_float(q.x & 0xFFFF0000u);
            v[4 * i + 2] = __uint_as_float(q.y << 16);
            v[4 * i + 3] = __uint_as_float(q.y & 0xFFFF0000u);
        }
    }
};

template <bool BF>
__global__ __launch_bounds__(TL_NT) void tdec_tail_kernel(const DecLastDesc d) {
    // phase 3: z rows [TL_NT][TZ_LD], over the dead phase-1 tile.  Row pitch 20 floats: the 16-lane groups of the
    // b128 row writes (16 consecutive rows) and row reads (thread = row) then cover 16 distinct 4-bank sets (pitch 16
    // put 4 rows on each set: 4-way conflicts on the writes, 16-way on the former per-float reads)
    constexpr int TZ_LD = 20;
    constexpr int GS_BYTES = TtRow<BF>::BYTES > TL_NT * TZ_LD * 4 ? TtRow<BF>::BYTES : TL_NT * TZ_LD * 4;
    __shared__ __attribute__((aligned(16))) char gsm[GS_BYTES];
    float* zb = reinterpret_cast<float*>(gsm);
    // 1-D block index -> (segment region g = (seg, bx), prompt), as fdec_tail: XCD x runs regions g = x, x + 8, ...
    // with the P prompts of each back to back, so the skip rows of a region are read once into that XCD's L2 and
    // served to the other P - 1 prompts from it
    const int Lin = d.H;
    const int nbx = (Lin + TL_IN - 1) / TL_IN;
    const int L8 = blockIdx.x, x8 = L8 & 7, jj = L8 >> 3;
    const int g = 8 * (jj / d.P) + x8, pr = jj % d.P;
    if (g >= nbx * (d.NI / d.P)) return;                   // block-uniform
    const int64_t seg = g / nbx;
    const int bxi = g % nbx;
    const int64_t item = seg * d.P + pr;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if ATHD_TDEC_PAD == 3
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");   // A/B: the same delay at the kernel start
#endif
    float mean, rstd;
    gn_params(d.stats, item, d.gn_count, mean, rstd);
    int r0;
    const int nr = tt_span(bxi, Lin, d.Hg, r0);
    const int64_t gb = (item * d.Hg + r0) * (int64_t)DL_C;
    for (int i = tid; i < nr * (DL_C / 8); i += TL_NT) {
        const int rr = i / (DL_C / 8), q = i % (DL_C / 8);
        float a[8];
        ld8(d.g, BF, gb + (int64_t)rr * DL_C + 8 * q, a);
        if constexpr (BF) {            // GroupNorm affine folded into one FMA, GELU pairs on packed ops
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const athd_f2v ga = (athd_f2v){d.gn_w[8 * q + j], d.gn_w[8 * q + j + 1]} * (athd_f2v){rstd, rstd};
                const athd_f2v gc = (athd_f2v){d.gn_b[8 * q + j], d.gn_b[8 * q + j + 1]} - (athd_f2v){mean, mean} * ga;
                const athd_f2v v = gelu_fast_pk(__builtin_elementwise_fma((athd_f2v){a[j], a[j + 1]}, ga, gc));
                a[j] = v.x;
                a[j + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = gn_act<BF>(a[j], mean, rstd, d.gn_w[8 * q + j], d.gn_b[8 * q + j]);
        }
        TtRow<BF>::put8(gsm, rr, 8 * q, a);
    }
    __syncthreads();
    const int p = lane & 15, cg = lane >> 4, ch0 = 12 * cg;
    float wA[12];
#pragma unroll
    for (int s = 0; s < 12; ++s) wA[s] = d.fold[p * DL_C + ch0 + s];     // Q [8][2][48]: row p = 2 k + j
    f32x4_t z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int r = 64 * k + 16 * wave + p;
        const int u = bxi * TL_IN - 1 + r;
        float x[12];
#pragma unroll
        for (int s = 0; s < 12; ++s) x[s] = 0.f;      // x = 0 outside [0, Lin): zero taps
        if (u >= 0 && u < Lin) {
            const LinIdx li = lin_index(u, d.Hg, Lin);
            const LinIdx lj = lin_index(u, d.H_skip2, Lin);
            Slice12<BF> sl;
            sl.load(2, d.skip2, (seg * d.H_skip2 + lj.i0) * (int64_t)d.C_skip2 + ch0);
            sl.load(3, d.skip2, (seg * d.H_skip2 + lj.i1) * (int64_t)d.C_skip2 + ch0);
            float ga[12], gq[12];
            TtRow<BF>::get12(gsm, li.i0 - r0, ch0, ga);
            TtRow<BF>::get12(gsm, li.i1 - r0, ch0, gq);
#pragma unroll
            for (int s = 0; s < 12; ++s) {
                const float sv = (lj.l0 * sl.get(2, s) + lj.l1 * sl.get(3, s)) * 0.1f;
                x[s] = (li.l0 * ga[s] + li.l1 * gq[s]) + sv;
            }
        }
        // the MFMAs run wave-converged (a matrix op reads every lane's operands whatever EXEC says)
        z[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 12; ++s) z[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[s], x[s], z[k], 0, 0, 0);
    }
    __syncthreads();                             // every wave is done reading the phase-1 tile
    // Round 5 put an explicit 48-state pad here: ~100 of 8.5 M outputs (channel 0) differed run to run with the two
    // branch streams, never with ATHD_SERIAL=1, and the pad made 9 of 9 comparisons identical.  The explanation given
    // then - that hipcc's padding between the last MFMA of a chain and the LDS store of its result is too short on
    // gfx950 - does NOT hold.  Round 6 (tools/hazard/README.md, profiles/r06_hazard.txt):
    //   - probes: v_mfma_f32_16x16x4_f32 results stored after exactly N wait states, single and at the end of 12-MFMA
    //     chains, alone and beside a matrix-saturating kernel: stale at 0 and 4 states, 0 stale in 2.6e8 lane-stores
    //     at 9, 10 and 16 (hipcc emits 9-10); the reverse order (LDS store, then an MFMA overwriting its data registers
    //     1 state later): 0;
    //   - builds (tools/diag_det4.py, 3 forwards each): no pad (ATHD_TDEC_PAD=0) 110 / 30 / 203 outputs differ; the pad's
    //     sched_barrier fence alone, the same instruction order as the pad build without its wait states (2): 158 / 141;
    //     the same 48 states at the kernel START instead (3): 0 / 0 / 0 / 0; no pad with ATHD_SERIAL=1: 0 / 0.
    // So the wait states matter only as a delay of the workgroup relative to the kernels of the other branch stream,
    // not as a hazard pad between MFMA and store: a timing-dependent interaction with the concurrent frequency-branch
    // kernels (the differing outputs are confined to the first-scheduled segment and to channel 0).  Its root cause is
    // not established; the pad is kept as the measured mitigation, guarded by test_bf16_forward_reproducible.
#ifndef ATHD_TDEC_PAD
#define ATHD_TDEC_PAD 1
#endif
#if ATHD_TDEC_PAD == 1
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#elif ATHD_TDEC_PAD == 2 || ATHD_TDEC_PAD == 3
    __builtin_amdgcn_sched_barrier(0);               // A/B: the pad's scheduling fence without its wait states
#endif
#pragma unroll
    for (int k = 0; k < 4; ++k)
        *reinterpret_cast<float4*>(zb + (64 * k + 16 * wave + p) * TZ_LD + 4 * cg) = make_float4(z[k][0], z[k][1], z[k][2], z[k][3]);
    __syncthreads();
    const int u = bxi * TL_IN - 1 + tid;
    if (!(tid > 0 && tid < TL_NT - 1 && u < Lin)) return;
    const float* F = d.fold;
    const float* cb = F + 16 * DL_C;             // P b (2), then tb (2), then 0.1 P (8)
    const float* S = cb + 4;
    const float c0 = cb[0] + cb[2], c1 = cb[1] + cb[3];
    float sbv[4][2];
    const int64_t sk = seg * d.H_skip * d.C_skip;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const LinIdx lj = lin_index(4 * u + r, d.H_skip, (int)d.T);
        float a[4], b[4], s[4];
        ld_skip4(d.skip, BF, sk + (int64_t)lj.i0 * d.C_skip, a);
        ld_skip4(d.skip, BF, sk + (int64_t)lj.i1 * d.C_skip, b);
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] = lj.l0 * a[q] + lj.l1 * b[q];
        sbv[r][0] = c0 + (S[0] * s[0] + S[1] * s[1] + S[2] * s[2] + S[3] * s[3]);
        sbv[r][1] = c1 + (S[4] * s[0] + S[5] * s[1] + S[6] * s[2] + S[7] * s[3]);
    }
    // taps of row u: [z0 z1 | z2 z3 | z4 z5 | z6 z7] x 2 channels; row u - 1 feeds rows 4u + {0, 1} through taps 6, 7,
    // row u + 1 feeds rows 4u + {2, 3} through taps 0, 1
    const float* zc = zb + tid * TZ_LD;
    const float4 c4 = *reinterpret_cast<const float4*>(zc + 4), c8 = *reinterpret_cast<const float4*>(zc + 8);
    const float4 l12 = *reinterpret_cast<const float4*>(zc - TZ_LD + 12);
    const float4 h0 = *reinterpret_cast<const float4*>(zc + TZ_LD);
    float4 o0, o1;
    o0.x = (c4.x + l12.x) + sbv[0][0];
    o0.y = (c4.y + l12.y) + sbv[0][1];
    o0.z = (c4.z + l12.z) + sbv[1][0];
    o0.w = (c4.w + l12.w) + sbv[1][1];
    o1.x = (c8.x + h0.x) + sbv[2][0];
    o1.y = (c8.y + h0.y) + sbv[2][1];
    o1.z = (c8.z + h0.z) + sbv[3][0];
    o1.w = (c8.w + h0.w) + sbv[3][1];
    float4* o = reinterpret_cast<float4*>(d.out + (item * (int64_t)d.T + 4 * (int64_t)u) * 2);
    o[0] = o0;
    o[1] = o1;
}

int fdec_tail_launch(const DecLastDesc& d, hipStream_t s) {
    if (d.g_bf16 != d.skip2_bf16 || d.g_bf16 != d.skip_bf16 || d.g_bf16 != d.fast_gelu ||d.P < 1 || d.NI % d.P != 0 || d.H < 1 || d.W < 1 || d.C_skip < 4 || d.H_skip < 1 || !d.g || !d.stats ||
        d.C_skip2 < DL_C || d.C_skip2 % 8 != 0 || d.H_skip2 < 1)
        return -1;
    const int nch = (d.H + FT_DC - 1) / FT_DC;
    const int waves = nch * ((d.W + 15) / 16);
    const int nreg = (waves + 3) / 4;                  // blocks per item
    const int64_t nseg = d.NI / d.P;
    // 8 XCD lanes x ceil(regions / 8) x P prompts (fdec_tail_kernel's block order); spare blocks return at once
    const int64_t per_x = (nreg * nseg + 7) / 8;
    const dim3 grid((unsigned)(8 * per_x * d.P));
    KScope ks(s);
    if (ks.on()) {
        // the two kept ConvT rows per output row once, level-2 skip rows (48 channels, 2 per output row) and level-3
        // skip rows (4 channels) once per segment, FO once
        const double eg = d.g_bf16 ? 2 : 4, es2 = d.skip2_bf16 ? 2 : 4, es = d.skip_bf16 ? 2 : 4;
        const double segs = d.NI / d.P;
        const double by = (double)d.NI * 2 * d.H * d.W * DL_C * eg + segs * std::min(d.H_skip2, 2 * d.H) * d.W * DL_C * es2 +
                          segs * 2 * d.H * d.W * 4 * es + (double)d.NI * d.H * d.W * 2 * 4;
        ks.begin(d.g_bf16 ? "fdec_tail_kernel<true>" : "fdec_tail_kernel<false>", 0.0, by);
    }
    if (d.g_bf16) hipLaunchKernelGGL(fdec_tail_kernel<true>, grid, dim3(256), 0, s, d, nreg);
    else hipLaunchKernelGGL(fdec_tail_kernel<false>, grid, dim3(256), 0, s, d, nreg);
    return (int)hipGetLastError();
}

bool tdec_tail_supported(const DecLastDesc& d) {
    if (4 * (int64_t)d.H != d.T || d.H < 1 || d.Hg < 1 || !d.g || !d.stats || d.C_skip2 < DL_C || d.C_skip2 % 8 != 0)
        return false;
    const int nb = (d.H + TL_IN - 1) / TL_IN;
    for (int bx = 0; bx < nb; ++bx) {
        int r0;
        const int nr = tt_span(bx, d.H, d.Hg, r0);
        if (nr < 1 || nr > TT_ROWS || r0 < 0 || r0 + nr > d.Hg) return false;
    }
    return true;
}

int tdec_tail_launch(const DecLastDesc& d, hipStream_t s) {
    if (d.g_bf16 != d.skip2_bf16 || d.g_bf16 != d.skip_bf16 || d.g_bf16 != d.fast_gelu ||d.P < 1 || d.NI % d.P != 0 || d.C_skip < 4 || d.H_skip < 1 || d.H_skip2 < 1 || !tdec_tail_supported(d)) return -1;
    KScope ks(s);
    if (ks.on()) {
        const double eg = d.g_bf16 ? 2 : 4, es2 = d.skip2_bf16 ? 2 : 4, es = d.skip_bf16 ? 2 : 4;
        const double segs = d.NI / d.P;
        const double by = (double)d.NI * d.Hg * DL_C * eg + segs * d.H_skip2 * DL_C * es2 + segs * d.H_skip * 4 * es +
                          (double)d.NI * d.T * 2 * 4;
        ks.begin(d.g_bf16 ? "tdec_tail_kernel<true>" : "tdec_tail_kernel<false>", 0.0, by);
    }
    // 8 XCD lanes x ceil(regions / 8) x P prompts (tdec_tail_kernel's block order); spare blocks return at once
    const int64_t regions = (int64_t)((d.H + TL_IN - 1) / TL_IN) * (d.NI / d.P);
    const dim3 grid((unsigned)(8 * ((regions + 7) / 8) * d.P));
    if (d.g_bf16) hipLaunchKernelGGL(tdec_tail_kernel<true>, grid, dim3(TL_NT), 0, s, d);
    else hipLaunchKernelGGL(tdec_tail_kernel<false>, grid, dim3(TL_NT), 0, s, d);
    return (int)hipGetLastError();
}

int fdec_last_launch(const DecLastDesc& d, hipStream_t s) {
    if (d.P < 1 || d.NI % d.P != 0 || d.H < 1 || d.W < 1 || d.C_skip < 4 || d.H_skip < 1) return -1;
    const int nch = (d.H + FL_DC - 1) / FL_DC;
    const dim3 grid((unsigned)((nch * d.W + 255) / 256), (unsigned)d.NI);
    KScope ks(s);
    if (ks.on()) {
        // the 48-channel input once (+ the chunk halo rows), skip rows (4 channels, 2 per output row, once per
        // segment), FO once
        const double eb = d.in_bf16 ? 2 : 4;
        const double by = (double)d.NI * d.H * d.W * DL_C * eb + (double)(d.NI / d.P) * 2 * d.H * d.W * 4 * (d.skip_bf16 ? 2 : 4) +
                          (double)d.NI * d.H * d.W * 2 * 4;
        ks.begin(d.in_bf16 ? "fdec_last_kernel<unsignedshort>" : "fdec_last_kernel<float>", 0.0, by);
    }
    if (d.in_bf16) hipLaunchKernelGGL(fdec_last_kernel<bf16_t>, grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL(fdec_last_kernel<float>, grid, dim3(256), 0, s, d);
    return (int)hipGetLastError();
}

int tdec_last_launch(const DecLastDesc& d, hipStream_t s) {
    if (d.P < 1 || d.NI % d.P != 0 || d.H < 1 || d.T < 1 || d.C_skip < 4 || d.H_skip < 1) return -1;
    const bool exact = 4 * (int64_t)d.H == d.T;
    KScope ks(s);
    if (ks.on()) {
        const double eb = d.in_bf16 ? 2 : 4;
        const double by = (double)d.NI * d.H * DL_C * eb + (double)(d.NI / d.P) * d.H_skip * 4 * (d.skip_bf16 ? 2 : 4) +
                          (double)d.NI * d.T * 2 * 4;
        ks.begin(klabel("%s<%s>", exact ? "tdec_last_kernel" : "tdec_last_generic_kernel", d.in_bf16 ? "unsignedshort" : "float"), 0.0, by);
    }
    if (exact) {
        const dim3 grid((unsigned)((d.H + TL_IN - 1) / TL_IN), (unsigned)d.NI);
        if (d.in_bf16) hipLaunchKernelGGL(tdec_last_kernel<bf16_t>, grid, dim3(TL_NT), 0, s, d);
        else hipLaunchKernelGGL(tdec_last_kernel<float>, grid, dim3(TL_NT), 0, s, d);
    } else {
        const dim3 grid((unsigned)((d.T + 255) / 256), (unsigned)d.NI);
        if (d.in_bf16) hipLaunchKernelGGL(tdec_last_generic_kernel<bf16_t>, grid, dim3(256), 0, s, d);
        else hipLaunchKernelGGL(tdec_last_generic_kernel<float>, grid, dim3(256), 0, s, d);
    }
    return (int)hipGetLastError();
}

}  // namespace athd
