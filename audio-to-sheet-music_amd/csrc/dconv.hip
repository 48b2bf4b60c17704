// DConv (demucs residual dilated-conv branch) for the narrow levels (C = 48, 96; hidden
// H = C/8 = 6, 12).  These layers are HBM-bound with K or N far below an MFMA tile, so they run as VALU kernels.
// x is [nb][L][C] in f32 (parity mode) or bf16 (throughput mode); h is [nb][L][H] f32.  One layer = 3 passes
// (each GroupNorm needs complete statistics before it can be applied):
//   c3:     h = b + W3 * x[t - dil], x[t], x[t + dil]          + GroupNorm statistics of h per group
//   c1stat: y = b1 + W1 * GELU(GN(h))   (2C outputs, never stored)  -> GroupNorm statistics of y per group
//   c1app:  x += scale * GLU(GN(y))     (y recomputed: K = H is tiny)
// A "group" is the GroupNorm(1) sample: one nb row of L positions (freq rows (b,f) along time, or time samples).
// Access pattern: c3 stages its x tile (+ dilation halo) in LDS with 16-B coalesced loads; the 1x1 passes map a
// lane to one position.  Every weight is read at a wave-uniform address (scalar loads, SGPR operands of the FMAs:
// no LDS traffic for weights).  Per-group GroupNorm parameters are finalised once per block into LDS.
#include <algorithm>

#include "common.h"
#include "prof.h"
#include "kernels.h"

namespace athd {

template <typename TS> struct XS;
template <> struct XS<float> {
    static ATHD_DEV float ld(const float* p, int64_t i) { return p[i]; }
};
template <> struct XS<bf16_t> {
    static ATHD_DEV float ld(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
};

// 16 B of x -> EPC floats
template <typename TS>
ATHD_DEV void unpack16(const uint4 q, float* v) {
    if constexpr (sizeof(TS) == 2) {
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w[i] << 16);
            v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
        }
    } else {
        v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
    }
}

// Block-level {sum, sumsq} per group.  Blocks cover <= 256 consecutive positions, so with L >= 256 a block spans
// at most two groups (g0 and g0 + 1).  Shorter rows fall back to per-thread atomics.
ATHD_DEV void group_stats_add(double* __restrict__ st, int64_t p0, int64_t p, bool valid, int64_t L, float s1, float s2,
                              double* sh) {
    if (L < 256) {
        if (valid) {
            atomicAdd(&st[2 * (p / L)], (double)s1);
            atomicAdd(&st[2 * (p / L) + 1], (double)s2);
        }
        return;
    }
    const int64_t g0 = p0 / L;
    const bool second = valid && (p / L) != g0;
    double a0 = (valid && !second) ? s1 : 0.0, b0 = (valid && !second) ? s2 : 0.0;
    double a1 = second ? s1 : 0.0, b1 = second ? s2 : 0.0;
    a0 = wave_sum_d(a0); b0 = wave_sum_d(b0); a1 = wave_sum_d(a1); b1 = wave_sum_d(b1);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[4 * w] = a0; sh[4 * w + 1] = b0; sh[4 * w + 2] = a1; sh[4 * w + 3] = b1; }
    __syncthreads();
    if (threadIdx.x < 4) {
        double v = 0.0;
        for (int i = 0; i < 4; ++i) v += sh[4 * i + threadIdx.x];
        const int64_t g = g0 + (threadIdx.x >= 2 ? 1 : 0);
        if (v != 0.0) atomicAdd(&st[2 * g + (threadIdx.x & 1)], v);
    }
}

ATHD_DEV void gn_mr(const double* st, int64_t g, double cnt, float& mean, float& rstd) {
    const double mm = st[2 * g] / cnt;
    double var = st[2 * g + 1] / cnt - mm * mm;
    if (var < 0) var = 0;
    mean = (float)mm;
    rstd = (float)(1.0 / sqrt(var + 1e-5));
}

// ---- c3: TILE positions per block, TPP = 256 / TILE threads per position, each computing H / TPP outputs
template <int C, typename TS>
__global__ __launch_bounds__(256) void dconv_c3_kernel(const TS* __restrict__ x, int64_t nb, int64_t L, int dil,
                                                       const float* __restrict__ W, const float* __restrict__ bias,
                                                       float* __restrict__ h, double* __restrict__ st) {
    constexpr int H = C / 8, K = 3 * C, HALO = 2;
    constexpr int TILE = sizeof(TS) == 2 ? 256 : 128;
    constexpr int TPP = 256 / TILE, HJ = H / TPP;
    constexpr int ROWS = TILE + 2 * HALO;
    constexpr int EPC = 16 / sizeof(TS);                    // elements per 16-B chunk
    constexpr int CPR = C / EPC;                             // chunks per row
    __shared__ __attribute__((aligned(16))) TS xs[ROWS * C];
    __shared__ double sh[16];
    const int64_t P = nb * L;
    const int64_t p0 = (int64_t)blockIdx.x * TILE;
    for (int i = threadIdx.x; i < ROWS * CPR; i += 256) {
        const int r = i / CPR, ch = i - r * CPR;
        const int64_t pp = p0 - HALO + r;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (pp >= 0 && pp < P) v = *reinterpret_cast<const uint4*>(x + pp * C + ch * EPC);
        *reinterpret_cast<uint4*>(&xs[r * C + ch * EPC]) = v;
    }
    __syncthreads();
    const int lp = threadIdx.x / TPP, sub = threadIdx.x % TPP;
    const int64_t p = p0 + lp;
    const bool valid = p < P;
    float s1 = 0.f, s2 = 0.f;
    if (valid) {
        const int64_t t = p % L;
        float acc[HJ];
#pragma unroll
        for (int j = 0; j < HJ; ++j) acc[j] = bias[sub * HJ + j];
#pragma unroll
        for (int tap = 0; tap < 3; ++tap) {
            const int64_t tt = t + (tap - 1) * dil;
            if (tt < 0 || tt >= L) continue;                 // zero padding of the group row
            const TS* xr = &xs[(lp + HALO + (tap - 1) * dil) * C];
#pragma unroll 2
            for (int c0 = 0; c0 < C; c0 += EPC) {
                float v[EPC];
                unpack16<TS>(*reinterpret_cast<const uint4*>(xr + c0), v);
#pragma unroll
                for (int e = 0; e < EPC; ++e)
#pragma unroll
                    for (int j = 0; j < HJ; ++j) acc[j] += W[(sub * HJ + j) * K + tap * C + c0 + e] * v[e];
            }
        }
        float* hr = h + p * H + sub * HJ;
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
            hr[j] = acc[j];
            s1 += acc[j];
            s2 += acc[j] * acc[j];
        }
    }
    group_stats_add(st, p0, p, valid, L, s1, s2, sh);
}

// GELU(GroupNorm(h)) of one position (the first GroupNorm of the layer, fused into both 1x1 passes)
template <int H, bool FAST>
ATHD_DEV void load_hg(const float* __restrict__ h, int64_t p, float mean, float rstd, const float* g1w, const float* g1b,
                      float* hv) {
#pragma unroll
    for (int j = 0; j < H; ++j) hv[j] = gelu<FAST>((h[p * H + j] - mean) * rstd * g1w[j] + g1b[j]);
}

// GroupNorm (mean, rstd) of the groups [g_first, g_first + n) a block touches, into LDS (n <= GN_TAB); the caller
// synchronises.  Blocks touching more groups (very short rows) compute per thread.
constexpr int GN_TAB = 8;
ATHD_DEV void gn_table(const double* st, double cnt, int64_t g_first, int64_t n, float* tm, float* tr) {
    if (n <= GN_TAB && (int64_t)threadIdx.x < n) gn_mr(st, g_first + threadIdx.x, cnt, tm[threadIdx.x], tr[threadIdx.x]);
}
ATHD_DEV void gn_lookup(const double* st, double cnt, int64_t g, int64_t g_first, int64_t n, const float* tm,
                        const float* tr, float& mean, float& rstd) {
    if (n <= GN_TAB) {
        mean = tm[g - g_first];
        rstd = tr[g - g_first];
    } else {
        gn_mr(st, g, cnt, mean, rstd);
    }
}

// ---- c1stat: one thread per position.  y = W h + b (2C channels) only feeds the GroupNorm statistics, and
// sum_n y_n = sum b + ws.h, sum_n y_n^2 = sum b^2 + 2 v.h + h^T G h with the 1x1 conv's moments (G = W^T W, v = W^T b,
// ws = W^T 1: ctx.h DConvW::gram1, computed in fp64 at pack time): H^2 + 3H FMAs per position instead of 2 x 2C x H
template <int C, bool FAST>
__global__ __launch_bounds__(256) void dconv_c1_stats_kernel(const float* __restrict__ h, int64_t nb, int64_t L,
                                                             const double* __restrict__ st_h,
                                                             const float* __restrict__ g1w, const float* __restrict__ g1b,
                                                             const float* __restrict__ gram, double* __restrict__ st_y) {
    constexpr int H = C / 8;
    __shared__ float tm[GN_TAB], tr[GN_TAB];
    __shared__ double sh[16];
    const int64_t P = nb * L;
    const int64_t p0 = (int64_t)blockIdx.x * 256;
    const int64_t gf = p0 / L, ng = (std::min<int64_t>(p0 + 255, P - 1)) / L - gf + 1;
    gn_table(st_h, (double)L * H, gf, ng, tm, tr);
    __syncthreads();
    const int64_t p = p0 + threadIdx.x;
    const bool valid = p < P;
    float s1 = 0.f, s2 = 0.f;
    if (valid) {
        float mean, rstd;
        gn_lookup(st_h, (double)L * H, p / L, gf, ng, tm, tr, mean, rstd);
        float hv[H];
        load_hg<H, FAST>(h, p, mean, rstd, g1w, g1b, hv);
        const float* G = gram;
        const float* v = gram + H * H;
        const float* ws = v + H;
        float q = 0.f, lv = 0.f, lw = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) {
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < H; ++k) t += G[j * H + k] * hv[k];
            q += hv[j] * t;
            lv += v[j] * hv[j];
            lw += ws[j] * hv[j];
        }
        s1 = ws[H] + lw;
        s2 = ws[H + 1] + (2.f * lv + q);
    }
    group_stats_add(st_y, p0, p, valid, L, s1, s2, sh);
}

// ---- c1app: one thread per position, all C channels: x[p][:] += scale * GLU(GN(y)); every weight / affine read is
// wave-uniform (scalar loads), x moves in 16-B chunks
template <int C, typename TS, bool FAST>
__global__ __launch_bounds__(256) void dconv_c1_apply_kernel(TS* __restrict__ x, const float* __restrict__ h, int64_t nb,
                                                             int64_t L, const double* __restrict__ st_h,
                                                             const float* __restrict__ g1w, const float* __restrict__ g1b,
                                                             const float* __restrict__ W, const float* __restrict__ bias,
                                                             const double* __restrict__ st_y,
                                                             const float* __restrict__ g2w, const float* __restrict__ g2b,
                                                             const float* __restrict__ scale) {
    constexpr int H = C / 8, N = 2 * C;
    constexpr int EPC = 16 / sizeof(TS);
    __shared__ float tm1[GN_TAB], tr1[GN_TAB], tm2[GN_TAB], tr2[GN_TAB];
    const int64_t P = nb * L;
    const int64_t p0 = (int64_t)blockIdx.x * 256;
    const int64_t gf = p0 / L, ng = (std::min<int64_t>(p0 + 255, P - 1)) / L - gf + 1;
    gn_table(st_h, (double)L * H, gf, ng, tm1, tr1);
    gn_table(st_y, (double)L * N, gf, ng, tm2, tr2);
    __syncthreads();
    const int64_t p = p0 + threadIdx.x;
    if (p >= P) return;
    const int64_t g = p / L;
    float m1, r1, m2, r2;
    gn_lookup(st_h, (double)L * H, g, gf, ng, tm1, tr1, m1, r1);
    gn_lookup(st_y, (double)L * N, g, gf, ng, tm2, tr2, m2, r2);
    float hv[H];
    load_hg<H, FAST>(h, p, m1, r1, g1w, g1b, hv);
    TS* xp = x + p * C;
#pragma unroll 2
    for (int c0 = 0; c0 < C; c0 += EPC) {
        uint4 q = *reinterpret_cast<const uint4*>(xp + c0);
        float e[EPC];
        unpack16<TS>(q, e);
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
            const int c = c0 + k;
            float a = bias[c], gt = bias[C + c];
#pragma unroll
            for (int j = 0; j < H; ++j) {
                a += W[c * H + j] * hv[j];
                gt += W[(C + c) * H + j] * hv[j];
            }
            a = (a - m2) * r2 * g2w[c] + g2b[c];
            gt = (gt - m2) * r2 * g2w[C + c] + g2b[C + c];
            const float o = scale[c] * (a * sigmoid<FAST>(gt));
            e[k] += o;                                // rounded once below (pack2bf: RNE, as f2bf)
        }
        if constexpr (sizeof(TS) == 2)
            q = make_uint4(pack2bf(e[0], e[1]), pack2bf(e[2], e[3]), pack2bf(e[4], e[5]), pack2bf(e[6], e[7]));
        else
            q = make_uint4(__float_as_uint(e[0]), __float_as_uint(e[1]), __float_as_uint(e[2]), __float_as_uint(e[3]));
        *reinterpret_cast<uint4*>(xp + c0) = q;
    }
}

template <int C, typename TS, bool FAST>
static void dconv_small_t(void* x, float* h, int64_t nb, int64_t L, int dil, const float* w3, const float* b3,
                          const float* g1w, const float* g1b, const float* w1, const float* b1, const float* gram1,
                          const float* g2w, const float* g2b, const float* scale, double* st_h, double* st_y,
                          hipStream_t s) {
    constexpr int H = C / 8, TILE = sizeof(TS) == 2 ? 256 : 128;
    const int64_t P = nb * L;
    const double px = (double)P;
    const double xb = (double)sizeof(TS);
    const char* tn = sizeof(TS) == 2 ? "unsignedshort" : "float";   // (rocprofv3 symbol spelling)
    {
        KScope ks(s);
        if (ks.on()) ks.begin(klabel("dconv_c3_kernel<%d,%s>", C, tn), 2.0 * px * H * 3 * C, px * (C * xb + H * 4));
        hipLaunchKernelGGL((dconv_c3_kernel<C, TS>), dim3((unsigned)((P + TILE - 1) / TILE)), dim3(256), 0, s,
                           (const TS*)x, nb, L, dil, w3, b3, h, st_h);
    }
    {
        KScope ks(s);
        if (ks.on()) ks.begin(klabel("dconv_c1_stats_kernel<%d,%s>", C, FAST ? "true" : "false"), 2.0 * px * (H * H + 3 * H), px * H * 4);
        hipLaunchKernelGGL((dconv_c1_stats_kernel<C, FAST>), dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, h, nb,
                           L, st_h, g1w, g1b, gram1, st_y);
    }
    {
        KScope ks(s);
        if (ks.on()) ks.begin(klabel("dconv_c1_apply_kernel<%d,%s,%s>", C, tn, FAST ? "true" : "false"), 2.0 * px * 2 * C * H, px * (H * 4 + 2 * C * xb));
        hipLaunchKernelGGL((dconv_c1_apply_kernel<C, TS, FAST>), dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s,
                           (TS*)x, h, nb, L, st_h, g1w, g1b, w1, b1, st_y, g2w, g2b, scale);
    }
}

int dconv_small_launch(void* x, int x_bf16, float* h, int64_t nb, int64_t L, int C, int dil, const float* w3,
                       const float* b3, const float* g1w, const float* g1b, const float* w1, const float* b1,
                       const float* gram1, const float* g2w, const float* g2b, const float* scale, double* st_h,
                       double* st_y, hipStream_t s, bool fast) {
    if (dil < 1 || dil > 2 || !gram1) return -2;
#define ATHD_DC(CC, TS, FA) \
    dconv_small_t<CC, TS, FA>(x, h, nb, L, dil, w3, b3, g1w, g1b, w1, b1, gram1, g2w, g2b, scale, st_h, st_y, s)
    if (C == 48) {
        if (x_bf16) { if (fast) ATHD_DC(48, bf16_t, true); else ATHD_DC(48, bf16_t, false); }
        else { if (fast) ATHD_DC(48, float, true); else ATHD_DC(48, float, false); }
    } else if (C == 96) {
        if (x_bf16) { if (fast) ATHD_DC(96, bf16_t, true); else ATHD_DC(96, bf16_t, false); }
        else { if (fast) ATHD_DC(96, float, true); else ATHD_DC(96, float, false); }
    } else {
        return -2;
    }
#undef ATHD_DC
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------
// Wide levels (C = 192, 384; bf16 mode): the DConv 1x1 apply  x += LayerScale(GLU(GN(W1 hb + b1)))  as a weights-
// resident MFMA pass (the pattern of convt4.hip) instead of a tiled GEMM: K = H = C/8 (24, 48) is one or two 32-wide
// K-steps, so the tiled GEMM (gemm3 / gemm5, one K-tile per 256-row tile) was all prologue and epilogue at ~7 GB/s
// per CU.  Here the packed 1x1 weights ([2C][64] bf16, GLU-interleaved columns, 48 / 96 KB) are loaded into LDS once
// per workgroup (XOR-swizzled 16-B chunks, conflict-free fragment reads as gemm3), and every wave walks 16-row units
// with no workgroup barrier: per unit the lane's activation fragment (row m, 8 hidden channels per K-step) comes from
// global memory, all of the row's residual channels are loaded up front, and the 2C columns are processed one
// GLU pair (32 packed columns -> 16 output channels) at a time: 2 x KS MFMAs, GroupNorm -> GLU -> LayerScale ->
// residual on the lane's 4 channels of row m, one 8-B store.
struct DcApply {
    const uint16_t* hb;        // [M][H] bf16 GELU(GN(h))
    const uint16_t* w;         // [2C][kp] packed GLU-interleaved 1x1 weights (kp == 64)
    const float* bias;         // [2C] packed
    const double* st;          // per group {sum, sumsq} of the 1x1 output
    const float* gn_w;         // [2C] packed
    const float* gn_b;
    const float* scale;        // [C] LayerScale
    uint16_t* x;               // [M][C] bf16 residual stream, updated in place
    int64_t M, L, gn_count;
    int kp;
    // fused rewrite (RW, C = 48 / 96, the layer's second DConv layer): out = GLU(Wr x + br) of the updated rows
    // instead of storing x; rw [2C][rkp] GLU-interleaved rows with the K order of dconv_rewrite_perm
    const uint16_t* rw = nullptr;
    const float* rbias = nullptr;  // [2C] packed
    uint16_t* out = nullptr;       // [M][C] bf16
    uint16_t* c4 = nullptr;        // optional [M][4]: channels 0..3 of out again (the decoder's compact skip)
    int rkp = 0;
};

template <int C, int NW, bool RW = false>
__global__ __launch_bounds__(NW * 64) void dconv_apply_kernel(const DcApply d) {
    constexpr int H = C / 8, KS = (H + 31) / 32, NP = C / 16;      // K-steps, GLU pairs (16 output channels each)
    constexpr int HS = H % 8 == 0 ? H : (H + 15) / 16 * 16;       // hidden row stride (H = 6, 12: padded to 16)
    constexpr int RK = (C + 31) / 32;                              // rewrite K-steps
    constexpr int RPB = RW ? (RK * 4 + 7) / 8 * 128 : 0;           // rewrite LDS row bytes (chunks padded to 8 k)
    __shared__ __attribute__((aligned(16))) char wl[2 * C * 128 + 2 * C * RPB];
    // per packed column: bias, GroupNorm weight, bias; per output channel: LayerScale; (RW) per packed rewrite column:
    // bias
    __shared__ __attribute__((aligned(16))) float cst[3 * 2 * C + C + (RW ? 2 * C : 0)];
    for (int i = threadIdx.x; i < 2 * C * 8; i += NW * 64) {
        const int row = i >> 3, ch = i & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(d.w + (int64_t)row * d.kp + ch * 8);
        *reinterpret_cast<uint4*>(wl + row * 128 + ((ch ^ (row & 7)) * 16)) = v;
    }
    for (int i = threadIdx.x; i < 2 * C; i += NW * 64) {
        cst[i] = d.bias[i];
        cst[2 * C + i] = d.gn_w[i];
        cst[4 * C + i] = d.gn_b[i];
    }
    for (int i = threadIdx.x; i < C; i += NW * 64) cst[6 * C + i] = d.scale[i];
    char* const wr = wl + 2 * C * 128;
    if constexpr (RW) {
        for (int i = threadIdx.x; i < 2 * C * (RPB / 16); i += NW * 64) {
            const int row = i / (RPB / 16), ch = i % (RPB / 16);
            const uint4 v = ch < RK * 4 ? *reinterpret_cast<const uint4*>(d.rw + (int64_t)row * d.rkp + ch * 8)
                                        : make_uint4(0u, 0u, 0u, 0u);
            *reinterpret_cast<uint4*>(wr + row * RPB + ((ch ^ (row & 7)) * 16)) = v;
        }
        for (int i = threadIdx.x; i < 2 * C; i += NW * 64) cst[7 * C + i] = d.rbias[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, fr = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nunits = (d.M + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * NW;
    typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
    auto wfrag = [&](int t, int ks) -> bf16v8 {
        return *reinterpret_cast<const bf16v8*>(wl + (16 * t + fr) * 128 + (((4 * ks + g) ^ (fr & 7)) * 16));
    };
    for (int64_t u = (int64_t)blockIdx.x * NW + wave; u < nunits; u += stride) {
        const int64_t m = u * 16 + fr;
        const bool ok = m < d.M;
        const int64_t mm = ok ? m : d.M - 1;
        // activation fragments: hidden channels 32 ks + 8 g .. + 7 of row mm (zero past H)
        bf16v8 af[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int k0 = 32 * ks + 8 * g;
            af[ks] = k0 < H ? *reinterpret_cast<const bf16v8*>(d.hb + mm * HS + k0) : bf16v8{};
        }
        // the row's residual channels 16 p + 4 g .. + 3, PG pairs per group; the next group's loads are issued
        // before the current group's MFMAs (the first group's before the GroupNorm parameters)
        constexpr int PG = NP % 6 == 0 ? 6 : NP, NG = NP / PG;
        static_assert(NP % PG == 0, "pair groups");
        static_assert(!RW || NG == 1, "the fused rewrite keeps all of the row's pairs in registers");
        uint2 xk[RW ? NP : 1];            // (RW) the updated bf16 x channels 16 p + 4 g .. + 3 of row m
        const uint16_t* xr = d.x + mm * C + 4 * g;
        uint2 rr[PG];
#pragma unroll
        for (int p = 0; p < PG; ++p) rr[p] = *reinterpret_cast<const uint2*>(xr + 16 * p);
        float gm, gr;
        gn_params(d.st, mm / d.L, d.gn_count, gm, gr);
        uint2* const xo = reinterpret_cast<uint2*>(d.x + mm * C + 4 * g);
#pragma unroll 1
        for (int gi = 0; gi < NG; ++gi) {
            uint2 rn[PG];
            if (gi + 1 < NG) {
#pragma unroll
                for (int p = 0; p < PG; ++p) rn[p] = *reinterpret_cast<const uint2*>(xr + 16 * (PG * (gi + 1) + p));
            }
            // (an opaque per-group LDS base: the column constants are read here, not hoisted out of the loops)
            int cb = 0;
            asm volatile("v_mov_b32 %0, 0" : "=v"(cb));
            const float* cs = cst + cb;
#pragma unroll
            for (int pp = 0; pp < PG; ++pp) {
                const int p = PG * gi + pp;
                f32x4_t aa = {0.f, 0.f, 0.f, 0.f}, ag = aa;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    aa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfrag(2 * p, ks), af[ks], aa, 0, 0, 0);
                    ag = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfrag(2 * p + 1, ks), af[ks], ag, 0, 0, 0);
                }
                const int na = 32 * p + 4 * g, oc = 16 * p + 4 * g;
                const float4 ba = *reinterpret_cast<const float4*>(cs + na), bg = *reinterpret_cast<const float4*>(cs + na + 16);
                const float4 wa = *reinterpret_cast<const float4*>(cs + 2 * C + na), wg = *reinterpret_cast<const float4*>(cs + 2 * C + na + 16);
                const float4 ca = *reinterpret_cast<const float4*>(cs + 4 * C + na), cg = *reinterpret_cast<const float4*>(cs + 4 * C + na + 16);
                const float4 sc = *reinterpret_cast<const float4*>(cs + 6 * C + oc);
                const float bav[4] = {ba.x, ba.y, ba.z, ba.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
                const float wav[4] = {wa.x, wa.y, wa.z, wa.w}, wgv[4] = {wg.x, wg.y, wg.z, wg.w};
                const float cav[4] = {ca.x, ca.y, ca.z, ca.w}, cgv[4] = {cg.x, cg.y, cg.z, cg.w};
                const float scv[4] = {sc.x, sc.y, sc.z, sc.w};
                const uint2 q = rr[pp];
                const float r4[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                                     __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u)};
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float a = (aa[e] + bav[e] - gm) * gr * wav[e] + cav[e];
                    const float gt = (ag[e] + bgv[e] - gm) * gr * wgv[e] + cgv[e];
                    o[e] = r4[e] + scv[e] * (a * sigmoid_fast(gt));
                }
                if constexpr (RW) xk[pp] = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
                else if (ok) xo[4 * p] = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
            }
            if (gi + 1 < NG) {
#pragma unroll
                for (int p = 0; p < PG; ++p) rr[p] = rn[p];
            }
        }
        if constexpr (RW) {
            // rewrite: the lane's x values of K-step ks are channels 32 ks + 4 g + {0..3} (pair 2 ks) and
            // 32 ks + 16 + 4 g + {0..3} (pair 2 ks + 1), which is the K order the packed rewrite weights carry, so the
            // B fragments are the registers as they are
            bf16v8 bx[RK];
#pragma unroll
            for (int ks = 0; ks < RK; ++ks) {
                const uint2 lo = xk[2 * ks], hi = 2 * ks + 1 < NP ? xk[2 * ks + 1 < NP ? 2 * ks + 1 : 0] : make_uint2(0u, 0u);
                const uint32_t w4[4] = {lo.x, lo.y, hi.x, hi.y};
                bx[ks] = __builtin_bit_cast(bf16v8, w4);
            }
            uint16_t* const orow = d.out + mm * C + 4 * g;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                f32x4_t aa = {0.f, 0.f, 0.f, 0.f}, ag = aa;
#pragma unroll
                for (int ks = 0; ks < RK; ++ks) {
                    const bf16v8 fa = *reinterpret_cast<const bf16v8*>(wr + (32 * q + fr) * RPB + (((4 * ks + g) ^ (fr & 7)) * 16));
                    const bf16v8 fg = *reinterpret_cast<const bf16v8*>(wr + (32 * q + 16 + fr) * RPB + (((4 * ks + g) ^ (fr & 7)) * 16));
                    aa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, bx[ks], aa, 0, 0, 0);
                    ag = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fg, bx[ks], ag, 0, 0, 0);
                }
                const int na = 32 * q + 4 * g;
                const float4 ba = *reinterpret_cast<const float4*>(cst + 7 * C + na);
                const float4 bg = *reinterpret_cast<const float4*>(cst + 7 * C + na + 16);
                const float bav[4] = {ba.x, ba.y, ba.z, ba.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (aa[e] + bav[e]) * sigmoid_fast(ag[e] + bgv[e]);
                const uint2 v = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
                if (ok) {
                    *reinterpret_cast<uint2*>(orow + 16 * q) = v;
                    if (q == 0 && g == 0 && d.c4) *reinterpret_cast<uint2*>(d.c4 + mm * 4) = v;
                }
            }
        }
    }
}

// Wide levels: the DConv conv3 (C -> H = C/8, 3 taps at dilation dil, zero padding at the GroupNorm row's ends)
// + the GroupNorm statistics of h, as a weights-resident pass (the pattern above; the tiled 256 x 32 GEMM streamed
// the taps' 64-wide K-tiles through LDS at ~2 TB/s).  The packed conv3 weights (H rows padded to 16 NT, K = 3C) sit in
// LDS with XOR-swizzled 16-B chunks; each wave walks a contiguous range of 16-row units (the tap rows +-dil stay in its
// L2 neighbourhood), loads its B fragments x[m + (tap - 1) dil][32 ks + 8 g ..] straight from global memory, and keeps
// the GroupNorm sums in fp64 per lane until the group changes (one wave reduction + atomic pair per change).
struct DcConv3 {
    const uint16_t* x;         // [M][C] bf16
    const uint16_t* w;         // [>= 16 NT][kp] packed conv3 weights, K = tap * C + ci
    const float* bias;         // [H]
    float* h;                  // [M][HF] f32 (HF = H, or 8 for H = 6)
    double* st;                // per group {sum, sumsq}
    int64_t M, L;
    int kp, dil;
};

template <int C, int NW>
__global__ __launch_bounds__(NW * 64) void dconv_conv3_kernel(const DcConv3 d) {
    constexpr int H = C / 8, NT = (H + 15) / 16, KS = (C + 31) / 32, K = 3 * C;
    constexpr int HF = H % 4 == 0 ? H : (H + 7) / 8 * 8;   // f32 hidden row stride (16-B stores)
    constexpr int RB = (K / 8 + 7) / 8 * 128;               // LDS row bytes (chunks padded to a multiple of 8: the
                                                            // XOR swizzle stays inside the row, e.g. C = 96: 36 -> 40)
    __shared__ __attribute__((aligned(16))) char wl[16 * NT * RB];
    for (int i = threadIdx.x; i < 16 * NT * (RB / 16); i += NW * 64) {    // (padding chunks zeroed: the masked
        const int row = i / (RB / 16), q = i % (RB / 16);                      // K-steps of C = 48 multiply them by 0)
        const uint4 v = q < K / 8 ? *reinterpret_cast<const uint4*>(d.w + (int64_t)row * d.kp + q * 8)
                                  : make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(wl + row * RB + ((q ^ (row & 7)) * 16)) = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, fr = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
    const int64_t nunits = (d.M + 15) / 16;
    const int64_t nw = (int64_t)gridDim.x * NW, wid = (int64_t)blockIdx.x * NW + wave;
    const int64_t u0 = nunits * wid / nw, u1 = nunits * (wid + 1) / nw;
    float bj[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) bj[j][e] = 16 * j + 4 * g + e < H ? d.bias[16 * j + 4 * g + e] : 0.f;
    int64_t cur_b = -1;
    double r1 = 0.0, r2 = 0.0;
    auto flush = [&]() {
        if (cur_b >= 0) {
            const double t1 = wave_sum_d(r1), t2 = wave_sum_d(r2);
            if (lane == 0) {
                atomicAdd(&d.st[2 * cur_b], t1);
                atomicAdd(&d.st[2 * cur_b + 1], t2);
            }
        }
        r1 = r2 = 0.0;
    };
    // unit epilogue: h store + GroupNorm sums (the unit's rows belong to group gb0 of its first row or, past a
    // boundary, gb0 + 1: L >= 16)
    auto finish = [&](int64_t u, const f32x4_t* acc) {
        const int64_t m = u * 16 + fr;
        const bool ok = m < d.M;
        const int64_t mm = ok ? m : d.M - 1;
        const int64_t gb = mm / d.L;
        const int64_t gb0 = (u * 16) / d.L;
        float s1a = 0.f, s2a = 0.f, s1b = 0.f, s2b = 0.f;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[j][e] + bj[j][e];
            const int c0 = 16 * j + 4 * g;
            if (ok && c0 < H) {        // (H = 6: channels 6, 7 of the second chunk are 0 - zero weight rows and bias)
                *reinterpret_cast<float4*>(d.h + mm * HF + c0) = make_float4(v[0], v[1], v[2], v[3]);
                const float p1 = (v[0] + v[1]) + (v[2] + v[3]);
                const float p2 = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
                if (gb == gb0) { s1a += p1; s2a += p2; } else { s1b += p1; s2b += p2; }
            }
        }
        if (gb0 != cur_b) {
            flush();
            cur_b = gb0;
        }
        r1 += (double)s1a;
        r2 += (double)s2a;
        const bool split = __any(gb != gb0);
        if (split) {
            flush();
            cur_b = gb0 + 1;
            r1 = (double)s1b;
            r2 = (double)s2b;
        }
    };
    // C = 96, 192: steps (unit, tap) in ping-pong buffers (below); C = 48, 384 measured slower that way (one box: 0.34
    // -> 0.37 and 0.17 -> 0.18 ms) and keep one tap at a time with the zeroing at the load
    constexpr bool PP = C == 96 || C == 192;
    // lane row of unit u (clamped) and its position in the group row (32-bit: M < 2^31, launcher)
    auto unit_row = [&](int64_t u, int64_t& mm, int& t) {
        const int64_t m = u * 16 + fr;
        mm = m < d.M ? m : d.M - 1;
        t = (int)((uint32_t)mm % (uint32_t)d.L);
    };
    // B fragments of one tap: x[mm + (tap - 1) dil][32 ks + 8 g ..]; returns whether the tap row lies inside the group
    // row.  PP: the loads are unconditional (rows outside the group read the lane's own row, K-steps past C its first
    // chunk) and the fragments are zeroed where they are used, so a prefetched step is not waited for at the load.
    auto load_tap = [&](int64_t mm, int t, int tap, bf16v8* bf) -> bool {
        const int tt = t + (tap - 1) * d.dil;
        const bool in = tt >= 0 && tt < (int)d.L;
        const uint16_t* xr = d.x + (mm + (in ? (int64_t)(tap - 1) * d.dil : 0)) * C + 8 * g;
        if constexpr (PP) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                bf[ks] = *reinterpret_cast<const bf16v8*>(xr + (32 * ks + 8 * g < C ? 32 * ks : 0));
        } else {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                bf[ks] = in && 32 * ks + 8 * g < C ? *reinterpret_cast<const bf16v8*>(xr + 32 * ks) : bf16v8{};
        }
        return in;
    };
    auto mfma_tap = [&](int tap, bool in, const bf16v8* bf, f32x4_t* acc) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int q = (tap * C + 32 * ks) / 8 + g;
            const bf16v8 b = !PP || (in && 32 * ks + 8 * g < C) ? bf[ks] : bf16v8{};
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const bf16v8 af = *reinterpret_cast<const bf16v8*>(wl + (16 * j + fr) * RB + ((q ^ (fr & 7)) * 16));
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b, acc[j], 0, 0, 0);
            }
        }
    };
    f32x4_t acc[NT];
    if constexpr (PP) {
        // the load side runs one step ahead of the compute side: the next step's fragments are in flight during
        // this step's MFMAs and the unit epilogue (registers: 2 x 4 KS)
        int64_t lu = u0, lmm = 0, cu = u0;
        int ltap = 0, lt = 0, ctap = 0;
        if (u0 < u1) unit_row(u0, lmm, lt);
        auto advance = [&]() {
            if (++ltap == 3) {
                ltap = 0;
                if (++lu < u1) unit_row(lu, lmm, lt);
            }
        };
        auto compute = [&](bool in, const bf16v8* bf) {
            if (ctap == 0) {
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
            mfma_tap(ctap, in, bf, acc);
            if (ctap == 2) {
                finish(cu, acc);
                ctap = 0;
                ++cu;
            } else {
                ++ctap;
            }
        };
        bf16v8 ba[KS], bb[KS];
        bool ia = false, ib = false;
        if (lu < u1) { ia = load_tap(lmm, lt, ltap, ba); advance(); }
#pragma unroll 1
        while (cu < u1) {
            if (lu < u1) { ib = load_tap(lmm, lt, ltap, bb); advance(); }
            compute(ia, ba);
            if (cu >= u1) break;
            if (lu < u1) { ia = load_tap(lmm, lt, ltap, ba); advance(); }
            compute(ib, bb);
        }
    } else {
        for (int64_t u = u0; u < u1; ++u) {
            int64_t mm;
            int t;
            unit_row(u, mm, t);
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
            for (int tap = 0; tap < 3; ++tap) {
                bf16v8 bf[KS];
                const bool in = load_tap(mm, t, tap, bf);
                mfma_tap(tap, in, bf, acc);
            }
            finish(u, acc);
        }
    }
    flush();
}

bool dconv_conv3_supported(int C, int H, int kp, int64_t L) {
    return (C == 48 || C == 96 || C == 192 || C == 384) && H == C / 8 && kp >= 3 * C && L >= 16;
}

int dconv_conv3_launch(const uint16_t* x, const uint16_t* w, int kp, const float* bias, float* h, double* st,
                       int64_t M, int64_t L, int C, int dil, hipStream_t s) {
    if (!dconv_conv3_supported(C, C / 8, kp, L) || M <= 0 || M >= (1LL << 31)) return -1;
    DcConv3 d;
    d.x = x; d.w = w; d.bias = bias; d.h = h; d.st = st; d.M = M; d.L = L; d.kp = kp; d.dil = dil;
    const int cus = device_cus();
    KScope ks(s);
    if (ks.on()) {
        const double H = C / 8;
        ks.begin(klabel("dconv_conv3_kernel<%d>", C), 2.0 * M * H * 3 * C, (double)M * (C * 2 + H * 4));
    }
    const int64_t units = (M + 15) / 16;
    if (C == 48) {       // 6 KB of weights
        const int64_t blocks = std::min<int64_t>(3LL * cus, (units + 7) / 8);
        hipLaunchKernelGGL((dconv_conv3_kernel<48, 8>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else if (C == 96) {       // 10 KB of weights
        const int64_t blocks = std::min<int64_t>(3LL * cus, (units + 7) / 8);
        hipLaunchKernelGGL((dconv_conv3_kernel<96, 8>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else if (C == 192) {      // 36 KB of weights: 2 eight-wave workgroups per CU
        const int64_t blocks = std::min<int64_t>(2LL * cus, (units + 7) / 8);
        hipLaunchKernelGGL((dconv_conv3_kernel<192, 8>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else {             // 110 KB: one 16-wave workgroup per CU
        const int64_t blocks = std::min<int64_t>((int64_t)cus, (units + 15) / 16);
        hipLaunchKernelGGL((dconv_conv3_kernel<384, 16>), dim3((unsigned)blocks), dim3(1024), 0, s, d);
    }
    return (int)hipGetLastError();
}

bool dconv_apply_supported(int C, int H, int kp, int64_t M) {
    return (C == 48 || C == 96 || C == 192 || C == 384) && H == C / 8 && kp == 64 && M > 0;
}

int dconv_apply_launch(const uint16_t* hb, const uint16_t* w, int kp, const float* bias, const double* st,
                       const float* gn_w, const float* gn_b, const float* scale, uint16_t* x, int64_t M, int64_t L,
                       int C, hipStream_t s, const DcRewrite* rwd) {
    if (!dconv_apply_supported(C, C / 8, kp, M)) return -1;
    if (rwd && !(C == 48 || C == 96)) return -1;
    DcApply d;
    d.hb = hb; d.w = w; d.bias = bias; d.st = st; d.gn_w = gn_w; d.gn_b = gn_b; d.scale = scale; d.x = x;
    d.M = M; d.L = L; d.gn_count = L * 2 * C; d.kp = kp;
    if (rwd) {
        if (rwd->kp < (C + 31) / 32 * 32) return -1;
        d.rw = rwd->w; d.rkp = rwd->kp; d.rbias = rwd->bias; d.out = rwd->out; d.c4 = rwd->c4;
    }
    const int cus = device_cus();
    KScope ks(s);
    if (ks.on()) {
        const double H = C / 8;
        if (rwd)
            ks.begin(klabel("dconv_apply_kernel<%d,rewrite>", C), 2.0 * M * 2 * C * (H + C),
                     (double)M * (H * 2 + 2.0 * C * 2 + (rwd->c4 ? 8 : 0)));
        else
            ks.begin(klabel("dconv_apply_kernel<%d>", C), 2.0 * M * 2 * C * H, (double)M * (H * 2 + 2.0 * C * 2));
    }
    const int64_t units = (M + 15) / 16;
    if (rwd) {           // C = 48: 25 KB of LDS, C = 96: 77 KB
        const int64_t blocks = std::min<int64_t>((C == 48 ? 3LL : 2LL) * cus, (units + 7) / 8);
        if (C == 48) hipLaunchKernelGGL((dconv_apply_kernel<48, 8, true>), dim3((unsigned)blocks), dim3(512), 0, s, d);
        else hipLaunchKernelGGL((dconv_apply_kernel<96, 8, true>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else if (C == 48) {
        const int64_t blocks = std::min<int64_t>(3LL * cus, (units + 7) / 8);
        hipLaunchKernelGGL((dconv_apply_kernel<48, 8>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else if (C == 96) {       // (time-branch level 1: hidden rows padded to 16 channels by gn_gelu_mom; 27 KB of LDS)
        const int64_t blocks = std::min<int64_t>(3LL * cus, (units + 7) / 8);
        hipLaunchKernelGGL((dconv_apply_kernel<96, 8>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else if (C == 192) {      // 48 KB of weights: two 8-wave workgroups per CU
        const int64_t blocks = std::min<int64_t>(2LL * cus, (units + 7) / 8);
        hipLaunchKernelGGL((dconv_apply_kernel<192, 8>), dim3((unsigned)blocks), dim3(512), 0, s, d);
    } else {             // 96 KB: one 16-wave workgroup per CU
        const int64_t blocks = std::min<int64_t>((int64_t)cus, (units + 15) / 16);
        hipLaunchKernelGGL((dconv_apply_kernel<384, 16>), dim3((unsigned)blocks), dim3(1024), 0, s, d);
    }
    return (int)hipGetLastError();
}

}  // namespace athd
