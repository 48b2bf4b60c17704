// FreqDecoder level 1 computed from the 32-row level-0 output instead of the 259-row resized tensor
// (ATHTDemucs_v2.py:90-103 for i = 0, 1).
//
// The reference materialises D0 = resize_H(S, 32 -> Hd) + 0.1 * resize_H(skip3, 8 -> Hd) (S = GELU(GN(ConvT0(x)))),
// then runs ConvTranspose2d (8,1)/(4,1)/(2,0) on it.  Everything between S and the level-1 ConvT output Y is linear,
// so with Z_k[j] = W_k S[j] and Zs_k[m] = W_k skip3[m] (one GEMM each, N = 8 taps x Co, K = Ci; forward.cpp):
//   T_u[k]   = W_k D0[u] = lerp(Z_k[i0(u)], Z_k[i1(u)]) + 0.1 * lerp(Zs_k[p0(u)], Zs_k[p1(u)])
//   Y[4u+r]  = b + T_u[r+2] + (r < 2 ? T_{u-1}[r+6] : T_{u+1}[r-2])            (k = o + 2 - 4u)
// This is the same arithmetic re-associated: 8x fewer MACs than the ConvT on Hd rows, and D0 never exists.
// Two passes, both sweeping u in order per (item, w, 4 channels) with the Z rows the resize touches held in
// registers (a row changes every ~Hd/32 steps):
//   fdec_lr_stats_kernel: GroupNorm(1) {sum, sumsq} over all 4*Hd ConvT rows;
//   fdec_lr_merge_kernel: rows 4d+1, 4d+2 (the only rows the exact /4 bilinear resize reads) -> GN -> GELU ->
//                         lerp -> + 0.1 * resize_H(skip2) -> D1 [item][d][w][Co].
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace athd {

namespace {

template <typename ZT>
ATHD_DEV void ld4(const ZT* p, float* v) {
    if constexpr (sizeof(ZT) == 2) {
        const uint2 q = *reinterpret_cast<const uint2*>(p);
        const bf16_t* h = reinterpret_cast<const bf16_t*>(&q);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = bf2f(h[j]);
    } else {
        const float4 a = *reinterpret_cast<const float4*>(p);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    }
}

// tap index of slot t: all 8 taps (stats pass) or {0, 3, 4, 7} (merge pass: rows 4d+1, 4d+2)
template <int NT>
ATHD_DEV constexpr int tap_of(int t) { return NT == 8 ? t : (t == 0 ? 0 : t == 1 ? 3 : t == 2 ? 4 : 7); }

// The two rows (i0, i1) a lerp reads, as r0 = scale * row[i0] and dr = scale * (row[i1] - row[i0]) per tap slot.
template <typename ZT, int NT>
struct LerpRows {
    float r0[NT][4], dr[NT][4];
    int c0 = -1, c1 = -1;
    ATHD_DEV void update(const ZT* base, int64_t rowpitch, int Co, const LinIdx& li, float scale) {
        if (li.i0 == c0 && li.i1 == c1) return;
        c0 = li.i0;
        c1 = li.i1;
        float a[NT][4], b[NT][4];
#pragma unroll
        for (int t = 0; t < NT; ++t) ld4(base + (int64_t)li.i0 * rowpitch + tap_of<NT>(t) * Co, a[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) ld4(base + (int64_t)li.i1 * rowpitch + tap_of<NT>(t) * Co, b[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                r0[t][j] = a[t][j] * scale;
                dr[t][j] = (b[t][j] - a[t][j]) * scale;
            }
    }
    ATHD_DEV float at(int t, int j, float l1) const { return fmaf(l1, dr[t][j], r0[t][j]); }
};

struct LrThread {
    int item, seg, w, c;
    bool active;
};

ATHD_DEV LrThread lr_thread(const LowRankDesc& d) {
    LrThread t;
    const int cg = d.Co / 4;
    const int q = blockIdx.x * 256 + threadIdx.x;
    t.active = q < d.W * cg;
    t.w = t.active ? q / cg : 0;
    t.c = t.active ? (q % cg) * 4 : 0;
    t.item = blockIdx.y;
    t.seg = t.item / d.P;
    return t;
}

}  // namespace

template <typename ZT>
__global__ __launch_bounds__(256) void fdec_lr_stats_kernel(const LowRankDesc d) {
    const LrThread th = lr_thread(d);
    const int N8 = 8 * d.Co;
    const int64_t rp = (int64_t)d.W * N8;
    const ZT* zb = (const ZT*)d.Z + (int64_t)th.item * d.Hs * rp + (int64_t)th.w * N8 + th.c;
    const ZT* sb = (const ZT*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    float bias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bias[j] = d.bias[th.c + j];
    LerpRows<ZT, 8> zr, sr;
    float prev[4][4] = {};     // T_{v-1}[4..7]
    double s1 = 0.0, s2 = 0.0;
    if (th.active) {
        for (int v = 0; v <= d.Hd; ++v) {
            float T[8][4];
            if (v < d.Hd) {
                const LinIdx a = lin_index(v, d.Hs, d.Hd);
                const LinIdx k = lin_index(v, d.Hk, d.Hd);
                zr.update(zb, rp, d.Co, a, 1.0f);
                sr.update(sb, rp, d.Co, k, 0.1f);
#pragma unroll
                for (int t = 0; t < 8; ++t)
#pragma unroll
                    for (int j = 0; j < 4; ++j) T[t][j] = zr.at(t, j, a.l1) + sr.at(t, j, k.l1);
            } else {
#pragma unroll
                for (int t = 0; t < 8; ++t)
#pragma unroll
                    for (int j = 0; j < 4; ++j) T[t][j] = 0.f;
            }
            float p1 = 0.f, p2 = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (v >= 1) {     // rows 4(v-1)+2, 4(v-1)+3
                    const float y2 = bias[j] + prev[0][j] + T[0][j];
                    const float y3 = bias[j] + prev[1][j] + T[1][j];
                    p1 += y2 + y3;
                    p2 += y2 * y2 + y3 * y3;
                }
                if (v < d.Hd) {   // rows 4v, 4v+1
                    const float y0 = bias[j] + T[2][j] + prev[2][j];
                    const float y1 = bias[j] + T[3][j] + prev[3][j];
                    p1 += y0 + y1;
                    p2 += y0 * y0 + y1 * y1;
                }
            }
            s1 += (double)p1;
            s2 += (double)p2;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) prev[t][j] = T[4 + t][j];
        }
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    __shared__ double sh[2][4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][wv] = s1; sh[1][wv] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&d.stats[2 * th.item], sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3]);
        atomicAdd(&d.stats[2 * th.item + 1], sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3]);
    }
}

template <typename ZT, bool FAST>
__global__ __launch_bounds__(256) void fdec_lr_merge_kernel(const LowRankDesc d) {
    const LrThread th = lr_thread(d);
    if (!th.active) return;
    const int N8 = 8 * d.Co;
    const int64_t rp = (int64_t)d.W * N8;
    const ZT* zb = (const ZT*)d.Z + (int64_t)th.item * d.Hs * rp + (int64_t)th.w * N8 + th.c;
    const ZT* sb = (const ZT*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    float mean, rstd;
    gn_params(d.stats, th.item, 4LL * d.Hd * d.W * d.Co, mean, rstd);
    float bias[4], gw[4], gb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bias[j] = d.bias[th.c + j];
        gw[j] = d.gn_w[th.c + j];
        gb[j] = d.gn_b[th.c + j];
    }
    // skip2 [seg][H_skip][W][C_skip], channels [0, Co)
    const int64_t kp = (int64_t)d.W * d.C_skip;
    const int64_t kb = (int64_t)th.seg * d.H_skip * kp + (int64_t)th.w * d.C_skip + th.c;
    int k0c = -1, k1c = -1;
    float ka[4] = {}, kbv[4] = {};
    const int64_t ob = (int64_t)th.item * d.Hd * d.W * d.Co + (int64_t)th.w * d.Co + th.c;
    const int64_t op = (int64_t)d.W * d.Co;

    LerpRows<ZT, 4> zr, sr;       // slots: taps 0, 3, 4, 7
    float cur3[4] = {}, cur4[4] = {}, cur7[4] = {}, prev7[4] = {};
    for (int v = 0; v <= d.Hd; ++v) {
        float T[4][4];
        if (v < d.Hd) {
            const LinIdx a = lin_index(v, d.Hs, d.Hd);
            const LinIdx k = lin_index(v, d.Hk, d.Hd);
            zr.update(zb, rp, d.Co, a, 1.0f);
            sr.update(sb, rp, d.Co, k, 0.1f);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) T[t][j] = zr.at(t, j, a.l1) + sr.at(t, j, k.l1);
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) T[t][j] = 0.f;
        }
        if (v >= 1) {
            const int dd = v - 1;     // output row: resize of ConvT rows 4dd+1 (i0) and 4dd+2 (i1)
            const LinIdx rr = lin_index(dd, 4 * d.Hd, d.Hd);
            const LinIdx lj = lin_index(dd, d.H_skip, d.Hd);
            if (lj.i0 != k0c || lj.i1 != k1c) {
                k0c = lj.i0;
                k1c = lj.i1;
                if (d.skip_bf16) {
                    ld4((const bf16_t*)d.skip + kb + (int64_t)lj.i0 * kp, ka);
                    ld4((const bf16_t*)d.skip + kb + (int64_t)lj.i1 * kp, kbv);
                } else {
                    ld4((const float*)d.skip + kb + (int64_t)lj.i0 * kp, ka);
                    ld4((const float*)d.skip + kb + (int64_t)lj.i1 * kp, kbv);
                }
            }
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float y1 = bias[j] + cur3[j] + prev7[j];
                const float y2 = bias[j] + cur4[j] + T[0][j];
                const float g1 = gelu<FAST>((y1 - mean) * rstd * gw[j] + gb[j]);
                const float g2 = gelu<FAST>((y2 - mean) * rstd * gw[j] + gb[j]);
                const float sv = (lj.l0 * ka[j] + lj.l1 * kbv[j]) * 0.1f;
                o[j] = (rr.l0 * g1 + rr.l1 * g2) + sv;
            }
            const int64_t oi = ob + (int64_t)dd * op;
            if (d.out_bf16) {
                bf16_t h[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) h[j] = f2bf(o[j]);
                *reinterpret_cast<uint2*>((bf16_t*)d.out + oi) = *reinterpret_cast<uint2*>(h);
            } else {
                *reinterpret_cast<float4*>((float*)d.out + oi) = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            prev7[j] = cur7[j];
            cur3[j] = T[1][j];
            cur4[j] = T[2][j];
            cur7[j] = T[3][j];
        }
    }
}

static bool lr_ok(const LowRankDesc& d) {
    return d.Z && d.Zs && d.bias && d.stats && d.Co % 4 == 0 && d.Hd > 0 && d.W > 0 && d.P > 0 && d.NI % d.P == 0 &&
           d.Hs > 0 && d.Hk > 0;
}

int fdec_lr_stats_launch(const LowRankDesc& d, hipStream_t s) {
    if (!lr_ok(d)) return -1;
    const dim3 grid((unsigned)((d.W * (d.Co / 4) + 255) / 256), (unsigned)d.NI);
    KScope ks(s);
    if (ks.on()) {
        // unique bytes: Z of every item + Zs of every segment, read once
        const double ze = d.z_bf16 ? 2.0 : 4.0;
        const double by = ze * 8.0 * d.Co * d.W * ((double)d.NI * d.Hs + (double)(d.NI / d.P) * d.Hk);
        ks.begin(d.z_bf16 ? "fdec_lr_stats_kernel<unsignedshort>" : "fdec_lr_stats_kernel<float>", 0.0, by);
    }
    if (d.z_bf16) hipLaunchKernelGGL(fdec_lr_stats_kernel<bf16_t>, grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL(fdec_lr_stats_kernel<float>, grid, dim3(256), 0, s, d);
    return (int)hipGetLastError();
}

int fdec_lr_merge_launch(const LowRankDesc& d, hipStream_t s) {
    if (!lr_ok(d) || !d.gn_w || !d.gn_b || !d.skip || !d.out || d.C_skip < d.Co || d.C_skip % 4 != 0) return -1;
    const dim3 grid((unsigned)((d.W * (d.Co / 4) + 255) / 256), (unsigned)d.NI);
    KScope ks(s);
    if (ks.on()) {
        // unique bytes: half the taps of Z / Zs, the skip rows the resize touches (once per segment), the output
        const double ze = d.z_bf16 ? 2.0 : 4.0;
        const double skip_rows = std::min<double>(d.H_skip, 2.0 * d.Hd);
        const double by = ze * 4.0 * d.Co * d.W * ((double)d.NI * d.Hs + (double)(d.NI / d.P) * d.Hk) +
                          (double)(d.NI / d.P) * skip_rows * d.W * d.Co * (d.skip_bf16 ? 2 : 4) +
                          (double)d.NI * d.Hd * d.W * d.Co * (d.out_bf16 ? 2 : 4);
        ks.begin(klabel("fdec_lr_merge_kernel<%s,%s>", d.z_bf16 ? "unsignedshort" : "float",
                        d.fast_gelu ? "true" : "false"), 0.0, by);
    }
    if (d.z_bf16) {
        if (d.fast_gelu) hipLaunchKernelGGL((fdec_lr_merge_kernel<bf16_t, true>), grid, dim3(256), 0, s, d);
        else hipLaunchKernelGGL((fdec_lr_merge_kernel<bf16_t, false>), grid, dim3(256), 0, s, d);
    } else {
        if (d.fast_gelu) hipLaunchKernelGGL((fdec_lr_merge_kernel<float, true>), grid, dim3(256), 0, s, d);
        else hipLaunchKernelGGL((fdec_lr_merge_kernel<float, false>), grid, dim3(256), 0, s, d);
    }
    return (int)hipGetLastError();
}

}  // namespace athd
