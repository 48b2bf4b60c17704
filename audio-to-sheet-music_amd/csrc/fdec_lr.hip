// FreqDecoder level 1 computed from the 32-row level-0 output instead of the 259-row resized tensor
// (ATHTDemucs_v2.py:90-103 for i = 0, 1).
//
// The reference materialises D0 = resize_H(S, 32 -> Hd) + 0.1 * resize_H(skip3, 8 -> Hd) (S = GELU(GN(ConvT0(x)))),
// then runs ConvTranspose2d (8,1)/(4,1)/(2,0) on it.  Everything between S and the level-1 ConvT output Y is linear,
// so with Z_k[j] = W_k S[j] and Zs_k[m] = W_k skip3[m] (one GEMM each, N = 8 taps x Co, K = Ci; forward.cpp):
//   T_u[k]   = W_k D0[u] = lerp(Z_k[i0(u)], Z_k[i1(u)]) + 0.1 * lerp(Zs_k[p0(u)], Zs_k[p1(u)])
//   Y[4u+r]  = b + T_u[r+2] + (r < 2 ? T_{u-1}[r+6] : T_{u+1}[r-2])            (k = o + 2 - 4u)
// This is the same arithmetic re-associated: 8x fewer MACs than the ConvT on Hd rows, and D0 never exists.
// Two passes, both sweeping u in order per (item, w, channel pair) with the Z rows the resize touches held in
// registers (a row changes every ~Hd/32 steps) and the per-step resize indices read from an LDS table.  Both
// passes are VALU-bound: the arithmetic runs on packed fp32 pairs (v_pk_fma_f32), the bias and the skip row
// base are folded into one per-row-change base so a step costs two packed FMAs per tap:
//   fdec_lr_stats_kernel: GroupNorm(1) {sum, sumsq} over all 4*Hd ConvT rows;
//   fdec_lr_merge_kernel: rows 4d+1, 4d+2 (the only rows the exact /4 bilinear resize reads) -> GN -> GELU ->
//                         lerp -> + 0.1 * resize_H(skip2) -> D1 [item][d][w][Co].
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace athd {

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));

ATHD_DEV f2 splat(float v) { return (f2){v, v}; }
ATHD_DEV f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <typename T>
ATHD_DEV f2 ld2(const T* p) {
    if constexpr (sizeof(T) == 2) {
        const uint32_t q = *reinterpret_cast<const uint32_t*>(p);
        return (f2){__uint_as_float(q << 16), __uint_as_float(q & 0xFFFF0000u)};
    } else {
        return *reinterpret_cast<const f2*>(p);
    }
}

// GELU on a packed pair: common.h::gelu_fast's tanh form (bf16 mode) or exact erf (f32 mode)
template <bool FAST>
ATHD_DEV f2 gelu2(f2 x) {
    if constexpr (!FAST) {
        return (f2){gelu_erf(x.x), gelu_erf(x.y)};
    } else {
        return (f2){gelu_fast(x.x), gelu_fast(x.y)};
    }
}

// Per-step resize indices of lin_index(v, in, Hd), tabulated once per block in LDS for v < LR_TAB.
constexpr int LR_TAB = 1024;
struct LrTab {
    int ij;     // i0 | i1 << 16
    float l1;
};
ATHD_DEV void lr_fill(LrTab* t, int n, int in, int out) {
    for (int v = threadIdx.x; v < n && v < LR_TAB; v += blockDim.x) {
        const LinIdx li = lin_index(v, in, out);
        t[v].ij = li.i0 | (li.i1 << 16);
        t[v].l1 = li.l1;
    }
}
struct Lerp {
    int i0, i1;
    float l1;
};
ATHD_DEV Lerp lr_get(const LrTab* t, int v, int in, int out) {
    Lerp r;
    if (v < LR_TAB) {
        const LrTab e = t[v];
        const int ij = __builtin_amdgcn_readfirstlane(e.ij);
        r.i0 = ij & 0xFFFF;
        r.i1 = ij >> 16;
        r.l1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(e.l1)));
    } else {
        const LinIdx li = lin_index(v, in, out);
        r.i0 = li.i0;
        r.i1 = li.i1;
        r.l1 = li.l1;
    }
    return r;
}

// tap index of slot t: all 8 taps (stats pass) or {0, 3, 4, 7} (merge pass: rows 4d+1, 4d+2)
template <int NT>
ATHD_DEV constexpr int tap_of(int t) { return NT == 8 ? t : (t == 0 ? 0 : t == 1 ? 3 : t == 2 ? 4 : 7); }

// The two rows (i0, i1) one lerp reads: r0 = scale * row[i0], dr = scale * (row[i1] - row[i0]) per tap slot, so the
// lerp is fma(l1, dr, r0) (same value as l0 * a + l1 * b up to rounding; l0 = 1 - l1).
template <typename ZT, int NT>
struct LerpRows {
    f2 r0[NT], dr[NT];
    int c0 = -1, c1 = -1;
    ATHD_DEV bool update(const ZT* base, int64_t rowpitch, int Co, const Lerp& li, float scale) {
        if (li.i0 == c0 && li.i1 == c1) return false;
        c0 = li.i0;
        c1 = li.i1;
        f2 a[NT], b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) a[t] = ld2(base + (int64_t)li.i0 * rowpitch + tap_of<NT>(t) * Co);
#pragma unroll
        for (int t = 0; t < NT; ++t) b[t] = ld2(base + (int64_t)li.i1 * rowpitch + tap_of<NT>(t) * Co);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            r0[t] = a[t] * splat(scale);
            dr[t] = (b[t] - a[t]) * splat(scale);
        }
        return true;
    }
};

struct LrThread {
    int item, seg, w, c;
    bool active;
};

ATHD_DEV LrThread lr_thread(const LowRankDesc& d) {
    LrThread t;
    const int cg = d.Co / 2;
    const int q = blockIdx.x * 256 + threadIdx.x;
    t.active = q < d.W * cg;
    t.w = t.active ? q / cg : 0;
    t.c = t.active ? (q % cg) * 2 : 0;
    t.item = blockIdx.y;
    t.seg = t.item / d.P;
    return t;
}

}  // namespace

template <typename ZT>
__global__ __launch_bounds__(256) void fdec_lr_stats_kernel(const LowRankDesc d) {
    __shared__ LrTab tz[LR_TAB], tk[LR_TAB];
    lr_fill(tz, d.Hd, d.Hs, d.Hd);
    lr_fill(tk, d.Hd, d.Hk, d.Hd);
    __syncthreads();
    const LrThread th = lr_thread(d);
    const int N8 = 8 * d.Co;
    const int64_t rp = (int64_t)d.W * N8;
    const ZT* zb = (const ZT*)d.Z + (int64_t)th.item * d.Hs * rp + (int64_t)th.w * N8 + th.c;
    const ZT* sb = (const ZT*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    const f2 bias = ld2(d.bias + th.c);
    LerpRows<ZT, 8> zr, sr;
    f2 base[8];                // r0(Z) + r0(Zs) (+ bias on taps 2..5: every output row has exactly one of those)
    f2 prev[4] = {};           // T_{v-1}[4..7]
    double s1 = 0.0, s2 = 0.0;
    if (th.active) {
        for (int v0 = 0; v0 <= d.Hd; v0 += 16) {
            f2 a1 = {}, a2 = {};
            const int v1 = min(v0 + 16, d.Hd + 1);
            for (int v = v0; v < v1; ++v) {
                f2 T[8];
                if (v < d.Hd) {
                    const Lerp a = lr_get(tz, v, d.Hs, d.Hd);
                    const Lerp k = lr_get(tk, v, d.Hk, d.Hd);
                    const bool cz = zr.update(zb, rp, d.Co, a, 1.0f);
                    const bool cs = sr.update(sb, rp, d.Co, k, 0.1f);
                    if (cz || cs) {
#pragma unroll
                        for (int t = 0; t < 8; ++t) base[t] = zr.r0[t] + sr.r0[t] + ((t >= 2 && t <= 5) ? bias : f2{});
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t) T[t] = pfma(splat(a.l1), zr.dr[t], pfma(splat(k.l1), sr.dr[t], base[t]));
                } else {
#pragma unroll
                    for (int t = 0; t < 8; ++t) T[t] = f2{};
                }
                if (v >= 1) {          // rows 4(v-1)+2, 4(v-1)+3
                    const f2 y2 = prev[0] + T[0];
                    const f2 y3 = prev[1] + T[1];
                    a1 += y2 + y3;
                    a2 = pfma(y2, y2, pfma(y3, y3, a2));
                }
                if (v < d.Hd) {        // rows 4v, 4v+1
                    const f2 y0 = T[2] + prev[2];
                    const f2 y1 = T[3] + prev[3];
                    a1 += y0 + y1;
                    a2 = pfma(y0, y0, pfma(y1, y1, a2));
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) prev[t] = T[4 + t];
            }
            s1 += (double)a1.x + (double)a1.y;
            s2 += (double)a2.x + (double)a2.y;
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
    __shared__ LrTab tz[LR_TAB], tk[LR_TAB], tj[LR_TAB];
    lr_fill(tz, d.Hd, d.Hs, d.Hd);
    lr_fill(tk, d.Hd, d.Hk, d.Hd);
    lr_fill(tj, d.Hd, d.H_skip, d.Hd);
    __syncthreads();
    const LrThread th = lr_thread(d);
    if (!th.active) return;
    const int N8 = 8 * d.Co;
    const int64_t rp = (int64_t)d.W * N8;
    const ZT* zb = (const ZT*)d.Z + (int64_t)th.item * d.Hs * rp + (int64_t)th.w * N8 + th.c;
    const ZT* sb = (const ZT*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    float mean, rstd;
    gn_params(d.stats, th.item, 4LL * d.Hd * d.W * d.Co, mean, rstd);
    const f2 bias = ld2(d.bias + th.c);
    const f2 gsc = ld2(d.gn_w + th.c) * splat(rstd);     // (y - mean) * rstd * w + b  as  (y - mean) * gsc + b
    const f2 gb = ld2(d.gn_b + th.c);
    // skip2 [seg][H_skip][W][C_skip], channels [0, Co): 0.1 * lerp, rows cached like the Z rows
    const int64_t kp = (int64_t)d.W * d.C_skip;
    const int64_t kb = (int64_t)th.seg * d.H_skip * kp + (int64_t)th.w * d.C_skip + th.c;
    int k0c = -1, k1c = -1;
    f2 ka = {}, kd = {};
    const int64_t ob = (int64_t)th.item * d.Hd * d.W * d.Co + (int64_t)th.w * d.Co + th.c;
    const int64_t op = (int64_t)d.W * d.Co;

    LerpRows<ZT, 4> zr, sr;       // slots: taps 0, 3, 4, 7
    f2 base[4];
    f2 cur3 = {}, cur4 = {}, cur7 = {}, prev7 = {};
    for (int v = 0; v <= d.Hd; ++v) {
        f2 T[4];
        if (v < d.Hd) {
            const Lerp a = lr_get(tz, v, d.Hs, d.Hd);
            const Lerp k = lr_get(tk, v, d.Hk, d.Hd);
            const bool cz = zr.update(zb, rp, d.Co, a, 1.0f);
            const bool cs = sr.update(sb, rp, d.Co, k, 0.1f);
            if (cz || cs) {
#pragma unroll
                for (int t = 0; t < 4; ++t) base[t] = zr.r0[t] + sr.r0[t] + ((t == 1 || t == 2) ? bias : f2{});
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) T[t] = pfma(splat(a.l1), zr.dr[t], pfma(splat(k.l1), sr.dr[t], base[t]));
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) T[t] = f2{};
        }
        if (v >= 1) {
            // output row dd: the exact /4 bilinear resize of the 4*Hd ConvT rows reads rows 4dd+1 and 4dd+2 with
            // weights 0.5 / 0.5 (src = 4dd + 1.5, exact in fp32)
            const int dd = v - 1;
            const Lerp lj = lr_get(tj, dd, d.H_skip, d.Hd);
            if (lj.i0 != k0c || lj.i1 != k1c) {
                k0c = lj.i0;
                k1c = lj.i1;
                f2 a, b;
                if (d.skip_bf16) {
                    a = ld2((const bf16_t*)d.skip + kb + (int64_t)lj.i0 * kp);
                    b = ld2((const bf16_t*)d.skip + kb + (int64_t)lj.i1 * kp);
                } else {
                    a = ld2((const float*)d.skip + kb + (int64_t)lj.i0 * kp);
                    b = ld2((const float*)d.skip + kb + (int64_t)lj.i1 * kp);
                }
                ka = a * splat(0.1f);
                kd = (b - a) * splat(0.1f);
            }
            const f2 y1 = cur3 + prev7;
            const f2 y2 = cur4 + T[0];
            const f2 g1 = gelu2<FAST>(pfma(y1 - splat(mean), gsc, gb));
            const f2 g2 = gelu2<FAST>(pfma(y2 - splat(mean), gsc, gb));
            const f2 o = pfma(g1 + g2, splat(0.5f), pfma(splat(lj.l1), kd, ka));
            const int64_t oi = ob + (int64_t)dd * op;
            if (d.out_bf16) {
                const bf2_t h = __builtin_convertvector(o, bf2_t);
                *reinterpret_cast<bf2_t*>((bf16_t*)d.out + oi) = h;
            } else {
                *reinterpret_cast<f2*>((float*)d.out + oi) = o;
            }
        }
        prev7 = cur7;
        cur3 = T[1];
        cur4 = T[2];
        cur7 = T[3];
    }
}

static bool lr_ok(const LowRankDesc& d) {
    return d.Z && d.Zs && d.bias && d.stats && d.Co % 2 == 0 && d.Hd > 0 && d.Hd < 65536 && d.W > 0 && d.P > 0 &&
           d.NI % d.P == 0 && d.Hs > 0 && d.Hk > 0;
}

int fdec_lr_stats_launch(const LowRankDesc& d, hipStream_t s) {
    if (!lr_ok(d)) return -1;
    const dim3 grid((unsigned)((d.W * (d.Co / 2) + 255) / 256), (unsigned)d.NI);
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
    if (!lr_ok(d) || !d.gn_w || !d.gn_b || !d.skip || !d.out || d.C_skip < d.Co || d.C_skip % 2 != 0 ||
        d.H_skip <= 0)
        return -1;
    const dim3 grid((unsigned)((d.W * (d.Co / 2) + 255) / 256), (unsigned)d.NI);
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
