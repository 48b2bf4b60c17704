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
//   fdec_lr_stats{2,3}_kernel: GroupNorm(1) {sum, sumsq} over all 4*Hd ConvT rows;
//   fdec_lr_merge{2,3}_kernel: rows 4d+1, 4d+2 (the only rows the exact /4 bilinear resize reads) -> GN -> GELU ->
//                         lerp -> + 0.1 * resize_H(skip2) -> D1 [item][d][w][Co].
#include <algorithm>
#include <cstdlib>

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

// packed tanh-form GELU: the arithmetic of common.h::gelu_fast on both lanes of the pair (the polynomial and the
// scaling as v_pk ops, the exp2 / rcp per lane)
ATHD_DEV f2 gelu2_pk(f2 x) {
    const f2 u = x * pfma(splat(0.044715f * 1.5957691216057308f), x * x, splat(1.5957691216057308f));
    const f2 t = u * splat(-1.4426950408889634f);
    const f2 den = (f2){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + splat(1.0f);
    return x * (f2){__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
}

// rows i0, i1 of a [H][W][8 Co] tap matrix at the thread's (w, channel pair): r0 = scale row[i0], dr = scale (row[i1] -
// row[i0]) for the NT tap slots (tap_of); i0 / i1 are wave-uniform (scalar offsets)
template <typename ZT, int NT>
ATHD_DEV void load_rows(const ZT* base, int64_t rowpitch, int Co, int i0, int i1, float scale, f2 (&r0)[NT],
                        f2 (&dr)[NT]);

// tap index of slot t: all 8 taps (stats pass) or {0, 3, 4, 7} (merge pass: rows 4d+1, 4d+2)
template <int NT>
ATHD_DEV constexpr int tap_of(int t) { return NT == 8 ? t : (t == 0 ? 0 : t == 1 ? 3 : t == 2 ? 4 : 7); }

template <typename ZT, int NT>
ATHD_DEV void load_rows(const ZT* base, int64_t rowpitch, int Co, int i0, int i1, float scale, f2 (&r0)[NT],
                        f2 (&dr)[NT]) {
    f2 a[NT], b[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) a[t] = ld2(base + (int64_t)i0 * rowpitch + tap_of<NT>(t) * Co);
#pragma unroll
    for (int t = 0; t < NT; ++t) b[t] = ld2(base + (int64_t)i1 * rowpitch + tap_of<NT>(t) * Co);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        r0[t] = a[t] * splat(scale);
        dr[t] = (b[t] - a[t]) * splat(scale);
    }
}

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

// ---------------------------------------------------------------------------------------------------------
// v2 passes (f32 mode, and bf16 without strict upsampling, i.e. Tspec <= 32): the per-step resize lerps and
// row-change flags are read from a step table in global memory (fdec_lr_steps_kernel, once per forward): the step
// index is wave-uniform, so the entry arrives through scalar loads and the lerp weights feed the packed FMAs as SGPR
// operands (round 1's per-block LDS index tables cost about half the VALU instructions of a step; that version is
// gone), and the GELU pair runs packed.
// step entry v through the constant address space: the index is wave-uniform, so this is a scalar load (through a
// generic pointer the compiler may use a vector load, which the step then waits on)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const u32x4_t c_u32x4;
ATHD_DEV LrStep lr_step(const LrStep* steps, int v) {
    static_assert(sizeof(LrStep) == 32, "LrStep layout");
    const c_u32x4* p = (const c_u32x4*)steps + 2 * __builtin_amdgcn_readfirstlane(v);
    const u32x4_t a = p[0], b = p[1];
    LrStep e;
    e.lz = __uint_as_float(a.x);
    e.lk = __uint_as_float(a.y);
    e.lj = __uint_as_float(a.z);
    e.zk = a.w;
    e.jj = b.x;
    e.flags = b.y;
    return e;
}

__global__ __launch_bounds__(256) void fdec_lr_steps_kernel(LrStep* steps, int Hd, int Hs, int Hk, int H_skip) {
    for (int v = threadIdx.x; v <= Hd; v += blockDim.x) {
        LrStep e = {};
        int z0 = -1, z1 = -1, k0 = -1, k1 = -1, j0 = -1, j1 = -1, pz0 = -2, pz1 = -2, pk0 = -2, pk1 = -2, pj0 = -2,
            pj1 = -2;
        if (v < Hd) {
            const LinIdx a = lin_index(v, Hs, Hd), k = lin_index(v, Hk, Hd);
            z0 = a.i0; z1 = a.i1; k0 = k.i0; k1 = k.i1;
            e.lz = a.l1;
            e.lk = k.l1;
        }
        if (v >= 1) {
            const LinIdx j = lin_index(v - 1, H_skip, Hd);
            j0 = j.i0; j1 = j.i1;
            e.lj = j.l1;
            if (v - 1 < Hd) {
                const LinIdx pa = lin_index(v - 1, Hs, Hd), pk = lin_index(v - 1, Hk, Hd);
                pz0 = pa.i0; pz1 = pa.i1; pk0 = pk.i0; pk1 = pk.i1;
            }
            if (v >= 2) {
                const LinIdx pj = lin_index(v - 2, H_skip, Hd);
                pj0 = pj.i0; pj1 = pj.i1;
            }
        }
        e.zk = (uint32_t)(z0 & 0xFF) | (uint32_t)(z1 & 0xFF) << 8 | (uint32_t)(k0 & 0xFF) << 16 | (uint32_t)(k1 & 0xFF) << 24;
        e.jj = (uint32_t)(j0 & 0xFFFF) | (uint32_t)(j1 & 0xFFFF) << 16;
        e.flags = (v < Hd && (z0 != pz0 || z1 != pz1) ? 1u : 0u) | (v < Hd && (k0 != pk0 || k1 != pk1) ? 2u : 0u) |
                  (v >= 1 && (j0 != pj0 || j1 != pj1) ? 4u : 0u);
        steps[v] = e;
    }
}

template <typename ZT>
__global__ __launch_bounds__(256) void fdec_lr_stats2_kernel(const LowRankDesc d) {
    const LrThread th = lr_thread(d);
    const int N8 = 8 * d.Co;
    const int64_t rp = (int64_t)d.W * N8;
    const ZT* zb = (const ZT*)d.Z + (int64_t)th.item * d.Hs * rp + (int64_t)th.w * N8 + th.c;
    const ZT* sb = (const ZT*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    const f2 bias = ld2(d.bias + th.c);
    f2 zr0[8], zdr[8], sr0[8], sdr[8];
    f2 base[8];                // r0(Z) + r0(Zs) (+ bias on taps 2..5: every output row has exactly one of those)
    f2 prev[4] = {};           // T_{v-1}[4..7]
    double s1 = 0.0, s2 = 0.0;
    LrStep nx = lr_step(d.steps, 0);
    if (th.active) {
        for (int v0 = 0; v0 <= d.Hd; v0 += 16) {
            f2 a1 = {}, a2 = {};
            const int v1 = min(v0 + 16, d.Hd + 1);
            for (int v = v0; v < v1; ++v) {
                f2 T[8];
                const LrStep st = nx;             // the next step's entry is in flight during this step
                if (v < d.Hd) nx = lr_step(d.steps, v + 1);
                if (v < d.Hd) {
                    if (st.flags & 3u) {
                        if (st.flags & 1u)
                            load_rows<ZT, 8>(zb, rp, d.Co, st.zk & 0xFF, (st.zk >> 8) & 0xFF, 1.0f, zr0, zdr);
                        if (st.flags & 2u)
                            load_rows<ZT, 8>(sb, rp, d.Co, (st.zk >> 16) & 0xFF, st.zk >> 24, 0.1f, sr0, sdr);
#pragma unroll
                        for (int t = 0; t < 8; ++t) base[t] = zr0[t] + sr0[t] + ((t >= 2 && t <= 5) ? bias : f2{});
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t) T[t] = pfma(splat(st.lz), zdr[t], pfma(splat(st.lk), sdr[t], base[t]));
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

// v3 statistics pass (bf16 mode, strict upsampling Hd > Hs, Hd > Hk): there every row change of a lerp moves (i0, i1)
// to (i1, min(i1 + 1, H - 1)), so a change needs ONE new row, and that row is known at the previous change.  The pass
// keeps the scaled i1 row (hi) and the row difference (dr) per tap, updates the lerp base incrementally (base += dr:
// the i0 row becomes the old i1 row), and prefetches the next i1 row as raw bf16 pairs right after each change, so
// its load latency hides under the ~Hd/H steps of VALU work before it is needed (v2 loads both rows at the change and
// waits for them).  Half the Z / Zs loads; rounding differs from v2 by the incremental base only (bf16 mode).
ATHD_DEV f2 bf2u(uint32_t q) { return (f2){__uint_as_float(q << 16), __uint_as_float(q & 0xFFFF0000u)}; }

__global__ __launch_bounds__(256) void fdec_lr_stats3_kernel(const LowRankDesc d) {
    const LrThread th = lr_thread(d);
    const int N8 = 8 * d.Co;
    const int64_t rp = (int64_t)d.W * N8;
    const bf16_t* zb = (const bf16_t*)d.Z + (int64_t)th.item * d.Hs * rp + (int64_t)th.w * N8 + th.c;
    const bf16_t* sb = (const bf16_t*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    const f2 bias = ld2(d.bias + th.c);
    f2 zhi[8], zdr[8], shi[8], sdr[8], base[8];
    uint32_t zpf[8], spf[8];
    double s1 = 0.0, s2 = 0.0;
    auto ldrow = [&](const bf16_t* p, int row, uint32_t (&r)[8]) {
#pragma unroll
        for (int t = 0; t < 8; ++t) r[t] = *reinterpret_cast<const uint32_t*>(p + (int64_t)row * rp + t * d.Co);
    };
    if (th.active) {
        const LrStep s0 = lr_step(d.steps, 0);
        int zr = (s0.zk >> 8) & 0xFF, kr = s0.zk >> 24;          // current i1 rows (wave-uniform)
        {
            uint32_t za[8], ka[8];
            ldrow(zb, s0.zk & 0xFF, za);
            ldrow(zb, zr, zpf);
            ldrow(sb, (s0.zk >> 16) & 0xFF, ka);
            ldrow(sb, kr, spf);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const f2 a = bf2u(za[t]), b = bf2u(zpf[t]);
                const f2 ka2 = bf2u(ka[t]) * splat(0.1f), kb2 = bf2u(spf[t]) * splat(0.1f);
                zhi[t] = b;
                zdr[t] = b - a;
                shi[t] = kb2;
                sdr[t] = kb2 - ka2;
                base[t] = a + ka2 + ((t >= 2 && t <= 5) ? bias : f2{});
            }
        }
        ldrow(zb, min(zr + 1, d.Hs - 1), zpf);
        ldrow(sb, min(kr + 1, d.Hk - 1), spf);
        // T of step v from the current rows (row changes applied first)
        auto tstep = [&](const LrStep& st, f2 (&T)[8]) {
            if (st.flags & 1u) {                  // Z rows (i0, i1) -> (i1, i1 + 1)
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const f2 nb = bf2u(zpf[t]);
                    base[t] += zdr[t];
                    zdr[t] = nb - zhi[t];
                    zhi[t] = nb;
                }
                zr = min(zr + 1, d.Hs - 1);
                ldrow(zb, min(zr + 1, d.Hs - 1), zpf);
            }
            if (st.flags & 2u) {                  // Zs rows
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const f2 nb = bf2u(spf[t]) * splat(0.1f);
                    base[t] += sdr[t];
                    sdr[t] = nb - shi[t];
                    shi[t] = nb;
                }
                kr = min(kr + 1, d.Hk - 1);
                ldrow(sb, min(kr + 1, d.Hk - 1), spf);
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) T[t] = pfma(splat(st.lz), zdr[t], pfma(splat(st.lk), sdr[t], base[t]));
        };
        // step 0 (rows 0, 1 only; its rows were loaded above)
        f2 pv[4];                                 // T[4..7] of the previous step
        f2 a1 = {}, a2 = {};
        {
            f2 T[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) T[t] = pfma(splat(s0.lz), zdr[t], pfma(splat(s0.lk), sdr[t], base[t]));
            a1 += T[2] + T[3];
            a2 = pfma(T[2], T[2], pfma(T[3], T[3], a2));
#pragma unroll
            for (int t = 0; t < 4; ++t) pv[t] = T[4 + t];
        }
        // steps 1 .. Hd-1: rows 4(v-1)+2, 4(v-1)+3 and 4v, 4v+1; no per-step conditions besides the row changes
        LrStep nx = lr_step(d.steps, 1);
        for (int v0 = 1; v0 < d.Hd; v0 += 16) {
            const int v1 = min(v0 + 16, d.Hd);
            for (int v = v0; v < v1; ++v) {
                const LrStep st = nx;
                nx = lr_step(d.steps, v + 1);
                f2 T[8];
                tstep(st, T);
                const f2 y2 = pv[0] + T[0], y3 = pv[1] + T[1];
                const f2 y0 = T[2] + pv[2], y1 = T[3] + pv[3];
                a1 += (y2 + y3) + (y0 + y1);
                a2 = pfma(y2, y2, pfma(y3, y3, a2));
                a2 = pfma(y0, y0, pfma(y1, y1, a2));
#pragma unroll
                for (int t = 0; t < 4; ++t) pv[t] = T[4 + t];
            }
            s1 += (double)a1.x + (double)a1.y;
            s2 += (double)a2.x + (double)a2.y;
            a1 = f2{};
            a2 = f2{};
        }
        // step Hd: rows 4(Hd-1)+2, 4(Hd-1)+3 only (T = 0)
        a1 += pv[0] + pv[1];
        a2 = pfma(pv[0], pv[0], pfma(pv[1], pv[1], a2));
        s1 += (double)a1.x + (double)a1.y;
        s2 += (double)a2.x + (double)a2.y;
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

// v3 merge pass (bf16 mode, strict upsampling Hd > Hs, Hk, H_skip): the one-new-row updates and next-row prefetches
// of fdec_lr_stats3_kernel for the Z / Zs rows (taps 0, 3, 4, 7) and the skip2 rows, and the first / last steps
// peeled so that the step loop carries no per-step conditions besides the row changes.
__global__ __launch_bounds__(256) void fdec_lr_merge3_kernel(const LowRankDesc d) {
    const LrThread th = lr_thread(d);
    if (!th.active) return;
    constexpr int NT = 4;
    const int N8 = 8 * d.Co, NZ = d.z_taps * d.Co;      // Zs rows: 8 taps; Z rows: 8 taps or taps 0, 3, 4, 7 only
    const int64_t rp = (int64_t)d.W * N8, rpz = (int64_t)d.W * NZ;
    const bool z4 = d.z_taps == 4;
    // 4-tap Z (fdec1f.hip): [item][j][w][channel group of 16][tap][16]: 128 B per (w, group) for the Gram pass's stores
    const bf16_t* zb = (const bf16_t*)d.Z + (int64_t)th.item * d.Hs * rpz + (int64_t)th.w * NZ +
                       (z4 ? (th.c >> 4) * 64 + (th.c & 15) : th.c);
    const bf16_t* sb = (const bf16_t*)d.Zs + (int64_t)th.seg * d.Hk * rp + (int64_t)th.w * N8 + th.c;
    float mean, rstd;
    gn_params(d.stats, th.item, 4LL * d.Hd * d.W * d.Co, mean, rstd);
    const f2 bias = ld2(d.bias + th.c);
    const f2 gsc = ld2(d.gn_w + th.c) * splat(rstd);     // (y - mean) * rstd * w + b  as  (y - mean) * gsc + b
    const f2 gb = ld2(d.gn_b + th.c) - splat(mean) * gsc; // ... as y * gsc + gb'
    const int64_t kp = (int64_t)d.W * d.C_skip;
    const bf16_t* kbp = (const bf16_t*)d.skip + (int64_t)th.seg * d.H_skip * kp + (int64_t)th.w * d.C_skip + th.c;
    bf2_t* op = (bf2_t*)((bf16_t*)d.out + (int64_t)th.item * d.Hd * d.W * d.Co + (int64_t)th.w * d.Co + th.c);
    const int64_t ostep = (int64_t)d.W * d.Co / 2;        // bf2 elements between output rows

    auto ldrow = [&](const bf16_t* p, int row, uint32_t (&r)[NT], bool compact) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
            r[t] = *reinterpret_cast<const uint32_t*>(p + (int64_t)row * (compact ? rpz : rp) +
                                                      (compact ? t * 16 : tap_of<NT>(t) * d.Co));
    };
    f2 zhi[NT], zdr[NT], shi[NT], sdr[NT], base[NT];
    uint32_t zpf[NT], spf[NT];
    const LrStep s0 = lr_step(d.steps, 0);
    int zr = (s0.zk >> 8) & 0xFF, kr = s0.zk >> 24;
    {
        uint32_t za[NT], ka[NT];
        ldrow(zb, s0.zk & 0xFF, za, z4);
        ldrow(zb, zr, zpf, z4);
        ldrow(sb, (s0.zk >> 16) & 0xFF, ka, false);
        ldrow(sb, kr, spf, false);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const f2 a = bf2u(za[t]), b = bf2u(zpf[t]);
            const f2 ka2 = bf2u(ka[t]) * splat(0.1f), kb2 = bf2u(spf[t]) * splat(0.1f);
            zhi[t] = b;
            zdr[t] = b - a;
            shi[t] = kb2;
            sdr[t] = kb2 - ka2;
            base[t] = a + ka2 + ((t == 1 || t == 2) ? bias : f2{});
        }
    }
    ldrow(zb, min(zr + 1, d.Hs - 1), zpf, z4);
    ldrow(sb, min(kr + 1, d.Hk - 1), spf, false);
    // skip2 rows of output row 0 (step 1's entry), then the next one prefetched
    const LrStep s1e = lr_step(d.steps, 1);
    int jr = (int)(s1e.jj >> 16);
    f2 khi, kdr;
    uint32_t jpf;
    {
        const f2 a = bf2u(*reinterpret_cast<const uint32_t*>(kbp + (int64_t)(s1e.jj & 0xFFFF) * kp)) * splat(0.1f);
        khi = bf2u(*reinterpret_cast<const uint32_t*>(kbp + (int64_t)jr * kp)) * splat(0.1f);
        kdr = khi - a;
    }
    jpf = *reinterpret_cast<const uint32_t*>(kbp + (int64_t)min(jr + 1, d.H_skip - 1) * kp);
    f2 kbase = khi - kdr;                                 // 0.1 * skip row j0

    auto tstep = [&](const LrStep& st, f2 (&T)[NT]) {
        if (st.flags & 1u) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f2 nb = bf2u(zpf[t]);
                base[t] += zdr[t];
                zdr[t] = nb - zhi[t];
                zhi[t] = nb;
            }
            zr = min(zr + 1, d.Hs - 1);
            ldrow(zb, min(zr + 1, d.Hs - 1), zpf, z4);
        }
        if (st.flags & 2u) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f2 nb = bf2u(spf[t]) * splat(0.1f);
                base[t] += sdr[t];
                sdr[t] = nb - shi[t];
                shi[t] = nb;
            }
            kr = min(kr + 1, d.Hk - 1);
            ldrow(sb, min(kr + 1, d.Hk - 1), spf, false);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) T[t] = pfma(splat(st.lz), zdr[t], pfma(splat(st.lk), sdr[t], base[t]));
    };
    // output row dd = v - 1 from rows 4dd+1 (cur3 + prev7) and 4dd+2 (cur4 + T0): the exact /4 resize (0.5 / 0.5)
    auto emit = [&](const LrStep& st, f2 y1, f2 y2, int dd) {
        if (dd >= 1 && (st.flags & 4u)) {                 // skip2 rows (j0, j1) -> (j1, j1 + 1)
            const f2 nb = bf2u(jpf) * splat(0.1f);
            kbase += kdr;
            kdr = nb - khi;
            khi = nb;
            jr = min(jr + 1, d.H_skip - 1);
            jpf = *reinterpret_cast<const uint32_t*>(kbp + (int64_t)min(jr + 1, d.H_skip - 1) * kp);
        }
        // the exact /4 resize: 0.5 GELU(y1) + 0.5 GELU(y2) with one reciprocal per element (common.h)
        const f2 gs = gelu_fast_wsum_pk(splat(0.5f), pfma(y1, gsc, gb), splat(0.5f), pfma(y2, gsc, gb));
        const f2 o = gs + pfma(splat(st.lj), kdr, kbase);
        op[(int64_t)dd * ostep] = __builtin_convertvector(o, bf2_t);
    };
    f2 cur3, cur4, cur7, prev7 = {};
    {
        f2 T[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) T[t] = pfma(splat(s0.lz), zdr[t], pfma(splat(s0.lk), sdr[t], base[t]));
        cur3 = T[1];
        cur4 = T[2];
        cur7 = T[3];
    }
    LrStep nx = s1e;
    for (int v = 1; v < d.Hd; ++v) {
        const LrStep st = nx;
        nx = lr_step(d.steps, v + 1);
        f2 T[NT];
        tstep(st, T);
        emit(st, cur3 + prev7, cur4 + T[0], v - 1);
        prev7 = cur7;
        cur3 = T[1];
        cur4 = T[2];
        cur7 = T[3];
    }
    emit(nx, cur3 + prev7, cur4, d.Hd - 1);               // step Hd: T = 0
}

template <typename ZT, bool FAST>
__global__ __launch_bounds__(256) void fdec_lr_merge2_kernel(const LowRankDesc d) {
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
    const int64_t kp = (int64_t)d.W * d.C_skip;
    const int64_t kb = (int64_t)th.seg * d.H_skip * kp + (int64_t)th.w * d.C_skip + th.c;
    f2 ka = {}, kd = {};
    const int64_t ob = (int64_t)th.item * d.Hd * d.W * d.Co + (int64_t)th.w * d.Co + th.c;
    const int64_t op = (int64_t)d.W * d.Co;

    f2 zr0[4], zdr[4], sr0[4], sdr[4];   // slots: taps 0, 3, 4, 7
    f2 base[4];
    f2 cur3 = {}, cur4 = {}, cur7 = {}, prev7 = {};
    LrStep nx = lr_step(d.steps, 0);
    for (int v = 0; v <= d.Hd; ++v) {
        const LrStep st = nx;                     // the next step's entry is in flight during this step
        if (v < d.Hd) nx = lr_step(d.steps, v + 1);
        f2 T[4];
        if (v < d.Hd) {
            if (st.flags & 3u) {
                if (st.flags & 1u) load_rows<ZT, 4>(zb, rp, d.Co, st.zk & 0xFF, (st.zk >> 8) & 0xFF, 1.0f, zr0, zdr);
                if (st.flags & 2u) load_rows<ZT, 4>(sb, rp, d.Co, (st.zk >> 16) & 0xFF, st.zk >> 24, 0.1f, sr0, sdr);
#pragma unroll
                for (int t = 0; t < 4; ++t) base[t] = zr0[t] + sr0[t] + ((t == 1 || t == 2) ? bias : f2{});
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) T[t] = pfma(splat(st.lz), zdr[t], pfma(splat(st.lk), sdr[t], base[t]));
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) T[t] = f2{};
        }
        if (v >= 1) {
            // output row dd = v - 1: the exact /4 bilinear resize of the 4*Hd ConvT rows reads rows 4dd+1 and 4dd+2
            // with weights 0.5 / 0.5 (src = 4dd + 1.5, exact in fp32)
            const int dd = v - 1;
            if (st.flags & 4u) {
                const int j0 = (int)(st.jj & 0xFFFF), j1 = (int)(st.jj >> 16);
                f2 a, b;
                if (d.skip_bf16) {
                    a = ld2((const bf16_t*)d.skip + kb + (int64_t)j0 * kp);
                    b = ld2((const bf16_t*)d.skip + kb + (int64_t)j1 * kp);
                } else {
                    a = ld2((const float*)d.skip + kb + (int64_t)j0 * kp);
                    b = ld2((const float*)d.skip + kb + (int64_t)j1 * kp);
                }
                ka = a * splat(0.1f);
                kd = (b - a) * splat(0.1f);
            }
            const f2 y1 = cur3 + prev7;
            const f2 y2 = cur4 + T[0];
            f2 g1, g2;
            if constexpr (FAST) {
                g1 = gelu2_pk(pfma(y1 - splat(mean), gsc, gb));
                g2 = gelu2_pk(pfma(y2 - splat(mean), gsc, gb));
            } else {
                g1 = gelu2<false>(pfma(y1 - splat(mean), gsc, gb));
                g2 = gelu2<false>(pfma(y2 - splat(mean), gsc, gb));
            }
            const f2 o = pfma(g1 + g2, splat(0.5f), pfma(splat(st.lj), kd, ka));
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

int fdec_lr_steps_launch(LrStep* steps, int Hd, int Hs, int Hk, int H_skip, hipStream_t s) {
    if (!steps || Hd <= 0 || Hs <= 0 || Hs > 256 || Hk <= 0 || Hk > 256 || H_skip <= 0 || H_skip > 65536) return -1;
    KScope ks(s);
    if (ks.on()) ks.begin("fdec_lr_steps_kernel", 0.0, (double)(Hd + 1) * sizeof(LrStep));
    hipLaunchKernelGGL(fdec_lr_steps_kernel, dim3(1), dim3(256), 0, s, steps, Hd, Hs, Hk, H_skip);
    return (int)hipGetLastError();
}

static bool lr_ok(const LowRankDesc& d) {
    return d.Z && d.Zs && d.bias && d.stats && d.steps && d.Co % 2 == 0 && d.Hd > 0 && d.Hd < 65536 && d.W > 0 && d.P > 0 &&
           d.NI % d.P == 0 && d.Hs > 0 && d.Hk > 0;
}

int fdec_lr_stats_launch(const LowRankDesc& d, hipStream_t s) {
    if (!lr_ok(d) || d.z_taps != 8) return -1;
    const dim3 grid((unsigned)((d.W * (d.Co / 2) + 255) / 256), (unsigned)d.NI);
    KScope ks(s);
    if (ks.on()) {
        // unique bytes: Z of every item + Zs of every segment, read once
        const double ze = d.z_bf16 ? 2.0 : 4.0;
        const double by = ze * 8.0 * d.Co * d.W * ((double)d.NI * d.Hs + (double)(d.NI / d.P) * d.Hk);
        ks.begin(d.z_bf16 && d.Hd > d.Hs && d.Hd > d.Hk ? "fdec_lr_stats3_kernel"
                 : d.z_bf16 ? "fdec_lr_stats2_kernel<unsignedshort>" : "fdec_lr_stats2_kernel<float>", 0.0, by);
    }
    if (d.z_bf16 && d.Hd > d.Hs && d.Hd > d.Hk)
        hipLaunchKernelGGL(fdec_lr_stats3_kernel, grid, dim3(256), 0, s, d);
    else if (d.z_bf16)
        hipLaunchKernelGGL(fdec_lr_stats2_kernel<bf16_t>, grid, dim3(256), 0, s, d);
    else
        hipLaunchKernelGGL(fdec_lr_stats2_kernel<float>, grid, dim3(256), 0, s, d);
    return (int)hipGetLastError();
}

// v3 merge: bf16 mode with strict upsampling of all three lerps (every row change advances by one row)
static bool merge3(const LowRankDesc& d) {
    return d.z_bf16 && d.skip_bf16 && d.out_bf16 && d.fast_gelu && d.Hd > d.Hs && d.Hd > d.Hk && d.Hd > d.H_skip;
}

int fdec_lr_merge_launch(const LowRankDesc& d, hipStream_t s) {
    if (!lr_ok(d) || !d.gn_w || !d.gn_b || !d.skip || !d.out || d.C_skip < d.Co || d.C_skip % 2 != 0 ||
        d.H_skip <= 0 || (d.z_taps != 8 && !(d.z_taps == 4 && merge3(d))))
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
        ks.begin(merge3(d) ? std::string("fdec_lr_merge3_kernel")
                            : klabel("fdec_lr_merge2_kernel<%s,%s>", d.z_bf16 ? "unsignedshort" : "float",
                                     d.fast_gelu ? "true" : "false"), 0.0, by);
    }
    if (merge3(d)) {
        hipLaunchKernelGGL(fdec_lr_merge3_kernel, grid, dim3(256), 0, s, d);
    } else if (d.z_bf16) {
        if (d.fast_gelu) hipLaunchKernelGGL((fdec_lr_merge2_kernel<bf16_t, true>), grid, dim3(256), 0, s, d);
        else hipLaunchKernelGGL((fdec_lr_merge2_kernel<bf16_t, false>), grid, dim3(256), 0, s, d);
    } else {
        if (d.fast_gelu) hipLaunchKernelGGL((fdec_lr_merge2_kernel<float, true>), grid, dim3(256), 0, s, d);
        else hipLaunchKernelGGL((fdec_lr_merge2_kernel<float, false>), grid, dim3(256), 0, s, d);
    }
    return (int)hipGetLastError();
}

}  // namespace athd
