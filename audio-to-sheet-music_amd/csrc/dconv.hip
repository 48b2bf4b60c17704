// DConv (demucs residual dilated-conv branch) for narrow levels (C = 48, 96; hidden
// H = C/8 = 6, 12) on gfx950.  These layers are HBM-bound with K or N far below an MFMA tile, so they run as
// VALU kernels, one thread per position, weights staged in LDS (broadcast reads):
//   c3:     h[p][j] = b[j] + sum_{tap,c} W[j][tap*C+c] x[p+(tap-1)dil][c]     + GroupNorm stats of h per group
//   c1stat: y[p][n] = b[n] + sum_j W[n][j] h[p][j]  (2C outputs)               -> GroupNorm stats of y per group
//   c1app:  x[p][c] += scale[c] * GLU(GN(y))[c]                                 (recomputes y: K = H is tiny)
// A "group" is the GroupNorm(1) sample: nb index of [nb][L][C] (freq rows (b,f) along time, or time samples).
#include "common.h"
#include "prof.h"
#include "kernels.h"

namespace athd {

// Block-level {sum, sumsq} per group: blocks cover 256 consecutive positions, so with L >= 256 a block spans at
// most two groups (first group g0 of the block and g0 + 1).  Shorter rows fall back to per-thread atomics.
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

template <int C>
__global__ __launch_bounds__(256) void dconv_c3_kernel(const float* __restrict__ x, int64_t nb, int64_t L, int dil,
                                                       const float* __restrict__ W, const float* __restrict__ bias,
                                                       float* __restrict__ h, double* __restrict__ st) {
    constexpr int H = C / 8, K = 3 * C;
    __shared__ float wl[H * K];
    __shared__ double sh[16];
    for (int i = threadIdx.x; i < H * K; i += 256) wl[i] = W[i];
    __syncthreads();
    const int64_t P = nb * L;
    const int64_t p0 = (int64_t)blockIdx.x * 256;
    const int64_t p = p0 + threadIdx.x;
    const bool valid = p < P;
    float s1 = 0.f, s2 = 0.f;
    if (valid) {
        const int64_t g = p / L, t = p - g * L;
        float acc[H];
#pragma unroll
        for (int j = 0; j < H; ++j) acc[j] = bias[j];
#pragma unroll
        for (int tap = 0; tap < 3; ++tap) {
            const int64_t tt = t + (tap - 1) * dil;
            if (tt < 0 || tt >= L) continue;
            const float4* xr = reinterpret_cast<const float4*>(x + (g * L + tt) * C);
#pragma unroll 4
            for (int c4 = 0; c4 < C / 4; ++c4) {
                const float4 v = xr[c4];
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    const float* wr = &wl[j * K + tap * C + 4 * c4];
                    acc[j] += wr[0] * v.x + wr[1] * v.y + wr[2] * v.z + wr[3] * v.w;
                }
            }
        }
        float* hr = h + p * H;
#pragma unroll
        for (int j = 0; j < H; ++j) {
            hr[j] = acc[j];
            s1 += acc[j];
            s2 += acc[j] * acc[j];
        }
    }
    group_stats_add(st, p0, p, valid, L, s1, s2, sh);
}

template <int C, bool APPLY>
__global__ __launch_bounds__(256) void dconv_c1_kernel(float* __restrict__ x, const float* __restrict__ h, int64_t nb,
                                                       int64_t L, const float* __restrict__ W,
                                                       const float* __restrict__ bias, double* __restrict__ st,
                                                       const float* __restrict__ gw, const float* __restrict__ gb,
                                                       const float* __restrict__ scale) {
    constexpr int H = C / 8, N = 2 * C;
    __shared__ float wl[N * H];
    __shared__ float bl[N], gwl[N], gbl[N], scl[C];
    __shared__ double sh[16];
    for (int i = threadIdx.x; i < N * H; i += 256) wl[i] = W[i];
    for (int i = threadIdx.x; i < N; i += 256) {
        bl[i] = bias[i];
        if (APPLY) { gwl[i] = gw[i]; gbl[i] = gb[i]; }
    }
    if (APPLY) for (int i = threadIdx.x; i < C; i += 256) scl[i] = scale[i];
    __syncthreads();
    const int64_t P = nb * L;
    const int64_t p0 = (int64_t)blockIdx.x * 256;
    const int64_t p = p0 + threadIdx.x;
    const bool valid = p < P;
    float hv[H];
    if (valid) {
#pragma unroll
        for (int j = 0; j < H; ++j) hv[j] = h[p * H + j];
    }
    if (!APPLY) {
        float s1 = 0.f, s2 = 0.f;
        if (valid) {
#pragma unroll 4
            for (int n = 0; n < N; ++n) {
                float y = bl[n];
#pragma unroll
                for (int j = 0; j < H; ++j) y += wl[n * H + j] * hv[j];
                s1 += y;
                s2 += y * y;
            }
        }
        group_stats_add(st, p0, p, valid, L, s1, s2, sh);
    } else {
        if (!valid) return;
        const int64_t g = p / L;
        const double cnt = (double)L * N;
        const double mm = st[2 * g] / cnt;
        double var = st[2 * g + 1] / cnt - mm * mm;
        if (var < 0) var = 0;
        const float mean = (float)mm, rstd = (float)(1.0 / sqrt(var + 1e-5));
        float4* xr = reinterpret_cast<float4*>(x + p * C);
#pragma unroll 2
        for (int c4 = 0; c4 < C / 4; ++c4) {
            float4 xv = xr[c4];
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int c = 4 * c4 + q;
                float a = bl[c], gt = bl[C + c];
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    a += wl[c * H + j] * hv[j];
                    gt += wl[(C + c) * H + j] * hv[j];
                }
                a = (a - mean) * rstd * gwl[c] + gbl[c];
                gt = (gt - mean) * rstd * gwl[C + c] + gbl[C + c];
                o[q] = scl[c] * (a * sigmoidf_(gt));
            }
            xv.x += o[0]; xv.y += o[1]; xv.z += o[2]; xv.w += o[3];
            xr[c4] = xv;
        }
    }
}

int dconv_small_launch(float* x, float* h, int64_t nb, int64_t L, int C, int dil, const float* w3, const float* b3,
                       const float* g1w, const float* g1b, const float* w1, const float* b1, const float* g2w,
                       const float* g2b, const float* scale, double* st_h, double* st_y, hipStream_t s, bool fast) {
    const int64_t P = nb * L;
    const dim3 grid((unsigned)((P + 255) / 256));
    const int H = C / 8;
    const double px = (double)P;
    if (C != 48 && C != 96) return -2;
    {
        KScope ks(s);
        if (ks.on()) ks.begin(klabel("dconv_c3_kernel<%d>", C), 2.0 * px * H * 3 * C, px * (C + H) * 4);
        if (C == 48) hipLaunchKernelGGL((dconv_c3_kernel<48>), grid, dim3(256), 0, s, x, nb, L, dil, w3, b3, h, st_h);
        else hipLaunchKernelGGL((dconv_c3_kernel<96>), grid, dim3(256), 0, s, x, nb, L, dil, w3, b3, h, st_h);
    }
    gn_gelu_launch(h, (int)nb, L * H, H, st_h, g1w, g1b, s, fast);
    {
        KScope ks(s);
        if (ks.on()) ks.begin(klabel("dconv_c1_kernel<%d,false>", C), 2.0 * px * 2 * C * H, px * H * 4);
        if (C == 48) hipLaunchKernelGGL((dconv_c1_kernel<48, false>), grid, dim3(256), 0, s, x, h, nb, L, w1, b1, st_y, g2w, g2b, scale);
        else hipLaunchKernelGGL((dconv_c1_kernel<96, false>), grid, dim3(256), 0, s, x, h, nb, L, w1, b1, st_y, g2w, g2b, scale);
    }
    {
        KScope ks(s);
        if (ks.on()) ks.begin(klabel("dconv_c1_kernel<%d,true>", C), 2.0 * px * 2 * C * H, px * (H + 2 * C) * 4);
        if (C == 48) hipLaunchKernelGGL((dconv_c1_kernel<48, true>), grid, dim3(256), 0, s, x, h, nb, L, w1, b1, st_y, g2w, g2b, scale);
        else hipLaunchKernelGGL((dconv_c1_kernel<96, true>), grid, dim3(256), 0, s, x, h, nb, L, w1, b1, st_y, g2w, g2b, scale);
    }
    return (int)hipGetLastError();
}

}  // namespace athd
