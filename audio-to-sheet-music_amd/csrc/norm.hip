#include <algorithm>
// Normalisation, elementwise, resize/merge and table kernels of the hot path (gfx950).
// GroupNorm/LayerNorm statistics are accumulated in fp64 (sum, sum of squares) so that the one-pass
// variance matches PyTorch's fp32 two-pass/Welford results to rounding.
#include <cstdlib>

#include "common.h"
#include "prof.h"
#include "kernels.h"

namespace athd {

// --------------------------------------------------------------------------------------------- statistics
__global__ __launch_bounds__(256) void stats_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ st) {
    const int64_t b = blockIdx.y;
    const float* p = x + b * n;
    double s1 = 0.0, s2 = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double v = p[i];
        s1 += v;
        s2 += v * v;
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    __shared__ double sh[2][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = s1; sh[1][w] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&st[2 * b], sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3]);
        atomicAdd(&st[2 * b + 1], sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3]);
    }
}

void stats_launch(const float* x, int nb, int64_t n, double* stats, hipStream_t s) {
    int blocks = (int)((n + 256 * 16 - 1) / (256 * 16));
    if (blocks > 512) blocks = 512;
    if (blocks < 1) blocks = 1;
    KScope ks(s);
    if (ks.on()) ks.begin("stats_kernel", 0.0, (double)nb * n * 4);
    hipLaunchKernelGGL(stats_kernel, dim3(blocks, nb), dim3(256), 0, s, x, n, stats);
}

__global__ void input_norm_params_kernel(const double* st, int nb, int64_t n, float* mean_div, float* mean_std) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const double mean = st[2 * b] / (double)n;
    double var = (st[2 * b + 1] - st[2 * b] * mean) / (double)(n - 1);     // unbiased (torch.std default)
    if (var < 0) var = 0;
    const float stdv = (float)sqrt(var);
    mean_div[2 * b] = (float)mean;
    mean_div[2 * b + 1] = 1e-5f + stdv;
    if (mean_std) { mean_std[2 * b] = (float)mean; mean_std[2 * b + 1] = stdv; }
}

void input_norm_params_launch(const double* stats, int nb, int64_t n, float* mean_div, float* mean_std, hipStream_t s) {
    hipLaunchKernelGGL(input_norm_params_kernel, dim3((nb + 63) / 64), dim3(64), 0, s, stats, nb, n, mean_div, mean_std);
}


// --------------------------------------------------------------------------------------------- GroupNorm users
template <bool FAST>
__global__ __launch_bounds__(256) void gn_gelu_kernel(float* __restrict__ h, int64_t per_batch, int H,
                                                      const double* __restrict__ st, const float* __restrict__ w,
                                                      const float* __restrict__ bb) {
    const int64_t b = blockIdx.y;
    float mean, rstd;
    gn_params(st, b, per_batch, mean, rstd);
    float* p = h + b * per_batch;
    const int n = (int)per_batch;      // < 2^31 per batch on every use
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int c = i % H;
        p[i] = gelu<FAST>((p[i] - mean) * rstd * w[c] + bb[c]);
    }
}

// bf16-mode variant writing a separate bf16 copy (the input stays intact): 8 elements per thread; the input is fp32,
// or bf16 (IB: the decoder's level-0 ConvT output, whose statistics its GEMM epilogue took before rounding)
template <bool IB>
__global__ __launch_bounds__(256) void gn_gelu_bf16_kernel(const void* __restrict__ h, bf16_t* __restrict__ out,
                                                           int64_t per_batch, int H, const double* __restrict__ st,
                                                           const float* __restrict__ w, const float* __restrict__ bb) {
    const int64_t b = blockIdx.y;
    float mean, rstd;
    gn_params(st, b, per_batch, mean, rstd);
    bf16_t* o = out + b * per_batch;
    const int n8 = (int)(per_batch / 8);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n8; i += gridDim.x * 256) {
        float x[8];
        if constexpr (IB) {
            const uint4 q = *reinterpret_cast<const uint4*>((const bf16_t*)h + b * per_batch + 8 * (int64_t)i);
            const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[2 * k] = __uint_as_float(qq[k] << 16);
                x[2 * k + 1] = __uint_as_float(qq[k] & 0xFFFF0000u);
            }
        } else {
            const float* p = (const float*)h + b * per_batch;
            const float4 u = *reinterpret_cast<const float4*>(p + 8 * (int64_t)i);
            const float4 v = *reinterpret_cast<const float4*>(p + 8 * (int64_t)i + 4);
            x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w; x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
        }
        const int c0 = (8 * i) % H;
        bf16_t r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = f2bf(gelu_fast((x[j] - mean) * rstd * w[c0 + j] + bb[c0 + j]));
        *reinterpret_cast<uint4*>(o + 8 * (int64_t)i) = *reinterpret_cast<const uint4*>(r);
    }
}

void gn_gelu_bf16_launch(const float* h, bf16_t* out, int nb, int64_t per_batch, int H, const double* stats,
                         const float* w, const float* b, hipStream_t s) {
    int blocks = (int)((per_batch / 8 + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    KScope ks(s);
    if (ks.on()) ks.begin("gn_gelu_bf16_kernel<false>", 0.0, (double)nb * per_batch * (4 + 2));
    hipLaunchKernelGGL(gn_gelu_bf16_kernel<false>, dim3(blocks, nb), dim3(256), 0, s, h, out, per_batch, H, stats, w, b);
}

// Wide DConv levels (H = C/8 = 24, 48; bf16 mode): gn_gelu_bf16_kernel's output plus the GroupNorm statistics of the
// following 1x1 conv's 2C outputs from its moments (ctx.h conv1x1_moments on the bf16-rounded weights: G = W^T W,
// v = W^T b, u = W^T 1, sum b, sum b^2), so no separate statistics GEMM pass over the 1x1 (forward.cpp dconv):
//   sum_n y_n = sum b + u.x,   sum_n y_n^2 = sum b^2 + 2 v.x + x^T G x,   x = the bf16 GELU(GN(h)) row the GEMM reads.
// One lane per position (row of H channels); groups of L >= 64 positions, so a wave spans at most two groups (its
// sums go to the first active lane's group and, for lanes past a boundary, to the last lane's group).
constexpr int GN_MOM_RMAX = 4;

template <int H, bool MULTI>
__global__ __launch_bounds__(256) void gn_gelu_mom_kernel(const float* __restrict__ h, bf16_t* __restrict__ out,
                                                          int64_t npos, int64_t L, int R_,
                                                          const double* __restrict__ st,
                                                          const float* __restrict__ w, const float* __restrict__ bb,
                                                          const float* __restrict__ gram, double* __restrict__ st_y) {
    __shared__ float wb[2 * H];
    // per (pass, wave) the segmented sums of its <= 2 groups; merged in position order into one atomic pair per
    // group and workgroup (one pair per wave put up to ~260 waves on each group's line: atomic-bound at large L)
    __shared__ double rs[GN_MOM_RMAX * 4 * 2][2];
    __shared__ int64_t rgid[GN_MOM_RMAX * 4 * 2];
    for (int i = threadIdx.x; i < 2 * H; i += 256) wb[i] = i < H ? w[i] : bb[i - H];
    __syncthreads();
    const int wv = threadIdx.x >> 6;
    const int R = MULTI ? R_ : 1;     // (MULTI = false: one pass, no loop - the H = 24, 48 loop bodies spill SGPRs)
#pragma unroll 1
    for (int it = 0; it < R; ++it) {
        const int64_t p0 = ((int64_t)blockIdx.x * R + it) * 256;
        const int64_t p = p0 + threadIdx.x;
        const bool act = p < npos;
        const int64_t pp = act ? p : npos - 1;
        const int64_t g = pp / L;
        float mean, rstd;
        gn_params(st, g, L * H, mean, rstd);
        constexpr int HF = H % 4 == 0 ? H : (H + 7) / 8 * 8;       // f32 input row stride (H = 6: 8, dconv_conv3)
        float x[HF];
        const float4* hr = reinterpret_cast<const float4*>(h + pp * HF);
#pragma unroll
        for (int q = 0; q < HF / 4; ++q) {
            const float4 v = hr[q];
            x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
        }
        constexpr int OS = H % 8 == 0 ? H : (H + 15) / 16 * 16;     // output row stride (H = 12: rows padded to 16)
        uint32_t pk[OS / 2];
#pragma unroll
        for (int j = 0; j < H; j += 2) {
            pk[j / 2] = pack2bf(gelu_fast((x[j] - mean) * rstd * wb[j] + wb[H + j]),
                                gelu_fast((x[j + 1] - mean) * rstd * wb[j + 1] + wb[H + j + 1]));
            x[j] = __uint_as_float(pk[j / 2] << 16);                 // the bf16 values the 1x1 GEMM multiplies
            x[j + 1] = __uint_as_float(pk[j / 2] & 0xFFFF0000u);
        }
#pragma unroll
        for (int j = H / 2; j < OS / 2; ++j) pk[j] = 0u;
        if (act) {
            uint4* o = reinterpret_cast<uint4*>(out + pp * OS);
#pragma unroll
            for (int q = 0; q < OS / 8; ++q) o[q] = make_uint4(pk[4 * q], pk[4 * q + 1], pk[4 * q + 2], pk[4 * q + 3]);
        }
        // the moments are wave-uniform: scalar loads, one G row per step (the pointer is made opaque per row, so the
        // compiler cannot hoist all H*H loads to the front, which needed ~2300 registers and spilled)
        typedef __attribute__((address_space(4))) const float cfloat;    // constant address space: scalar loads
        float qf = 0.f, lv = 0.f, lw = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) {
            cfloat* gr = (cfloat*)(gram + j * H);
            asm volatile("" : "+s"(gr), "+v"(qf));              // row j's loads after row j-1's products
            float t4[4] = {0.f, 0.f, 0.f, 0.f};                 // 4 independent chains (the FMA latency, not issue)
#pragma unroll
            for (int k0 = 0; k0 < H; k0 += 24) {               // (at most 24 row values in SGPRs at a time)
                cfloat* gk = gr + k0;
                if (k0 > 0) asm volatile("" : "+s"(gk), "+v"(t4[0]));
#pragma unroll
                for (int k = 0; k < (H - k0 < 24 ? H - k0 : 24); ++k) t4[k & 3] = fmaf(gk[k], x[k0 + k], t4[k & 3]);
            }
            qf = fmaf(x[j], (t4[0] + t4[1]) + (t4[2] + t4[3]), qf);
            lv = fmaf(gr[H * (H - j) + j], x[j], lv);            // gram[H*H + j]      = (W^T b)_j
            lw = fmaf(gr[H * (H - j) + H + j], x[j], lw);        // gram[H*H + H + j]  = (W^T 1)_j
        }
        cfloat* gt = (cfloat*)(gram + H * H + 2 * H);
        const float sb = gt[0], sb2 = gt[1];
        const double s1 = act ? (double)(sb + lw) : 0.0;
        const double s2 = act ? (double)(sb2 + (2.f * lv + qf)) : 0.0;
        // segmented wave sums: group gA of the first lane, gB of the last active lane (gA <= g <= gB, gB <= gA + 1)
        const int64_t gA = __builtin_amdgcn_readfirstlane((int)g);
        const int64_t last = p0 + wv * 64 + 63;
        const int64_t gB = (last < npos ? last : npos - 1) / L;
        const bool inA = g == gA;
        const double a1 = wave_sum_d(inA ? s1 : 0.0), a2 = wave_sum_d(inA ? s2 : 0.0);
        double b1 = 0.0, b2 = 0.0;
        if (gB != gA) {
            b1 = wave_sum_d(inA ? 0.0 : s1);
            b2 = wave_sum_d(inA ? 0.0 : s2);
        }
        if ((threadIdx.x & 63) == 0) {
            const int e = (it * 4 + wv) * 2;
            rgid[e] = gA; rs[e][0] = a1; rs[e][1] = a2;
            rgid[e + 1] = gB != gA ? gB : -1; rs[e + 1][0] = b1; rs[e + 1][1] = b2;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {          // entries in position order: groups non-decreasing
        int64_t cg = -1;
        double c1 = 0.0, c2 = 0.0;
        for (int e = 0; e < R * 8; ++e) {
            const int64_t ge = rgid[e];
            if (ge < 0) continue;
            if (ge != cg) {
                if (cg >= 0) {
                    atomicAdd(&st_y[2 * cg], c1);
                    atomicAdd(&st_y[2 * cg + 1], c2);
                }
                cg = ge;
                c1 = c2 = 0.0;
            }
            c1 += rs[e][0];
            c2 += rs[e][1];
        }
        if (cg >= 0) {
            atomicAdd(&st_y[2 * cg], c1);
            atomicAdd(&st_y[2 * cg + 1], c2);
        }
    }
}

// H = 48 with the quadratic form split over the workgroup's 4 waves: a workgroup takes 64 positions, wave w
// writes GELU(GN(h)) of channels [w H/4, (w + 1) H/4) of all 64 (one lane per position) and its bf16-rounded values
// into an LDS row per position, then takes G rows [w H/4, (w + 1) H/4) (scalar loads, as above) against the whole row;
// wave 0 adds the 4 partial forms.  4x the waves of gn_gelu_mom_kernel and a quarter of its serial G-row chain per
// wave: level 3 has only 66 k / 132 k positions, so the one-wave-per-64-positions form left the CUs idle (fenc3
// 0.104 -> 0.075 ms, tenc3 0.103 -> 0.051 for two launches; at H = 24 the split measured slower and is not used).
template <int H>
__global__ __launch_bounds__(256) void gn_gelu_mom_split_kernel(const float* __restrict__ h, bf16_t* __restrict__ out,
                                                                int64_t npos, int64_t L,
                                                                const double* __restrict__ st,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bb,
                                                                const float* __restrict__ gram,
                                                                double* __restrict__ st_y) {
    constexpr int QJ = H / 4;
    static_assert(QJ % 2 == 0, "channel pairs");
    __shared__ float wb[2 * H];
    __shared__ float xs[64][H + 1];          // (odd pitch: the row reads of 64 lanes hit distinct banks)
    __shared__ float red[4][64][3];
    for (int i = threadIdx.x; i < 2 * H; i += 256) wb[i] = i < H ? w[i] : bb[i - H];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t p = (int64_t)blockIdx.x * 64 + lane;
    const bool act = p < npos;
    const int64_t pp = act ? p : npos - 1;
    const int64_t g = pp / L;
    float mean, rstd;
    gn_params(st, g, L * H, mean, rstd);
    {
        const int c0 = QJ * wv;
        const float2* hr = reinterpret_cast<const float2*>(h + pp * H + c0);
        uint32_t* o = reinterpret_cast<uint32_t*>(out + pp * H + c0);
#pragma unroll
        for (int q = 0; q < QJ / 2; ++q) {
            const float2 v = hr[q];
            const int c = c0 + 2 * q;
            const uint32_t pk = pack2bf(gelu_fast((v.x - mean) * rstd * wb[c] + wb[H + c]),
                                        gelu_fast((v.y - mean) * rstd * wb[c + 1] + wb[H + c + 1]));
            if (act) o[q] = pk;
            xs[lane][c] = __uint_as_float(pk << 16);
            xs[lane][c + 1] = __uint_as_float(pk & 0xFFFF0000u);
        }
    }
    __syncthreads();
    float x[H];
#pragma unroll
    for (int k = 0; k < H; ++k) x[k] = xs[lane][k];
    typedef __attribute__((address_space(4))) const float cfloat;    // constant address space: scalar loads
    float qf = 0.f, lv = 0.f, lw = 0.f;
    const int j0 = __builtin_amdgcn_readfirstlane(QJ * wv);
#pragma unroll
    for (int jj = 0; jj < QJ; ++jj) {
        const int j = j0 + jj;
        cfloat* gr = (cfloat*)(gram + j * H);
        asm volatile("" : "+s"(gr), "+v"(qf));              // row j's loads after row j-1's products
        float t4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < H; k0 += 24) {
            cfloat* gk = gr + k0;
            if (k0 > 0) asm volatile("" : "+s"(gk), "+v"(t4[0]));
#pragma unroll
            for (int k = 0; k < (H - k0 < 24 ? H - k0 : 24); ++k) t4[k & 3] = fmaf(gk[k], x[k0 + k], t4[k & 3]);
        }
        const float xj = xs[lane][j];
        qf = fmaf(xj, (t4[0] + t4[1]) + (t4[2] + t4[3]), qf);
        lv = fmaf(gr[H * (H - j) + j], xj, lv);             // gram[H*H + j]      = (W^T b)_j
        lw = fmaf(gr[H * (H - j) + H + j], xj, lw);         // gram[H*H + H + j]  = (W^T 1)_j
    }
    red[wv][lane][0] = qf;
    red[wv][lane][1] = lv;
    red[wv][lane][2] = lw;
    __syncthreads();
    if (wv != 0) return;
    qf = (red[0][lane][0] + red[1][lane][0]) + (red[2][lane][0] + red[3][lane][0]);
    lv = (red[0][lane][1] + red[1][lane][1]) + (red[2][lane][1] + red[3][lane][1]);
    lw = (red[0][lane][2] + red[1][lane][2]) + (red[2][lane][2] + red[3][lane][2]);
    cfloat* gt = (cfloat*)(gram + H * H + 2 * H);
    const float sb = gt[0], sb2 = gt[1];
    const double s1 = act ? (double)(sb + lw) : 0.0;
    const double s2 = act ? (double)(sb2 + (2.f * lv + qf)) : 0.0;
    const int64_t gA = __builtin_amdgcn_readfirstlane((int)g);
    const int64_t last = (int64_t)blockIdx.x * 64 + 63;
    const int64_t gB = (last < npos ? last : npos - 1) / L;
    const bool inA = g == gA;
    const double a1 = wave_sum_d(inA ? s1 : 0.0), a2 = wave_sum_d(inA ? s2 : 0.0);
    if (lane == 0) {
        atomicAdd(&st_y[2 * gA], a1);
        atomicAdd(&st_y[2 * gA + 1], a2);
    }
    if (gB != gA) {
        const double b1 = wave_sum_d(inA ? 0.0 : s1), b2 = wave_sum_d(inA ? 0.0 : s2);
        if (lane == 0) {
            atomicAdd(&st_y[2 * gB], b1);
            atomicAdd(&st_y[2 * gB + 1], b2);
        }
    }
}

int gn_gelu_mom_launch(const float* h, uint16_t* out, int nb, int64_t L, int H, const double* stats, const float* w,
                       const float* b, const float* gram, double* st_y, hipStream_t s) {
    if (L < 64 || (H != 6 && H != 12 && H != 24 && H != 48)) return -1;
    const int64_t npos = (int64_t)nb * L;
    // 256-position passes per workgroup: as many as keep >= 2048 workgroups (8 per CU), at most GN_MOM_RMAX
    const int64_t passes = (npos + 255) / 256;
    const int R = H <= 12 ? (int)std::max<int64_t>(1, std::min<int64_t>(GN_MOM_RMAX, passes / 2048)) : 1;
    const dim3 grid((unsigned)((passes + R - 1) / R));
    KScope ks(s);
    if (ks.on())
        ks.begin(klabel(H <= 24 ? "gn_gelu_mom_kernel<%d>" : "gn_gelu_mom_split_kernel<%d>", H), 2.0 * npos * (H * H + 2 * H),
                 (double)npos * H * (4 + 2));
    if (H == 6) hipLaunchKernelGGL((gn_gelu_mom_kernel<6, true>), grid, dim3(256), 0, s, h, out, npos, L, R, stats, w, b, gram, st_y);
    else if (H == 12) hipLaunchKernelGGL((gn_gelu_mom_kernel<12, true>), grid, dim3(256), 0, s, h, out, npos, L, R, stats, w, b, gram, st_y);
    else if (H == 24) hipLaunchKernelGGL((gn_gelu_mom_kernel<24, false>), grid, dim3(256), 0, s, h, out, npos, L, R, stats, w, b, gram, st_y);
    else hipLaunchKernelGGL((gn_gelu_mom_split_kernel<48>), dim3((unsigned)((npos + 63) / 64)), dim3(256), 0, s, h, out, npos, L, stats, w, b, gram, st_y);
    return (int)hipGetLastError();
}

void gn_gelu_bf16in_launch(const uint16_t* h, uint16_t* out, int nb, int64_t per_batch, int H, const double* stats,
                           const float* w, const float* b, hipStream_t s) {
    int blocks = (int)((per_batch / 8 + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    KScope ks(s);
    if (ks.on()) ks.begin("gn_gelu_bf16_kernel<true>", 0.0, (double)nb * per_batch * (2 + 2));
    hipLaunchKernelGGL(gn_gelu_bf16_kernel<true>, dim3(blocks, nb), dim3(256), 0, s, h, out, per_batch, H, stats, w, b);
}

void gn_gelu_launch(float* h, int nb, int64_t per_batch, int H, const double* stats, const float* w, const float* b,
                    hipStream_t s, bool fast) {
    int blocks = (int)((per_batch + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    KScope ks(s);
    if (ks.on()) ks.begin(fast ? "gn_gelu_kernel<true>" : "gn_gelu_kernel<false>", 0.0, 2.0 * nb * per_batch * 4);
    if (fast) hipLaunchKernelGGL(gn_gelu_kernel<true>, dim3(blocks, nb), dim3(256), 0, s, h, per_batch, H, stats, w, b);
    else hipLaunchKernelGGL(gn_gelu_kernel<false>, dim3(blocks, nb), dim3(256), 0, s, h, per_batch, H, stats, w, b);
}

__global__ __launch_bounds__(256) void gn_apply_kernel(float* __restrict__ x, int64_t per_batch, int C,
                                                       const double* __restrict__ st, const float* __restrict__ w,
                                                       const float* __restrict__ bb) {
    const int64_t b = blockIdx.y;
    float mean, rstd;
    gn_params(st, b, per_batch, mean, rstd);
    float* p = x + b * per_batch;
    const int n = (int)per_batch;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int c = i % C;
        p[i] = (p[i] - mean) * rstd * w[c] + bb[c];
    }
}

void gn_apply_launch(float* x, int nb, int64_t N, int C, const double* stats, const float* w, const float* b,
                     hipStream_t s) {
    int64_t per = N * C;
    int blocks = (int)((per + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    KScope ks(s);
    if (ks.on()) ks.begin("gn_apply_kernel", 0.0, 2.0 * nb * per * 4);
    hipLaunchKernelGGL(gn_apply_kernel, dim3(blocks, nb), dim3(256), 0, s, x, per, C, stats, w, b);
}

// --------------------------------------------------------------------------------------------- LayerNorm
// One wave per token row of C = 64 * PER channels.  PER == 8 (C = 512): each lane owns 8 consecutive channels, so a
// row is read as two float4 per lane (one 2 KB coalesced row per instruction pair) and the bf16 output leaves as one
// 16-B store per lane; other PER: strided channels lane + 64 j.
ATHD_DEV void ld8(const float* p, float* o) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <int PER>
__global__ __launch_bounds__(256) void layernorm_kernel(const LnDesc d) {
    constexpr int C = PER * 64;
    constexpr bool VEC = PER == 8;
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t rows = (int64_t)d.nb * d.N;
    if (row >= rows) return;
    const int64_t b = row / d.N;
    const int64_t tok = row % d.N;
    float* xr = d.x + row * C;
    auto chan = [&](int j) { return VEC ? 8 * lane + j : lane + 64 * j; };
    float v[PER];
    if (VEC) {
        ld8(xr + 8 * lane, v);
    } else {
#pragma unroll
        for (int j = 0; j < PER; ++j) v[j] = xr[chan(j)];
    }
    if (d.gn_stats) {
        float gm, gr;
        gn_params(d.gn_stats, b, d.N * (int64_t)C, gm, gr);
        if (VEC) {
            float gw[8], gb[8];
            ld8(d.gn_w + 8 * lane, gw);
            ld8(d.gn_b + 8 * lane, gb);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (v[j] - gm) * gr * gw[j] + gb[j];
            float4* xo = reinterpret_cast<float4*>(xr + 8 * lane);
            xo[0] = make_float4(v[0], v[1], v[2], v[3]);
            xo[1] = make_float4(v[4], v[5], v[6], v[7]);
        } else {
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const int c = chan(j);
                v[j] = (v[j] - gm) * gr * d.gn_w[c] + d.gn_b[c];
                xr[c] = v[j];
            }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) s += v[j];
    const float mean = wave_sum(s) * (1.f / C);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) { const float t = v[j] - mean; q += t * t; }
    const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / C) + 1e-5f);
    float y[PER];
    if (VEC) {                                   // affine and positional rows as float4 pairs too
        float wv[8], bv[8], pv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        ld8(d.w + 8 * lane, wv);
        ld8(d.b + 8 * lane, bv);
        if (d.pos) ld8(d.pos + tok * C + 8 * lane, pv);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (v[j] - mean) * rstd * wv[j] + bv[j] + pv[j];
    } else {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = chan(j);
            y[j] = (v[j] - mean) * rstd * d.w[c] + d.b[c];
            if (d.pos) y[j] += d.pos[tok * C + c];
        }
    }
    if (VEC && d.out_bf16) {
        reinterpret_cast<uint4*>((bf16_t*)d.out + row * C)[lane] =
            make_uint4(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]), pack2bf(y[4], y[5]), pack2bf(y[6], y[7]));
    } else if (VEC) {
        float4* o = reinterpret_cast<float4*>((float*)d.out + row * C);
        o[2 * lane] = make_float4(y[0], y[1], y[2], y[3]);
        o[2 * lane + 1] = make_float4(y[4], y[5], y[6], y[7]);
    } else {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = chan(j);
            if (d.out_bf16) ((bf16_t*)d.out)[row * C + c] = f2bf(y[j]);
            else ((float*)d.out)[row * C + c] = y[j];
        }
    }
}

// C = 512 with RW rows per wave: every load of the wave's rows (and the affine rows) is issued before the first
// reduction, RW x 32 B in flight per lane instead of 32 B (one short row per wave left each wave mostly waiting on
// its single load).  Per row the arithmetic is layernorm_kernel<8>'s.
template <int RW>
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const LnDesc d) {
    constexpr int C = 512;
    const int lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RW;
    const int64_t rows = (int64_t)d.nb * d.N;
    if (row0 >= rows) return;
    float v[RW][8];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const int64_t row = row0 + r < rows ? row0 + r : rows - 1;
        ld8(d.x + row * C + 8 * lane, v[r]);
    }
    float wv[8], bv[8], wv2[8], bv2[8];
    ld8(d.w + 8 * lane, wv);
    ld8(d.b + 8 * lane, bv);
    if (d.out2) {
        ld8(d.w2 + 8 * lane, wv2);
        ld8(d.b2 + 8 * lane, bv2);
    }
    if (d.gn_stats) {
        float gw[8], gb[8];
        ld8(d.gn_w + 8 * lane, gw);
        ld8(d.gn_b + 8 * lane, gb);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int64_t row = row0 + r;
            if (row >= rows) break;
            float gm, gr;
            gn_params(d.gn_stats, row / d.N, d.N * (int64_t)C, gm, gr);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[r][j] = (v[r][j] - gm) * gr * gw[j] + gb[j];
            if (d.gn_writeback) {
                float4* xo = reinterpret_cast<float4*>(d.x + row * C + 8 * lane);
                xo[0] = make_float4(v[r][0], v[r][1], v[r][2], v[r][3]);
                xo[1] = make_float4(v[r][4], v[r][5], v[r][6], v[r][7]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const int64_t row = row0 + r;
        if (row >= rows) break;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[r][j];
        const float mean = wave_sum(s) * (1.f / C);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float t = v[r][j] - mean; q += t * t; }
        const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / C) + 1e-5f);
        float pv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};     // (positional rows: the input LayerNorms only)
        if (d.pos) ld8(d.pos + (row % d.N) * C + 8 * lane, pv);
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (v[r][j] - mean) * rstd * wv[j] + bv[j] + pv[j];
        if (d.out2) {
            float y2[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) y2[j] = (v[r][j] - mean) * rstd * wv2[j] + bv2[j];
            reinterpret_cast<uint4*>((bf16_t*)d.out2 + row * C)[lane] =
                make_uint4(pack2bf(y2[0], y2[1]), pack2bf(y2[2], y2[3]), pack2bf(y2[4], y2[5]), pack2bf(y2[6], y2[7]));
        }
        if (d.out_bf16) {
            reinterpret_cast<uint4*>((bf16_t*)d.out + row * C)[lane] =
                make_uint4(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]), pack2bf(y[4], y[5]), pack2bf(y[6], y[7]));
        } else {
            float4* o = reinterpret_cast<float4*>((float*)d.out + row * C);
            o[2 * lane] = make_float4(y[0], y[1], y[2], y[3]);
            o[2 * lane + 1] = make_float4(y[4], y[5], y[6], y[7]);
        }
    }
}

// rows per wave: 4 measured 1.80 ms per forward vs 1.83 for one row per wave (layernorm_kernel<8>); whole-step A/B of
// 1, 2 and 4 within noise (tools/gpu_r03f.sh)
constexpr int LN_RW = 4;

void layernorm_launch(const LnDesc& d0, hipStream_t s) {
    const int64_t rows = (int64_t)d0.nb * d0.N;
    LnDesc d = d0;
    // gn_writeback = 0 (the pending GroupNorm applied in registers only) exists only where ln_lazy_gn_ok holds (the
    // C = 512 row kernel, out2 fused into it): the out2 split below reads x again expecting the GroupNorm written back,
    // and layernorm_kernel<6> always writes it back.  forward.cpp requests the lazy form only under that predicate;
    // anything else is written back here
    if (!d.gn_writeback && !ln_lazy_gn_ok(d)) d.gn_writeback = 1;
    if (d.out2 && !(d.C == 512 && d.out_bf16 && !d.pos)) {   // (only the C = 512 bf16 row kernel has out2)
        LnDesc d2 = d0;
        d2.gn_stats = nullptr; d2.w = d0.w2; d2.b = d0.b2; d2.out = d0.out2; d2.out2 = nullptr; d2.pos = nullptr;
        d.out2 = nullptr;
        layernorm_launch(d, s);
        layernorm_launch(d2, s);          // reads x after the first launch applied the pending GroupNorm
        return;
    }
    if (d.C == 512) {
        const dim3 grid((unsigned)((rows + 4 * LN_RW - 1) / (4 * LN_RW)));
        KScope ks(s);
        if (ks.on()) {
            double by = (double)rows * d.C * (4 + (d.out_bf16 ? 2 : 4)) +
                        (d.gn_stats && d.gn_writeback ? (double)rows * d.C * 4 : 0.0);
            if (d.pos) by += (double)d.N * d.C * 4;
            if (d.out2) by += (double)rows * d.C * 2;
            ks.begin(klabel("layernorm_rows_kernel<%d>", LN_RW), 0.0, by);
        }
        hipLaunchKernelGGL(layernorm_rows_kernel<LN_RW>, grid, dim3(256), 0, s, d);
        return;
    }
    dim3 grid((unsigned)((rows + 3) / 4));
    KScope ks(s);
    if (ks.on()) {
        double by = (double)rows * d.C * (4 + (d.out_bf16 ? 2 : 4)) + (d.gn_stats ? (double)rows * d.C * 4 : 0.0);
        if (d.pos) by += (double)d.N * d.C * 4;
        ks.begin("layernorm_kernel<6>", 0.0, by);
    }
    hipLaunchKernelGGL(layernorm_kernel<6>, grid, dim3(256), 0, s, d);
}

// --------------------------------------------------------------------------------------------- text conditioning
// U[item] = X[item / P] + a[item] (row vector over C); float4 lanes.  Ub (optional, throughput mode): a bf16 copy of U,
// the A operand of the text MLP's first GEMM (U itself stays f32 for the residual of the second)
// bf16 copy of an fp32 tensor (n % 8 == 0), round-to-nearest-even as every GEMM's fp32-A conversion (f2bf): the
// segment features x_enc / xt_enc for the bf16-A text.mlp0 GEMM (numerically what gemm2's fp32-A path multiplies)
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, int64_t n8) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        const float4 a = reinterpret_cast<const float4*>(x)[2 * i], b = reinterpret_cast<const float4*>(x)[2 * i + 1];
        reinterpret_cast<uint4*>(y)[i] = make_uint4(pack2bf(a.x, a.y), pack2bf(a.z, a.w), pack2bf(b.x, b.y), pack2bf(b.z, b.w));
    }
}

void to_bf16_launch(const float* x, uint16_t* y, int64_t n, hipStream_t s) {
    const int64_t n8 = n / 8;
    const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 4096);
    KScope ks(s);
    if (ks.on()) ks.begin("to_bf16_kernel", 0.0, (double)n * 6);
    hipLaunchKernelGGL(to_bf16_kernel, dim3(blocks), dim3(256), 0, s, x, y, n8);
}

// The chain v = Wv t + bv -> vi = Wiv v + biv -> a = Wo vi + bo -> c0 = W0 a + b0 is affine in the text row t, so
// athd_finalize composes it in double into two 384 x 512 maps: a = Ma t + ma, c0 = Mc t + mc (stored transposed,
// [k][o]).  Grid (rows, 2 maps x 6 chunks of 64 outputs): lane o of a chunk sums a quarter of k per wave (coalesced
// [k][o] reads), the quarters meet in LDS.  text_per_item = 0 (forward_prompts): one row per PROMPT, written for
// every item of that prompt (item % P).  (Round 2 ran the four matvecs serially per item with [o][k] reads: 110 us.)
__global__ __launch_bounds__(256) void text_vec_kernel(const float* __restrict__ text, int NI, int P, int per_item,
                                                       const float* __restrict__ maT, const float* __restrict__ ma,
                                                       const float* __restrict__ mcT, const float* __restrict__ mc,
                                                       const float* __restrict__ b2, float* __restrict__ a,
                                                       float* __restrict__ c0, float* __restrict__ c2) {
    constexpr int D = 384, TD = 512;
    __shared__ float t[TD];
    __shared__ float red[4][64];
    const int src = blockIdx.x;                       // item (per_item) or prompt
    const int step = per_item ? NI : P;               // items sharing this row: src, src + step, ...
    const int mat = blockIdx.y / 6, o = (blockIdx.y % 6) * 64 + (threadIdx.x & 63), kq = threadIdx.x >> 6;
    const float* tp = text + (int64_t)src * TD;
    for (int i = threadIdx.x; i < TD; i += 256) t[i] = tp[i];
    __syncthreads();
    const float* mT = mat == 0 ? maT : mcT;
    float s = 0.f;
#pragma unroll 8
    for (int k = kq * 128; k < kq * 128 + 128; ++k) s += mT[(int64_t)k * D + o] * t[k];
    red[kq][threadIdx.x & 63] = s;
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const float v = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x])) +
                    (mat == 0 ? ma[o] : mc[o]);
    if (mat == 0) {
        //   (x + a) + mlp2(h) = x + W2 h + (a + b2)   ->  c2 = a + b2   (ATHTDemucs_v2.py:46-48)
        const float r2 = v + b2[o];
        for (int it = src; it < NI; it += step) {
            a[(int64_t)it * D + o] = v;
            c2[(int64_t)it * D + o] = r2;
        }
    } else if (c0) {
        //   mlp0(x + a) = W0 x + (W0 a + b0)   ->  c0 = W0 a + b0
        for (int it = src; it < NI; it += step) c0[(int64_t)it * D + o] = v;
    }
}

void text_vec_launch(const float* text, int NI, int P, int text_per_item, const float* maT, const float* ma,
                     const float* mcT, const float* mc, const float* b2, float* a, float* c0, float* c2, hipStream_t s) {
    const int nsrc = text_per_item ? NI : (P < NI ? P : NI);
    KScope ks(s);
    if (ks.on()) ks.begin("text_vec_kernel", 2.0 * nsrc * 2 * 512.0 * 384, 2 * 512.0 * 384 * 4);
    hipLaunchKernelGGL(text_vec_kernel, dim3(nsrc, 12), dim3(256), 0, s, text, NI, P, text_per_item, maT, ma, mcT, mc, b2,
                       a, c0, c2);
}

// --------------------------------------------------------------------------------------------- decoder merge
// out[item][ho][w][c] = resize_H(act(GN(src)))[ho][w][c] + 0.1 * resize_H(skip[item/P])[ho][w][c]   (FreqDecoder /
// TimeDecoder body, ATHTDemucs_v2.py:90-103 / :127-138).  Each thread produces V consecutive channels of one
// position (V = 8: one 16-B bf16 / two 16-B fp32 accesses per row touched).  Per-item counts are < 2^31.
template <int V>
ATHD_DEV void ldv(const void* p, int bf, int64_t i, float* v) {
    if constexpr (V == 8) {
        if (bf) {
            const uint4 q = *reinterpret_cast<const uint4*>((const bf16_t*)p + i);
            const bf16_t* h = reinterpret_cast<const bf16_t*>(&q);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = bf2f(h[j]);
        } else {
            const float4 a = *reinterpret_cast<const float4*>((const float*)p + i);
            const float4 b = *reinterpret_cast<const float4*>((const float*)p + i + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
    } else {   // V == 4
        if (bf) {
            const uint2 q = *reinterpret_cast<const uint2*>((const bf16_t*)p + i);
            const bf16_t* h = reinterpret_cast<const bf16_t*>(&q);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = bf2f(h[j]);
        } else {
            const float4 a = *reinterpret_cast<const float4*>((const float*)p + i);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        }
    }
}

template <int V>
ATHD_DEV void merge_src_v(const MergeDesc& d, int64_t item, int i, int w, int c, float mean, float rstd, float* x) {
    int slot = i;
    int rows = d.H_src;
    if (d.kept) {
        slot = 2 * (i >> 2) + ((i & 3) == 2 ? 1 : 0);
        rows = 2 * (d.H_src >> 2);
    }
    ldv<V>(d.src, d.src_bf16, item * (int64_t)rows * d.W * d.C + ((int64_t)slot * d.W + w) * d.C + c, x);
    if (d.stats) {
        if (d.fast_gelu) {
#pragma unroll
            for (int j = 0; j < V; ++j) x[j] = gelu_fast((x[j] - mean) * rstd * d.gn_w[c + j] + d.gn_b[c + j]);
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) x[j] = gelu_erf((x[j] - mean) * rstd * d.gn_w[c + j] + d.gn_b[c + j]);
        }
    }
}

// resize_H(act(GN(src)))[ho][w][c..c+V) of one item
template <int V>
ATHD_DEV void merge_src_lerp(const MergeDesc& d, int64_t item, int ho, int w, int c, float mean, float rstd, float* out) {
    if (d.H_src == d.H_out) {
        merge_src_v<V>(d, item, ho, w, c, mean, rstd, out);
    } else {
        float a[V], b[V];
        const LinIdx li = lin_index(ho, d.H_src, d.H_out);
        merge_src_v<V>(d, item, li.i0, w, c, mean, rstd, a);
        merge_src_v<V>(d, item, li.i1, w, c, mean, rstd, b);
#pragma unroll
        for (int j = 0; j < V; ++j) out[j] = li.l0 * a[j] + li.l1 * b[j];
    }
}

// 0.1 * resize_H(skip[seg])[ho][w][c..c+V): shared by the P prompt items of a segment, computed once
template <int V>
ATHD_DEV void merge_skip_v(const MergeDesc& d, int64_t seg, int ho, int w, int c, float* sv) {
    const int64_t sk = seg * (int64_t)d.H_skip * d.W * d.C_skip;
    float a[V], b[V];
    if (d.H_skip == d.H_out) {
        ldv<V>(d.skip, d.skip_bf16, sk + (int64_t)(ho * d.W + w) * d.C_skip + c, a);
#pragma unroll
        for (int j = 0; j < V; ++j) sv[j] = a[j] * 0.1f;
    } else {
        const LinIdx lj = lin_index(ho, d.H_skip, d.H_out);
        ldv<V>(d.skip, d.skip_bf16, sk + (int64_t)(lj.i0 * d.W + w) * d.C_skip + c, a);
        ldv<V>(d.skip, d.skip_bf16, sk + (int64_t)(lj.i1 * d.W + w) * d.C_skip + c, b);
#pragma unroll
        for (int j = 0; j < V; ++j) sv[j] = (lj.l0 * a[j] + lj.l1 * b[j]) * 0.1f;
    }
}

constexpr int MERGE_MAXP = 256;

// per-item GroupNorm (mean, rstd) of the block's segment into LDS
ATHD_DEV void merge_gn_lds(const MergeDesc& d, int64_t seg, float* s_mean, float* s_rstd) {
    for (int p = threadIdx.x; p < d.P; p += blockDim.x) {
        float mean = 0.f, rstd = 1.f;
        if (d.stats) gn_params(d.stats, seg * d.P + p, d.gn_count, mean, rstd);
        s_mean[p] = mean;
        s_rstd[p] = rstd;
    }
    __syncthreads();
}

// grid.y = segment; every thread reads the skip once and writes all P items of its segment
template <int V>
__global__ __launch_bounds__(256) void dec_merge_kernel(const MergeDesc d) {
    const int64_t seg = blockIdx.y;
    __shared__ float s_mean[MERGE_MAXP], s_rstd[MERGE_MAXP];
    merge_gn_lds(d, seg, s_mean, s_rstd);
    const int cv = d.C / V;
    const int n = d.H_out * d.W * cv;
    const int64_t per_item = (int64_t)d.H_out * d.W * d.C;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int c = (i % cv) * V;
        const int pw = i / cv;
        const int w = pw % d.W;
        const int ho = pw / d.W;
        float sv[V];
        merge_skip_v<V>(d, seg, ho, w, c, sv);
        for (int p = 0; p < d.P; ++p) {
            const int64_t item = seg * d.P + p;
            float v[V];
            merge_src_lerp<V>(d, item, ho, w, c, s_mean[p], s_rstd[p], v);
#pragma unroll
            for (int j = 0; j < V; ++j) v[j] = v[j] + sv[j];
            const int64_t o = item * per_item + (int64_t)pw * d.C + c;
            if (d.out_bf16) {
                bf16_t h[V];
#pragma unroll
                for (int j = 0; j < V; ++j) h[j] = f2bf(v[j]);
                if constexpr (V == 8) *reinterpret_cast<uint4*>((bf16_t*)d.out + o) = *reinterpret_cast<uint4*>(h);
                else *reinterpret_cast<uint2*>((bf16_t*)d.out + o) = *reinterpret_cast<uint2*>(h);
            } else {
#pragma unroll
                for (int j = 0; j < V; j += 4)
                    *reinterpret_cast<float4*>((float*)d.out + o + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
            }
        }
    }
}

// Time-branch merge (W = 1, all rows stored, V = 8 channels per thread, P prompt items per segment): each thread walks a
// run of DM_RUN consecutive output rows.  The H resize reads source rows (i0, i1) with i0 advancing by ~1 per output
// row, so the GroupNorm -> GELU'd rows are cached per item and each source row is loaded and activated once instead of
// twice (dec_merge_kernel: two rows per output row); the P items' rows are processed together (their loads in flight
// at once), the skip rows once per segment.  Same arithmetic as dec_merge_kernel, value for value.
constexpr int DM_RUN = 16;

template <int P, int PP, bool FAST>
__global__ __launch_bounds__(256) void dec_merge_w1_kernel(const MergeDesc d) {
    const int64_t seg = blockIdx.y;
    const int cv = d.C / 8;
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int run = t / cv, c = (t - run * cv) * 8;
    const int h0 = run * DM_RUN;
    if (h0 >= d.H_out) return;
    const int h1 = min(h0 + DM_RUN, d.H_out);
    const bool gn = d.stats != nullptr;
    float gw[8], gb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        gw[j] = gn ? d.gn_w[c + j] : 1.f;
        gb[j] = gn ? d.gn_b[c + j] : 0.f;
    }
    const int64_t src_item = (int64_t)d.H_src * d.C;
    const int64_t out_item = (int64_t)d.H_out * d.C;
    const int64_t sk = seg * (int64_t)d.H_skip * d.C_skip + c;
    // PP items per pass over the run (the skip rows are re-read per pass, from L2)
#pragma unroll 1
    for (int p0 = 0; p0 < P; p0 += PP) {
        float mean[PP], rstd[PP];
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            mean[p] = 0.f;
            rstd[p] = 1.f;
            if (gn) gn_params(d.stats, seg * P + p0 + p, d.gn_count, mean[p], rstd[p]);
        }
        // activated source row `row` of item p0 + p into x
        auto act_row = [&](int p, int row, float* x) {
            ldv<8>(d.src, d.src_bf16, (seg * P + p0 + p) * src_item + (int64_t)row * d.C + c, x);
            if (gn) {
                if constexpr (FAST) {      // GroupNorm affine folded into one FMA, GELU pairs on packed ops
#pragma unroll
                    for (int j = 0; j < 8; j += 2) {
                        const athd_f2v ga = (athd_f2v){gw[j], gw[j + 1]} * (athd_f2v){rstd[p], rstd[p]};
                        const athd_f2v gc = (athd_f2v){gb[j], gb[j + 1]} - (athd_f2v){mean[p], mean[p]} * ga;
                        const athd_f2v v = gelu_fast_pk(__builtin_elementwise_fma((athd_f2v){x[j], x[j + 1]}, ga, gc));
                        x[j] = v.x;
                        x[j + 1] = v.y;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) x[j] = gelu_erf((x[j] - mean[p]) * rstd[p] * gw[j] + gb[j]);
                }
            }
        };
        float r0[PP][8], r1[PP][8], ka[8], kb[8];
        int c0 = -1, c1 = -1, s0 = -1, s1 = -1;
        for (int ho = h0; ho < h1; ++ho) {
            const LinIdx li = lin_index(ho, d.H_src, d.H_out);
            const LinIdx lj = lin_index(ho, d.H_skip, d.H_out);
            if (li.i0 != c0) {
                if (li.i0 == c1) {
#pragma unroll
                    for (int p = 0; p < PP; ++p)
#pragma unroll
                        for (int j = 0; j < 8; ++j) r0[p][j] = r1[p][j];
                } else {
#pragma unroll
                    for (int p = 0; p < PP; ++p) act_row(p, li.i0, r0[p]);
                }
            }
            if (li.i1 != c1) {
                if (li.i1 == li.i0) {
#pragma unroll
                    for (int p = 0; p < PP; ++p)
#pragma unroll
                        for (int j = 0; j < 8; ++j) r1[p][j] = r0[p][j];
                } else {
#pragma unroll
                    for (int p = 0; p < PP; ++p) act_row(p, li.i1, r1[p]);
                }
            }
            c0 = li.i0;
            c1 = li.i1;
            if (lj.i0 != s0 || lj.i1 != s1) {
                ldv<8>(d.skip, d.skip_bf16, sk + (int64_t)lj.i0 * d.C_skip, ka);
                ldv<8>(d.skip, d.skip_bf16, sk + (int64_t)lj.i1 * d.C_skip, kb);
                s0 = lj.i0;
                s1 = lj.i1;
            }
            float sv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) sv[j] = d.H_skip == d.H_out ? ka[j] * 0.1f : (lj.l0 * ka[j] + lj.l1 * kb[j]) * 0.1f;
#pragma unroll
            for (int p = 0; p < PP; ++p) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float m = d.H_src == d.H_out ? r0[p][j] : li.l0 * r0[p][j] + li.l1 * r1[p][j];
                    v[j] = m + sv[j];
                }
                const int64_t o = (seg * P + p0 + p) * out_item + (int64_t)ho * d.C + c;
                if (d.out_bf16) {
                    bf16_t h[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) h[j] = f2bf(v[j]);
                    *reinterpret_cast<uint4*>((bf16_t*)d.out + o) = *reinterpret_cast<uint4*>(h);
                } else {
                    *reinterpret_cast<float4*>((float*)d.out + o) = make_float4(v[0], v[1], v[2], v[3]);
                    *reinterpret_cast<float4*>((float*)d.out + o + 4) = make_float4(v[4], v[5], v[6], v[7]);
                }
            }
        }
    }
}

// last freq level: C = 4 merged channels -> freq_out 1x1 (4 -> 2), FO^T [item][w][ho][2] (frame-major for the iSTFT)
__global__ __launch_bounds__(256) void dec_merge_proj_kernel(const MergeDesc d) {
    const int64_t seg = blockIdx.y;
    __shared__ float s_mean[MERGE_MAXP], s_rstd[MERGE_MAXP];
    merge_gn_lds(d, seg, s_mean, s_rstd);
    const int n = d.H_out * d.W;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int w = i % d.W;
        const int ho = i / d.W;
        float sv[4];
        merge_skip_v<4>(d, seg, ho, w, 0, sv);
        for (int p = 0; p < d.P; ++p) {
            const int64_t item = seg * d.P + p;
            float m[4];
            merge_src_lerp<4>(d, item, ho, w, 0, s_mean[p], s_rstd[p], m);
#pragma unroll
            for (int j = 0; j < 4; ++j) m[j] = m[j] + sv[j];
            float2 o;
            o.x = d.proj_b[0] + (d.proj_w[0] * m[0] + d.proj_w[1] * m[1] + d.proj_w[2] * m[2] + d.proj_w[3] * m[3]);
            o.y = d.proj_b[1] + (d.proj_w[4] * m[0] + d.proj_w[5] * m[1] + d.proj_w[6] * m[2] + d.proj_w[7] * m[3]);
            *reinterpret_cast<float2*>((float*)d.out + item * (int64_t)n * 2 + ((int64_t)w * d.H_out + ho) * 2) = o;
        }
    }
}

int dec_merge_launch(const MergeDesc& d, hipStream_t s) {
    if (d.P < 1 || d.P > MERGE_MAXP || d.NI % d.P != 0) return -1;
    const int V = (d.C % 8 == 0) ? 8 : 4;    // C is 192/96/48 (8) or 4
    const int64_t n = (int64_t)d.H_out * d.W * (d.proj_w ? 1 : d.C / V);
    int blocks = (int)((n + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    // time-branch levels (W = 1, all rows stored, 4 prompts): runs of DM_RUN output rows per thread (dec_merge_w1)
    const bool w1 = !d.proj_w && V == 8 && d.W == 1 && !d.kept && d.P == 4 && d.C_skip >= d.C;
    KScope ks(s);
    if (ks.on()) {
        // unique bytes: the source rows the H-resize touches (<= 2 per output row), the skip rows likewise (once per
        // segment, shared by its P prompt items), the output once
        const double src_rows = std::min<double>(d.kept ? d.H_src / 2 : d.H_src, 2.0 * d.H_out);
        const double skip_rows = std::min<double>(d.H_skip, 2.0 * d.H_out);
        const double by = (double)d.NI * src_rows * d.W * d.C * (d.src_bf16 ? 2 : 4) +
                          (double)(d.NI / d.P) * skip_rows * d.W * d.C_skip * (d.skip_bf16 ? 2 : 4) +
                          (double)d.NI * d.H_out * d.W * (d.proj_w ? 2 * 4 : d.C * (d.out_bf16 ? 2 : 4));
        ks.begin(w1 ? (d.fast_gelu ? "dec_merge_w1_kernel<4,2,true>" : "dec_merge_w1_kernel<4,2,false>")
                 : d.proj_w ? "dec_merge_proj_kernel" : (V == 8 ? "dec_merge_kernel<8>" : "dec_merge_kernel<4>"), 0.0, by);
    }
    const dim3 grid(blocks, d.NI / d.P);
    if (w1) {
        const int64_t threads = (int64_t)((d.H_out + DM_RUN - 1) / DM_RUN) * (d.C / 8);
        const dim3 g1((unsigned)((threads + 255) / 256), d.NI / d.P);
        if (d.fast_gelu) hipLaunchKernelGGL((dec_merge_w1_kernel<4, 2, true>), g1, dim3(256), 0, s, d);
        else hipLaunchKernelGGL((dec_merge_w1_kernel<4, 2, false>), g1, dim3(256), 0, s, d);
        return (int)hipGetLastError();
    }
    if (d.proj_w) hipLaunchKernelGGL(dec_merge_proj_kernel, grid, dim3(256), 0, s, d);
    else if (V == 8) hipLaunchKernelGGL(dec_merge_kernel<8>, grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL(dec_merge_kernel<4>, grid, dim3(256), 0, s, d);
    return (int)hipGetLastError();
}

// --------------------------------------------------------------------------------------------- waveform layout
// (B, 2, T) -> (B, T, 2): the time level-0 conv then reads its 8 taps x 2 channels as one contiguous K row
__global__ __launch_bounds__(256) void wav_interleave_kernel(const float* __restrict__ wav, int64_t T,
                                                             float* __restrict__ out) {
    const int64_t b = blockIdx.y;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const float* x = wav + b * 2 * T;
    *reinterpret_cast<float2*>(out + (b * T + t) * 2) = make_float2(x[t], x[T + t]);
}

void wav_interleave_launch(const float* wav, int nb, int64_t T, float* out, hipStream_t s) {
    KScope ks(s);
    if (ks.on()) ks.begin("wav_interleave_kernel", 0.0, 2.0 * nb * 2 * T * 4);
    hipLaunchKernelGGL(wav_interleave_kernel, dim3((unsigned)((T + 255) / 256), nb), dim3(256), 0, s, wav, T, out);
}

// --------------------------------------------------------------------------------------------- position tables
__global__ void pos2d_kernel(float* out, int Fr, int T1, int C) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = (int64_t)Fr * T1 * C;
    if (i >= n) return;
    const int c = (int)(i % C);
    const int64_t tok = i / C;
    const int t = (int)(tok % T1), f = (int)(tok / T1);
    const int half = C / 2;                              // d_model/2 channels per axis
    const float k = -(float)(log(10000.0) / (double)half);
    const int cc = c < half ? c : c - half;
    const float div = expf((float)(cc & ~1) * k);        // arange(0, half, 2)[cc/2] * -(ln(1e4)/half)
    const float pos = (float)(c < half ? t : f);         // first half: width (time) axis, second: height (freq)
    const float ph = pos * div;
    out[i] = (cc & 1) ? cosf(ph) : sinf(ph);
}

void pos2d_launch(float* out, int Fr, int T1, int C, hipStream_t s) {
    const int64_t n = (int64_t)Fr * T1 * C;
    hipLaunchKernelGGL(pos2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, Fr, T1, C);
}

__global__ void pos1d_kernel(float* out, int T2, int C) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)T2 * C) return;
    const int c = (int)(i % C);
    const int t = (int)(i / C);
    const int half = C / 2;
    const int a = c < half ? c : c - half;
    const float e = (float)a / (float)(half - 1);
    const float den = powf(10000.0f, e);
    const float ph = (float)t / den;
    out[i] = c < half ? cosf(ph) : sinf(ph);
}

void pos1d_launch(float* out, int T2, int C, hipStream_t s) {
    hipLaunchKernelGGL(pos1d_kernel, dim3((unsigned)(((int64_t)T2 * C + 255) / 256)), dim3(256), 0, s, out, T2, C);
}

}  // namespace athd
