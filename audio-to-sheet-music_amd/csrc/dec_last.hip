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
        ks.begin("fdec_last_kernel", 0.0, by);
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
        ks.begin(exact ? "tdec_last_kernel" : "tdec_last_generic_kernel", 0.0, by);
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
