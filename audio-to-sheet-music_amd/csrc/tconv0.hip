// Time encoder level 0 conv: HEncLayer(freq=False).conv = Conv1d(2, 48, 8, stride 4, padding 2) -> GELU on the raw
// (B, 2, T) waveform, with the per-sample time normalisation (wav - meant) / (1e-5 + stdt) applied on load
// (ATHTDemucs_v2.py:272-275, 201-206; demucs HEncLayer: right zero pad to a multiple of 4 = reads past T are 0).
//
// K = 16 (8 taps x 2 channels) is far too short for an MFMA tile to pay: as an implicit GEMM this layer ran at
// ~1 TB/s on its 48-channel output.  Here one lane computes one output position: 16 normalised samples in
// registers, the 48 x 16 fp32 weights read with wave-uniform addresses (scalar loads, SGPR operands of the FMAs),
// GELU, and 48 channels stored channels-last [B][Lo][48] (bf16 in throughput mode).  HBM-bound: wav in once
// (the 8-tap windows of neighbouring lanes overlap in L1), output out once.
// Round 6: the block's 256 output rows (96 B each in bf16: not whole 128-B lines) are staged in LDS and leave as one
// contiguous 24 KB run of 16-B-per-lane stores; the per-lane row stores wrote 1.55x the output bytes to memory
// (PMC WRITE_SIZE, profiles/pmc_traffic.json: partial-line writes).
#include "common.h"
#include "kernels.h"
#include "prof.h"

#include <type_traits>

namespace athd {

template <bool BF>
__global__ __launch_bounds__(256) void tconv0_kernel(const float* __restrict__ wav, int64_t T, int64_t Lo,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     const float* __restrict__ tnorm, void* __restrict__ out) {
    typedef typename std::conditional<BF, bf16_t, float>::type OT;
    __shared__ __attribute__((aligned(16))) OT tile[256 * 48];
    const int64_t b = blockIdx.y;
    const int64_t lo0 = (int64_t)blockIdx.x * 256;
    const int64_t lo = lo0 + threadIdx.x;
    const int nrow = (int)(Lo - lo0 < 256 ? Lo - lo0 : 256);
    const float sub = tnorm[2 * b], dv = tnorm[2 * b + 1];
    const float* x0 = wav + b * 2 * T;
    const float* x1 = x0 + T;
    float x[16];                                  // k = tap * 2 + channel (the packed GEMM K order)
#pragma unroll
    for (int tap = 0; tap < 8; ++tap) {
        const int64_t p = 4 * lo - 2 + tap;
        const bool in = p >= 0 && p < T;
        x[2 * tap] = in ? (x0[p] - sub) / dv : 0.f;
        x[2 * tap + 1] = in ? (x1[p] - sub) / dv : 0.f;
    }
#pragma unroll
    for (int n0 = 0; n0 < 48; n0 += 8) {
        float y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) s = fmaf(w[(n0 + i) * 16 + k], x[k], s);
            y[i] = gelu<BF>(s + bias[n0 + i]);
        }
        if constexpr (BF) {
            *reinterpret_cast<uint4*>(&tile[threadIdx.x * 48 + n0]) =
                make_uint4(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]), pack2bf(y[4], y[5]), pack2bf(y[6], y[7]));
        } else {
            float4* o = reinterpret_cast<float4*>(&tile[threadIdx.x * 48 + n0]);
            o[0] = make_float4(y[0], y[1], y[2], y[3]);
            o[1] = make_float4(y[4], y[5], y[6], y[7]);
        }
    }
    __syncthreads();
    // the block's rows are one contiguous run of nrow * 48 elements: 16-B pieces, consecutive lanes, whole lines
    constexpr int PER = 16 / (int)sizeof(OT);          // elements per 16-B piece
    const int pieces = nrow * 48 / PER;
    const uint4* src = reinterpret_cast<const uint4*>(tile);
    uint4* dst = reinterpret_cast<uint4*>((OT*)out + (b * Lo + lo0) * 48);
    for (int i = threadIdx.x; i < pieces; i += 256) dst[i] = src[i];
}

void tconv0_launch(const float* wav, int nb, int64_t T, int64_t Lo, const float* w, const float* bias,
                   const float* tnorm, void* out, int out_bf16, hipStream_t s) {
    dim3 grid((unsigned)((Lo + 255) / 256), nb);
    KScope ks(s);
    if (ks.on())
        ks.begin(out_bf16 ? "tconv0_kernel<true>" : "tconv0_kernel<false>", 2.0 * nb * Lo * 48 * 16,
                 (double)nb * 2 * T * 4 + (double)nb * Lo * 48 * (out_bf16 ? 2 : 4));
    if (out_bf16) hipLaunchKernelGGL(tconv0_kernel<true>, grid, dim3(256), 0, s, wav, T, Lo, w, bias, tnorm, out);
    else hipLaunchKernelGGL(tconv0_kernel<false>, grid, dim3(256), 0, s, wav, T, Lo, w, bias, tnorm, out);
}

}  // namespace athd
