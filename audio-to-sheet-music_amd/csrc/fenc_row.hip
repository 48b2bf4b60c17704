// One frequency-encoder level of the narrow levels (C = 48, 96) fused into one kernel: HEncLayer(freq=True) conv
// (8,1)/(4,1)/(2,0) -> GELU -> DConv (2 residual layers) -> rewrite 1x1 -> GLU (+ freq embedding after level 0)
// (demucs HEncLayer/DConv; call site ATHTDemucs_v2.py:197-217).
//
// DConv runs on (B*Fr, C, T): every GroupNorm(1) of a freq level is a statistic over ONE (b, f) row of T positions.
// So a whole level is row-local: one workgroup per (b, f) row keeps the residual stream x (C x T, fp32) in MFMA
// accumulator registers, its bf16 image in LDS for the convolutions, and writes only the level output.  The
// unfused path makes 8 HBM passes over the C x T activations per level (conv out, 2 x [conv3, 1x1 stats, 1x1
// apply], rewrite); this makes one read of the level input and one write of its output.
//
// Work split (6 waves): wave w owns x channel tile ct = w % (C/16) (16 channels) and the m-tiles (16 positions)
// mt = w / (C/16) + (6 / (C/16)) * i.  Every contraction is v_mfma_f32_16x16x32_bf16 with the weights as the A
// operand (rows = output channels) and the activations as the B operand, so a lane holds 4 consecutive channels
// of one position:  acc[r] = out[channel 16*tile + 4*(lane>>4) + r][position 16*mt + (lane&15)].
//   conv    K = 8*Cin  (level 0: the 8 taps x 4 CaC channels of the frame-major spectrogram, normalised on load;
//                       level 1: 2 taps x 48 channels per LDS stage)
//   conv3   K = 3C, N = C/8 (padded to 16 rows), m-tiles spread over all waves
//   1x1     K = C/8 (padded to 32), N = 2C GLU-interleaved: rows 32*ct + [0,16) = 'a', + [16,32) = gate, so the
//           lane's 'a' and gate values are the two halves of one x channel tile; computed twice (statistics pass,
//           then the GroupNorm -> GLU -> LayerScale -> residual pass) instead of being kept
//   rewrite K = C, N = 2C GLU-interleaved, output staged in LDS and stored as one contiguous T x C bf16 row.
// Throughput (bf16) mode only; T <= 16 * FR_MT_MAX (the forward falls back to the unfused path otherwise).
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace athd {

namespace {

constexpr int FR_NW = 6;             // waves per workgroup
constexpr int FR_NT = 64 * FR_NW;
constexpr int FR_HALO = 2;           // max DConv dilation

ATHD_DEV bf16x8_t ldfrag(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

ATHD_DEV f32x4_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

ATHD_DEV void st4bf(bf16_t* p, float a, float b, float c, float d) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(a, b), pack2bf(c, d));
}

// sum of (s1, s2) over the workgroup; `red` is a fresh [2][FR_NW] slot per call
ATHD_DEV void block_sum2(float& s1, float& s2, float* red) {
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[w] = s1;
        red[FR_NW + w] = s2;
    }
    __syncthreads();
    s1 = 0.f;
    s2 = 0.f;
#pragma unroll
    for (int i = 0; i < FR_NW; ++i) {
        s1 += red[i];
        s2 += red[FR_NW + i];
    }
}

ATHD_DEV void gn_from_sums(float s1, float s2, float cnt, float& mean, float& rstd) {
    mean = s1 / cnt;
    float var = s2 / cnt - mean * mean;
    var = var < 0.f ? 0.f : var;
    rstd = 1.0f / sqrtf(var + 1e-5f);
}

}  // namespace

template <int CIN, int C>
__global__ __launch_bounds__(FR_NT, CIN == 4 ? 3 : 1) void fenc_row_kernel(const FencRowDesc d) {
    constexpr int NCT = C / 16;                  // x channel tiles
    constexpr int MG = FR_NW / NCT;              // m-tile groups per channel tile
    constexpr int MTW = (FR_MT_MAX + MG - 1) / MG;
    constexpr int TPM = FR_MT_MAX * 16;
    constexpr int H = C / 8;
    constexpr int KC = 8 * CIN;                  // conv K
    constexpr int KS = CIN == 4 ? 32 : 2 * CIN;  // conv K per LDS stage
    constexpr int NSTAGE = KC / KS;
    constexpr int XIN_P = KS + 8;                // LDS pitches (elements): +16 B keeps 16-row fragment reads
    constexpr int XS_P = C + 8;                  //   on distinct banks
    constexpr int HS_P = 40;
    constexpr int K3 = 3 * C, K3S = (K3 + 31) / 32;
    constexpr int KRS = (C + 31) / 32;
    // LDS: the conv input stage and the DConv hidden tile share one buffer (the conv is done before the first
    // hidden tile is written); the output row is staged in xs once the rewrite has read it.  C = 48: 52.7 KB and
    // <= 168 VGPRs (launch bound: 3 waves per SIMD), so two 6-wave workgroups share a CU.
    constexpr int XIN_E = (TPM * XIN_P > TPM * HS_P) ? TPM * XIN_P : TPM * HS_P;
    static_assert(C % 16 == 0 && FR_NW % NCT == 0 && KC % KS == 0 && KS % 32 == 0 && (CIN == 4 || CIN % 8 == 0),
                  "fenc_row shape");
    static_assert(TPM * C <= (TPM + 2 * FR_HALO) * XS_P, "output staging fits xs");
    __shared__ __attribute__((aligned(16))) bf16_t xin[XIN_E];
    __shared__ __attribute__((aligned(16))) bf16_t xs[(TPM + 2 * FR_HALO) * XS_P];
    bf16_t* const hs = xin;
    __shared__ float red[4][2 * FR_NW];

    // row r -> block: the 8 XCDs each take a contiguous run of rows, so neighbouring output rows (which share 4 of
    // their 8 input rows) run on one XCD and re-read those rows from its L2
    const int R = d.B * d.Fout;
    const int per = (R + 7) / 8;
    const int r = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (r >= R) return;
    const int b = r / d.Fout, f = r % d.Fout;
    const int T = d.T;
    const int MT = (T + 15) >> 4;
    const int TP = MT * 16;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int l15 = lane & 15, l4 = lane >> 4;
    const int ct = wave % NCT, mg = wave / NCT;
    const int cb = ct * 16 + 4 * l4;             // first of this lane's 4 x channels

    // zero xs (conv3 zero padding: halo rows and positions >= T)
    for (int i = tid; i < (TPM + 2 * FR_HALO) * XS_P / 8; i += FR_NT)
        reinterpret_cast<uint4*>(xs)[i] = make_uint4(0u, 0u, 0u, 0u);

    // ---------------------------------------------------------------- conv (8,1)/(4,1)/(2,0) + GELU
    f32x4_t xr[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i) xr[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < NSTAGE; ++s) {
        if (s > 0) __syncthreads();
        for (int c = tid; c < TP * (KS / 8); c += FR_NT) {
            const int m = c / (KS / 8), q = c - m * (KS / 8);
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (CIN == 4) {
                // level 0: k = tap * 4 + ch over the frame-major, L|R-interleaved CaC spectrogram specT[b][t][F][4];
                // chunk q = taps 2q, 2q+1 = input rows 4f-2+2q, +1 (both in or both out of [0, Fin))
                const int fi = 4 * f - 2 + 2 * q;
                if (m < T && fi >= 0 && fi + 1 < d.Fin) {
                    const float* p = (const float*)d.in + (((int64_t)b * T + m) * d.Fin + fi) * 4;
                    const float4 u0 = *reinterpret_cast<const float4*>(p);
                    const float4 u1 = *reinterpret_cast<const float4*>(p + 4);
                    const float sub = d.a_norm[2 * b], rdv = 1.0f / d.a_norm[2 * b + 1];
                    v = make_uint4(pack2bf((u0.x - sub) * rdv, (u0.y - sub) * rdv), pack2bf((u0.z - sub) * rdv, (u0.w - sub) * rdv),
                                   pack2bf((u1.x - sub) * rdv, (u1.y - sub) * rdv), pack2bf((u1.z - sub) * rdv, (u1.w - sub) * rdv));
                }
            } else {
                const int k0 = s * KS + q * 8;
                const int tap = k0 / CIN, ci = k0 - tap * CIN;
                const int fi = 4 * f - 2 + tap;
                if (m < T && fi >= 0 && fi < d.Fin)
                    v = *reinterpret_cast<const uint4*>((const bf16_t*)d.in + (((int64_t)b * d.Fin + fi) * T + m) * CIN + ci);
            }
            *reinterpret_cast<uint4*>(&xin[m * XIN_P + q * 8]) = v;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KS / 32; ++ks) {
            const bf16x8_t wf = ldfrag(d.wc + (int64_t)(ct * 16 + l15) * d.wc_ld + s * KS + ks * 32 + 8 * l4);
#pragma unroll
            for (int i = 0; i < MTW; ++i) {
                const int mt = mg + MG * i;
                if (mt < MT) xr[i] = mfma(wf, ldfrag(&xin[(mt * 16 + l15) * XIN_P + ks * 32 + 8 * l4]), xr[i]);
            }
        }
    }
    {
        const float4 bc = *reinterpret_cast<const float4*>(d.bc + cb);
        const float bcv[4] = {bc.x, bc.y, bc.z, bc.w};
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            if (mt >= MT) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) xr[i][q] = m < T ? gelu_fast(xr[i][q] + bcv[q]) : 0.f;
            st4bf(&xs[(FR_HALO + m) * XS_P + cb], xr[i][0], xr[i][1], xr[i][2], xr[i][3]);
        }
    }
    __syncthreads();
    // the conv input stage is dead: zero the hidden tile's K padding columns 16..31 (columns 0..15 are written by
    // every conv3 pass, zeros past H included)
    for (int i = tid; i < TPM * 2; i += FR_NT)
        *reinterpret_cast<uint4*>(&hs[(i >> 1) * HS_P + 16 + 8 * (i & 1)]) = make_uint4(0u, 0u, 0u, 0u);

    // ---------------------------------------------------------------- DConv: x += LayerScale(GLU(GN(1x1(GELU(GN(conv3(x)))))))
#pragma unroll 1
    for (int dd = 0; dd < 2; ++dd) {
        const int dil = 1 << dd;
        // conv3 (C -> H, 3 taps, dilation dil, zero padding) on m-tiles wave, wave + 6, wave + 12
        f32x4_t ha[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) ha[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < K3S; ++ks) {
            const int k0 = ks * 32 + 8 * l4;
            const bf16x8_t wf = ldfrag(d.w3[dd] + (int64_t)l15 * d.w3_ld + k0);   // rows >= H and k >= 3C are zero
            const int tap = k0 / C, c0 = k0 - tap * C;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int mt = wave + FR_NW * i;
                if (mt >= MT) continue;
                bf16x8_t xf = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                if (k0 < K3) xf = ldfrag(&xs[(FR_HALO + mt * 16 + l15 + (tap - 1) * dil) * XS_P + c0]);
                ha[i] = mfma(wf, xf, ha[i]);
            }
        }
        float hb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) hb[q] = (4 * l4 + q < H) ? d.b3[dd][4 * l4 + q] : 0.f;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int mt = wave + FR_NW * i;
            const int m = mt * 16 + l15;
            if (mt >= MT || m >= T) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (4 * l4 + q < H) {
                    const float v = ha[i][q] + hb[q];
                    s1 += v;
                    s2 += v * v;
                }
            }
        }
        block_sum2(s1, s2, red[2 * dd]);
        float hm, hr;
        gn_from_sums(s1, s2, (float)(H * T), hm, hr);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int mt = wave + FR_NW * i;
            if (mt >= MT) continue;
            float g[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = 4 * l4 + q;
                g[q] = j < H ? gelu_fast((ha[i][q] + hb[q] - hm) * hr * d.g1w[dd][j] + d.g1b[dd][j]) : 0.f;
            }
            st4bf(&hs[(mt * 16 + l15) * HS_P + 4 * l4], g[0], g[1], g[2], g[3]);
        }
        __syncthreads();

        // 1x1 (H -> 2C), GLU-interleaved rows: 'a' = 32 ct + l15, gate = 32 ct + 16 + l15; K = 32 (H zero-padded)
        const bf16x8_t wa = ldfrag(d.w1[dd] + (int64_t)(32 * ct + l15) * d.w1_ld + 8 * l4);
        const bf16x8_t wg = ldfrag(d.w1[dd] + (int64_t)(32 * ct + 16 + l15) * d.w1_ld + 8 * l4);
        const int pa = 32 * ct + 4 * l4;           // packed column of this lane's 'a' values; gate = pa + 16
        float ba[4], bg[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ba[q] = d.b1[dd][pa + q];
            bg[q] = d.b1[dd][pa + 16 + q];
        }
        s1 = 0.f;
        s2 = 0.f;
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            if (mt >= MT) continue;               // wave-uniform: the MFMAs run on full waves
            const bf16x8_t hf = ldfrag(&hs[(mt * 16 + l15) * HS_P + 8 * l4]);
            const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const f32x4_t ya = mfma(wa, hf, z), yg = mfma(wg, hf, z);
            if (m >= T) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float a = ya[q] + ba[q], g = yg[q] + bg[q];
                s1 += a + g;
                s2 += a * a + g * g;
            }
        }
        block_sum2(s1, s2, red[2 * dd + 1]);
        float ym, yr;
        gn_from_sums(s1, s2, (float)(2 * C * T), ym, yr);
        float gwa[4], gba[4], gwg[4], gbg[4], sc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            gwa[q] = d.g2w[dd][pa + q];
            gba[q] = d.g2b[dd][pa + q];
            gwg[q] = d.g2w[dd][pa + 16 + q];
            gbg[q] = d.g2b[dd][pa + 16 + q];
            sc[q] = d.scale[dd][cb + q];
        }
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            if (mt >= MT) continue;
            const bf16x8_t hf = ldfrag(&hs[(mt * 16 + l15) * HS_P + 8 * l4]);
            const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const f32x4_t ya = mfma(wa, hf, z), yg = mfma(wg, hf, z);
            if (m >= T) continue;                 // positions >= T stay 0 in xr and xs
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float a = (ya[q] + ba[q] - ym) * yr * gwa[q] + gba[q];
                const float g = (yg[q] + bg[q] - ym) * yr * gwg[q] + gbg[q];
                xr[i][q] = xr[i][q] + sc[q] * (a * sigmoid_fast(g));
            }
            st4bf(&xs[(FR_HALO + m) * XS_P + cb], xr[i][0], xr[i][1], xr[i][2], xr[i][3]);
        }
        __syncthreads();
    }

    // ---------------------------------------------------------------- rewrite 1x1 (C -> 2C) + GLU (+ freq embedding)
    {
        const int pa = 32 * ct + 4 * l4;
        float ba[4], bg[4], ra[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ba[q] = d.br[pa + q];
            bg[q] = d.br[pa + 16 + q];
            if (d.row_add) ra[q] = d.row_add[(int64_t)f * C + cb + q];
        }
        bf16x8_t wa[KRS], wg[KRS];
#pragma unroll
        for (int ks = 0; ks < KRS; ++ks) {
            wa[ks] = ldfrag(d.wr + (int64_t)(32 * ct + l15) * d.wr_ld + ks * 32 + 8 * l4);
            wg[ks] = ldfrag(d.wr + (int64_t)(32 * ct + 16 + l15) * d.wr_ld + ks * 32 + 8 * l4);
        }
        uint2 ov[MTW];           // the wave's output values (bf16 x 4 per m-tile), held until xs is free
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            ov[i] = make_uint2(0u, 0u);
            if (mt >= MT) continue;
            f32x4_t za = f32x4_t{0.f, 0.f, 0.f, 0.f}, zg = za;
#pragma unroll
            for (int ks = 0; ks < KRS; ++ks) {
                const int k0 = ks * 32 + 8 * l4;
                bf16x8_t xf = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                if (k0 < C) xf = ldfrag(&xs[(FR_HALO + m) * XS_P + k0]);
                za = mfma(wa[ks], xf, za);
                zg = mfma(wg[ks], xf, zg);
            }
            if (m < T) {
                float o[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = (za[q] + ba[q]) * sigmoid_fast(zg[q] + bg[q]) + ra[q];
                ov[i] = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
            }
        }
        __syncthreads();         // every wave has read xs: stage the output row [T][C] there
        bf16_t* ob = xs;
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            if (mt < MT && m < T) *reinterpret_cast<uint2*>(&ob[m * C + cb]) = ov[i];
        }
        __syncthreads();
        bf16_t* dst = d.out + ((int64_t)b * d.Fout + f) * (int64_t)T * C;
        for (int i = tid; i < T * C / 8; i += FR_NT)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(ob)[i];
    }
}

bool fenc_row_supported(int cin, int c, int T) {
    return ((cin == 4 && c == 48) || (cin == 48 && c == 96)) && T >= 1 && T <= 16 * FR_MT_MAX;
}

int fenc_row_launch(const FencRowDesc& d, int cin, int c, hipStream_t s) {
    if (!fenc_row_supported(cin, c, d.T) || d.Fout * 4 != d.Fin) return -1;
    const int R = d.B * d.Fout;
    const dim3 grid((unsigned)(8 * ((R + 7) / 8)));
    KScope ks(s);
    if (ks.on()) {
        // flops: the level's MACs at true K; bytes: the level input once + the output once + weights
        const double T = d.T, rows = R;
        const double H = c / 8.0;
        const double macs = rows * T * (c * 8.0 * cin + 2 * (H * 3 * c + 2.0 * c * H) + 2.0 * c * c);
        const double in_b = cin == 4 ? (double)d.B * d.Fin * T * 4 * 4 : (double)d.B * d.Fin * T * cin * 2;
        ks.begin(klabel("fenc_row_kernel<%d,%d>", cin, c), 2.0 * macs, in_b + rows * T * c * 2);
    }
    if (cin == 4) hipLaunchKernelGGL((fenc_row_kernel<4, 48>), grid, dim3(FR_NT), 0, s, d);
    else hipLaunchKernelGGL((fenc_row_kernel<48, 96>), grid, dim3(FR_NT), 0, s, d);
    return (int)hipGetLastError();
}

}  // namespace athd
