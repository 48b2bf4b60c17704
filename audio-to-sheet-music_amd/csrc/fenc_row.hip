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
// Work split (level 0: 6 waves, level 1: 12): wave w owns x channel tile ct = w % (C/16) (16 channels) and the
// m-tiles (16 positions) mt = w / (C/16) + (NW / (C/16)) * i.  Every contraction is v_mfma_f32_16x16x32_bf16 with the weights as the A
// operand (rows = output channels) and the activations as the B operand, so a lane holds 4 consecutive channels
// of one position:  acc[r] = out[channel 16*tile + 4*(lane>>4) + r][position 16*mt + (lane&15)].
//   conv    K = 8*Cin  (level 0: the 8 taps x 4 CaC channels of the frame-major spectrogram, normalised on load;
//                       level 1: 2 taps x 48 channels per LDS stage)
//   conv3   K = 3C, N = C/8 (padded to 16 rows), m-tiles spread over all waves
//   1x1     K = C/8 (padded to 32), N = 2C GLU-interleaved: rows 32*ct + [0,16) = 'a', + [16,32) = gate, so the
//           lane's 'a' and gate values are the two halves of one x channel tile; computed twice (statistics pass,
//           then the GroupNorm -> GLU -> LayerScale -> residual pass) instead of being kept
//   rewrite K = C, N = 2C GLU-interleaved, stored from registers (the waves of a position complete its row in L2).
// Throughput (bf16) mode only; T <= 16 * FR_MT_MAX (the forward falls back to the unfused path otherwise).
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace athd {

namespace {

// waves per workgroup of fenc_row0_kernel.  8 (round 6): 4 channel-tile slots x 2 m-groups, the
// fourth slot's waves idle in the (channel tile, m-tile) phases and share the per-m-tile phases, so every working wave
// keeps the 6-wave form's 9 units while two 8-wave workgroups fit a CU (the 6-wave shape averaged 1.73,
// profiles/r05_occupancy.txt; 6-wave workgroups at 128 VGPRs reach only 1.5 per CU in r05_residency.txt).
#ifndef ATHD_F0_NW
#define ATHD_F0_NW 8
#endif
constexpr int FR_NW = ATHD_F0_NW;
static_assert(FR_NW == 6 || FR_NW == 8, "fenc_row0 wave count");
constexpr int FR_NT = 64 * FR_NW;
constexpr int FR_HALO = 2;           // max DConv dilation

ATHD_DEV bf16x8_t ldfrag(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

ATHD_DEV f32x4_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

ATHD_DEV void st4bf(bf16_t* p, float a, float b, float c, float d) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(a, b), pack2bf(c, d));
}

// sum of (s1, s2) over the workgroup of NW waves; `red` is a fresh [2][NW] slot per call
template <int NW>
ATHD_DEV void block_sum2(float& s1, float& s2, float* red) {
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[w] = s1;
        red[NW + w] = s2;
    }
    __syncthreads();
    s1 = 0.f;
    s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        s1 += red[i];
        s2 += red[NW + i];
    }
}

ATHD_DEV void gn_from_sums(float s1, float s2, float cnt, float& mean, float& rstd) {
    mean = s1 / cnt;
    float var = s2 / cnt - mean * mean;
    var = var < 0.f ? 0.f : var;
    rstd = 1.0f / sqrtf(var + 1e-5f);
}

}  // namespace

#ifdef ATHD_FR_STAMP
// measurement build only (-DATHD_FR_STAMP, tools/fr_stamps.py): s_memtime at the phase boundaries of
// fenc_row0_kernel and fenc_row1_kernel, wave 0 of every workgroup -> g_fr_stamp[block][16]; read back with athd_fr_stamps
__device__ uint64_t g_fr_stamp[65536 * 16];
#define FR_STAMP(k) do { if (threadIdx.x == 0) g_fr_stamp[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define FR_STAMP(k) do { } while (0)
#endif

#define FR_SCHED() __builtin_amdgcn_sched_barrier(0)      // (no instruction is scheduled across it)

// ---------------------------------------------------------------------------------------------------------
// Level 0 (Cin = 4 CaC channels, C = 48) as a branch-free kernel: the contractions and arithmetic above (round 2's
// generic kernel), restructured for latency:
//   - a fixed 18-tile (288-position) row: wave w owns channel tile w % 3 and m-tiles w / 3 + 2 i (i < 9), conv3
//     m-tiles w + 6 i (i < 3); positions >= T are computed and masked with selects instead of per-tile branches
//     (the data-dependent `mt < MT` / `m < T` branches of the generic kernel cost exec-mask save/restore and
//     accumulator copies on every tile);
//   - the input gather is 3 fixed chunks per thread, all six 16-B loads in flight at once;
//   - weight fragments and per-channel parameters of the next phase are loaded before the barrier that ends the
//     current one, so their L2 latency overlaps it;
//   - workgroup sums by DPP row rotations + 4 readlanes (no LDS round trips inside the wave reduction);
//   - <= 128 VGPRs, so two 6-wave workgroups are always co-resident on a CU whatever their SIMD placement.
namespace {

constexpr int F0_NT = 18;                 // m-tiles per row
constexpr int F0_TP = 16 * F0_NT;         // positions per row (T <= 288)
constexpr int F0_C = 48, F0_H = 6;
// LDS images (bf16 elements).  xs (the residual stream x, 2 halo rows each side): 112-B rows (7 chunks of 16 B: an
// odd chunk count, so 16 consecutive rows start in 16 distinct chunk slots of the 256-B bank space and every 16-row
// fragment read - the conv3 taps shift rows by 0, +-1, +-2 - is conflict-free); xin (conv input) and hs (DConv
// hidden) share one buffer of 64-B rows, chunk XOR (row >> 1) & 3.
// Round 5: the 112-B rows replace round 4's 160-B rows (chunk XOR (row >> 2) & 1): 65.8 -> 51.7 KB of LDS per
// workgroup, 2.23 -> 1.68 ms per forward (serialised events), whole step 1861 -> 1898 segments/s (one box); the
// register target stays 4 waves per SIMD (ATHD_F0_WPE=5 reaches 96 VGPRs with 26 spilled: 1.87 ms).  The LDS size,
// not the bank pattern, made the difference (56.4 KB with 80-B hidden rows: 2.16 ms).
// (round 3's padded pitches 56 / 40 cost 1.9 extra LDS cycles per LDS instruction, SQ_LDS_BANK_CONFLICT, with the
// 40-element hidden rows; pitch 80 with the swizzle is kept as ATHD_F0_XSP=80)
#ifndef ATHD_F0_XSP
#define ATHD_F0_XSP 56
#endif
#ifndef ATHD_F0_WPE
#define ATHD_F0_WPE 4       // (waves per SIMD the register allocation targets)
#endif
#ifndef ATHD_F0_HSP
#define ATHD_F0_HSP 32
#endif
constexpr int F0_XIN_P = ATHD_F0_HSP, F0_XS_P = ATHD_F0_XSP, F0_HS_P = ATHD_F0_HSP;
ATHD_DEV int xs_off(int row, int col) {
    if constexpr (F0_XS_P == 80) return row * F0_XS_P + (((col >> 3) ^ ((row >> 2) & 1)) << 3) + (col & 7);
    else return row * F0_XS_P + col;      // (an odd number of 16-B chunks per row: 16-row fragment reads conflict-free)
}
ATHD_DEV int hs_off(int row, int col) {
    if constexpr (F0_HS_P == 32) return row * F0_HS_P + (((col >> 3) ^ ((row >> 1) & 3)) << 3) + (col & 7);
    else return row * F0_HS_P + col;      // (F0_HS_P = 40: 5 chunks per row; 56.4 KB in all: 2.16 ms, measured)
}
// (both swizzles repeat every 8 rows, so an m-tile's image is the lane's offset at row l15 (+ halo, + tap shift) plus
// mt * 16 rows: the per-tile part stays an immediate offset)

ATHD_DEV float dpp_row_sum(float v) {     // every lane: the sum over its row of 16 lanes
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1032
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2301
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));  // row_ror 4
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));  // row_ror 8
    return v;
}
ATHD_DEV float wave_sum_dpp(float v) {
    v = dpp_row_sum(v);
    return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}
// workgroup sum of (s1, s2); `red` is a fresh [2][FR_NW] slot per call.  Ends synced.
ATHD_DEV void block_sum2_dpp(float& s1, float& s2, float* red) {
    s1 = wave_sum_dpp(s1);
    s2 = wave_sum_dpp(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[w] = s1;
        red[FR_NW + w] = s2;
    }
    __syncthreads();
    if constexpr (FR_NW == 8) {
        s1 = ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
        s2 = ((red[FR_NW + 0] + red[FR_NW + 1]) + (red[FR_NW + 2] + red[FR_NW + 3])) +
             ((red[FR_NW + 4] + red[FR_NW + 5]) + (red[FR_NW + 6] + red[FR_NW + 7]));
    } else {
        s1 = ((red[0] + red[1]) + (red[2] + red[3])) + (red[4] + red[5]);
        s2 = ((red[FR_NW + 0] + red[FR_NW + 1]) + (red[FR_NW + 2] + red[FR_NW + 3])) + (red[FR_NW + 4] + red[FR_NW + 5]);
    }
}

ATHD_DEV float4 ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
// keeps the next m-tile's LDS fragment loads (and the MFMAs fed by them) below this point: without it the scheduler
// hoists all nine tiles' loads and MFMAs of a pass for ILP and the pass needs ~200 VGPRs
#define FR_PIN() asm volatile("" ::: "memory")

// the lane index made opaque per phase: per-tile LDS addresses and position masks are recomputed in each phase
// instead of being computed once and held in registers across the whole kernel (~40 VGPRs)
// a pointer the compiler cannot see through: loads from it stay in the phase that issues them (weights are
// otherwise treated as invariant and hoisted into earlier phases, where they occupy registers)
template <typename T>
ATHD_DEV const T* launder(const T* p) {
    uint64_t v = (uint64_t)p;
    asm volatile("" : "+s"(v));
    return (const T*)v;
}
ATHD_DEV int opaque_lane() {
    int l;
    asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"((int)(threadIdx.x & 63)));
    return l;
}

}  // namespace


__global__ __launch_bounds__(FR_NT, ATHD_F0_WPE) void fenc_row0_kernel(const FencRowDesc d) {
    constexpr int C = F0_C, H = F0_H, NCT = 3, MTW = 9;
    __shared__ __attribute__((aligned(16))) bf16_t xin[F0_TP * F0_XIN_P];    // conv input, then the hidden tile
    __shared__ __attribute__((aligned(16))) bf16_t xs[(F0_TP + 2 * FR_HALO) * F0_XS_P];
    bf16_t* const hs = xin;
    __shared__ float red[4][2 * FR_NW];
    __shared__ float gsh[2][52];                 // the 1x1 convs' moments (50 floats per layer)

    FR_STAMP(0);
    const int R = d.B * d.Fout;
    const int per = (R + 7) / 8;
    const int r = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (r >= R) return;
    const int b = r / d.Fout, f = r % d.Fout;
    const int T = d.T;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l15 = lane & 15, l4 = lane >> 4;
    // channel-tile slot and m-group of the wave (FR_NW = 8: slot 3 holds no channel tile - those waves skip the
    // (channel tile, m-tile) phases; ctl = the tile their addresses use, never read through)
    constexpr int NCS = FR_NW == 8 ? 4 : NCT;
    const int ct = wave % NCS, mg = wave / NCS;
    const bool cwork = ct < NCT;                 // wave-uniform
    const int ctl = cwork ? ct : NCT - 1;
    const int cb = ctl * 16 + 4 * l4;            // first of this lane's 4 x channels
    const int pa = 32 * ctl + 4 * l4;            // packed GLU column of this lane's 'a' values (gate: pa + 16)

    // ---- input gather: chunk c = tid + FR_NT i (< 4 F0_TP) -> position c / 4, taps 2 (c % 4), +1 (8 floats = 2 x 16 B)
    constexpr int NGC = (4 * F0_TP + FR_NT - 1) / FR_NT;
    float4 u[NGC][2];
#pragma unroll
    for (int i = 0; i < NGC; ++i) {
        const int c = tid + FR_NT * i, m = c >> 2, q = c & 3;
        const int fi = 4 * f - 2 + 2 * q;
        if (c < 4 * F0_TP && m < T && fi >= 0 && fi + 1 < d.Fin) {
            const float* p = (const float*)d.in + (((int64_t)b * T + m) * d.Fin + fi) * 4;
            u[i][0] = ld4f(p);
            u[i][1] = ld4f(p + 4);
        } else {
            u[i][0] = u[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    const bf16x8_t wf = ldfrag(d.wc + (int64_t)(ctl * 16 + l15) * d.wc_ld + 8 * l4);
    const float4 bc = ld4f(d.bc + cb);
    const float sub = d.a_norm[2 * b], rdv = 1.0f / d.a_norm[2 * b + 1];
    if (tid < 100) gsh[tid / 50][tid % 50] = d.gram[tid / 50][tid % 50];
    // halo rows of xs (conv3 zero padding); positions >= T are written as zeros by the conv epilogue
    if (tid < 2 * FR_HALO * F0_XS_P / 8) {
        const int hr = tid / (F0_XS_P / 8), hc = tid % (F0_XS_P / 8);
        const int row = hr < FR_HALO ? hr : F0_TP + hr;
        *reinterpret_cast<uint4*>(&xs[row * F0_XS_P + hc * 8]) = make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < NGC; ++i) {
        const int c = tid + FR_NT * i, m = c >> 2, q = c & 3;
        if (c >= 4 * F0_TP) break;
        const bool ok = m < T && 4 * f - 2 + 2 * q >= 0 && 4 * f - 2 + 2 * q + 1 < d.Fin;
        const float4 a = u[i][0], e = u[i][1];
        uint4 v = make_uint4(pack2bf((a.x - sub) * rdv, (a.y - sub) * rdv), pack2bf((a.z - sub) * rdv, (a.w - sub) * rdv),
                             pack2bf((e.x - sub) * rdv, (e.y - sub) * rdv), pack2bf((e.z - sub) * rdv, (e.w - sub) * rdv));
        if (!ok) v = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(&xin[hs_off(m, q * 8)]) = v;
    }
    __syncthreads();
    FR_STAMP(1);

    // ---- conv (8,1)/(4,1)/(2,0): one K-step of 32 + bias + GELU; residual stream xr in registers
    f32x4_t xr[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i) xr[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (cwork) {
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
        const int mt = mg + 2 * i;
        if (i % 3 == 0) FR_SCHED();
        xr[i] = mfma(wf, ldfrag(&xin[hs_off(l15, 8 * l4) + mt * 16 * F0_XIN_P]), f32x4_t{0.f, 0.f, 0.f, 0.f});
    }
    {
        const float bcv[4] = {bc.x, bc.y, bc.z, bc.w};
        const int l15 = opaque_lane() & 15;
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + 2 * i;
            const int m = mt * 16 + l15;
#pragma unroll
            for (int q = 0; q < 4; ++q) xr[i][q] = gelu_fast(xr[i][q] + bcv[q]);
            if (mt * 16 + 16 > T) {               // (wave-uniform) the tile holding position T: zero the tail
#pragma unroll
                for (int q = 0; q < 4; ++q) xr[i][q] = m < T ? xr[i][q] : 0.f;
            }
            st4bf(&xs[xs_off(FR_HALO + l15, cb) + mt * 16 * F0_XS_P], xr[i][0], xr[i][1], xr[i][2], xr[i][3]);
        }
    }
    }   // cwork
    __syncthreads();
    FR_STAMP(2);
    // the conv input is dead: zero the hidden tile's K padding columns 16..31
    for (int i = tid; i < F0_TP * 2; i += FR_NT)
        *reinterpret_cast<uint4*>(&hs[hs_off(i >> 1, 16 + 8 * (i & 1))]) = make_uint4(0u, 0u, 0u, 0u);

    // ---- DConv: x += LayerScale(GLU(GN(1x1(GELU(GN(conv3(x)))))))
#pragma unroll 1
    for (int dd = 0; dd < 2; ++dd) {
        const int dil = 1 << dd;
        const int l15 = opaque_lane() & 15;
        f32x4_t ha[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) ha[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            const int k0 = ks * 32 + 8 * l4;
            const int tap = k0 / C, c0 = k0 - tap * C;
            const bool kok = k0 < 3 * C;
            FR_SCHED();
            // (rows >= H and k >= 3C are zero in the packed matrix)
            const bf16x8_t w3f = ldfrag(d.w3[dd] + (int64_t)l15 * d.w3_ld + k0);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int mt = wave + FR_NW * i;
                if (mt >= F0_NT) break;                  // (wave-uniform; FR_NW = 8: waves 2..7 have 2 m-tiles)
                bf16x8_t xf = ldfrag(&xs[xs_off(FR_HALO + l15 + (kok ? (tap - 1) * dil : 0), kok ? c0 : 0) + mt * 16 * F0_XS_P]);
                if (!kok) xf = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                ha[i] = mfma(w3f, xf, ha[i]);
            }
        }
        float hb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) hb[q] = d.b3[dd][min(4 * l4 + q, H - 1)];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const bool ok = (wave + FR_NW * i) * 16 + l15 < T;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float v = ha[i][q] + hb[q];
                const bool use = ok && 4 * l4 + q < H;
                s1 += use ? v : 0.f;
                s2 += use ? v * v : 0.f;
            }
        }
        float g1w[4], g1b[4];             // (issued before the reduction's barrier)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            g1w[q] = d.g1w[dd][min(4 * l4 + q, H - 1)];
            g1b[q] = d.g1b[dd][min(4 * l4 + q, H - 1)];
        }
        FR_STAMP(3 + 4 * dd);
        block_sum2_dpp(s1, s2, red[2 * dd]);
        FR_STAMP(4 + 4 * dd);
        float hm, hr;
        gn_from_sums(s1, s2, (float)(H * T), hm, hr);
        // GELU(GN(h)) -> hs (bf16); then the 1x1 output's GroupNorm statistics from the moments of the 1x1 conv
        // (sum_n y = sum b + ws.x, sum_n y^2 = sum b^2 + 2 v.x + x^T G x over the bf16 x the MFMAs multiply), one
        // position per lane (l4 = 0) from its hidden row: this replaces a full 1x1 MFMA pass over the row
        const float* G = gsh[dd];
        s1 = 0.f;
        s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int mt = wave + FR_NW * i;
            if (mt >= F0_NT) break;
            FR_SCHED();
            float g[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float v = gelu_fast((ha[i][q] + hb[q] - hm) * hr * g1w[q] + g1b[q]);
                g[q] = 4 * l4 + q < H ? v : 0.f;
            }
            *reinterpret_cast<uint2*>(&hs[hs_off(l15, 4 * l4) + mt * 16 * F0_HS_P]) =
                make_uint2(pack2bf(g[0], g[1]), pack2bf(g[2], g[3]));
        }
        // (the hidden rows of this wave's positions were written by this wave: LDS order within a wave suffices)
        // lane group l4 < 3 takes the positions of m-tile wave + FR_NW l4: the wave's 48 positions in one pass
        {
            const int mt = wave + FR_NW * l4;
            if (l4 < 3 && mt * 16 + l15 < T) {
                const uint4 hq = *reinterpret_cast<const uint4*>(&hs[hs_off(l15, 0) + mt * 16 * F0_HS_P]);
                const float x[6] = {__uint_as_float(hq.x << 16), __uint_as_float(hq.x & 0xFFFF0000u),
                                    __uint_as_float(hq.y << 16), __uint_as_float(hq.y & 0xFFFF0000u),
                                    __uint_as_float(hq.z << 16), __uint_as_float(hq.z & 0xFFFF0000u)};
                float q = 0.f, lv = 0.f, lw = 0.f;
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    float t = 0.f;
#pragma unroll
                    for (int kk = 0; kk < 6; ++kk) t += G[j * 6 + kk] * x[kk];
                    q += x[j] * t;
                    lv += G[36 + j] * x[j];
                    lw += G[42 + j] * x[j];
                }
                s1 += G[48] + lw;
                s2 += G[49] + (2.f * lv + q);
            }
        }
        // the apply pass's 1x1 weights and GroupNorm affine (issued before the reduction's barrier)
        const bf16x8_t wa = ldfrag(d.w1[dd] + (int64_t)(32 * ctl + l15) * d.w1_ld + 8 * l4);
        const bf16x8_t wg = ldfrag(d.w1[dd] + (int64_t)(32 * ctl + 16 + l15) * d.w1_ld + 8 * l4);
        const float4 ba = ld4f(d.b1[dd] + pa), bg = ld4f(d.b1[dd] + pa + 16);
        const float bav[4] = {ba.x, ba.y, ba.z, ba.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
        const float4 gwa = ld4f(d.g2w[dd] + pa), gba = ld4f(d.g2b[dd] + pa);
        const float4 gwg = ld4f(d.g2w[dd] + pa + 16), gbg = ld4f(d.g2b[dd] + pa + 16);
        const float4 sc4 = ld4f(d.scale[dd] + cb);
        block_sum2_dpp(s1, s2, red[2 * dd + 1]);
        FR_STAMP(5 + 4 * dd);
        float ym, yr;
        gn_from_sums(s1, s2, (float)(2 * C * T), ym, yr);
        // (y + b - mean) * rstd * w + beta  as  y * wa + ca  (wa = rstd w, ca = (b - mean) wa + beta); the 'a' half
        // carries the LayerScale, the gate half -log2(e): x += a' / (1 + 2^g')
        const float scv[4] = {sc4.x, sc4.y, sc4.z, sc4.w};
        const float gwa4[4] = {gwa.x * yr, gwa.y * yr, gwa.z * yr, gwa.w * yr};
        const float gwg4[4] = {gwg.x * yr, gwg.y * yr, gwg.z * yr, gwg.w * yr};
        const float gba4[4] = {gba.x, gba.y, gba.z, gba.w}, gbg4[4] = {gbg.x, gbg.y, gbg.z, gbg.w};
        float gwav[4], cav[4], gwgv[4], cgv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            gwav[q] = gwa4[q] * scv[q];
            cav[q] = ((bav[q] - ym) * gwa4[q] + gba4[q]) * scv[q];
            gwgv[q] = gwg4[q] * -1.4426950408889634f;
            cgv[q] = ((bgv[q] - ym) * gwg4[q] + gbg4[q]) * -1.4426950408889634f;
        }
        // pass 2: GroupNorm -> GLU -> LayerScale -> residual
        const int l15c = opaque_lane() & 15;
        if (cwork) {
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + 2 * i;
            const int m = mt * 16 + l15c;
            FR_SCHED();
            const bf16x8_t hf = ldfrag(&hs[hs_off(l15c, 8 * l4) + mt * 16 * F0_HS_P]);
            const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const f32x4_t ya = mfma(wa, hf, z), yg = mfma(wg, hf, z);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float a = ya[q] * gwav[q] + cav[q];
                const float g = yg[q] * gwgv[q] + cgv[q];
                xr[i][q] = a * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(g)) + xr[i][q];
            }
            if (mt * 16 + 16 > T) {               // (wave-uniform) positions >= T stay 0 in xr and xs
#pragma unroll
                for (int q = 0; q < 4; ++q) xr[i][q] = m < T ? xr[i][q] : 0.f;
            }
            st4bf(&xs[xs_off(FR_HALO + l15c, cb) + mt * 16 * F0_XS_P], xr[i][0], xr[i][1], xr[i][2], xr[i][3]);
        }
        }   // cwork
        __syncthreads();
        FR_STAMP(6 + 4 * dd);
    }

    // ---- rewrite 1x1 (C -> 2C) + GLU + freq embedding
    if (cwork) {
        const float* br = launder(d.br);
        const uint16_t* wr = launder(d.wr);
        const float4 ba = ld4f(br + pa), bg = ld4f(br + pa + 16);
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f);
        if (d.row_add) ra = ld4f(launder(d.row_add) + (int64_t)f * C + cb);
        bf16x8_t wa[2], wg[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            wa[ks] = ldfrag(wr + (int64_t)(32 * ctl + l15) * d.wr_ld + ks * 32 + 8 * l4);
            wg[ks] = ldfrag(wr + (int64_t)(32 * ctl + 16 + l15) * d.wr_ld + ks * 32 + 8 * l4);
        }
        const float bav[4] = {ba.x, ba.y, ba.z, ba.w};
        const float bgv[4] = {bg.x * -1.4426950408889634f, bg.y * -1.4426950408889634f, bg.z * -1.4426950408889634f,
                              bg.w * -1.4426950408889634f};
        const float rav[4] = {ra.x, ra.y, ra.z, ra.w};
        uint2 ov[MTW];
        const int l15 = opaque_lane() & 15;
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int m = (mg + 2 * i) * 16 + l15;
            FR_PIN();
            f32x4_t za = f32x4_t{0.f, 0.f, 0.f, 0.f}, zg = za;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int k0 = ks * 32 + 8 * l4;
                bf16x8_t xf = ldfrag(&xs[xs_off(FR_HALO + l15, k0 < C ? k0 : 0) + (m - l15) * F0_XS_P]);
                if (k0 >= C) xf = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                za = mfma(wa[ks], xf, za);
                zg = mfma(wg[ks], xf, zg);
            }
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                o[q] = (za[q] + bav[q]) * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(zg[q] * -1.4426950408889634f + bgv[q])) + rav[q];
            ov[i] = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
        }
        FR_STAMP(11);
        // straight from registers (8 B per lane, 32 B per position and wave-instruction; the 3 channel-tile waves of a
        // position complete its 96-B row in L2): no LDS staging and its two barriers
        bf16_t* dst = d.out + ((int64_t)b * d.Fout + f) * (int64_t)T * C;
        uint2* d4 = d.out4 ? reinterpret_cast<uint2*>(d.out4 + ((int64_t)b * d.Fout + f) * (int64_t)T * 4) : nullptr;
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int m = (mg + 2 * i) * 16 + l15;
            if (m < T) {
                *reinterpret_cast<uint2*>(&dst[(int64_t)m * C + cb]) = ov[i];
                if (cb == 0 && d4) d4[m] = ov[i];    // the decoder's level-3 skip reads channels 0..3: a compact copy
            }
        }
        FR_STAMP(12);
    }
}

// ---------------------------------------------------------------------------------------------------------
// Level 1 (Cin = 48, C = 96, 12 waves, one workgroup per CU; round 5, replacing the generic kernel of rounds 2-4, 1.40
// -> 1.05 ms per launch): the contractions and arithmetic above with the latency taken out of the generic kernel's two
// longest phases (s_memtime phase stamps, tools/fr_stamps.py FR_LEVEL=1: the four register-staged conv stages took
// 36 % of a row, the two conv3 passes with their weights read from global memory another 17 %):
//   - conv: one stage per tap.  The [T][48] input rows of one frequency row are one contiguous slab of T x 96 B; it is
//     moved by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip) as a linear copy into a 3-deep ring of 272-row
//     images (96-B rows; rows >= T and taps outside [0, Fin) from a zero page), so taps t + 1 and t + 2 are in flight
//     while tap t's MFMAs run.  The tap's weights ([96][48], 112-B rows: conflict-free 16-row fragment reads) arrive
//     the same way one tap ahead in a 2-deep ring.  Nothing but LDS-DMA is in flight in the loop: a VGPR-returning
//     global load among the DMAs makes the compiler's wait counting give up (vmcnt(0) before the next MFMA, i.e. the
//     ring serialised).  Every wave issues exactly 4 pieces per stage (surplus pieces load the zero page into a
//     scratch KB), so the explicit counted waits are exact.  A tap's 48 channels are two 16x16x32 MFMAs (the second
//     half zero weights).
//   - conv3 weights of both DConv layers moved into the dead tap ring at the end of the conv and read from LDS.
//   - the 1x1 weights issued before the barrier that precedes their use.
namespace {
constexpr int F1_C = 96, F1_CIN = 48, F1_H = 12, F1_NW = 12, F1_NT = 64 * F1_NW;
constexpr int F1_NCT = F1_C / 16, F1_MG = F1_NW / F1_NCT, F1_MTW = (FR_MT_MAX + F1_MG - 1) / F1_MG;
constexpr int F1_TPM = 16 * FR_MT_MAX;          // 272 positions
constexpr int F1_PIECES = (F1_TPM * 96 + 1023) / 1024;   // 26 DMA pieces of 1 KB per tap image
constexpr int F1_STB = F1_PIECES * 1024;        // one tap image (bytes), 96-B rows
constexpr int F1_RING = 3;
constexpr int F1_WROW = 112;                    // tap weight rows in LDS (bytes): 96 used
constexpr int F1_WPC = (F1_C * F1_WROW + 1023) / 1024;   // 11 pieces per tap's weights
constexpr int F1_WSB = F1_WPC * 1024;
constexpr int F1_XS_P = F1_C + 8;               // residual image pitch (elements)
constexpr int F1_HS_P = 40;                     // hidden tile pitch (elements)
constexpr int F1_W3_P = 3 * F1_C + 8;           // conv3 weight rows in LDS (elements): 592 B, 16 rows on distinct banks
constexpr int F1_W3C = F1_W3_P / 8;             // 37 chunks per conv3 row (36 used)
constexpr int F1_W3PC = (2 * 16 * F1_W3C * 16 + 1023) / 1024;   // 19 pieces for both layers
constexpr int F1_K3S = 3 * F1_C / 32;           // 9 conv3 K-steps
constexpr int F1_WRC = 13;                      // rewrite weight rows in LDS: 13 chunks (208 B, 192 used; conflict-free)
constexpr int F1_WRB = 2 * F1_C * F1_WRC * 16;  // rewrite weight image (bytes)
constexpr int F1_W3B = 2 * 16 * F1_W3_P * 2;    // conv3 weight image (bytes)
constexpr int F1_LPC = F1_WRB / 1024;           // DMA pieces of the rewrite weight image
constexpr int F1_C3I = (FR_MT_MAX + F1_NW - 1) / F1_NW;
constexpr int F1_GSZ = F1_H * F1_H + 2 * F1_H + 2;
static_assert((F1_TPM - 1) * 96 + 128 <= F1_STB && F1_TPM * F1_HS_P * 2 <= F1_STB && F1_W3PC * 1024 <= F1_STB,
              "fenc_row1 LDS layout");
static_assert(F1_PIECES <= 3 * F1_NW && F1_WPC <= F1_NW && F1_W3PC <= 2 * F1_NW && F1_LPC <= 4 * F1_NW,
              "DMA pieces per wave");
// after the conv the ring is reused: slot 0 = hidden tile, slot 1 + weight ring = rewrite weights, slot 2 = conv3 weights
static_assert(F1_WRB <= F1_STB + 2 * F1_WSB && F1_W3B <= F1_STB && F1_WRB % 1024 == 0, "late images");
typedef __attribute__((address_space(3))) void f1_lds_void;
typedef __attribute__((address_space(1))) void f1_gbl_void;
__device__ __attribute__((aligned(64))) uint4 g_zero_f1[4];
}  // namespace

__global__ __launch_bounds__(F1_NT, 1) void fenc_row1_kernel(const FencRowDesc d) {
    constexpr int C = F1_C, H = F1_H, NW = F1_NW, MG = F1_MG, MTW = F1_MTW, TPM = F1_TPM;
    constexpr int XS_P = F1_XS_P, HS_P = F1_HS_P;
    // [slot 0 | slot 1 | tap weight ring (2) | slot 2]: the 3-deep tap image ring and the weight ring; after the conv
    // the hidden tile (slot 0), the rewrite weights (slot 1 + weight ring) and the conv3 weights (slot 2)
    // One LDS array with the LDS-DMA destinations first (the rings, then the scratch KB the surplus pieces go to),
    // then the residual image and the small tables
    constexpr int O_SINK = 3 * F1_STB + 2 * F1_WSB, O_XS = O_SINK + 1024;
    constexpr int O_RED = O_XS + (TPM + 2 * FR_HALO) * XS_P * 2, O_GSH = O_RED + 4 * 2 * NW * 4;
    constexpr int O_P3 = O_GSH + 2 * F1_GSZ * 4, O_END = O_P3 + 2 * 3 * 16 * 4;
    __shared__ __attribute__((aligned(1024))) char smem1[O_END];
    char* const stg = smem1;
    char* const wring = stg + 2 * F1_STB;
    char* const dma_sink = smem1 + O_SINK;
    auto slot = [&](int k) -> char* { return stg + (k == 2 ? 2 * F1_STB + 2 * F1_WSB : k * F1_STB); };
    bf16_t* const xs = reinterpret_cast<bf16_t*>(smem1 + O_XS);
    float (*const red)[2 * NW] = reinterpret_cast<float (*)[2 * NW]>(smem1 + O_RED);
    float (*const gsh)[F1_GSZ] = reinterpret_cast<float (*)[F1_GSZ]>(smem1 + O_GSH);
    float (*const p3)[3][16] = reinterpret_cast<float (*)[3][16]>(smem1 + O_P3);   // conv3 bias, GN affine (padded)
    bf16_t* const hs = reinterpret_cast<bf16_t*>(stg);
    char* const late2 = stg + 2 * F1_STB + 2 * F1_WSB;                              // slot 2
    const bf16_t* const w3s = reinterpret_cast<const bf16_t*>(late2);               // [2][16][F1_W3_P]
    const char* const wrs = stg + F1_STB;                                           // [2C][F1_WRC chunks]

    FR_STAMP(0);
    const int R = d.B * d.Fout;
    const int per = (R + 7) / 8;
    const int r = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (r >= R) return;
    const int b = r / d.Fout, f = r % d.Fout;
    const int T = d.T;
    const int MT = (T + 15) >> 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l15 = lane & 15, l4 = lane >> 4;
    const int ct = wave % F1_NCT, mg = wave / F1_NCT;
    const int cb = ct * 16 + 4 * l4;

    const char* const zero = reinterpret_cast<const char*>(g_zero_f1);
    auto dma = [&](const char* src, char* dst) {
        __builtin_amdgcn_global_load_lds((f1_gbl_void*)src, (f1_lds_void*)dst, 16, 0, 0);
    };
    // tap t's input image -> ring slot t % 3: a linear copy of the T x 96 B slab, piece p = image bytes
    // [1024 p, 1024 p + 1024), wave w: pieces w, w + 12, w + 24 (past 26: zero page -> scratch)
    auto dma_tap = [&](int t) {
        const int fi = 4 * f - 2 + t;
        const bool fok = fi >= 0 && fi < d.Fin;
        const char* slab = (const char*)d.in + ((int64_t)b * d.Fin + (fok ? fi : 0)) * (int64_t)T * (F1_CIN * 2);
        char* dst = slot(t % F1_RING);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int p = wave + NW * j;
            const int byte = 1024 * p + 16 * lane;
            dma(fok && byte < T * (F1_CIN * 2) ? slab + byte : zero, p < F1_PIECES ? dst + p * 1024 : dma_sink);
        }
    };
    // tap t's weights [96 rows][48] -> wring[t & 1], 112-B rows (16 B of zeros): wave w loads piece w (< 11)
    auto dma_wt = [&](int t) {
        const int e = 1024 * wave + 16 * lane;
        const int row = e / F1_WROW, col = e - row * F1_WROW;
        const bool ok = wave < F1_WPC && row < C && col < 96;
        dma(ok ? (const char*)d.wc + (int64_t)row * d.wc_ld * 2 + t * 96 + col : zero,
            wave < F1_WPC ? wring + (t & 1) * F1_WSB + 1024 * wave : dma_sink);
    };
    // the conv3 weights of both layers [2][16][296] -> ring slot 2 (free once tap 5 is read): 19 pieces, 2 per wave.
    // (the two base pointers laundered into SGPRs: a per-lane select between two kernel-argument fields otherwise
    // becomes a per-lane load of the field, a VGPR-returning load among the DMAs)
    const char* const w3g0 = launder((const char*)d.w3[0]);
    const char* const w3g1 = launder((const char*)d.w3[1]);
    auto dma_w3 = [&]() {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int p = wave + NW * j;
            const int e = (1024 * p + 16 * lane) >> 4;                   // chunk index in the LDS image
            const int lr = e / F1_W3C, ch = e - lr * F1_W3C;             // (layer * 16 + row), chunk
            const int dd = lr >> 4, row = lr & 15;
            const bool ok = p < F1_W3PC && dd < 2 && ch < 3 * C / 8;
            const char* w3g = dd ? w3g1 : w3g0;
            dma(ok ? w3g + ((int64_t)row * d.w3_ld + 8 * ch) * 2 : zero,
                p < F1_W3PC ? late2 + 1024 * p : dma_sink);
        }
    };
    // after the conv: the rewrite weights [2C][C] (rows of F1_WRC chunks), 4 pieces per wave
    const char* const wrg0 = launder((const char*)d.wr);
    auto dma_late = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = wave + NW * j;
            const int e = (1024 * p + 16 * lane) >> 4;                  // 16-B chunk of the image
            const int row = e / F1_WRC, ch = e - row * F1_WRC;
            const bool ok = p < F1_LPC && ch < C / 8;
            dma(ok ? wrg0 + ((int64_t)row * d.wr_ld + 8 * ch) * 2 : zero, p < F1_LPC ? (char*)wrs + 1024 * p : dma_sink);
        }
    };
    for (int i = tid; i < 2 * F1_GSZ; i += F1_NT) gsh[i / F1_GSZ][i % F1_GSZ] = d.gram[i / F1_GSZ][i % F1_GSZ];
    if (tid < 2 * 3 * 16) {      // (in LDS: a VGPR-returning load while the late DMA is in flight would wait it out)
        const int dd = tid / 48, k = (tid / 16) % 3, j = tid % 16;
        const float* src = k == 0 ? d.b3[dd] : k == 1 ? d.g1w[dd] : d.g1b[dd];
        p3[dd][k][j] = j < H ? src[j] : 0.f;
    }
    for (int i = tid; i < (TPM + 2 * FR_HALO) * XS_P / 8; i += F1_NT)
        reinterpret_cast<uint4*>(xs)[i] = make_uint4(0u, 0u, 0u, 0u);
    const float4 bc = *reinterpret_cast<const float4*>(d.bc + cb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // (only LDS-DMA in flight from here on)
    // VMEM issue order, for the counted waits below: img(0), wt(0), img(1); stage t: wt(t + 1), img(t + 2) (stage 6:
    // wt(7), the conv3 weights)
    // (the counted waits rely on this issue order: a compiler fence between the groups keeps the scheduler from
    // interleaving them - they are independent memory operations to it)
    auto order = []() { asm volatile("" ::: "memory"); };
    dma_tap(0);
    order();
    dma_wt(0);
    order();
    dma_tap(1);
    order();

    // ---------------------------------------------------------------- conv (8,1)/(4,1)/(2,0): 8 tap stages
    f32x4_t xr[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i) xr[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int wrow = (ct * 16 + l15) * F1_WROW;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        // this wave's img(t) and wt(t) landed: only the 3 pieces issued after wt(t) (img(t + 1); at t = 7 the conv3
        // weights' 2) may still be in flight
        if (t == 7) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        // every wave's pieces landed; tap t - 1's reads done.  (A raw s_barrier: __syncthreads' fences would add a
        // full vmcnt(0).)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < 8) dma_wt(t + 1);
        order();
        if (t + 2 < 8) dma_tap(t + 2);                        // into the slot tap t - 1 was read from
        if (t == 6) dma_w3();                                 // slot 2 held tap 5
        order();
        const char* img = slot(t % F1_RING);
        const char* wl = wring + (t & 1) * F1_WSB + wrow;
        // K-step 0: channels 0..31; K-step 1: channels 32..47 in lanes l4 = 0, 1 and zero weights in l4 = 2 (the row's
        // zero padding) and l4 = 3 (the next row's first chunk, zeroed here), so the B lanes l4 >= 2 - the next image
        // row's first channels - contribute nothing.  (A 16x16x16 MFMA for channels 32..47 in the same accumulation
        // chain made the results nondeterministic on gfx950: measured, not kept.)
        const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(wl + 16 * l4);
        bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(wl + 64 + 16 * l4);
        if (l4 == 3) a1 = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            // branch-free: a tile past MT reads rows clamped into the image and its accumulators are never used
            const int mt = min(mg + MG * i, FR_MT_MAX - 1);
            if (i % 3 == 0) FR_SCHED();           // (else all nine tiles' fragment reads are hoisted: spills)
            const char* rp = img + (mt * 16 + l15) * (F1_CIN * 2);
            xr[i] = mfma(a0, *reinterpret_cast<const bf16x8_t*>(rp + 16 * l4), xr[i]);
            xr[i] = mfma(a1, *reinterpret_cast<const bf16x8_t*>(rp + 64 + 16 * l4), xr[i]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // the conv3 weights landed (published by the barrier below)
    FR_STAMP(1);
    {
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
    FR_STAMP(2);
    dma_late();              // (the ring is dead; waited for before the last DConv barrier)
    // the tap ring is dead: zero the hidden tile's K padding columns 16..31 (columns 0..15 are written by every conv3)
    for (int i = tid; i < TPM * 2; i += F1_NT)
        *reinterpret_cast<uint4*>(&hs[(i >> 1) * HS_P + 16 + 8 * (i & 1)]) = make_uint4(0u, 0u, 0u, 0u);

    // ---------------------------------------------------------------- DConv: x += LayerScale(GLU(GN(1x1(GELU(GN(conv3(x)))))))
#pragma unroll 1
    for (int dd = 0; dd < 2; ++dd) {
        const int dil = 1 << dd;
        f32x4_t ha[F1_C3I];
#pragma unroll
        for (int i = 0; i < F1_C3I; ++i) ha[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < F1_K3S; ++ks) {
            const int k0 = ks * 32 + 8 * l4;
            const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(&w3s[(dd * 16 + l15) * F1_W3_P + k0]);
            const int tap = k0 / C, c0 = k0 - tap * C;
#pragma unroll
            for (int i = 0; i < F1_C3I; ++i) {
                const int mt = wave + NW * i;
                if (mt >= MT) continue;
                ha[i] = mfma(wf, ldfrag(&xs[(FR_HALO + mt * 16 + l15 + (tap - 1) * dil) * XS_P + c0]), ha[i]);
            }
        }
        float hb[4], g1w[4], g1b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            hb[q] = p3[dd][0][4 * l4 + q];
            g1w[q] = p3[dd][1][4 * l4 + q];
            g1b[q] = p3[dd][2][4 * l4 + q];
        }
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < F1_C3I; ++i) {
            const int mt = wave + NW * i;
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
        FR_STAMP(3 + 4 * dd);
        block_sum2<NW>(s1, s2, red[2 * dd]);
        FR_STAMP(4 + 4 * dd);
        float hm, hr;
        gn_from_sums(s1, s2, (float)(H * T), hm, hr);
#pragma unroll
        for (int i = 0; i < F1_C3I; ++i) {
            const int mt = wave + NW * i;
            if (mt >= MT) continue;
            float g[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                g[q] = 4 * l4 + q < H ? gelu_fast((ha[i][q] + hb[q] - hm) * hr * g1w[q] + g1b[q]) : 0.f;
            st4bf(&hs[(mt * 16 + l15) * HS_P + 4 * l4], g[0], g[1], g[2], g[3]);
        }
        // the 1x1 output's GroupNorm statistics from the 1x1 conv's moments over the hidden rows this wave wrote
        s1 = 0.f;
        s2 = 0.f;
        {
            const float* G = gsh[dd];
#pragma unroll
            for (int i = 0; i < F1_C3I; ++i) {
                const int mt = wave + NW * i;
                if (mt >= MT || mt * 16 + l15 >= T) continue;
                FR_SCHED();
                float x[16];
                const uint4* hr_ = reinterpret_cast<const uint4*>(&hs[(mt * 16 + l15) * HS_P]);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint4 hq = hr_[u];
                    const uint32_t w4[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        x[8 * u + 2 * e] = __uint_as_float(w4[e] << 16);
                        x[8 * u + 2 * e + 1] = __uint_as_float(w4[e] & 0xFFFF0000u);
                    }
                }
                float qf = 0.f, lv = 0.f, lw = 0.f;
#pragma unroll
                for (int jj = 0; jj < H / 4; ++jj) {
                    const int j = 4 * jj + l4;
                    const float xj = x[j];
                    float tq = 0.f;
#pragma unroll
                    for (int kk = 0; kk < H; ++kk) tq += G[j * H + kk] * x[kk];
                    qf += xj * tq;
                    lv += G[H * H + j] * xj;
                    lw += G[H * H + H + j] * xj;
                }
                s1 += (l4 == 0 ? G[H * H + 2 * H] : 0.f) + lw;
                s2 += (l4 == 0 ? G[H * H + 2 * H + 1] : 0.f) + (2.f * lv + qf);
            }
        }
        // the apply pass's 1x1 weights and GroupNorm affine (issued before the reduction's barrier)
        const bf16x8_t wa = ldfrag(d.w1[dd] + (int64_t)(32 * ct + l15) * d.w1_ld + 8 * l4);
        const bf16x8_t wg = ldfrag(d.w1[dd] + (int64_t)(32 * ct + 16 + l15) * d.w1_ld + 8 * l4);
        const int pa = 32 * ct + 4 * l4;
        const float4 ba4 = *reinterpret_cast<const float4*>(d.b1[dd] + pa);
        const float4 bg4 = *reinterpret_cast<const float4*>(d.b1[dd] + pa + 16);
        const float4 gwa = *reinterpret_cast<const float4*>(d.g2w[dd] + pa);
        const float4 gba = *reinterpret_cast<const float4*>(d.g2b[dd] + pa);
        const float4 gwg = *reinterpret_cast<const float4*>(d.g2w[dd] + pa + 16);
        const float4 gbg = *reinterpret_cast<const float4*>(d.g2b[dd] + pa + 16);
        const float4 sc4 = *reinterpret_cast<const float4*>(d.scale[dd] + cb);
        block_sum2<NW>(s1, s2, red[2 * dd + 1]);      // (its barrier also publishes hs)
        FR_STAMP(5 + 4 * dd);
        float ym, yr;
        gn_from_sums(s1, s2, (float)(2 * C * T), ym, yr);
        const float ba[4] = {ba4.x, ba4.y, ba4.z, ba4.w}, bg[4] = {bg4.x, bg4.y, bg4.z, bg4.w};
        const float gwav[4] = {gwa.x, gwa.y, gwa.z, gwa.w}, gbav[4] = {gba.x, gba.y, gba.z, gba.w};
        const float gwgv[4] = {gwg.x, gwg.y, gwg.z, gwg.w}, gbgv[4] = {gbg.x, gbg.y, gbg.z, gbg.w};
        const float scv[4] = {sc4.x, sc4.y, sc4.z, sc4.w};
        float wav[4], cav[4], wgv[4], cgv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float wa_ = gwav[q] * yr, wg_ = gwgv[q] * yr;
            wav[q] = wa_ * scv[q];
            cav[q] = ((ba[q] - ym) * wa_ + gbav[q]) * scv[q];
            wgv[q] = wg_ * -1.4426950408889634f;
            cgv[q] = ((bg[q] - ym) * wg_ + gbgv[q]) * -1.4426950408889634f;
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
                const float a = ya[q] * wav[q] + cav[q];
                const float g = yg[q] * wgv[q] + cgv[q];
                xr[i][q] = a * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(g)) + xr[i][q];
            }
            st4bf(&xs[(FR_HALO + m) * XS_P + cb], xr[i][0], xr[i][1], xr[i][2], xr[i][3]);
        }
        if (dd == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's rewrite-weight pieces landed ...
        __syncthreads();                                                 // ... and every wave's are published
        FR_STAMP(6 + 4 * dd);
    }

    // ---------------------------------------------------------------- rewrite 1x1 (C -> 2C) + GLU
    {
        const int l15 = opaque_lane() & 15;      // (per-tile addresses recomputed here, not held across the DConv)
        const int pa = 32 * ct + 4 * l4;
        float ba[4], bg[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ba[q] = d.br[pa + q];
            bg[q] = d.br[pa + 16 + q];
        }
        bf16x8_t wra[3], wrg[3];                 // (from the LDS image)
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            wra[ks] = *reinterpret_cast<const bf16x8_t*>(wrs + ((32 * ct + l15) * F1_WRC + 4 * ks + l4) * 16);
            wrg[ks] = *reinterpret_cast<const bf16x8_t*>(wrs + ((32 * ct + 16 + l15) * F1_WRC + 4 * ks + l4) * 16);
        }
        uint2 ov[MTW];
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            ov[i] = make_uint2(0u, 0u);
            if (mt >= MT) continue;
            f32x4_t za = f32x4_t{0.f, 0.f, 0.f, 0.f}, zg = za;
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
                const bf16x8_t xf = ldfrag(&xs[(FR_HALO + m) * XS_P + ks * 32 + 8 * l4]);
                za = mfma(wra[ks], xf, za);
                zg = mfma(wrg[ks], xf, zg);
            }
            if (m < T) {
                float o[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = (za[q] + ba[q]) * sigmoid_fast(zg[q] + bg[q]);
                ov[i] = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
            }
        }
        FR_STAMP(11);
        // straight from registers: 8 B per lane, 32 B per position and wave-instruction; the 6 channel-tile waves of a
        // position complete its 192-B row in L2 (the LDS-staged form took two more barriers: 7.8k cycles per row)
        bf16_t* dst = d.out + ((int64_t)b * d.Fout + f) * (int64_t)T * C;
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
            const int mt = mg + MG * i;
            const int m = mt * 16 + l15;
            if (mt < MT && m < T) *reinterpret_cast<uint2*>(&dst[(int64_t)m * C + cb]) = ov[i];
        }
        FR_STAMP(12);
    }
}

bool fenc_row_supported(int cin, int c, int T) {
    return ((cin == 4 && c == 48) || (cin == 48 && c == 96)) && T >= 1 && T <= 16 * FR_MT_MAX;
}

#ifdef ATHD_FR_STAMP
extern "C" int athd_fr_stamps(void* host, int blocks) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fr_stamp), (size_t)blocks * 16 * 8, 0, hipMemcpyDeviceToHost);
}
#endif

int fenc_row_launch(const FencRowDesc& d, int cin, int c, hipStream_t s) {
    // (the 1x1 convs' GroupNorm statistics come from their moments, d.gram)
    if (!fenc_row_supported(cin, c, d.T) || d.Fout * 4 != d.Fin || !d.gram[0] || !d.gram[1]) return -1;
    const int R = d.B * d.Fout;
    const dim3 grid((unsigned)(8 * ((R + 7) / 8)));
    KScope ks(s);
    if (ks.on()) {
        // flops: the level's MACs at true K; bytes: the level input once + the output once + weights
        const double T = d.T, rows = R;
        const double H = c / 8.0;
        const double macs = rows * T * (c * 8.0 * cin + 2 * (H * 3 * c + 2.0 * c * H) + 2.0 * c * c);
        const double in_b = cin == 4 ? (double)d.B * d.Fin * T * 4 * 4 : (double)d.B * d.Fin * T * cin * 2;
        ks.begin(cin == 4 ? "fenc_row0_kernel" : "fenc_row1_kernel", 2.0 * macs, in_b + rows * T * c * 2);
    }
    if (cin == 4) hipLaunchKernelGGL(fenc_row0_kernel, grid, dim3(FR_NT), 0, s, d);
    else hipLaunchKernelGGL(fenc_row1_kernel, grid, dim3(F1_NT), 0, s, d);
    return (int)hipGetLastError();
}

}  // namespace athd
