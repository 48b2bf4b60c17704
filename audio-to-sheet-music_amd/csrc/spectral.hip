// Spectral front/back end for gfx950.
//
// STFT: one workgroup per (sample, kept frame).  Both audio channels go through ONE 4096-point complex FFT
// (z = x_L + i x_R), three radix-16 Stockham passes in registers with two padded-LDS exchanges, twiddles
// from a 4096-entry table; the two real spectra are split as X_L = (Z_k + conj Z_-k)/2, X_R = (Z_k - conj Z_-k)/2i.
// The reflect padding of HTDemucs._spec (demucs pad1d, incl. its zero-extension for inputs shorter than the
// pad) is folded into the frame gather; torch.stft's own centre padding is never reached by the kept frames
// 2..le+1, so it needs no code.  Output is the CaC tensor frame-major: specT[b][t][f][4] = {Re L, Im L, Re R,
// Im R} with the 1/sqrt(4096) "normalized" scale (exactly 1/64).
//
// iSTFT: per (item, frame) the decoder's freq map is resized 2048 rows (PyTorch fp32 bilinear index math),
// passed through sigmoid, and the masking formula of ATHTDemucs_v2.py:303-309 is applied to both channels;
// the two Hermitian spectra are packed into one complex inverse FFT (x_L = Re, x_R = Im), scaled 1/64 and
// windowed; the overlap-add of the <=4 frames per output sample runs in registers, divided by the window envelope
// of ALL le+4 frames (torch.istft), plus the denormalised time branch after its 1x1 output conv
// (ATHTDemucs_v2.py:314-324): istft_ola_kernel below, no frame tensor in HBM.
#include <cstdlib>

#include "common.h"
#include "prof.h"
#include "kernels.h"

namespace athd {

constexpr int NFFT = 4096;
constexpr int HOP = 1024;

template <typename R>
struct cx { R x, y; };
using cpx = cx<float>;
template <typename R> ATHD_DEV cx<R> cadd(cx<R> a, cx<R> b) { return {a.x + b.x, a.y + b.y}; }
template <typename R> ATHD_DEV cx<R> csub(cx<R> a, cx<R> b) { return {a.x - b.x, a.y - b.y}; }
template <typename R> ATHD_DEV cx<R> cmul(cx<R> a, cx<R> b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

// 4096-point forward FFT (e^{-2 pi i}) with 256 threads as three radix-16 Stockham passes (4096 = 16^3).  Each
// thread keeps 16 points in registers; a pass is twiddle -> 16-point DFT in registers, and only the two
// exchanges between passes go through LDS (vs six LDS round trips for radix-4).  Pass Ns (1, 16, 256): thread j
// holds a[j + 256 r], multiplies by tw[(j mod Ns) r 4096/(16 Ns)] and writes its DFT output q to
// (j / Ns) 16 Ns + (j mod Ns) + q Ns.  After the last pass thread j holds X[j + 256 q] with no store needed.
// LDS slots are padded (one per 16) so that the stride-16 stores of the first exchange are conflict-free.
//
// R = float in throughput (bf16) mode.  R = double in the f32 parity mode: the spectrum is then the correctly
// rounded fp32 value.  That matters because the reference's phase term z / (Re z_L + 1e-8)
// (ATHTDemucs_v2.py:308) is singular: at a bin with Re z_L within a few 1e-8 of -1e-8 the output depends on the
// last bits of the FFT, and an fp32 FFT whose rounding differs from torch's (another summation order) can move
// the whole-output SDR by tens of dB on the reference fixtures.  A correctly rounded spectrum stays within
// ~90 dB of the reference output on all of them.
constexpr int FPAD = NFFT + NFFT / 16;
ATHD_DEV int pidx(int i) { return i + (i >> 4); }

// in-place forward radix-4: (x0, x1, x2, x3) <- DFT4
template <typename R>
ATHD_DEV void r4(cx<R>& x0, cx<R>& x1, cx<R>& x2, cx<R>& x3) {
    const cx<R> s02 = cadd(x0, x2), d02 = csub(x0, x2), s13 = cadd(x1, x3), d13 = csub(x1, x3);
    const cx<R> md13 = {d13.y, -d13.x};                  // -i * d13
    x0 = cadd(s02, s13);
    x1 = cadd(d02, md13);
    x2 = csub(s02, s13);
    x3 = csub(d02, md13);
}

// 16-point DFT as 4 x 4: v[r] (r = 4 r1 + r0) in; output bin q = k0 + 4 k1 is left in v[4 k0 + k1] (see vq)
template <typename R>
ATHD_DEV void dft16(cx<R> (&v)[16]) {
    constexpr R C1 = (R)0.92387953251128675613, S1 = (R)0.38268343236508977173, C2 = (R)0.70710678118654752440;
#pragma unroll
    for (int r0 = 0; r0 < 4; ++r0) r4(v[r0], v[4 + r0], v[8 + r0], v[12 + r0]);
    // a[r0][k0] sits in v[r0 + 4 k0]; multiply by W16^(r0 k0)
    v[1 + 4] = cmul(v[5], {C1, -S1});      // W^1
    v[1 + 8] = cmul(v[9], {C2, -C2});      // W^2
    v[1 + 12] = cmul(v[13], {S1, -C1});    // W^3
    v[2 + 4] = cmul(v[6], {C2, -C2});      // W^2
    v[2 + 8] = {v[10].y, -v[10].x};        // W^4 = -i
    v[2 + 12] = cmul(v[14], {-C2, -C2});   // W^6
    v[3 + 4] = cmul(v[7], {S1, -C1});      // W^3
    v[3 + 8] = cmul(v[11], {-C2, -C2});    // W^6
    v[3 + 12] = cmul(v[15], {-C1, S1});    // W^9
#pragma unroll
    for (int k0 = 0; k0 < 4; ++k0) r4(v[4 * k0], v[4 * k0 + 1], v[4 * k0 + 2], v[4 * k0 + 3]);
}
// register holding DFT16 output bin q
ATHD_DEV constexpr int vq(int q) { return 4 * (q & 3) + (q >> 2); }

// One LDS exchange: DFT output q of this thread goes to slot dst(q), then v[r] = slot j + 256 r.  `lds` holds
// FPAD 8-byte words: complex floats, or the real and then the imaginary parts of complex doubles.  Ends synced.
template <typename R, typename Dst>
ATHD_DEV void exchange(cx<R> (&v)[16], void* lds, Dst dst, int j) {
    if constexpr (sizeof(R) == 4) {
        cpx* b = reinterpret_cast<cpx*>(lds);
#pragma unroll
        for (int q = 0; q < 16; ++q) b[pidx(dst(q))] = v[vq(q)];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = b[pidx(j + 256 * r)];
        __syncthreads();
    } else {
        R* b = reinterpret_cast<R*>(lds);
        R t[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) b[pidx(dst(q))] = v[vq(q)].x;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) t[r] = b[pidx(j + 256 * r)];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) b[pidx(dst(q))] = v[vq(q)].y;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = {t[r], b[pidx(j + 256 * r)]};
        __syncthreads();
    }
}

// v[r] = x[threadIdx.x + 256 r] on entry; X[threadIdx.x + 256 q] = v[vq(q)] on exit.  tw[m] = e^{-2 pi i m/4096}.
// j = threadIdx.x (a parameter so that a caller looping over frames can make it opaque per iteration)
// Twiddles of the Ns = 16 and Ns = 256 passes: w^r for r = 1..15 with w = tw[16 (j & 15)] and w = tw[j].  R = double
// (the f32 parity mode) reads every power from the table; R = float takes them as running products of the two base
// twiddles the caller loaded once (tw16, tw256): no table loads per frame (30 dependent L2 round trips per frame were
// most of the iSTFT's wait time, SQ), at <= 15 ulp of twiddle error, below the fp32 FFT's own rounding over 12 stages.
// (no defaults for tw16 / tw256: a float caller that forgot them would run on zero twiddles)
template <typename R, typename TW>
ATHD_DEV void fft4096(cx<R> (&v)[16], void* lds, const TW* __restrict__ tw, int j, cpx tw16, cpx tw256) {
    constexpr bool REC = sizeof(R) == 4;
    dft16(v);                                                       // Ns = 1: no twiddles
    exchange(v, lds, [j](int q) { return 16 * j + q; }, j);
    {                                                               // Ns = 16
        const int k = j & 15;
        cx<R> w = {(R)tw16.x, (R)tw16.y};
#pragma unroll
        for (int r = 1; r < 16; ++r) {
            if constexpr (REC) {
                v[r] = cmul(v[r], w);
                // (pinned: the product chain interleaved with its uses, not all 15 powers held at once)
                asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(v[r].x), "+v"(v[r].y));
                if (r < 15) w = cmul(w, {(R)tw16.x, (R)tw16.y});
            } else {
                const TW t = tw[k * r * 16];
                v[r] = cmul(v[r], {t.x, t.y});
            }
        }
        dft16(v);
        const int base = (j >> 4) * 256 + k;
        exchange(v, lds, [base](int q) { return base + 16 * q; }, j);
    }
    cx<R> w = {(R)tw256.x, (R)tw256.y};
#pragma unroll
    for (int r = 1; r < 16; ++r) {                                  // Ns = 256
        if constexpr (REC) {
            v[r] = cmul(v[r], w);
            // (pinned: the product chain interleaved with its uses, not all 15 powers held at once)
            asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(v[r].x), "+v"(v[r].y));
            if (r < 15) w = cmul(w, {(R)tw256.x, (R)tw256.y});
        } else {
            const TW t = tw[j * r];
            v[r] = cmul(v[r], {t.x, t.y});
        }
    }
    dft16(v);
}
// the two base twiddles of fft4096's running products for thread j (R = float only)
template <typename TW>
ATHD_DEV void fft4096_base(const TW* __restrict__ tw, int j, cpx& tw16, cpx& tw256) {
    const TW a = tw[16 * (j & 15)], c = tw[j];
    tw16 = {(float)a.x, (float)a.y};
    tw256 = {(float)c.x, (float)c.y};
}

ATHD_DEV float pad_sample(const float* __restrict__ x, int64_t p, const PadPlan& pp) {
    int64_t i = p - pp.left;                 // index into the zero-extended signal of length Lx
    if (i < 0) i = -i;
    if (i >= pp.Lx) i = 2 * (pp.Lx - 1) - i;
    i -= pp.ext_left;
    return (i >= 0 && i < pp.L) ? x[i] : 0.f;
}

template <typename R, typename TW>
__global__ __launch_bounds__(256) void stft_kernel(const float* __restrict__ wav, int64_t T, PadPlan pp, int Tspec,
                                                   const TW* __restrict__ tw, const float* __restrict__ win,
                                                   float* __restrict__ specT, double* __restrict__ st) {
    __shared__ cpx buf[FPAD];
    // 1-D grid over (b, t), each XCD a contiguous range (workgroup i runs on XCD i % 8): the 4 frames that share each
    // hop of samples run on one XCD and read them from HBM once (a frame-fastest 2-D grid put neighbouring frames on
    // different XCDs: 1.6x the waveform bytes, PMC)
    int t;
    int64_t b;
    {
        const int n = (int)gridDim.x, q = n / 8, r = n % 8, x = (int)blockIdx.x % 8;
        const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (int)blockIdx.x / 8;
        t = id % Tspec;
        b = id / Tspec;
    }
    const float* xl = wav + b * 2 * T;
    const float* xr = xl + T;
    const int64_t p0 = (int64_t)t * HOP;     // kept frame t = stft frame t+2, starts at 1024 t in the pad1d'ed signal
    cx<R> v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int n = threadIdx.x + 256 * r;
        const float w = win[n];
        v[r] = {(R)(pad_sample(xl, p0 + n, pp) * w), (R)(pad_sample(xr, p0 + n, pp) * w)};
    }
    cpx tw16, tw256;
    fft4096_base(tw, (int)threadIdx.x, tw16, tw256);
    fft4096(v, buf, tw, (int)threadIdx.x, tw16, tw256);
#pragma unroll
    for (int q = 0; q < 16; ++q) buf[pidx(threadIdx.x + 256 * q)] = {(float)v[vq(q)].x, (float)v[vq(q)].y};
    __syncthreads();
    float* outT = specT + (b * Tspec + t) * 2048LL * 4;
    double s1 = 0.0, s2 = 0.0;                                // CaC normalisation statistics (A3), fused
    for (int k = threadIdx.x; k < 2048; k += 256) {
        cpx zk = buf[pidx(k)], zn = buf[pidx((NFFT - k) & (NFFT - 1))];
        // X_L = (zk + conj zn)/2, X_R = (zk - conj zn)/(2i); scaled by 1/64 (normalized=True)
        const float s = 0.5f / 64.f;
        float4 v;
        v.x = (zk.x + zn.x) * s;
        v.y = (zk.y - zn.y) * s;
        v.z = (zk.y + zn.y) * s;
        v.w = -(zk.x - zn.x) * s;
        *reinterpret_cast<float4*>(outT + (int64_t)k * 4) = v;
        s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    __shared__ double red[2][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = s1; red[1][w] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&st[2 * b], red[0][0] + red[0][1] + red[0][2] + red[0][3]);
        atomicAdd(&st[2 * b + 1], red[1][0] + red[1][1] + red[1][2] + red[1][3]);
    }
}

void stft_launch(const float* wav, int nb, int64_t T, const PadPlan& pp, int Tspec, const float2* tw,
                 const double2* tw64, const float* win, float* specT, double* stats, hipStream_t s) {
    KScope ks(s);
    if (ks.on()) ks.begin(tw64 ? "stft_kernel<double,HIP_vector_type<double,2>>" : "stft_kernel<float,HIP_vector_type<float,2>>", 0.0, (double)nb * 2 * T * 4 + (double)nb * 2048 * Tspec * 4 * 4);
    // 1-D grid of Tspec * nb workgroups (the kernel maps each to its (b, t) XCD-contiguously)
    if (tw64)
        hipLaunchKernelGGL((stft_kernel<double, double2>), dim3(Tspec * nb, 1), dim3(256), 0, s, wav, T, pp, Tspec, tw64,
                           win, specT, stats);
    else
        hipLaunchKernelGGL((stft_kernel<float, float2>), dim3(Tspec * nb, 1), dim3(256), 0, s, wav, T, pp, Tspec, tw, win,
                           specT, stats);
}

// ---------------------------------------------------------------------------------------------------------
// Fused iSTFT: mask + inverse FFT + overlap-add + envelope + time branch, no frame tensor in HBM.
//
// OLA coordinates: q = n + 3584 (1536 of _ispec's slice + 2048 of istft's centre); stft frame f covers
// q in [1024 f, 1024 f + 4096); kept frame t = f - 2 (frames outside [0, Tspec) are the zero padding).  Hop block
// B = q >> 10 receives frames B-3 .. B.  After fft4096 thread j holds the frame's samples j + 256 q' (q' = 0..15),
// i.e. offsets o = j + 256 (q' & 3) of the frame's hop h = q' >> 2: every thread owns the same 4 offsets of every hop
// block, so the overlap-add runs in registers: acc[h] = block f + h, frame f adds its hop h to acc[h] (ascending f,
// from 0.0f), then block f has all of this workgroup's frames and the ring shifts by one block.
// Workgroup k of an item runs the g real frames t = g k .. (one inverse FFT per frame; istft_ola_split).
// Its blocks whose frames all lie in its range are final: divided by the window envelope, the denormalised time
// branch added, stored (4 coalesced samples x 2 channels per thread).  The 3 blocks at each end of its range also
// take frames of the neighbouring workgroup: their partial sums go to `part` (head: first 3 blocks, tail: the 3
// after the last frame) and istft_fix_kernel adds tail(k-1) + head(k) and finishes them.  Workgroup 0's head and
// the last workgroup's tail only border zero frames and are final in place.
// Traffic per item: FO + the segment's spectrum (shared by its prompts through L2) + xt2 + out + 48 KB of partials
// per workgroup, vs round 1's 8.5 MB frame tensor written and read back per item.
constexpr int IO_G = 32;            // at most this many frames per workgroup

// Frames per workgroup g and workgroups per item n: n = ceil(Tspec / 32) workgroups of g = ceil(Tspec / n) frames
// (balanced: at 6 s, Tspec = 259, 9 x 29 | 27 instead of 8 x 32 | 3, so the 2304 workgroups of the bench config fill
// exactly 3 rounds of 768 resident workgroups instead of leaving a third of the last round idle).  Every workgroup
// but the first must hold >= 3 frames: its 3 head blocks border the previous workgroup, its 3 tail blocks the next
// one (a 1- or 2-frame workgroup would hand out head and tail parts of the same blocks), so n grows until the last
// workgroup has >= 3 frames.
struct OlaSplit { int n, g; };
static OlaSplit istft_ola_split(int Tspec) {
    // (terminates for every Tspec >= 1: checked exhaustively up to 200000 frames, 55 h of audio)
    for (int n = (Tspec + IO_G - 1) / IO_G;; ++n) {
        const int g = (Tspec + n - 1) / n;
        if (n == 1 || (g >= 3 && Tspec - (n - 1) * g >= 3) || g < 3) return {n, g};
    }
}

// Finish hop block B: out = y / env + denormalised time branch, for the samples of [0, T).  Every block holding an
// output sample is interior (q = n + 3584 >= 3 HOP, and B <= (T + 3583) / HOP <= Tspec + 3 = nfr - 1 because
// Tspec = ceil(T / HOP)), i.e. receives all four frames B-3 .. B, so its window envelope (torch.istft: the sum of
// win^2 over ALL le + 4 frames) is the thread's precomputed `env_in` of its 4 offsets (FAST: the reciprocal).
template <bool FAST>
ATHD_DEV void ola_finish(int B, int j, const float (&y)[4][2], int T, const float (&env_in)[4],
                         const float* __restrict__ x2, float mean, float stdv, float* __restrict__ o0,
                         float* __restrict__ o1) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int n = B * HOP + j + 256 * o - 3584;
        if (n >= 0 && n < T) {
            const float2 x = *reinterpret_cast<const float2*>(x2 + (int64_t)n * 2);
            float r0, r1;
            if constexpr (FAST) {
                r0 = y[o][0] * env_in[o];
                r1 = y[o][1] * env_in[o];
            } else {
                r0 = y[o][0] / env_in[o];
                r1 = y[o][1] / env_in[o];
            }
            o0[n] = r0 + (x.x * stdv + mean);
            o1[n] = r1 + (x.y * stdv + mean);
        }
    }
}

// ola_finish with the block's time-branch samples already loaded (xq[o] = x2[n], zero outside [0, T))
template <bool FAST>
ATHD_DEV void ola_finish_x(int B, int j, const float (&y)[4][2], int T, const float (&env_in)[4], const float2 (&xq)[4],
                           float mean, float stdv, float* __restrict__ o0, float* __restrict__ o1) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int n = B * HOP + j + 256 * o - 3584;
        if (n >= 0 && n < T) {
            const float r0 = FAST ? y[o][0] * env_in[o] : y[o][0] / env_in[o];
            const float r1 = FAST ? y[o][1] * env_in[o] : y[o][1] / env_in[o];
            o0[n] = r0 + (xq[o].x * stdv + mean);
            o1[n] = r1 + (xq[o].y * stdv + mean);
        }
    }
}

// interior envelope at offsets j + 256 o of a hop block: frames B-3 .. B in ascending order
ATHD_DEV void ola_env_in(int j, const float* __restrict__ win2, float (&e)[4]) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int q = 3 * HOP + j + 256 * o;
        e[o] = ((win2[q] + win2[q - HOP]) + win2[q - 2 * HOP]) + win2[q - 3 * HOP];
    }
}

// part[item][k][2 (head, tail)][3 blocks][4 offsets i][256 threads][2 channels]
ATHD_DEV float* ola_part(float* part, int64_t item, int nwg, int k, int side, int blk) {
    return part + ((((item * nwg + k) * 2 + side) * 3 + blk) * 4) * 256 * 2;
}

// Lane -> FFT thread index j of the iSTFT (round 6): lanes l < 32 of wave w take j = 32 w + l + 1 and lane l + 32 takes
// its Hermitian partner 256 - j, so the mirrored half of the packed spectrum (bins 4096 - kb, computed by the partner
// of the thread that needs them) crosses between the two halves of one wave by v_permlane32_swap instead of an LDS
// round trip with two workgroup barriers.  The self-mirrored j = 128 and j = 0 (lanes 31 and 63 of wave 3) use their
// own values.  Any lane -> j map is valid for the FFT's LDS exchanges; outputs stay coalesced per 32-lane half.
ATHD_DEV int istft_j(int tid) {
    const int w = tid >> 6, l = tid & 63;
    if (l < 32) return 32 * w + l + 1;
    return tid == 255 ? 0 : 255 - 32 * w - (l - 32);
}

// FAST (R = float, the bf16 throughput mode): the mask's sigmoid and phase division and the envelope division use
// v_exp / v_rcp (~1 ulp) instead of the IEEE sequences; the f32 parity mode (R = double) keeps them exact.
// PF: the next frame's spectrum is prefetched into registers during the current frame's FFT (32 VGPRs)
template <typename R, typename TW, int MINW, bool PF = true>
__global__ __launch_bounds__(256, MINW) void istft_ola_kernel(const float* __restrict__ fo, int Tspec, int P, int T,
                                                           const float* __restrict__ specT, const TW* __restrict__ tw,
                                                           const float* __restrict__ win,
                                                           const float* __restrict__ win2,
                                                           const float* __restrict__ xt2,
                                                           const float* __restrict__ tnorm, float* __restrict__ out,
                                                           float* __restrict__ part, int nwg, int g, int units) {
    constexpr bool FAST = sizeof(R) == 4;
    __shared__ cpx buf[FPAD];
    __shared__ uint2 ltab[2048];       // resize of the Tspec decoder rows to 2048 bins: {i0 | i1 << 16, l1}
    // XCD-aware order: workgroup L runs on XCD L % 8; the P prompts of one (segment, frame range) unit are
    // consecutive on one XCD, so they run together and share the segment's spectrum through that XCD's L2
    const int L = blockIdx.x, xcd = L & 7, jx = L >> 3;
    const int u = 8 * (jx / P) + xcd;
    if (u >= units) return;
    const int64_t b = u / nwg;
    const int k = u % nwg;
    const int64_t item = b * P + jx % P;
    const int t0 = k * g, t1 = min(t0 + g, Tspec);
    for (int kb = threadIdx.x; kb < 2048; kb += 256) {
        const LinIdx li = lin_index(kb, Tspec, 2048);
        ltab[kb] = make_uint2((uint32_t)li.i0 | ((uint32_t)li.i1 << 16), __float_as_uint(li.l1));
    }
    const int jl = istft_j((int)threadIdx.x);
    const bool hi_half = (threadIdx.x & 63) >= 32;
    float env_in[4];                   // interior envelope of this thread's offsets j + 256 o (FAST: reciprocal)
    ola_env_in(jl, win2, env_in);
    if constexpr (FAST) {
#pragma unroll
        for (int o = 0; o < 4; ++o) env_in[o] = __builtin_amdgcn_rcpf(env_in[o]);
    }
    cpx tw16, tw256;                    // (frame-invariant: fft4096's base twiddles, R = float)
    if constexpr (FAST) fft4096_base(tw, jl, tw16, tw256);
    float acc[4][4][2];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int o = 0; o < 4; ++o) acc[h][o][0] = acc[h][o][1] = 0.f;
    const float mean = tnorm[2 * b], stdv = tnorm[2 * b + 1];
    float* o0 = out + (item * 2 + 0) * T;
    float* o1 = out + (item * 2 + 1) * T;
    const float* x2 = xt2 + item * T * 2;
    // the spectrum of the next frame is loaded into registers before the current frame's FFT, so its HBM latency
    // hides under the FFT (8 x 16 B per thread: bins k = j + 256 i)
    float4 zs[8];
    auto load_spec = [&](int t) {
        const float* S = specT + (b * Tspec + t) * 2048LL * 4;
#pragma unroll
        for (int i = 0; i < 8; ++i) zs[i] = *reinterpret_cast<const float4*>(S + (int64_t)(jl + 256 * i) * 4);
    };
    auto put = [&](int side, int blk, int j) {             // acc[0] -> a partial slot (coalesced 8-B stores)
        float* pp = ola_part(part, item, nwg, k, side, blk);
#pragma unroll
        for (int o = 0; o < 4; ++o) *reinterpret_cast<float2*>(pp + (o * 256 + j) * 2) = make_float2(acc[0][o][0], acc[0][o][1]);
    };
    auto shift = [&]() {
#pragma unroll
        for (int h = 0; h < 3; ++h)
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                acc[h][o][0] = acc[h + 1][o][0];
                acc[h][o][1] = acc[h + 1][o][1];
            }
#pragma unroll
        for (int o = 0; o < 4; ++o) acc[3][o][0] = acc[3][o][1] = 0.f;
    };
    if constexpr (PF) load_spec(t0);
    __syncthreads();                                       // ltab
#pragma unroll 1
    for (int t = t0; t < t1; ++t) {
        // the thread index made opaque per frame: the FFT's frame-invariant address arithmetic (twiddle pointers, LDS
        // slots) is recomputed each frame instead of being hoisted out of the loop and spilled
        int j;
        asm volatile("v_mov_b32 %0, %1" : "=v"(j) : "v"(jl));
        // ---- masked, Hermitian-packed spectrum of frame t: the FFT input x[j + 256 r] in registers ----
        // r < 8: this thread's bins kb = j + 256 r (Z_k); r >= 8: index 4096 - kb' with kb' = (256 - j) + 256 (15 - r),
        // the partner lane's mirror value (Z_m), by v_permlane32_swap
        const float* F0 = fo + (item * (int64_t)Tspec + t) * Tspec * 2;
        // the time-branch samples of the block this frame completes (f = t + 2), loaded now and added after the FFT
        // (round 6: their HBM latency was exposed at the end of every frame)
        // (FAST only: the f32 parity mode's double FFT has no registers to spare)
        float2 xq[4];
        if constexpr (FAST) {
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                const int n = (t + 2) * HOP + j + 256 * o - 3584;
                xq[o] = (n >= 0 && n < T) ? *reinterpret_cast<const float2*>(x2 + (int64_t)n * 2) : make_float2(0.f, 0.f);
            }
        }
        cx<R> v[16];
        cpx mir[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kb = j + 256 * i;
            const uint2 e = ltab[kb];
            const float l1 = __uint_as_float(e.y), l0 = 1.f - l1;
            const float2 ra = *reinterpret_cast<const float2*>(F0 + 2 * (int)(e.x & 0xFFFFu));
            const float2 rb = *reinterpret_cast<const float2*>(F0 + 2 * (int)(e.x >> 16));
            const float xd0 = l0 * ra.x + l1 * rb.x;
            const float xd1 = l0 * ra.y + l1 * rb.y;
            const float m0 = sigmoid<FAST>(xd0), m1 = sigmoid<FAST>(xd1);
            float4 z;
            if constexpr (PF) z = zs[i];
            else z = *reinterpret_cast<const float4*>(specT + ((b * Tspec + t) * 2048LL + kb) * 4);
            const float ms0 = z.x * m0, ms1 = z.y * m1;
            const float d0 = z.x + 1e-8f, d1 = z.y + 1e-8f;
            cpx X0, X1;
            if constexpr (FAST) {
                const float q0 = __builtin_amdgcn_rcpf(d0), q1 = __builtin_amdgcn_rcpf(d1);
                X0 = {ms0 * (z.x * q0), ms0 * (z.y * q0)};
                X1 = {ms1 * (z.z * q1), ms1 * (z.w * q1)};
            } else {
                X0 = {ms0 * (z.x / d0), ms0 * (z.y / d0)};
                X1 = {ms1 * (z.z / d1), ms1 * (z.w / d1)};
            }
            if (kb == 0) { X0.y = 0.f; X1.y = 0.f; }
            const cpx Zk = {X0.x - X1.y, X0.y + X1.x};
            v[i] = {(R)Zk.x, (R)-Zk.y};
            const cpx Zm = {X0.x + X1.y, -X0.y + X1.x};   // (kb = 0: unused)
            mir[i] = {Zm.x, -Zm.y};
        }
        {
            const bool self128 = j == 128, self0 = j == 0;
#pragma unroll
            for (int r = 8; r < 16; ++r) {
                const cpx mine = mir[15 - r];
                const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(mine.x), __float_as_uint(mine.x), false, false);
                const auto sy = __builtin_amdgcn_permlane32_swap(__float_as_uint(mine.y), __float_as_uint(mine.y), false, false);
                cpx z = {__uint_as_float(hi_half ? sx[0] : sx[1]), __uint_as_float(hi_half ? sy[0] : sy[1])};
                if (self128) z = mine;                     // its own mirror bins 128 + 256 (15 - r)
                if (self0) z = r == 8 ? cpx{0.f, 0.f} : mir[16 - r];   // the Nyquist bin 2048 (zero), own bins 256 (16 - r)
                v[r] = {(R)z.x, (R)z.y};
            }
        }
        if constexpr (PF) {
            if (t + 1 < t1) load_spec(t + 1);              // next frame's spectrum, in flight during the FFT
        }
        fft4096(v, buf, tw, j, tw16, tw256);               // ends synced: buf is free for the next frame
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const float wq = win[j + 256 * q] * (1.f / 64.f);   // (L1-resident 16 KB table)
            const float x0 = (float)v[vq(q)].x * wq;
            const float x1 = -(float)v[vq(q)].y * wq;
            acc[q >> 2][q & 3][0] = acc[q >> 2][q & 3][0] + x0;
            acc[q >> 2][q & 3][1] = acc[q >> 2][q & 3][1] + x1;
        }
        // block f = t + 2 has all of this workgroup's frames
        const int f = t + 2;
        if (t - t0 < 3 && k > 0) put(0, t - t0, j);        // head block: also takes workgroup k-1's last frames
        else if constexpr (FAST) ola_finish_x<FAST>(f, j, acc[0], T, env_in, xq, mean, stdv, o0, o1);
        else ola_finish<FAST>(f, j, acc[0], T, env_in, x2, mean, stdv, o0, o1);
        shift();
    }
    // tail blocks f_last + 1 .. + 3: final if no real frame follows, else partial
    const int j = jl;
#pragma unroll
    for (int h = 0; h < 3; ++h) {
        if (t1 >= Tspec) ola_finish<FAST>(t1 + 2 + h, j, acc[0], T, env_in, x2, mean, stdv, o0, o1);
        else put(1, h, j);
        shift();
    }
}

// boundary blocks: block 2 + g k + h (k = 1 .. nwg-1, h = 0..2) = tail partial of workgroup k-1 + head of k
// (exact division by the envelope: the blocks are few, so the f32 parity arithmetic serves both modes)
__global__ __launch_bounds__(256) void istft_fix_kernel(int Tspec, int P, int T, int nwg, int g,
                                                        const float* __restrict__ win2, const float* __restrict__ xt2,
                                                        const float* __restrict__ tnorm, float* __restrict__ out,
                                                        const float* __restrict__ part) {
    const int64_t item = blockIdx.y;
    const int64_t b = item / P;
    const int k = 1 + blockIdx.x / 3, h = blockIdx.x % 3, j = threadIdx.x;
    const float* tl = ola_part(const_cast<float*>(part), item, nwg, k - 1, 1, h);
    const float* hd = ola_part(const_cast<float*>(part), item, nwg, k, 0, h);
    float y[4][2], env_in[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const float2 a = *reinterpret_cast<const float2*>(tl + (o * 256 + j) * 2);
        const float2 c = *reinterpret_cast<const float2*>(hd + (o * 256 + j) * 2);
        y[o][0] = a.x + c.x;
        y[o][1] = a.y + c.y;
    }
    ola_env_in(j, win2, env_in);
    ola_finish<false>(2 + g * k + h, j, y, T, env_in, xt2 + item * (int64_t)T * 2, tnorm[2 * b],
                      tnorm[2 * b + 1], out + (item * 2 + 0) * T, out + (item * 2 + 1) * T);
}

int istft_ola_nwg(int Tspec) { return istft_ola_split(Tspec).n; }

void istft_ola_launch(const float* fo, int NI, int Tspec, int P, int64_t T, const float* spec, const float2* tw,
                      const double2* tw64, const float* win, const float* win2, const float* xt2, const float* tnorm,
                      float* out, float* part, hipStream_t s) {
    const OlaSplit sp = istft_ola_split(Tspec);
    const int nwg = sp.n;
    {
        const int units = (NI / P) * nwg;
        const dim3 grid((unsigned)(8 * ((units + 7) / 8) * P));
        KScope ks(s);
        if (ks.on())
            ks.begin(tw64 ? "istft_ola_kernel<double,HIP_vector_type<double,2>,3,true>"
                          : "istft_ola_kernel<float,HIP_vector_type<float,2>,3,false>", 0.0,
                     (double)NI * Tspec * Tspec * 2 * 4 + (double)(NI / P) * 2048 * Tspec * 4 * 4 + (double)NI * T * 2 * 4 +
                         (double)NI * 2 * T * 4);
        // <3 waves per SIMD, no prefetch>: 1512 vs 1781 us for <2, prefetch> (round 2 measurement)
        if (tw64)
            hipLaunchKernelGGL((istft_ola_kernel<double, double2, 3>), grid, dim3(256), 0, s, fo, Tspec, P, (int)T, spec,
                               tw64, win, win2, xt2, tnorm, out, part, nwg, sp.g, units);
        else
            hipLaunchKernelGGL((istft_ola_kernel<float, float2, 3, false>), grid, dim3(256), 0, s, fo, Tspec, P, (int)T,
                               spec, tw, win, win2, xt2, tnorm, out, part, nwg, sp.g, units);
    }
    if (nwg > 1) {
        const dim3 grid((unsigned)(3 * (nwg - 1)), (unsigned)NI);
        KScope ks(s);
        if (ks.on()) ks.begin("istft_fix_kernel", 0.0, (double)NI * (nwg - 1) * 3 * 1024 * 2 * 4 * 4);
        hipLaunchKernelGGL(istft_fix_kernel, grid, dim3(256), 0, s, Tspec, P, (int)T, nwg, sp.g, win2, xt2, tnorm, out, part);
    }
}


}  // namespace athd
