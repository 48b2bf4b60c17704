// Spectral front/back end for gfx950.
//
// STFT: one workgroup per (sample, kept frame).  Both audio channels go through ONE 4096-point complex FFT
// (z = x_L + i x_R), radix-4 Stockham (6 stages) ping-ponging between two 32 KiB LDS buffers, twiddles from
// a 4096-entry table; the two real spectra are split as X_L = (Z_k + conj Z_-k)/2, X_R = (Z_k - conj Z_-k)/2i.
// The reflect padding of HTDemucs._spec (demucs pad1d, incl. its zero-extension for inputs shorter than the
// pad) is folded into the frame gather; torch.stft's own centre padding is never reached by the kept frames
// 2..le+1, so it needs no code.  Output is the CaC tensor channels-last: spec[b][f][t][4] = {Re L, Im L, Re R,
// Im R} with the 1/sqrt(4096) "normalized" scale (exactly 1/64).
//
// iSTFT: per (item, frame) the decoder's freq map is resized 2048 rows (PyTorch fp32 bilinear index math),
// passed through sigmoid, and the masking formula of ATHTDemucs_v2.py:303-309 is applied to both channels;
// the two Hermitian spectra are packed into one complex inverse FFT (x_L = Re, x_R = Im), scaled 1/64 and
// windowed into a frame buffer.  The combine kernel then gathers the <=4 overlapping frames per output sample,
// divides by the window envelope of ALL le+4 frames (torch.istft), and adds the denormalised time branch after
// its 1x1 output conv (ATHTDemucs_v2.py:314-324).
#include "common.h"
#include "prof.h"
#include "kernels.h"

namespace athd {

constexpr int NFFT = 4096;
constexpr int HOP = 1024;

struct cpx { float x, y; };
ATHD_DEV cpx cadd(cpx a, cpx b) { return {a.x + b.x, a.y + b.y}; }
ATHD_DEV cpx csub(cpx a, cpx b) { return {a.x - b.x, a.y - b.y}; }
ATHD_DEV cpx cmul(cpx a, cpx b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

// In-LDS radix-4 Stockham FFT (forward, e^{-2 pi i}) of 4096 points with 256 threads.  Result in the buffer
// returned (a or b).
ATHD_DEV cpx* fft4096(cpx* a, cpx* b, const float2* __restrict__ tw) {
    const int tid = threadIdx.x;
    for (int L = 1; L < NFFT; L *= 4) {
        const int tstride = NFFT / (4 * L);
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int j = tid + 256 * it;
            const int k = j & (L - 1);
            cpx a0 = a[j], a1 = a[j + NFFT / 4], a2 = a[j + NFFT / 2], a3 = a[j + 3 * NFFT / 4];
            if (L > 1) {
                float2 w1 = tw[(k * tstride) & (NFFT - 1)];
                float2 w2 = tw[(2 * k * tstride) & (NFFT - 1)];
                float2 w3 = tw[(3 * k * tstride) & (NFFT - 1)];
                a1 = cmul(a1, {w1.x, w1.y});
                a2 = cmul(a2, {w2.x, w2.y});
                a3 = cmul(a3, {w3.x, w3.y});
            }
            cpx s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
            cpx md13 = {d13.y, -d13.x};                    // -i * d13
            const int base = (j - k) * 4 + k;
            b[base] = cadd(s02, s13);
            b[base + L] = cadd(d02, md13);
            b[base + 2 * L] = csub(s02, s13);
            b[base + 3 * L] = csub(d02, md13);
        }
        __syncthreads();
        cpx* t = a; a = b; b = t;
    }
    return a;
}

ATHD_DEV float pad_sample(const float* __restrict__ x, int64_t p, const PadPlan& pp) {
    int64_t i = p - pp.left;                 // index into the zero-extended signal of length Lx
    if (i < 0) i = -i;
    if (i >= pp.Lx) i = 2 * (pp.Lx - 1) - i;
    i -= pp.ext_left;
    return (i >= 0 && i < pp.L) ? x[i] : 0.f;
}

__global__ __launch_bounds__(256) void stft_kernel(const float* __restrict__ wav, int64_t T, PadPlan pp, int Tspec,
                                                   const float2* __restrict__ tw, const float* __restrict__ win,
                                                   float* __restrict__ spec, float* __restrict__ specT) {
    __shared__ cpx bufA[NFFT];
    __shared__ cpx bufB[NFFT];
    const int t = blockIdx.x;
    const int64_t b = blockIdx.y;
    const float* xl = wav + b * 2 * T;
    const float* xr = xl + T;
    const int64_t p0 = (int64_t)t * HOP;     // kept frame t = stft frame t+2, starts at 1024 t in the pad1d'ed signal
    for (int n = threadIdx.x; n < NFFT; n += 256) {
        const float w = win[n];
        bufA[n] = {pad_sample(xl, p0 + n, pp) * w, pad_sample(xr, p0 + n, pp) * w};
    }
    __syncthreads();
    cpx* Z = fft4096(bufA, bufB, tw);
    float* out = spec + ((b * 2048) * Tspec + t) * 4;
    float* outT = specT + (b * Tspec + t) * 2048LL * 4;      // frame-major copy for the iSTFT (contiguous)
    for (int k = threadIdx.x; k < 2048; k += 256) {
        cpx zk = Z[k], zn = Z[(NFFT - k) & (NFFT - 1)];
        // X_L = (zk + conj zn)/2, X_R = (zk - conj zn)/(2i); scaled by 1/64 (normalized=True)
        const float s = 0.5f / 64.f;
        float4 v;
        v.x = (zk.x + zn.x) * s;
        v.y = (zk.y - zn.y) * s;
        v.z = (zk.y + zn.y) * s;
        v.w = -(zk.x - zn.x) * s;
        *reinterpret_cast<float4*>(out + (int64_t)k * Tspec * 4) = v;
        *reinterpret_cast<float4*>(outT + (int64_t)k * 4) = v;
    }
}

void stft_launch(const float* wav, int nb, int64_t T, const PadPlan& pp, int Tspec, const float2* tw,
                 const float* win, float* spec, float* specT, hipStream_t s) {
    KScope ks(s);
    if (ks.on()) ks.begin("stft_kernel", 0.0, (double)nb * 2 * T * 4 + 2.0 * nb * 2048 * Tspec * 4 * 4);
    hipLaunchKernelGGL(stft_kernel, dim3(Tspec, nb), dim3(256), 0, s, wav, T, pp, Tspec, tw, win, spec, specT);
}

// ---------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void istft_frames_kernel(const float* __restrict__ fo, int Tspec, int P,
                                                           const float* __restrict__ specT,
                                                           const float2* __restrict__ tw,
                                                           const float* __restrict__ win,
                                                           float* __restrict__ frames) {
    __shared__ cpx bufA[NFFT];
    __shared__ cpx bufB[NFFT];
    const int t = blockIdx.x;
    const int64_t item = blockIdx.y;
    const int64_t b = item / P;
    const float* F0 = fo + (item * (int64_t)Tspec + t) * Tspec * 2;   // FO^T: [item][t][row][2]
    const float* S = specT + (b * Tspec + t) * 2048LL * 4;             // [b][t][k][4]
    for (int k = threadIdx.x; k < 2048; k += 256) {
        const LinIdx li = lin_index(k, Tspec, 2048);
        const float* r0 = F0 + (int64_t)li.i0 * 2;
        const float* r1 = F0 + (int64_t)li.i1 * 2;
        const float xd0 = li.l0 * r0[0] + li.l1 * r1[0];
        const float xd1 = li.l0 * r0[1] + li.l1 * r1[1];
        const float m0 = sigmoidf_(xd0), m1 = sigmoidf_(xd1);
        const float4 z = *reinterpret_cast<const float4*>(S + (int64_t)k * 4);
        // masked_z = (mag*mask) * (z / (mag + 1e-8)); ch0: z_L with mag = Re z_L; ch1: z_R with mag = Im z_L
        const float ms0 = z.x * m0, ms1 = z.y * m1;
        const float d0 = z.x + 1e-8f, d1 = z.y + 1e-8f;
        cpx X0 = {ms0 * (z.x / d0), ms0 * (z.y / d0)};
        cpx X1 = {ms1 * (z.z / d1), ms1 * (z.w / d1)};
        if (k == 0) { X0.y = 0.f; X1.y = 0.f; }          // c2r ignores the imaginary part of the DC bin
        // Z = X0 + i X1 (k), and its Hermitian mirror at N-k: conj(X0) + i conj(X1); conj() for the inverse
        // (ifft(Z) = conj(fft(conj(Z))))
        cpx Zk = {X0.x - X1.y, X0.y + X1.x};
        bufA[k] = {Zk.x, -Zk.y};
        if (k > 0) {
            cpx Zm = {X0.x + X1.y, -X0.y + X1.x};
            bufA[NFFT - k] = {Zm.x, -Zm.y};
        }
    }
    if (threadIdx.x == 0) bufA[2048] = {0.f, 0.f};    // Nyquist bin padded with zero (HTDemucs._ispec)
    __syncthreads();
    cpx* Z = fft4096(bufA, bufB, tw);
    float* o = frames + (item * Tspec + t) * 2LL * NFFT;
    for (int n = threadIdx.x; n < NFFT; n += 256) {
        const float w = win[n] * (1.f / 64.f);
        o[n] = Z[n].x * w;             // conj(fft(conj Z)) -> real part unchanged
        o[NFFT + n] = -Z[n].y * w;     // imag part negated
    }
}

void istft_frames_launch(const float* fo, int NI, int Tspec, int P, const float* spec, const float2* tw,
                         const float* win, float* frames, hipStream_t s) {
    KScope ks(s);
    if (ks.on())
        ks.begin("istft_frames_kernel", 0.0, (double)NI * Tspec * Tspec * 2 * 4 + (double)(NI / P) * 2048 * Tspec * 4 * 4 +
                                                 (double)NI * Tspec * 2 * 4096 * 4);
    hipLaunchKernelGGL(istft_frames_kernel, dim3(Tspec, NI), dim3(256), 0, s, fo, Tspec, P, spec, tw, win, frames);
}

// out[item][c][n] = OLA(frames)/env + xt2[item][n][c] * stdt[b] + meant[b]   (ATHTDemucs_v2.py:310-324; xt2 is
// time_out of the time decoder, dec_last.hip)
__global__ __launch_bounds__(256) void combine_kernel(const float* __restrict__ frames, int Tspec, int64_t T,
                                                      const float* __restrict__ win2, const float* __restrict__ xt2,
                                                      const float* __restrict__ tnorm, int P,
                                                      float* __restrict__ out) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t item = blockIdx.y;
    if (n >= T) return;
    const int64_t b = item / P;
    const int64_t q = n + 3584;                      // OLA index: 1536 (_ispec slice) + 2048 (istft centre)
    const int nfr = Tspec + 4;
    int f_lo;                                        // first frame f' with 1024 f' + 4096 > q
    if (q - NFFT + 1 <= 0) f_lo = 0;
    else f_lo = (int)((q - NFFT + 1 + HOP - 1) / HOP);
    int f_hi = (int)(q / HOP);
    if (f_hi > nfr - 1) f_hi = nfr - 1;
    float env = 0.f, y0 = 0.f, y1 = 0.f;
    for (int f = f_lo; f <= f_hi; ++f) {
        const int j = (int)(q - (int64_t)f * HOP);
        env += win2[j];
        const int t = f - 2;
        if (t >= 0 && t < Tspec) {
            const float* fr = frames + (item * Tspec + t) * 2LL * NFFT;
            y0 += fr[j];
            y1 += fr[NFFT + j];
        }
    }
    const float2 x2 = *reinterpret_cast<const float2*>(xt2 + (item * T + n) * 2);
    const float mean = tnorm[2 * b], stdv = tnorm[2 * b + 1];
    out[(item * 2 + 0) * T + n] = y0 / env + (x2.x * stdv + mean);
    out[(item * 2 + 1) * T + n] = y1 / env + (x2.y * stdv + mean);
}

void combine_launch(const float* frames, int NI, int Tspec, int64_t T, const float* win2, const float* xt2,
                    const float* tnorm, int P, float* out, hipStream_t s) {
    dim3 grid((unsigned)((T + 255) / 256), NI);
    KScope ks(s);
    if (ks.on())
        ks.begin("combine_kernel", 0.0, (double)NI * Tspec * 2 * 4096 * 4 + (double)NI * T * 2 * 4 + (double)NI * 2 * T * 4);
    hipLaunchKernelGGL(combine_kernel, grid, dim3(256), 0, s, frames, Tspec, T, win2, xt2, tnorm, P, out);
}

}  // namespace athd
