// Track level: the window loop of test_inference.py:92-141 and sdr_loss (src/loss.py:9-30).
//
// overlap-add: the reference runs windows start_k = k*hop (hop = chunk - overlap), end_k = min(start_k + chunk, L),
// applies torchaudio Fade(fade_in_k = k ? overlap : 0, fade_out_k = end_k < L ? overlap : 0, 'linear') and does
// final[..., start_k:end_k] += out_k in ascending k.  Here every output sample GATHERS its <= 2 covering windows in
// ascending k, starting from 0.0f - the same fp32 additions in the same order, no atomics.  The window plan is
// analytic, so no table is needed; [k0, k1) selects a window range (sharded runs) whose output span starts at
// start_k0.
#include <algorithm>

#include "common.h"
#include "prof.h"
#include "kernels.h"

// The reference rounds every product before the sum (out = fade(out); final += out) and torch.linspace rounds
// step*i before the subtraction: no fma contraction anywhere in this file (__fmul_rn / __fadd_rn are plain
// header functions compiled with contraction on): plain operators under a contract(off) pragma in each function.

namespace athd {

// torch.linspace(0, 1, n)[i] in fp32 (ATen range-factory formula: the first half counts up from start, the second
// half down from end), explicit roundings so the compiler cannot contract into an fma.
ATHD_DEV float linspace01(int64_t i, int64_t n) {
#pragma clang fp contract(off)
    if (n == 1) return 0.f;
    const float step = 1.f / (float)(n - 1);
    if (i < n / 2) return step * (float)i;
    return 1.f - step * (float)(n - i - 1);
}

struct OlaDesc {
    const float* win;          // [(k1-k0)][S][2][chunk]  window k's samples in its first len_k entries
    float* out;                // [S][2][span]
    int64_t L, chunk, overlap, hop, k0, k1, n, span, t0;
    int S;
};

__global__ __launch_bounds__(256) void ola_kernel(const OlaDesc d) {
#pragma clang fp contract(off)
    const int64_t t_loc = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int sc = blockIdx.y;                      // stem * 2 + channel
    if (t_loc >= d.span) return;
    const int64_t t = d.t0 + t_loc;
    // windows covering t: start_k <= t < end_k  ->  k in [ceil((t - chunk + 1) / hop), floor(t / hop)]
    int64_t ka = t - d.chunk + 1 <= 0 ? 0 : (t - d.chunk + 1 + d.hop - 1) / d.hop;
    int64_t kb = t / d.hop;
    if (ka < d.k0) ka = d.k0;
    if (kb > d.k1 - 1) kb = d.k1 - 1;
    float acc = 0.f;
    for (int64_t k = ka; k <= kb; ++k) {
        const int64_t st = k * d.hop;
        const int64_t en = st + d.chunk < d.L ? st + d.chunk : d.L;
        if (t >= en) continue;
        const int64_t len = en - st, j = t - st;
        const int64_t fin = k == 0 ? 0 : d.overlap;
        const int64_t fout = en < d.L ? d.overlap : 0;
        float fi = j < fin ? linspace01(j, fin) : 1.f;
        float fo = j >= len - fout ? 1.f - linspace01(j - (len - fout), fout) : 1.f;
        fi = fminf(fmaxf(fi, 0.f), 1.f);
        fo = fminf(fmaxf(fo, 0.f), 1.f);
        const float x = d.win[((k - d.k0) * (2 * d.S) + sc) * d.chunk + j];
        const float w = fi * fo;
        acc = acc + w * x;
    }
    d.out[(int64_t)sc * d.span + t_loc] = acc;
}

// torch.linspace(1, 0, n)[i] in fp32: step = (0 - 1) / (n - 1) = -s; first half 1 + step * i, second half
// 0 - step * (n - i - 1) = s * (n - i - 1) (exact negations).
ATHD_DEV float linspace10(int64_t i, int64_t n) {
#pragma clang fp contract(off)
    if (n == 1) return 1.f;
    const float step = -(1.f / (float)(n - 1));
    if (i < n / 2) return 1.f + step * (float)i;
    return -step * (float)(n - i - 1);
}

// benchmark.py protocol (OurModel._chunked_inference, benchmark.py:155-204).  Every window's model input was
// zero-padded to `chunk` (only its first len_k outputs are used); fade_len_k = min(overlap, len_k / 2);
// chunk_weight = 1 with [:fade_len] = linspace(0, 1) if start_k > 0 and [-fade_len:] = linspace(1, 0) if
// end_k < L (the two ramps never overlap: 2 fade_len <= len_k); output[t] += out_k * w, weight[t] += w in ascending
// k from 0; output / weight.clamp(min=1e-8).  wsum == nullptr: out = the normalised track span.  wsum != nullptr:
// out = sum w x and wsum = sum w (unnormalised partial spans of a sharded run, finished by ola_normalize).
__global__ __launch_bounds__(256) void ola_weighted_kernel(const OlaDesc d, float* __restrict__ wsum) {
#pragma clang fp contract(off)
    const int64_t t_loc = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int sc = blockIdx.y;
    if (t_loc >= d.span) return;
    const int64_t t = d.t0 + t_loc;
    int64_t ka = t - d.chunk + 1 <= 0 ? 0 : (t - d.chunk + 1 + d.hop - 1) / d.hop;
    int64_t kb = t / d.hop;
    if (ka < d.k0) ka = d.k0;
    if (kb > d.k1 - 1) kb = d.k1 - 1;
    float acc = 0.f, ws = 0.f;
    for (int64_t k = ka; k <= kb; ++k) {
        const int64_t st = k * d.hop;
        const int64_t en = st + d.chunk < d.L ? st + d.chunk : d.L;
        if (t >= en) continue;
        const int64_t len = en - st, j = t - st;
        const int64_t fl = d.overlap < len / 2 ? d.overlap : len / 2;
        float w = 1.f;
        if (st > 0 && fl > 0 && j < fl) w = linspace01(j, fl);
        if (en < d.L && fl > 0 && j >= len - fl) w = linspace10(j - (len - fl), fl);
        const float x = d.win[((k - d.k0) * (2 * d.S) + sc) * d.chunk + j];
        acc = acc + x * w;
        ws = ws + w;
    }
    if (wsum) {
        d.out[(int64_t)sc * d.span + t_loc] = acc;
        if (sc == 0) wsum[t_loc] = ws;
    } else {
        d.out[(int64_t)sc * d.span + t_loc] = acc / fmaxf(ws, 1e-8f);
    }
}

__global__ __launch_bounds__(256) void ola_normalize_kernel(float* __restrict__ out, const float* __restrict__ wsum,
                                                            int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    out[(int64_t)blockIdx.y * n + t] = out[(int64_t)blockIdx.y * n + t] / fmaxf(wsum[t], 1e-8f);
}

int ola_normalize_launch(float* out, const float* wsum, int rows, int64_t n, hipStream_t s) {
    if (!out || !wsum || rows <= 0 || n <= 0 || rows > 65535) return -1;
    KScope ks(s);
    if (ks.on()) ks.begin("ola_normalize_kernel", 0.0, (double)n * 4 * (2 * rows + 1));
    hipLaunchKernelGGL(ola_normalize_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)rows), dim3(256), 0, s, out,
                       wsum, n);
    return (int)hipGetLastError();
}

int ola_launch(const float* win, int64_t L, int64_t chunk, int64_t overlap, int S, int64_t k0, int64_t k1, float* out,
               hipStream_t s, int mode, float* wsum) {
    if (!win || !out || L <= 0 || chunk <= 0 || overlap < 0 || overlap >= chunk || S <= 0 || 2 * S > 65535)
        return -1;
    if (mode != 0 && mode != 1) return -1;
    OlaDesc d;
    d.win = win;
    d.out = out;
    d.L = L;
    d.chunk = chunk;
    d.overlap = overlap;
    d.hop = chunk - overlap;
    d.n = (L + d.hop - 1) / d.hop;     // while start < L: start += hop
    if (k0 < 0 || k1 > d.n || k0 >= k1) return -1;
    d.k0 = k0;
    d.k1 = k1;
    d.S = S;
    d.t0 = k0 * d.hop;
    const int64_t last_end = std::min<int64_t>((k1 - 1) * d.hop + chunk, L);
    d.span = last_end - d.t0;
    KScope ks(s);
    const dim3 grid((unsigned)((d.span + 255) / 256), 2 * S);
    if (mode == 0) {
        if (ks.on()) ks.begin("ola_kernel", 0.0, (double)(k1 - k0) * 2 * S * chunk * 4 + (double)2 * S * d.span * 4);
        hipLaunchKernelGGL(ola_kernel, grid, dim3(256), 0, s, d);
    } else {
        if (ks.on())
            ks.begin("ola_weighted_kernel", 0.0,
                     (double)(k1 - k0) * 2 * S * chunk * 4 + (double)(2 * S + (wsum ? 1 : 0)) * d.span * 4);
        hipLaunchKernelGGL(ola_weighted_kernel, grid, dim3(256), 0, s, d, wsum);
    }
    return (int)hipGetLastError();
}

// ---- SI-SDR of src/loss.py:33-68 (benchmark.py:573-588): per row, est and target centred on their means,
//      s_target = (<e, t> / (|t|^2 + 1e-8)) t, e_noise = e - s_target, clamp(10 log10((|s_target|^2 + 1e-8) /
//      (|e_noise|^2 + 1e-8)), -30, 30), mean over rows.  Two passes in fp64: row means, then the centred sums
//      <e,t>, |t|^2, |e|^2; |s_target|^2 = a^2 |t|^2 and |e_noise|^2 = |e|^2 - 2 a <e,t> + a^2 |t|^2 with
//      a = <e,t> / (|t|^2 + 1e-8).
__global__ __launch_bounds__(256) void sisdr_sums_kernel(const float* __restrict__ est, const float* __restrict__ tgt,
                                                         int64_t n, const double* __restrict__ mean,
                                                         double* __restrict__ sums, int pass) {
    const int64_t r = blockIdx.y;
    const float* e = est + r * n;
    const float* g = tgt + r * n;
    double a = 0.0, b = 0.0, c = 0.0;
    const double me = pass ? mean[2 * r] / (double)n : 0.0, mt = pass ? mean[2 * r + 1] / (double)n : 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double ev = (double)e[i] - me, tv = (double)g[i] - mt;
        if (pass) {
            a += ev * tv;
            b += tv * tv;
            c += ev * ev;
        } else {
            a += ev;
            b += tv;
        }
    }
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    c = wave_sum_d(c);
    __shared__ double sh[12];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[3 * w] = a; sh[3 * w + 1] = b; sh[3 * w + 2] = c; }
    __syncthreads();
    if (threadIdx.x < 3) {
        const double v = sh[threadIdx.x] + sh[3 + threadIdx.x] + sh[6 + threadIdx.x] + sh[9 + threadIdx.x];
        if (pass || threadIdx.x < 2) atomicAdd(&sums[(pass ? 3 : 2) * r + threadIdx.x], v);
    }
}

__global__ void sisdr_final_kernel(const double* __restrict__ sums, int64_t rows, float* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double m = 0.0;
    for (int64_t r = 0; r < rows; ++r) {
        const double et = sums[3 * r], tt = sums[3 * r + 1], ee = sums[3 * r + 2];
        const double al = et / (tt + 1e-8);
        const double st = al * al * tt;
        double en = ee - 2.0 * al * et + al * al * tt;
        en = en < 0.0 ? 0.0 : en;
        double v = 10.0 * log10((st + 1e-8) / (en + 1e-8));
        v = v < -30.0 ? -30.0 : (v > 30.0 ? 30.0 : v);
        m += v;
    }
    out[0] = (float)(m / (double)rows);
}

// scratch: 5 * rows doubles (2 for the means, 3 for the centred sums)
int sisdr_launch(const float* est, const float* tgt, int64_t rows, int64_t n, double* scratch, float* out,
                 hipStream_t s) {
    if (!est || !tgt || !scratch || !out || rows <= 0 || n <= 0 || rows > 65535) return -1;
    HIP_CHECK_RET(hipMemsetAsync(scratch, 0, (size_t)rows * 5 * sizeof(double), s));
    const int bx = (int)std::min<int64_t>((n + 255) / 256, 1024);
    double* mean = scratch;
    double* sums = scratch + 2 * rows;
    hipLaunchKernelGGL(sisdr_sums_kernel, dim3(bx, (unsigned)rows), dim3(256), 0, s, est, tgt, n, mean, mean, 0);
    hipLaunchKernelGGL(sisdr_sums_kernel, dim3(bx, (unsigned)rows), dim3(256), 0, s, est, tgt, n, mean, sums, 1);
    hipLaunchKernelGGL(sisdr_final_kernel, dim3(1), dim3(64), 0, s, sums, rows, out);
    return (int)hipGetLastError();
}

// ---- SDR: per row r, num = sum tgt^2, den = sum (tgt - est)^2 (fp64 partial sums), then
//      sdr_r = clamp(10 log10((num + 1e-8) / (den + 1e-8)), -30, 30) and mean over rows.
__global__ __launch_bounds__(256) void sdr_sums_kernel(const float* __restrict__ est, const float* __restrict__ tgt,
                                                       int64_t n, double* __restrict__ sums) {
    const int64_t r = blockIdx.y;
    const float* e = est + r * n;
    const float* g = tgt + r * n;
    double a = 0.0, b = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double tv = g[i], dv = (double)g[i] - (double)e[i];
        a += tv * tv;
        b += dv * dv;
    }
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    __shared__ double sh[8];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[2 * w] = a; sh[2 * w + 1] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&sums[2 * r], sh[0] + sh[2] + sh[4] + sh[6]);
        atomicAdd(&sums[2 * r + 1], sh[1] + sh[3] + sh[5] + sh[7]);
    }
}

__global__ void sdr_final_kernel(const double* __restrict__ sums, int64_t rows, float* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double m = 0.0;
    for (int64_t r = 0; r < rows; ++r) {
        double v = 10.0 * log10((sums[2 * r] + 1e-8) / (sums[2 * r + 1] + 1e-8));
        v = v < -30.0 ? -30.0 : (v > 30.0 ? 30.0 : v);
        m += v;
    }
    out[0] = (float)(m / (double)rows);
}

int sdr_launch(const float* est, const float* tgt, int64_t rows, int64_t n, double* sums, float* out, hipStream_t s) {
    if (!est || !tgt || !sums || !out || rows <= 0 || n <= 0) return -1;
    HIP_CHECK_RET(hipMemsetAsync(sums, 0, (size_t)rows * 2 * sizeof(double), s));
    int bx = (int)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(sdr_sums_kernel, dim3(bx, (unsigned)rows), dim3(256), 0, s, est, tgt, n, sums);
    hipLaunchKernelGGL(sdr_final_kernel, dim3(1), dim3(64), 0, s, sums, rows, out);
    return (int)hipGetLastError();
}

}  // namespace athd
