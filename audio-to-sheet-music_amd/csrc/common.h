// Shared device helpers for the athd HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ATHD_DEV __device__ __forceinline__

// CUs of the CURRENT device, cached per device id (a process may drive GPUs of different CU counts);
// 256 (MI355X) if the query fails
inline int device_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    int& c = cache[dev & 63];
    if (c == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        c = n;
    }
    return c;
}
#define ATHD_HD __host__ __device__ __forceinline__

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // 8 bf16 = one MFMA 16x16x32 operand fragment
typedef __attribute__((ext_vector_type(4))) float f32x4_t;    // 16x16 accumulator fragment
typedef uint16_t bf16_t;                                      // raw bf16 storage

// Round-to-nearest-even f32 -> bf16 (NaN stays NaN through the plain cast path in hipcc; we only feed finite
// activations here, and the explicit form keeps the rounding identical across host and device).
ATHD_DEV bf16_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (bf16_t)(u >> 16);
}
// Two floats -> packed bf16 pair (lo = a) by v_cvt_pk_bf16_f32: the same round-to-nearest-even as f2bf for finite
// values, one instruction for both.
typedef __attribute__((ext_vector_type(2))) float athd_f2v;
typedef __attribute__((ext_vector_type(2))) __bf16 athd_b2v;
ATHD_DEV uint32_t pack2bf(float a, float b) {
    const athd_b2v r = __builtin_convertvector((athd_f2v){a, b}, athd_b2v);
    return __builtin_bit_cast(uint32_t, r);
}
ATHD_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

ATHD_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }
// bf16-mode GELU: branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 absolute), ~15 VALU ops vs ~60
// with two branches for erff.  The f32 parity mode always uses gelu_erf.
ATHD_DEV float erf_fast(float x) {
    const float ax = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    p *= t;
    const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
    return copysignf(fmaf(-p, e, 1.0f), x);
}
// bf16-mode GELU: the tanh form x * sigmoid(sqrt(8/pi) (x + 0.044715 x^3)) on v_exp_f32 + v_rcp_f32, 7 VALU ops.
// |gelu_fast - gelu_erf| <= 4.8e-4 absolute (at x ~ 2.7, value 2.69: 1.8e-4 relative, below half a bf16 ulp).
ATHD_DEV float gelu_fast(float x) {
    constexpr float K0 = -1.5957691216057308f * 1.4426950408889634f, K1 = K0 * 0.044715f;   // (-log2(e) folded in)
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * fmaf(K1, x * x, K0)));
}
template <bool FAST>
ATHD_DEV float gelu(float x) { if constexpr (FAST) return gelu_fast(x); else return gelu_erf(x); }
// gelu_fast on a pair: the polynomial and scaling on packed f32 ops (v_pk_mul / v_pk_fma), exp2 / rcp per lane
// (the -log2(e) of the exp2 folded into the polynomial's constants: 4 packed ops + 2 x (exp, rcp) per pair)
ATHD_DEV athd_f2v gelu_fast_pk(athd_f2v x) {
    constexpr float K0 = -1.5957691216057308f * 1.4426950408889634f, K1 = K0 * 0.044715f;
    const athd_f2v t = x * __builtin_elementwise_fma((athd_f2v){K1, K1}, x * x, (athd_f2v){K0, K0});
    const athd_f2v den = (athd_f2v){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + (athd_f2v){1.0f, 1.0f};
    return x * (athd_f2v){__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
}
// wa * gelu_fast(a) + wb * gelu_fast(b) on pairs with ONE reciprocal per element instead of two (the decoder merges
// only need the resize's weighted sum of two rows' GELUs): (wa a (1 + eb) + wb b (1 + ea)) / ((1 + ea)(1 + eb)).  The
// exp2 argument is clamped at 60 so that the product of the denominators stays finite (there the term is x 2^-60).
ATHD_DEV athd_f2v gelu_fast_wsum_pk(athd_f2v wa, athd_f2v a, athd_f2v wb, athd_f2v b) {
    constexpr float K0 = -1.5957691216057308f * 1.4426950408889634f, K1 = K0 * 0.044715f;
    const athd_f2v lim = {60.0f, 60.0f}, one = {1.0f, 1.0f};
    const athd_f2v ta = __builtin_elementwise_min(a * __builtin_elementwise_fma((athd_f2v){K1, K1}, a * a, (athd_f2v){K0, K0}), lim);
    const athd_f2v tb = __builtin_elementwise_min(b * __builtin_elementwise_fma((athd_f2v){K1, K1}, b * b, (athd_f2v){K0, K0}), lim);
    const athd_f2v da = (athd_f2v){__builtin_amdgcn_exp2f(ta.x), __builtin_amdgcn_exp2f(ta.y)} + one;
    const athd_f2v db = (athd_f2v){__builtin_amdgcn_exp2f(tb.x), __builtin_amdgcn_exp2f(tb.y)} + one;
    const athd_f2v den = da * db;
    return __builtin_elementwise_fma(wa * a, db, wb * b * da) *
           (athd_f2v){__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
}
ATHD_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// bf16-mode sigmoid: v_exp_f32 + v_rcp_f32 (~1 ulp each; 4 instructions vs ~25 for expf and an IEEE divide).  The
// f32 parity mode keeps sigmoidf_.
ATHD_DEV float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
template <bool FAST>
ATHD_DEV float sigmoid(float x) { if constexpr (FAST) return sigmoid_fast(x); else return sigmoidf_(x); }

ATHD_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
ATHD_DEV double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
ATHD_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// PyTorch-faithful fp32 source index for linear/bilinear resize with align_corners=False and no explicit scale
// (ATen UpSample.h area_pixel_compute_scale / area_pixel_compute_source_index / guard_index_and_lambda).
struct LinIdx { int i0, i1; float l0, l1; };
ATHD_HD LinIdx lin_index(int dst, int in_size, int out_size) {
    LinIdx r;
    if (in_size == out_size) { r.i0 = r.i1 = dst; r.l0 = 1.f; r.l1 = 0.f; return r; }
    float scale = (float)in_size / (float)out_size;
    float src = scale * ((float)dst + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    int i0 = (int)floorf(src);
    if (i0 > in_size - 1) i0 = in_size - 1;
    float lam = src - (float)i0;
    lam = fminf(fmaxf(lam, 0.f), 1.f);
    r.i0 = i0;
    r.i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
    r.l1 = lam;
    r.l0 = 1.f - lam;
    return r;
}

// GroupNorm(1) (mean, 1/sqrt(var + 1e-5)) of batch b from fp64 {sum, sumsq} over `count` elements
ATHD_DEV void gn_params(const double* st, int64_t b, int64_t count, float& mean, float& rstd) {
    const double m = st[2 * b] / (double)count;
    double var = st[2 * b + 1] / (double)count - m * m;
    if (var < 0) var = 0;
    mean = (float)m;
    rstd = (float)(1.0 / sqrt(var + 1e-5));
}

#define HIP_CHECK_RET(x)                                                       \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) return (int)e_;                                  \
    } while (0)
