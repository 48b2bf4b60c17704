// Implicit-GEMM convolution / linear layer on MFMA (gfx950).
//
// One descriptor covers every contraction on the hot path:
//   Conv2d (k,1) / Conv1d along the "H" axis of a channels-last tensor [nb][H][W][C] with `ntaps` taps,
//   1x1 convs and Linear layers (ntaps = 1), and one residue class of a stride-4 ConvTranspose (2 taps).
//   out[b][ho*os+oo][w][n] = epi( sum_{tap,ci} A[b][ho*s+off+tap*dil][w][ci] * Wp[n][tap*C_in+ci] + bias[n] )
// Weights are pre-packed [N][Kp] (k contiguous, zero padded to Kp % 32 == 0) in the compute dtype.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace athd {

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_GLU = 2 };

// n / d for 0 <= n < 2^31 as a multiply-high and a shift (Granlund-Montgomery with a 31+l bit reciprocal:
// mul = ceil(2^(31+l) / d), l = ceil(log2 d), exact for every n < 2^31).  Filled by gemm_launch; the kernels' row
// index decompositions (m -> w, h, b) and GroupNorm group indices use it instead of the ~30-instruction integer
// division sequence.
struct FastDivU {
    uint32_t mul = 0, shift = 0, d = 1;
};
inline FastDivU make_fastdiv(uint32_t d) {
    FastDivU f;
    f.d = d;
    if (d <= 1) return f;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.mul = (uint32_t)((((uint64_t)1 << (31 + l)) + d - 1) / d);
    f.shift = l - 1;
    return f;
}
#if defined(__HIPCC__)
__device__ inline uint32_t fdiv(uint32_t n, const FastDivU& f) { return f.d == 1 ? n : __umulhi(n, f.mul) >> f.shift; }
#endif

struct GemmDesc {
    // A operand (activations), channels-last
    const void* A = nullptr;
    int a_bf16 = 0;           // A stored as bf16 (else f32)
    int nb = 1;               // batch count (GEMM M = nb * H_out * W)
    int H_in = 1, W = 1, C_in = 0;
    int a_ld = 0;             // elements between consecutive positions (>= C_in)
    int64_t a_cs = 1;         // elements between channels (1 = channels-last; the raw (B,2,T) waveform uses T)
    int64_t a_bs = -1;        // elements between batches (-1: H_in*W*a_ld)
    int64_t a_hs = -1;        // elements between consecutive input rows h (-1: W*a_ld).  a_hs == C_in with dil == 1
                              // makes the whole (tap, ci) K row contiguous ("flat K", used when C_in < 8)
    int ntaps = 1, in_stride = 1, in_off = 0, dil = 1;
    int H_out = 1;            // output rows computed per batch
    const float* a_norm = nullptr;    // optional per-batch {sub, div} on in-bounds A: (a - sub[b]) / div[b]
    // optional GroupNorm(1) on f32 A as it is loaded (gemm2's fp32-A path, ntaps == 1): a' = (a - mean[b]) * rstd[b] *
    // a_gn_w[ci] + a_gn_b[ci], statistics {sum, sumsq} over a_gn_count elements per batch
    const double* a_gn_stats = nullptr;
    int64_t a_gn_count = 0;
    const float* a_gn_w = nullptr;
    const float* a_gn_b = nullptr;
    // B operand (packed weights [N][Kp]) and bias
    const void* Wp = nullptr;
    int N = 0, K = 0, Kp = 0;
    const float* bias = nullptr;
    // C output
    void* C = nullptr;
    int c_bf16 = 0;
    int H_out_total = 1;      // rows in the output tensor per batch
    int o_stride = 1, o_off = 0;
    int ldo = 0;              // elements between output positions
    int col_off = 0;
    int64_t c_bs = -1;        // elements between output batches (-1: H_out_total*W*ldo)
    int store = 1;            // 0: compute statistics only
    // GLU epilogue only: the first 4 output channels of every row also go to c4 [rows][4] (C's dtype), the compact
    // copy the decoders' last level reads as its skip (saved[0][:, :4], ATHTDemucs_v2.py:96-103 / :130-137)
    void* c4 = nullptr;
    int col_split = 0;        // >0: column group g = n / col_split goes to output row + g * hi_row_off, column
    int hi_row_off = 1;       //     n - g * col_split (ConvTranspose residue classes computed by one GEMM)
    int store_mask = 3;       //     bit g: store column group g
    int k_blk = 0;            // >0 (with col_split): the four-residue ConvT's zero blocks - column groups 0/1 read
                              //     only K [0, 2 k_blk), groups 2/3 only K [k_blk, 3 k_blk); k_blk % 32 == 0
    // epilogue
    int act = ACT_NONE;       // ACT_GLU: packed pairs [a(16) | gate(16)] per 32 columns, output N/2 channels
    const void* res = nullptr;        // residual (same layout as C; f32, or bf16 with res_bf16); out = res + rs[n]*v
    int res_bf16 = 0;
    const float* res_scale = nullptr;
    // optional GroupNorm(1) on the f32 residual as it is read (epilogue flag F_RGN, gemm5's residual epilogue): the
    // residual stream's pending GroupNorm, which the LayerNorm pass before this GEMM applied in registers only
    // (LnDesc::gn_writeback = 0): res' = (res - mean[b]) * rstd[b] * res_gn_w[n] + res_gn_b[n], statistics {sum, sumsq}
    // over res_gn_count elements per batch
    const double* res_gn_stats = nullptr;
    int64_t res_gn_count = 0;
    const float* res_gn_w = nullptr;
    const float* res_gn_b = nullptr;
    const float* row_add = nullptr;   // out += row_add[ho][n]   (freq embedding after encoder level 0)
    double* stats = nullptr;          // per-batch {sum, sumsq} of the final output value
    const double* gn_stats = nullptr; // GroupNorm(1) applied to v (after bias, before act) with per-batch
    FastDivU fd_w, fd_h, fd_hw;       // W, H_out, H_out * W (filled by the launchers: with_fastdiv)
    int64_t gn_count = 0;             //   statistics {sum, sumsq} over gn_count elements and per-column
    const float* gn_w = nullptr;      //   affine (packed in the same column order as the weights)
    const float* gn_b = nullptr;
    // per-batch bias (epilogue flag F_PB): v += pbias[ob][n] for output batch ob.  pfold > 1: every input batch b
    // (M rows) yields pfold output batches ob = b * pfold + p (the P prompts of one segment), each with its own
    // pbias row, stored at C + ob * c_bs.  res_div > 1: the residual of output batch ob is read from res batch
    // ob / res_div at stride res_bs (a per-segment residual shared by its P prompts).
    const float* pbias = nullptr;
    int pfold = 1, res_div = 1;
    int64_t res_bs = 0;
    // LayerNorm over each output row (epilogue flag F_LN; gemm3 with one N tile per row, N == BN): the row's values
    // v are stored as (v - mean) * rstd * ln_w[n] + ln_b[n] (eps 1e-5, two-pass statistics as layernorm_kernel)
    const float* ln_w = nullptr;
    const float* ln_b = nullptr;
    // with an f32 C and a residual (rowln.hip, N = 512): C keeps the rows, ln_out gets their LayerNorm as bf16
    void* ln_out = nullptr;
    // split-K tail (gemm5, residual-stream epilogues, dense rows; gemm5.hip): scratch for the f32 partial tiles of
    // the last, partial round of tiles (SK_WS_BYTES per stream).  Null: no split.  sk_full / sk_S are filled by the
    // launcher (tiles computed whole, K pieces per tail tile).
    float* sk_ws = nullptr;
    int sk_full = 0, sk_S = 1;
};

// per-stream scratch of the split-K tail: at most SK_MAX_PIECES f32 partial tiles of 256 x 256
constexpr int SK_MAX_PIECES = 320;
constexpr size_t SK_WS_BYTES = (size_t)SK_MAX_PIECES * 256 * 256 * 4;

// Algorithmic work of one launch (prof.h): 2 M N K flops; bytes = unique activations read once + packed weights +
// outputs (+ residual read).  mode 1 weights are bf16, mode 0 f32.
inline void gemm_work(const GemmDesc& d, int mode, double& flops, double& bytes) {
    const double M = (double)d.nb * d.H_out * d.W;
    flops = 2.0 * M * d.N * d.K;
    const double nout = d.act == ACT_GLU ? d.N / 2 : d.N;
    bytes = (double)d.nb * d.H_in * d.W * d.C_in * (d.a_bf16 ? 2 : 4) + (double)d.N * d.K * (mode == 1 ? 2 : 4);
    if (d.store) bytes += M * nout * (d.c_bf16 ? 2 : 4) * (d.pfold > 1 ? d.pfold : 1);
    if (d.res) bytes += M * nout * (d.res_bf16 ? 2 : 4) / (d.res_div > 1 ? d.res_div : 1);
    if (d.pbias) bytes += (double)d.nb * (d.pfold > 1 ? d.pfold : 1) * d.N * 4;
}

// mode: 0 = exact fp32 (v_mfma_f32_16x16x4_f32), 1 = bf16 (v_mfma_f32_16x16x32_bf16, fp32 accumulate)
int gemm_launch(const GemmDesc& d, int mode, hipStream_t s);
// the shapes the residual projection + LayerNorm pass (rowln.hip, GemmDesc::ln_out) handles
bool rowln_supported(const GemmDesc& d);
// d with its fast-division constants filled (every kernel launcher passes this copy to the kernel)
inline GemmDesc with_fastdiv(const GemmDesc& d) {
    GemmDesc e = d;
    e.fd_w = make_fastdiv((uint32_t)d.W);
    e.fd_h = make_fastdiv((uint32_t)d.H_out);
    e.fd_hw = make_fastdiv((uint32_t)d.H_out * (uint32_t)d.W);
    return e;
}

}  // namespace athd
