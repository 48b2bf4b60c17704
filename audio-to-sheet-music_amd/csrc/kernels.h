// Launchers for the non-GEMM kernels of the hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm.h"

namespace athd {

// demucs pad1d(reflect) plan for HTDemucs._spec: padded index p -> original sample (or 0)
struct PadPlan {
    int64_t L;          // original length
    int64_t left;       // reflect pad applied to the zero-extended signal
    int64_t ext_left;   // zero extension on the left (only when L <= max pad)
    int64_t Lx;         // zero-extended length
};

// tconv0.hip: time encoder level-0 conv + GELU on the raw waveform, normalisation on load; w = [48][tap*2 + c] f32
void tconv0_launch(const float* wav, int nb, int64_t T, int64_t Lo, const float* w, const float* bias,
                   const float* tnorm, void* out, int out_bf16, hipStream_t s);

// spectral.hip
// specT [b][t][f][4] (frame-major: level-0 encoder and iSTFT) + per-batch {sum, sumsq} of it into stats (zeroed)
// tw64 != nullptr (f32 parity mode): the FFT runs in double (spectral.hip)
void stft_launch(const float* wav, int nb, int64_t T, const PadPlan& pp, int Tspec, const float2* tw,
                 const double2* tw64, const float* win, float* specT, double* stats, hipStream_t s);
// fo: FO^T [item][t][row][2] (fdec_tail_kernel output); specT as above
// fused: mask + inverse FFT + overlap-add + envelope + time branch (round 1's frame tensor is gone); part:
// istft_ola_part_floats(NI, Tspec) floats of boundary partial sums
void istft_ola_launch(const float* fo, int NI, int Tspec, int P, int64_t T, const float* spec, const float2* tw,
                      const double2* tw64, const float* win, const float* win2, const float* xt2, const float* tnorm,
                      float* out, float* part, hipStream_t s);
int istft_ola_nwg(int Tspec);
inline int64_t istft_ola_part_floats(int64_t NI, int Tspec) { return NI * istft_ola_nwg(Tspec) * 2 * 3 * 1024 * 2; }

// norm.hip
// per-batch {sum, sumsq} (double) of x[b][0..n)
void stats_launch(const float* x, int nb, int64_t n, double* stats, hipStream_t s);
// input normalisation: per batch (mean, 1/(1e-5 + unbiased std)) as floats {mean, inv} and (mean, std)
void input_norm_params_launch(const double* stats, int nb, int64_t n, float* mean_inv, float* mean_std,
                              hipStream_t s);
// h[nb][L*H] = GELU(GN(h)) in place (GroupNorm(1,H), stats over L*H per nb)
void gn_gelu_launch(float* h, int nb, int64_t per_batch, int H, const double* stats, const float* w,
                    const float* b, hipStream_t s, bool fast);
// out[nb][per_batch] (bf16) = GELU_fast(GN(h)); per_batch % 8 == 0, H % 8 == 0
void gn_gelu_bf16_launch(const float* h, uint16_t* out, int nb, int64_t per_batch, int H, const double* stats,
                         const float* w, const float* b, hipStream_t s);
// gn_gelu_bf16 on [nb][L][H] (H = 24 / 48, L >= 64) plus the following 1x1 conv's GroupNorm {sum, sumsq} per nb
// into st_y from its moments `gram` (ctx.h conv1x1_moments, bf16-rounded weights); -1 if the shape is not covered
int gn_gelu_mom_launch(const float* h, uint16_t* out, int nb, int64_t L, int H, const double* stats, const float* w,
                       const float* b, const float* gram, double* st_y, hipStream_t s);
void gn_gelu_bf16in_launch(const uint16_t* h, uint16_t* out, int nb, int64_t per_batch, int H, const double* stats,
                           const float* w, const float* b, hipStream_t s);
// x[nb][N][C] = GN(x) in place
void gn_apply_launch(float* x, int nb, int64_t N, int C, const double* stats, const float* w, const float* b,
                     hipStream_t s);
// LayerNorm over C (384 or 512) of rows x[nb*N][C]; optional pending GroupNorm applied first (and written back
// to x), optional positional table pos[N][C] added after the norm, output f32 or bf16 (may alias x if f32).
struct LnDesc {
    float* x = nullptr; int nb = 1; int64_t N = 0; int C = 512;
    const float* w = nullptr; const float* b = nullptr;
    const double* gn_stats = nullptr; const float* gn_w = nullptr; const float* gn_b = nullptr;
    int gn_writeback = 1;    // 0: the pending GroupNorm is applied in registers only (x keeps its raw values; the next
                             // reader of x as a residual applies it again: GemmDesc::res_gn_*, bf16 mode)
    const float* pos = nullptr;
    void* out = nullptr; int out_bf16 = 0;
    // optional second affine of the same normalised rows -> out2 (C = 512, bf16, no pos): the cross layers' two
    // norms of one input (forward.cpp), one read of x instead of two
    const float* w2 = nullptr; const float* b2 = nullptr; void* out2 = nullptr;
};
// the LayerNorm pass can apply a pending GroupNorm in registers only (gn_writeback = 0): the C = 512 row kernel, with
// out2 (if any) fused into the same pass (bf16 output, no positional rows)
inline bool ln_lazy_gn_ok(const LnDesc& d) { return d.C == 512 && (!d.out2 || (d.out_bf16 && !d.pos)); }

void layernorm_launch(const LnDesc& d, hipStream_t s);
// y = bf16(x), n % 8 == 0 (round to nearest even)
void to_bf16_launch(const float* x, uint16_t* y, int64_t n, hipStream_t s);
// a[item] = out_proj(in_v(v_proj(text[item])))   (TextCrossAttention closed form, 384 <- 512), and the prompt's
// out_mlp row biases c0[item] = W0 a + b0, c2[item] = a + b2 (c0 == nullptr: a only)
void text_vec_launch(const float* text, int NI, int P, int text_per_item, const float* maT, const float* ma,
                     const float* mcT, const float* mc, const float* b2, float* a, float* c0, float* c2, hipStream_t s);
// decoder merge: out[item][ho][w][c] = resize_H(act(GN(src)))[ho][w][c] + 0.1 * resize_H(skip[item/P][..][c])
struct MergeDesc {
    const void* src = nullptr; int src_bf16 = 0; int H_src = 0;   // logical ConvT output rows
    int kept = 0;                                // src holds only rows 4d+1, 4d+2 as slots 2d, 2d+1
    int C = 0;                                   // channels of src and out
    const double* stats = nullptr; int64_t gn_count = 0; const float* gn_w = nullptr; const float* gn_b = nullptr;
    const void* skip = nullptr; int skip_bf16 = 0; int H_skip = 0; int C_skip = 0; int P = 1;
    void* out = nullptr; int out_bf16 = 0; int H_out = 0; int W = 1; int NI = 1;
    const float* proj_w = nullptr; const float* proj_b = nullptr;   // optional 1x1 C(=4) -> 2 projection
    int fast_gelu = 0;                            // bf16 mode: branch-free erf
};
int dec_merge_launch(const MergeDesc& d, hipStream_t s);   // -1: P > 256 or NI % P != 0
// fdec_lr.hip: FreqDecoder level 1 from the 32-row level-0 output (re-associated ConvT; see fdec_lr.hip).
// Z [NI][Hs][W][8*Co] = W_k S[j] per tap k; Zs [NI/P][Hk][W][8*Co] = W_k skip3[m]; skip [NI/P][H_skip][W][C_skip].
// per output-row step v of the level-1 low-rank decoder (fdec_lr.hip): the resize lerps of the Z rows (Hs -> Hd), the
// skip-projection rows (Hk -> Hd) and, for row dd = v - 1, the skip rows (H_skip -> Hd); flags: bit 0 / 1 / 2 = the
// z / k / j rows differ from step v - 1 (always set at v = 0)
struct LrStep {
    float lz, lk, lj;
    uint32_t zk;        // i0z | i1z << 8 | i0k << 16 | i1k << 24
    uint32_t jj;        // i0j | i1j << 16
    uint32_t flags;
    uint32_t pad[2];
};
struct LowRankDesc {
    const LrStep* steps = nullptr;                // Hd + 1 entries (fdec_lr_steps_launch)
    const void* Z = nullptr; const void* Zs = nullptr; int z_bf16 = 0;
    int z_taps = 8;                               // Z rows: [w][8 taps][Co], or 4 = taps 0, 3, 4, 7 as [w][Co / 16][4][16]
                                                  // (merge pass only; written by fdec1_gram_kernel)
    int Hs = 32, Hk = 8, Hd = 0, W = 0, Co = 0, P = 1, NI = 0;
    const float* bias = nullptr;                  // ConvT bias [Co]
    double* stats = nullptr;                      // per item {sum, sumsq} over the 4*Hd ConvT rows
    const float* gn_w = nullptr; const float* gn_b = nullptr; int fast_gelu = 0;
    const void* skip = nullptr; int skip_bf16 = 0; int H_skip = 0; int C_skip = 0;
    void* out = nullptr; int out_bf16 = 0;        // [NI][Hd][W][Co]
    // fused passes (fdec1f.hip): the GEMM operands of Z instead of Z itself
    const void* S = nullptr;                      // bf16 [NI][Hs][W][Ci]
    const void* Wt = nullptr; int w_ld = 0;       // bf16 tap weights [8 Co][w_ld] (row k Co + c)
    int Ci = 0;
    void* z4 = nullptr;                           // fdec1_gram_kernel also writes the merge pass's 4-tap Z here (bf16)
};
int fdec_lr_steps_launch(LrStep* steps, int Hd, int Hs, int Hk, int H_skip, hipStream_t s);
int fdec_lr_stats_launch(const LowRankDesc& d, hipStream_t s);
int fdec_lr_merge_launch(const LowRankDesc& d, hipStream_t s);
// fdec1f.hip: the statistics pass as Gram matrices of Z tiles computed in LDS (bf16 mode, Co = 96, Ci = 192, Hs = 32,
// Hk = 8, Hd > 32); gram: fdec1_gram_floats(NI, W) floats, gq: fdec1_gram_q_doubles() doubles of workspace
bool fdec1_gram_supported(const LowRankDesc& d);
int64_t fdec1_gram_floats(int64_t NI, int W);
int64_t fdec1_gram_q_doubles();
int fdec1_gram_launch(const LowRankDesc& d, float* gram, double* gq, hipStream_t s);
// fenc_row.hip: a whole narrow frequency-encoder level (conv + GELU + DConv + rewrite GLU) per (b, f) row, bf16 mode
constexpr int FR_MT_MAX = 17;        // T <= 272 positions (16-position tiles)
struct FencRowDesc {
    const void* in = nullptr;          // level 0: specT f32 [B][T][Fin][4]; level 1: bf16 [B][Fin][T][Cin]
    const float* a_norm = nullptr;     // level 0: per batch {sub, div}
    int B = 0, Fin = 0, Fout = 0, T = 0;
    const uint16_t* wc = nullptr; int wc_ld = 0; const float* bc = nullptr;        // conv [C][8 Cin]
    const uint16_t* w3[2] = {nullptr, nullptr}; int w3_ld = 0;                    // conv3 [16][3C] (rows >= C/8 zero)
    const float* b3[2] = {nullptr, nullptr};
    const float* g1w[2] = {nullptr, nullptr}; const float* g1b[2] = {nullptr, nullptr};
    const uint16_t* w1[2] = {nullptr, nullptr}; int w1_ld = 0;                    // 1x1 [2C][C/8] GLU-interleaved
    const float* b1[2] = {nullptr, nullptr};
    const float* g2w[2] = {nullptr, nullptr}; const float* g2b[2] = {nullptr, nullptr};   // packed order
    const float* gram[2] = {nullptr, nullptr};    // 1x1 moments (ctx.h conv1x1_moments, bf16-rounded weights)
    const float* scale[2] = {nullptr, nullptr};
    const uint16_t* wr = nullptr; int wr_ld = 0; const float* br = nullptr;      // rewrite [2C][C] GLU-interleaved
    const float* row_add = nullptr;    // level 0: freq embedding [Fout][C]
    uint16_t* out = nullptr;           // [B][Fout][T][C] bf16
    uint16_t* out4 = nullptr;          // level 0 (optional): channels 0..3 of out, [B][Fout][T][4] (decoder skip copy)
};
bool fenc_row_supported(int cin, int c, int T);
int fenc_row_launch(const FencRowDesc& d, int cin, int c, hipStream_t s);
// dec_last.hip: last decoder level (ConvT 48 -> 4 + resize + 0.1 skip + 1x1 projection to 2, folded) of either branch.
//   freq: in [NI][H][W][48] -> out FO^T [NI][W][H][2] (H = W = Tspec); fold = [Am | A0 | Ap] (3 x [2][48]), P b + pb (2),
//         0.1 P (8); skip [NI/P][H_skip][W][C_skip] (channels 0..3 used)
//   time: in [NI][H][48] (H = Lin) -> out xt2 [NI][T][2] = time_out(...) incl. bias; fold = Q_k (8 x [2][48]), P b (2),
//         tb (2), 0.1 P (8); skip [NI/P][H_skip][C_skip]
struct DecLastDesc {
    const void* in = nullptr; int in_bf16 = 0;
    int NI = 0, P = 1, H = 0, W = 1;
    int64_t T = 0;
    const float* fold = nullptr;
    const void* skip = nullptr; int skip_bf16 = 0; int H_skip = 0; int C_skip = 0;
    float* out = nullptr;
    // dec_tail: the level-2 merge (GroupNorm -> GELU -> resize -> + 0.1 resize(skip2[:, :48])) fused in front, so the
    // 48-channel input x is computed from the level-2 ConvT output g instead of read from `in`:
    //   freq: g = kept slots [NI][2H][W][48] (logical rows 4d+1, 4d+2); time: g = [NI][Hg][48] (Hg = 4 L2 rows)
    const void* g = nullptr; int g_bf16 = 0; int Hg = 0;
    const double* stats = nullptr; int64_t gn_count = 0; const float* gn_w = nullptr; const float* gn_b = nullptr;
    int fast_gelu = 0;
    const void* skip2 = nullptr; int skip2_bf16 = 0; int H_skip2 = 0; int C_skip2 = 0;
};
int fdec_last_launch(const DecLastDesc& d, hipStream_t s);
int tdec_last_launch(const DecLastDesc& d, hipStream_t s);
int fdec_tail_launch(const DecLastDesc& d, hipStream_t s);
bool tdec_tail_supported(const DecLastDesc& d);     // 4 H == T and every block's g rows fit its LDS tile
int tdec_tail_launch(const DecLastDesc& d, hipStream_t s);
// convt4.hip: decoder level-2 ConvTranspose (96 -> 48, k8 s4 p2) over rows (b, u, w) of x [nb][H][W][96] bf16, all
// four residues in one pass (bf16 mode).  w: [4 x 48 rows][192] bf16, row rho*48 + co, K = the residue pair's two
// input rows (u-1 | u for rho 0/1, u | u+1 for rho 2/3) x 96 channels; bias [48].  keep = 1: residues 1, 2 stored as
// rows 2t, 2t+1 of out [nb][2H][W][48]; keep = 0: out [nb][4H][W][48].  stats: per item fp64 {sum, sumsq} over all
// four residues (accumulated).
struct ConvT4Desc {
    const uint16_t* x = nullptr;
    const uint16_t* w = nullptr;
    const float* bias = nullptr;
    uint16_t* out = nullptr;
    double* stats = nullptr;
    int nb = 0, H = 0, W = 1, keep = 0;
    uint32_t M = 0;                       // filled by convt4_launch
    FastDivU fd_w, fd_h, fd_hw;           // filled by convt4_launch
};
bool convt4_supported(int cin, int cout, int64_t nb, int64_t H, int64_t W);
int convt4_launch(const ConvT4Desc& d, hipStream_t s);
// dconv.hip: one DConv layer (conv3 -> GN -> GELU -> 1x1 -> GN -> GLU -> LayerScale -> residual) for C in {48, 96}
// x: [nb][L][C] f32 or bf16 (x_bf16), updated in place; h: [nb][L][C/8] f32 scratch
// dconv.hip, bf16 mode, MFMA passes (C = 48, 96, 192, 384): the DConv 1x1 apply x += scale * GLU(GN(W1 hb + b1))
// (hb [M][HS] with HS = C/8, or 16 for C = 48, 96; x [M][C]; GroupNorm groups of L rows); -1 if the shape is not
// covered.  With rw (C = 48, 96) the updated rows are not stored: the encoder layer's rewrite out = GLU(Wr x + br)
// runs on them in registers (rw: [2C][kp] GLU-interleaved rows in the K order of ctx.h rewrite_perm).
struct DcRewrite {
    const uint16_t* w;
    int kp;
    const float* bias;
    uint16_t* out;     // [M][C] bf16
    uint16_t* c4;      // optional [M][4]
};
// conv3 (C -> C/8, 3 taps at dilation dil, zero padding at each group's ends) + GroupNorm {sum, sumsq} of h per group
// of L rows; x bf16 [M][C], h f32 [M][HF] (HF = C/8, or 8 for C = 48); -1 if the shape is not covered
int dconv_conv3_launch(const uint16_t* x, const uint16_t* w, int kp, const float* bias, float* h, double* st,
                       int64_t M, int64_t L, int C, int dil, hipStream_t s);
int dconv_apply_launch(const uint16_t* hb, const uint16_t* w, int kp, const float* bias, const double* st,
                       const float* gn_w, const float* gn_b, const float* scale, uint16_t* x, int64_t M, int64_t L,
                       int C, hipStream_t s, const DcRewrite* rw = nullptr);
int dconv_small_launch(void* x, int x_bf16, float* h, int64_t nb, int64_t L, int C, int dil, const float* w3,
                       const float* b3, const float* g1w, const float* g1b, const float* w1, const float* b1,
                       const float* gram1, const float* g2w, const float* g2b, const float* scale, double* st_h,
                       double* st_y, hipStream_t s, bool fast);
// (B, 2, T) -> (B, T, 2)
void wav_interleave_launch(const float* wav, int nb, int64_t T, float* out, hipStream_t s);
// positional tables of the cross-transformer (computed on device with the fp32 op order of demucs)
void pos2d_launch(float* out, int Fr, int T1, int C, hipStream_t s);   // out[(f*T1+t)][C]
void pos1d_launch(float* out, int T2, int C, hipStream_t s);           // out[t][C]

// track.hip: window overlap-add of test_inference.py:92-141 (mode 0) and benchmark.py:155-204 (mode 1, weighted;
// wsum != nullptr: unnormalised partial span + weight sums), sdr_loss / sisdr_loss (src/loss.py:9-68)
int ola_launch(const float* win, int64_t L, int64_t chunk, int64_t overlap, int S, int64_t k0, int64_t k1, float* out,
               hipStream_t s, int mode = 0, float* wsum = nullptr);
int ola_normalize_launch(float* out, const float* wsum, int rows, int64_t n, hipStream_t s);
int sdr_launch(const float* est, const float* tgt, int64_t rows, int64_t n, double* sums, float* out, hipStream_t s);
int sisdr_launch(const float* est, const float* tgt, int64_t rows, int64_t n, double* scratch, float* out,
                 hipStream_t s);

}  // namespace athd
