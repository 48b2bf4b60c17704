// Kernel micro-benchmark entry points (test tooling, not part of libathd.so): plain-C launchers for the GEMM and
// attention kernels on caller-provided device buffers, used by tools/kbench.py to time variants against
// torch/hipBLASLt on identical shapes in one process.
#include "../audio-to-sheet-music_amd/csrc/gemm.h"
#include "../audio-to-sheet-music_amd/csrc/attn.h"
#include <hip/hip_runtime.h>

using namespace athd;
namespace athd {
extern int g_attn_variant;
int gemm2_launch(const GemmDesc& d, hipStream_t s);
int gemm3_launch(const GemmDesc& d, hipStream_t s, int variant);
int gemm4_launch(const GemmDesc& d, hipStream_t s);
int gemm5_launch(const GemmDesc& d, hipStream_t s);
int gemm5_probe_launch(const GemmDesc& d, hipStream_t s, int probe);
}

extern "C" {
// out[M][N] = act(A[M][K] @ W[N][Kp]^T + bias); variant 1 = v1 kernel, 2 = v2 kernel
int kb_gemm(int variant, const void* A, int a_bf16, const void* W, const float* bias, void* C, int c_bf16, int M, int N,
            int K, int Kp, int act, void* stream) {
    GemmDesc d;
    d.A = A; d.a_bf16 = a_bf16; d.nb = 1; d.H_in = M; d.W = 1; d.C_in = K; d.a_ld = K; d.H_out = M;
    d.Wp = W; d.N = N; d.K = K; d.Kp = Kp; d.bias = bias; d.C = C; d.c_bf16 = c_bf16; d.H_out_total = M; d.ldo = N;
    d.act = act;
    if (variant >= 40 && N % 256 != 0) return -1;   // gemm4 reads whole 256-row weight tiles; W here has N rows
    if (variant == 40) return gemm4_launch(d, (hipStream_t)stream);
    if (variant == 50) return gemm5_launch(d, (hipStream_t)stream);
    if (variant > 50 && variant < 58) return gemm5_probe_launch(d, (hipStream_t)stream, variant - 50);
    if (variant == 41) { d.store = 0; return gemm4_launch(d, (hipStream_t)stream); }   // timing probe: no C stores
    if (variant == 42) { d.bias = nullptr; return gemm4_launch(d, (hipStream_t)stream); }   // timing probe: no bias
    if (variant == 2) return gemm2_launch(d, (hipStream_t)stream);
    if (variant >= 30) return gemm3_launch(d, (hipStream_t)stream, variant - 30);
    return gemm_launch(d, 1, (hipStream_t)stream);
}
// residual-stream GEMM as the transformer's out_proj / linear2 run it: C (f32, in place) = C + scale * (A @ W^T + bias),
// with stats != NULL also {sum, sumsq} of the result (one group: nb = 1)
int kb_gemm_res(int variant, const void* A, const void* W, const float* bias, float* C, const float* scale,
                double* stats, int M, int N, int K, int Kp, void* stream) {
    GemmDesc d;
    d.A = A; d.a_bf16 = 1; d.nb = 1; d.H_in = M; d.W = 1; d.C_in = K; d.a_ld = K; d.H_out = M;
    d.Wp = W; d.N = N; d.K = K; d.Kp = Kp; d.bias = bias; d.C = C; d.c_bf16 = 0; d.H_out_total = M; d.ldo = N;
    d.res = C; d.res_scale = scale; d.stats = stats;
    if (variant == 50) return N % 256 == 0 ? gemm5_launch(d, (hipStream_t)stream) : -1;
    if (variant >= 30) return gemm3_launch(d, (hipStream_t)stream, variant - 30);
    return gemm_launch(d, 1, (hipStream_t)stream);
}
// ConvT residue-pair GEMM as the decoder runs it (kept mode, pair 0): A (nb, H, W, Cin) bf16, 2 taps (rows u-1, u),
// N = 2*Cout columns split at Cout, only the high half stored into slot 2u of a (nb, 2H, W, Cout) bf16 output,
// GroupNorm statistics per nb.
int kb_convt(int variant, const void* A, const void* W, const float* bias, void* C, double* stats, int nb, int H,
             int Wd, int Cin, int Cout, int Kp, void* stream) {
    GemmDesc d;
    d.A = A; d.a_bf16 = 1; d.nb = nb; d.H_in = H; d.W = Wd; d.C_in = Cin; d.a_ld = Cin;
    d.ntaps = 2; d.in_stride = 1; d.in_off = -1; d.dil = 1; d.H_out = H;
    d.Wp = W; d.N = 2 * Cout; d.K = 2 * Cin; d.Kp = Kp; d.bias = bias;
    d.C = C; d.c_bf16 = 1; d.ldo = Cout; d.stats = stats; d.col_split = Cout;
    d.H_out_total = 2 * H; d.o_stride = 2; d.o_off = 0; d.hi_row_off = 0; d.store_mask = 2;
    if (variant == 2) return gemm2_launch(d, (hipStream_t)stream);
    if (variant >= 30) return gemm3_launch(d, (hipStream_t)stream, variant - 30);
    return gemm_launch(d, 1, (hipStream_t)stream);
}
// four-residue ConvT GEMM as the decoder runs it for level 2 (kept mode): K = rows u-1 | u | u+1, N = 4*Cout split
// at Cout, residues 1, 2 stored into slots 2u, 2u+1; kskip = 1 sets k_blk (zero-block skip)
int kb_convt_quad(int variant, int kskip, const void* A, const void* W, const float* bias, void* C, double* stats,
                  int nb, int H, int Wd, int Cin, int Cout, int Kp, void* stream) {
    GemmDesc d;
    d.A = A; d.a_bf16 = 1; d.nb = nb; d.H_in = H; d.W = Wd; d.C_in = Cin; d.a_ld = Cin;
    d.ntaps = 3; d.in_stride = 1; d.in_off = -1; d.dil = 1; d.H_out = H;
    d.Wp = W; d.N = 4 * Cout; d.K = 3 * Cin; d.Kp = Kp; d.bias = bias;
    d.C = C; d.c_bf16 = 1; d.ldo = Cout; d.stats = stats; d.col_split = Cout; d.hi_row_off = 1;
    d.H_out_total = 2 * H; d.o_stride = 2; d.o_off = -1; d.store_mask = 6;
    if (kskip) d.k_blk = Cin;
    if (kskip == 2) d.store_mask = 0;       // probe: no stores
    if (kskip == 3) d.stats = nullptr;      // probe: no statistics
    return gemm3_launch(d, (hipStream_t)stream, variant);
}
// variant: 0 = attn32<2>, 1 = attn_bf16 (16x16x32), 2 = attn32<3>; prescaled = Q already x ATTN_Q_PRESCALE
int kb_attn(int variant, int prescaled, const void* qkv, int nb, int N, void* out, void* stream) {
    g_attn_variant = variant;
    AttnDesc a;
    a.nb = nb; a.Nq = N; a.Nk = N; a.heads = 8; a.scale = prescaled ? ATTN_SCALE_PRESCALED : 0.125f;
    a.Q = qkv; a.q_bf16 = 1; a.q_bs = (int64_t)N * 1536; a.q_ld = 1536; a.q_off = 0;
    a.K = qkv; a.k_bf16 = 1; a.k_bs = (int64_t)N * 1536; a.k_ld = 1536; a.k_off = 512;
    a.V = qkv; a.v_bf16 = 1; a.v_bs = (int64_t)N * 1536; a.v_ld = 1536; a.v_off = 1024;
    a.O = out; a.o_bf16 = 1; a.o_bs = (int64_t)N * 512; a.o_ld = 512;
    return attn_launch(a, 1, (hipStream_t)stream);
}
}

// probe: lane -> elements returned by ds_read_b64_tr_b16 with the attention kernel's addressing
typedef short kb_v4i16 __attribute__((ext_vector_type(4)));
__global__ void kb_tr_kernel(short* out) {
    __shared__ __attribute__((aligned(16))) short t[64 * 72];
    for (int i = threadIdx.x; i < 64 * 72; i += 64) t[i] = (short)((i / 72) * 256 + (i % 72));
    __syncthreads();
    const int lane = threadIdx.x, g = lane >> 4, c16 = lane & 15;
    const short* base = &t[(4 * g + (c16 >> 2)) * 72 + 4 * (c16 & 3)];
    kb_v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) kb_v4i16*)base);
    for (int j = 0; j < 4; ++j) out[4 * lane + j] = v[j];
}
extern "C" int kb_tr(void* out) {
    hipLaunchKernelGGL(kb_tr_kernel, dim3(1), dim3(64), 0, 0, (short*)out);
    return (int)hipDeviceSynchronize();
}
