// Private: athd context (packed device weights) shared by athd_api.cpp and forward.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "prof.h"

namespace athd {

struct HostT {
    std::vector<float> v;
    std::vector<int64_t> shape;
};

struct GemmW {
    void* w = nullptr;
    float* bias = nullptr;
    int N = 0, K = 0, Kp = 0;
};

struct DConvW {
    GemmW c3[2], c1[2];
    GemmW c3p[2];           // bf16 mode, C <= 96: conv3 with its C/8 rows zero-padded to 16 (fenc_row.hip MFMA tile)
    float *g1w[2], *g1b[2], *g2w[2], *g2b[2], *scale[2];
    // natural-order fp32 copies for the VALU kernels of the narrow levels (C <= 96): conv3 [H][3C] (tap-major k),
    // 1x1 [2C][H], its bias and GroupNorm affine
    float *w3f[2] = {nullptr, nullptr}, *w1f[2] = {nullptr, nullptr}, *b1f[2] = {nullptr, nullptr};
    float *g2wf[2] = {nullptr, nullptr}, *g2bf[2] = {nullptr, nullptr};
    // moments of the 1x1 conv for its GroupNorm statistics (dconv.hip c1stat): G = W^T W [H][H], v = W^T b [H],
    // ws = W^T 1 [H], sum b, sum b^2 (so sum_n y_n and sum_n y_n^2 of y = W h + b come from h alone)
    float* gram1[2] = {nullptr, nullptr};
    float* gram1b[2] = {nullptr, nullptr};   // the same from the bf16-rounded weights (fenc_row.hip, bf16 mode)
};

struct EncW {
    int cin = 0, cout = 0;
    GemmW conv, rewrite;
    GemmW rewrite_perm;            // bf16 mode, C = 48, 96: rewrite in the K order of the fused DConv apply (dconv.hip)
    float* conv_f32 = nullptr;     // time level 0 only: [cout][tap * cin + ci] fp32 (tconv0.hip)
    DConvW dc;
};

struct TLayerW {
    bool cross = false;
    GemmW qkv, q, kv, out, l1, l2;
    float *n1w, *n1b, *n2w, *n2b, *n3w = nullptr, *n3b = nullptr, *now, *nob, *g1, *g2;
};

struct DecW {
    int cin = 0, cout = 0;
    GemmW pair[2];          // ConvTranspose residue pairs {0,1} (taps u-1,u) and {2,3} (taps u,u+1), N = 2*cout
    GemmW quad;             // levels 2: all four residues in one GEMM, rows [rho * cout + co], K = [row u-1 | u | u+1]
    uint16_t* ct4w = nullptr;   // level 2, bf16 mode: [rho * cout + co][2 cin] = the residue pair's two rows (convt4.hip)
    float* ct4b = nullptr;      //   and the bias [cout]
    GemmW taps;             // freq level 1 only: every tap as its own column block, N = 8*cout, K = cin (fdec_lr.hip)
    float* bias = nullptr;  // freq level 1 only: ConvT bias [cout]
    float *gnw = nullptr, *gnb = nullptr;
};

}  // namespace athd

namespace athd {
inline uint16_t host_f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// Moments of a 1x1 conv W [N][H] (row-major), b [N] for GroupNorm statistics from its input alone:
// [G = W^T W (H x H) | v = W^T b (H) | ws = W^T 1 (H) | sum b | sum b^2], accumulated in fp64; round_bf16: from the
// bf16-rounded weights the MFMA kernels multiply with
inline std::vector<float> conv1x1_moments(const std::vector<float>& w, const std::vector<float>& b, int N, int H,
                                          bool round_bf16) {
    std::vector<double> g((size_t)H * H + 2 * H + 2, 0.0);
    auto wv = [&](int n, int j) -> double {
        const float x = w[(size_t)n * H + j];
        if (!round_bf16) return x;
        const uint32_t u = (uint32_t)host_f2bf(x) << 16;
        float r;
        std::memcpy(&r, &u, 4);
        return r;
    };
    for (int n = 0; n < N; ++n) {
        const double bn = b[n];
        for (int j = 0; j < H; ++j) {
            const double wj = wv(n, j);
            for (int k = 0; k < H; ++k) g[(size_t)j * H + k] += wj * wv(n, k);
            g[(size_t)H * H + j] += bn * wj;
            g[(size_t)H * H + H + j] += wj;
        }
        g[(size_t)H * H + 2 * H] += bn;
        g[(size_t)H * H + 2 * H + 1] += bn * bn;
    }
    return std::vector<float>(g.begin(), g.end());
}
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t rup(int64_t a, int64_t b) { return cdiv(a, b) * b; }
constexpr int ENC_CH[4] = {48, 96, 192, 384};
constexpr int DEC_CH[5] = {384, 192, 96, 48, 4};
// ConvTranspose (k8 s4 p2) residue classes: output row 4u+rho = taps in rows u+in_off, u+in_off+1 with kernel
// indices {k0, k1}
constexpr int RES_OFF[4] = {-1, -1, 0, 0};
constexpr int RES_K0[4] = {6, 7, 4, 5};
constexpr int RES_K1[4] = {2, 3, 0, 1};

// Bump allocator over the caller's workspace (or sizing pass when base == nullptr).
struct Arena {
    char* base = nullptr;
    size_t off = 0;
    template <typename T>
    T* take(int64_t n) {
        size_t bytes = (size_t)rup((int64_t)(n * (int64_t)sizeof(T)), 256);
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += bytes;
        return p;
    }
};
}  // namespace athd

using namespace athd;

struct athd_ctx {
    int device = 0;
    // second stream + fork/join events: the transformer's time branch runs beside the frequency branch (forward.cpp)
    hipStream_t s_time = nullptr;
    hipEvent_t ev_f = nullptr, ev_t = nullptr;
    int mode = 1;
    // (segment, prompt) items per decode chunk (athd_set_decode_items): the decoder's workspace scales with it
    int64_t decode_items = 64;
    bool finalized = false;
    std::string err;
    std::map<std::string, HostT> host;
    std::vector<void*> allocs;
    athd::KProf* prof = nullptr;     // non-null between athd_profile_start / _stop
    athd::KProf prof_done;           // aggregated results of the last profile window

    EncW fenc[4], tenc[4];
    float* femb = nullptr;           // [512][48] = (w * 10) * 0.2
    GemmW up, down, up_t, down_t;
    float *nin_w, *nin_b, *nint_w, *nint_b;
    TLayerW L[5], Lt[5];
    // text cross-attention row vectors (text_vec_kernel): a = Ma t + ma, c0 = W0 a + b0 = Mc t + mc, composed in double
    // at finalize and stored transposed [512][384]; out_mlp.2 bias; norm_out affine
    float *ta_maT, *ta_ma, *ta_mcT, *ta_mc, *ta_m2b, *ta_nw, *ta_nb;
    GemmW mlp0, mlp2;
    DecW fdec[4], tdec[4];
    float *fout_w, *fout_b, *tout_w, *tout_b;
    float* flast = nullptr;          // folded last freq level + freq_out (dec_last.hip)
    float* tlast = nullptr;          // folded last time level + time_out
    float2* tw = nullptr;
    double2* tw64 = nullptr;       // FFT twiddles in double (f32 parity mode, spectral.hip)
    float* win = nullptr;
    float* win2 = nullptr;

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    template <typename T>
    T* dalloc(size_t n) {
        void* p = nullptr;
        if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) return nullptr;
        allocs.push_back(p);
        return (T*)p;
    }
    const HostT& W(const std::string& k) { return host.at(k); }
    bool upload_failed = false;
    void h2d(void* dst, const void* src, size_t bytes) {
        if (!dst || hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess) upload_failed = true;
    }
    float* up_f32(const std::vector<float>& v) {
        float* p = dalloc<float>(v.size());
        h2d(p, v.data(), v.size() * 4);
        return p;
    }
    float* up_key(const std::string& k) { return up_f32(W(k).v); }
    // Pack a [N][K] fp32 host matrix (row-major, k contiguous) into the compute dtype, Kp = roundup(K, 64).  The
    // allocation holds roundup(N, 256) rows, the extra ones zero: a 256-column GEMM tile (gemm5.hip) may read
    // whole tiles of rows past N.
    GemmW up_gemm(const std::vector<float>& w, int N, int K, const std::vector<float>& bias) {
        GemmW g;
        g.N = N;
        g.K = K;
        g.Kp = (int)rup(K, 64);
        const int Nalloc = (int)rup(N, 256);
        if (mode == 1) {
            std::vector<uint16_t> p((size_t)Nalloc * g.Kp, 0);
            for (int n = 0; n < N; ++n)
                for (int k = 0; k < K; ++k) p[(size_t)n * g.Kp + k] = host_f2bf(w[(size_t)n * K + k]);
            void* d = dalloc<uint16_t>(p.size());
            h2d(d, p.data(), p.size() * 2);
            g.w = d;
        } else {
            std::vector<float> p((size_t)Nalloc * g.Kp, 0.f);
            for (int n = 0; n < N; ++n)
                for (int k = 0; k < K; ++k) p[(size_t)n * g.Kp + k] = w[(size_t)n * K + k];
            g.w = up_f32(p);
        }
        g.bias = bias.empty() ? nullptr : up_f32(bias);
        return g;
    }
    // conv weight [Cout][Cin][taps] -> [Cout][tap*Cin + ci]
    GemmW conv_gemm(const std::string& wk, const std::string& bk, int cout, int cin, int taps, bool glu = false) {
        const auto& w = W(wk).v;
        std::vector<float> p((size_t)cout * taps * cin);
        for (int co = 0; co < cout; ++co)
            for (int ci = 0; ci < cin; ++ci)
                for (int t = 0; t < taps; ++t) p[((size_t)co * taps + t) * cin + ci] = w[((size_t)co * cin + ci) * taps + t];
        std::vector<float> b = W(bk).v;
        if (glu) {   // pair order: per 32 packed rows [a(16q..16q+15) | gate(C+16q..)]
            std::vector<float> q(p.size());
            const int K = taps * cin;
            for (int pr = 0; pr < cout; ++pr)
                std::memcpy(&q[(size_t)pr * K], &p[(size_t)glu_src(pr, cout) * K], K * 4);
            p.swap(q);
            b = glu_order(b);
        }
        return up_gemm(p, cout, taps * cin, b);
    }
    static int glu_src(int pr, int n) {
        const int C = n / 2, qq = pr / 32, s = pr % 32;
        return s < 16 ? 16 * qq + s : C + 16 * qq + (s - 16);
    }
    static std::vector<float> glu_order(const std::vector<float>& v) {
        std::vector<float> o(v.size());
        for (size_t i = 0; i < v.size(); ++i) o[i] = v[glu_src((int)i, (int)v.size())];
        return o;
    }
    // rows [row0, row0 + rows) of a [N][K] linear layer; the first `scaled_rows` of them (weights and bias) times
    // `scale` (the attention query prescale, see ATTN_Q_PRESCALE)
    GemmW lin_gemm(const std::string& wk, const std::string& bk, int row0 = 0, int rows = -1, int scaled_rows = 0,
                   float scale = 1.f) {
        const HostT& w = W(wk);
        int N = (int)w.shape[0], K = (int)w.shape[1];
        if (rows < 0) rows = N - row0;
        std::vector<float> p(w.v.begin() + (size_t)row0 * K, w.v.begin() + (size_t)(row0 + rows) * K);
        const auto& bb = W(bk).v;
        std::vector<float> b(bb.begin() + row0, bb.begin() + row0 + rows);
        for (int n = 0; n < scaled_rows && n < rows; ++n) {
            for (int k = 0; k < K; ++k) p[(size_t)n * K + k] *= scale;
            b[n] *= scale;
        }
        return up_gemm(p, rows, K, b);
    }
};

