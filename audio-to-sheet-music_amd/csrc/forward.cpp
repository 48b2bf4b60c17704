// athd forward orchestration: AudioTextHTDemucs.forward (ATHTDemucs_v2.py:250-326) as a sequence of HIP
// kernels on the caller's stream.  Workspace layout is computed by the same code path in a sizing pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/athd.h"
#include "attn.h"
#include "ctx.h"
#include "prof.h"
#include "gemm.h"
#include "kernels.h"

namespace {

struct Dims {
    int64_t B = 0, T = 0;
    int P = 1;
    int Tspec = 0;
    int F[5] = {2048, 512, 128, 32, 8};
    int64_t L[5] = {0, 0, 0, 0, 0};   // L[0] = T, L[i+1] = ceil(L[i]/4)
    int64_t Nf = 0, Nt = 0, Nmax = 0;
    int64_t Bc = 0;                   // samples per decode chunk
    int64_t chunks = 0;
};

Dims make_dims(const athd_ctx* c, int64_t B, int64_t T, int P) {
    Dims d;
    d.B = B;
    d.T = T;
    d.P = P;
    d.Tspec = (int)cdiv(T, 1024);
    d.L[0] = T;
    for (int i = 0; i < 4; ++i) d.L[i + 1] = cdiv(d.L[i], 4);
    d.Nf = 8LL * d.Tspec;
    d.Nt = d.L[4];
    d.Nmax = std::max(d.Nf, d.Nt);
    // (segment, prompt) items per decode chunk; the decoder's buffers scale with it.  Library default 64 (an 18 GB
    // workspace at B=64 x P=4); bench.py sets 256 = the whole bench batch in one chunk (51 GB, sized for the 288 GB
    // of HBM: fewer, larger decoder launches; measured 32 / 64 / 128 / 256 items: 1203 / 1238 / 1263 / 1284
    // segments/s).  ATHD_DECODE_ITEMS overrides the context's setting.
    int64_t items_per_chunk = c ? c->decode_items : 64;
    if (const char* e = std::getenv("ATHD_DECODE_ITEMS")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v > 0) items_per_chunk = v;
    }
    d.Bc = std::max<int64_t>(1, std::min<int64_t>(B, items_per_chunk / P));
    d.chunks = cdiv(B, d.Bc);
    return d;
}

struct Bufs {
    float* specT;
    double* stats;
    int64_t nstats;     // number of double pairs
    float *snorm, *tnorm_div, *tnorm_std;
    // encoder activations: f32 in parity mode, bf16 in throughput mode (Bufs::ea bytes per element)
    void* saved[4];
    void* saved_t[4];
    void* sk4;                        // channels 0..3 of saved[0] / saved_t[0] ([rows][4]): the decoders' level-3 skip
    void* sk4t;
    void* ybuf;
    void* ybuf_t;                     // the time encoder's level buffers (it runs on the second stream)
    float* hbuf_t;
    uint16_t* hbuf_b_t;
    float* hbuf;
    uint16_t* hbuf_b;                 // bf16 mode: GELU(GN(hbuf)) as bf16, the A operand of the wide DConv 1x1 GEMMs
    int ea = 4;
    float *X, *XT;
    void *H[4], *QKV, *O, *F1;
    void *QKVt, *Ot, *F1t;            // the time branch's scratch (it runs on its own stream beside the freq branch)
    float *Gt, *Dt;                   // the time decoder's ConvT / merge buffers (second stream too)
    float *pos2d, *pos1d, *x_enc, *xt_enc;
    uint16_t *x_enc_b, *xt_enc_b;     // bf16 copies (throughput mode): the A operand of text.mlp0
    // decode (per chunk)
    float *avec, *tc0, *tc2;         // per-prompt attention vector and out_mlp row biases (text_vec_kernel)
    float *Yb, *x_cond, *xt_cond;
    void* Hm;
    float* Ybt;         // the time branch's text cross-attention scratch (it runs on the second stream)
    void* Hmt;
    float *G, *D, *FO;
    float* FO2 = nullptr;             // second freq-output buffer (chunks > 1): chunk c's iSTFT reads FO[c & 1] while
                                      // chunk c + 1's decoder writes the other one
    float* ola_part;    // boundary partial sums of the fused iSTFT (spectral.hip)
    LrStep* lrsteps;    // level-1 low-rank decoder step table (fdec_lr.hip)
    float* gram;        // level-1 statistics Gram blocks / quadratic forms (fdec1f.hip, bf16 mode)
    double* gramq;
    void *S, *Z, *Zs;   // freq level 1 re-associated (fdec_lr.hip): per-tap products of the 32 / 8 source rows
    mutable float* xt2 = nullptr;   // time_out(time decoder) of the last decode chunk: D (fused tail) or G (ragged T)
    float* skw[2] = {nullptr, nullptr};   // split-K tail scratch of the freq / time stream (gemm5, GemmDesc::sk_ws)
};

size_t plan(Arena& ar, const Dims& d, Bufs& b, bool actbf) {
    const int64_t B = d.B, Ts = d.Tspec;
    const size_t ab = actbf ? 2 : 4;
    auto act = [&](int64_t n) -> void* { return (void*)ar.take<char>(n * (int64_t)ab); };
    // stats pool
    int64_t ns = 0;
    for (int i = 0; i < 4; ++i) ns += 4 * (B * d.F[i + 1]) + 4 * B;
    ns += 10 * B + 4 * B;
    ns += d.chunks * 6 * d.Bc * d.P;
    b.nstats = ns;
    b.stats = ar.take<double>(2 * ns);
    b.specT = ar.take<float>(B * 2048 * Ts * 4);
    b.snorm = ar.take<float>(2 * B);
    b.tnorm_div = ar.take<float>(2 * B);
    b.tnorm_std = ar.take<float>(2 * B);
    int64_t ymax = 0, hmax = 0, ymax_t = 0, hmax_t = 0;
    for (int i = 0; i < 4; ++i) {
        const int64_t C = ENC_CH[i];
        b.saved[i] = act(B * d.F[i + 1] * Ts * C);
        b.saved_t[i] = act(B * d.L[i + 1] * C);
        const int64_t rows = B * d.F[i + 1] * Ts, rows_t = B * d.L[i + 1];
        ymax = std::max(ymax, rows * C);
        const int64_t hs = C <= 96 ? 16 : C / 8;     // (C = 48, 96: hidden rows padded to 16 for the MFMA passes)
        hmax = std::max(hmax, rows * hs);
        ymax_t = std::max(ymax_t, rows_t * C);
        hmax_t = std::max(hmax_t, rows_t * hs);
    }
    b.sk4 = act(B * d.F[1] * Ts * 4);
    b.sk4t = act(B * d.L[1] * 4);
    b.ybuf_t = act(ymax_t);
    b.hbuf_t = ar.take<float>(hmax_t);
    b.hbuf_b_t = ab == 2 ? ar.take<uint16_t>(hmax_t) : nullptr;
    b.ybuf = act(ymax);
    b.ea = (int)ab;
    b.hbuf = ar.take<float>(hmax);
    b.hbuf_b = ab == 2 ? ar.take<uint16_t>(hmax) : nullptr;
    b.X = ar.take<float>(B * d.Nf * 512);
    b.XT = ar.take<float>(B * d.Nt * 512);
    for (int i = 0; i < 4; ++i) b.H[i] = act(B * d.Nmax * 512);
    b.QKV = act(B * d.Nmax * 1536);
    b.O = act(B * d.Nmax * 512);
    b.F1 = act(B * d.Nmax * 2048);
    b.QKVt = act(B * d.Nmax * 1536);
    b.Ot = act(B * d.Nt * 512);
    b.F1t = act(B * d.Nt * 2048);
    b.pos2d = ar.take<float>(d.Nf * 512);
    b.pos1d = ar.take<float>(d.Nt * 512);
    b.x_enc = ar.take<float>(B * d.Nf * 384);
    b.xt_enc = ar.take<float>(B * d.Nt * 384);
    b.x_enc_b = actbf ? ar.take<uint16_t>(B * d.Nf * 384) : nullptr;
    b.xt_enc_b = actbf ? ar.take<uint16_t>(B * d.Nt * 384) : nullptr;
    // decode chunk
    const int64_t NI = d.Bc * d.P;
    b.avec = ar.take<float>(NI * 384);
    b.tc0 = ar.take<float>(NI * 384);
    b.tc2 = ar.take<float>(NI * 384);
    b.Hm = act(NI * d.Nf * 384);
    b.Yb = ar.take<float>(NI * d.Nf * 384);
    b.Hmt = act(NI * d.Nt * 384);
    b.Ybt = ar.take<float>(NI * d.Nt * 384);
    b.x_cond = ar.take<float>(NI * d.Nf * 384);
    b.xt_cond = ar.take<float>(NI * d.Nt * 384);
    int64_t g = std::max<int64_t>(32 * Ts * 192, 2 * Ts * Ts * 96);
    g = std::max(g, 4 * d.Nt * 192);
    g = std::max(g, 4 * d.L[3] * 96);
    g = std::max(g, 4 * d.L[2] * 48);
    g = std::max(g, d.T * 2);                  // tdec_last output xt2 [NI][T][2]
    b.G = ar.take<float>(NI * g);
    int64_t dm = Ts * Ts * 192;
    dm = std::max(dm, d.L[3] * 192);
    dm = std::max(dm, d.L[2] * 96);
    dm = std::max(dm, d.L[1] * 48);
    b.D = ar.take<float>(NI * dm);
    int64_t gt = std::max<int64_t>(4 * d.Nt * 192, 4 * d.L[3] * 96);
    gt = std::max(gt, 4 * d.L[2] * 48);
    gt = std::max(gt, d.T * 2);
    b.Gt = ar.take<float>(NI * gt);
    int64_t dmt = std::max<int64_t>(d.L[3] * 192, d.L[2] * 96);
    dmt = std::max(dmt, d.L[1] * 48);
    b.Dt = ar.take<float>(NI * dmt);
    b.S = act(NI * 32 * Ts * DEC_CH[1]);
    b.Z = act(NI * 32 * Ts * 8 * DEC_CH[2]);
    b.Zs = act(d.Bc * 8 * Ts * 8 * DEC_CH[2]);
    b.FO = ar.take<float>(NI * Ts * Ts * 2);
    if (d.chunks > 1) b.FO2 = ar.take<float>(NI * Ts * Ts * 2);
    b.ola_part = ar.take<float>(istft_ola_part_floats(NI, (int)Ts));
    b.lrsteps = ar.take<LrStep>(Ts + 1);
    b.gram = actbf ? ar.take<float>(fdec1_gram_floats(NI, (int)Ts)) : nullptr;
    b.gramq = actbf ? ar.take<double>(fdec1_gram_q_doubles()) : nullptr;
    for (int i = 0; i < 2; ++i) b.skw[i] = actbf ? ar.take<float>(SK_WS_BYTES / 4) : nullptr;
    return ar.off;
}

// element offset into an encoder activation buffer (f32 or bf16 storage)
inline void* eoff(void* p, int64_t n, int ea) { return (char*)p + n * ea; }

struct Run {
    athd_ctx* c;
    hipStream_t s;
    const Bufs* b = nullptr;
    int mode;
    bool actbf;
    double* st_next;
    int err = 0;
    std::string what;

    double* stats(int64_t pairs) {
        double* p = st_next;
        st_next += 2 * pairs;
        return p;
    }
    void check(int rc, const char* w) {
        if (rc != 0 && err == 0) {
            err = rc;
            what = w;
        }
    }
    // Linear layer on token rows: out[nb][N][n] = A[nb][N][:] @ W^T (+ epilogue)
    GemmDesc lin(const GemmW& w, const void* A, int a_bf16, int nb, int64_t ntok, int ldA) {
        GemmDesc g;
        g.A = A;
        g.a_bf16 = a_bf16;
        g.nb = nb;
        g.H_in = (int)ntok;
        g.W = 1;
        g.C_in = w.K;
        g.a_ld = ldA;
        g.H_out = (int)ntok;
        g.Wp = w.w;
        g.N = w.N;
        g.K = w.K;
        g.Kp = w.Kp;
        g.bias = w.bias;
        g.H_out_total = (int)ntok;
        g.ldo = w.N;
        return g;
    }
    void gemm(const GemmDesc& g, const char* w) {
        KSite site(w);
        check(gemm_launch(g, mode, s), w);
    }
    // the split-K tail scratch of the stream this Run currently launches on (freq: caller's stream, time: s_time);
    // ATHD_SK=0 turns the split off (read at every call: tests/test_gpu_parity.py::test_splitk_tail_matches_unsplit)
    float* skws() const {
        const char* e = std::getenv("ATHD_SK");
        if (e && e[0] == '0') return nullptr;
        return b ? b->skw[s == c->s_time ? 1 : 0] : nullptr;
    }
};

// One encoder level's DConv (2 residual layers) on x viewed as [nb][L][C] (freq: nb = B*F rows along time).
// Per layer: h = conv3(x) (+stats) -> GN+GELU in place -> 1x1 conv twice: pass 1 only accumulates the GroupNorm
// statistics of its 2C outputs, pass 2 recomputes them (K = C/8 is tiny) and applies GN -> GLU -> LayerScale
// -> residual in the epilogue, writing x in place.  The 2C-channel intermediate never touches HBM.
// the second stream (time branch of the transformer and of the decoder) and its fork / join events, made once
// ATHD_SERIAL=1: both branches on the caller's stream (profiling runs whose per-kernel times should be the kernel's
// own; also the behaviour while an athd_profile window is open)
// round-5 A/B switch: ATHD_ROWLN=0 keeps out_proj and the FFN's LayerNorm as two launches; read at every forward
// (tests/test_gpu_parity.py::test_rowln_off_matches_default switches it between calls)
static bool rowln_enabled() {
    const char* e = std::getenv("ATHD_ROWLN");
    return !(e && e[0] == '0');
}

bool serial_branches(const Run& r) {
    static int env = -1;
    if (env < 0) {
        const char* e = std::getenv("ATHD_SERIAL");
        env = (e && *e && *e != '0') ? 1 : 0;
    }
    return env == 1 || r.c->prof != nullptr;
}

// ATHD_FDEC1_FUSED=0: the unfused level-1 frequency decoder (Z stored by a GEMM, fdec_lr.hip's two passes) instead
// of fdec1f.hip; read at every forward (A/B and parity runs switch it between calls)
bool fdec1_fused_enabled() {
    const char* e = std::getenv("ATHD_FDEC1_FUSED");
    return !(e && *e == '0');
}

// (created by athd_finalize: a forward creates no HIP objects, so it can be graph-captured from the first call)
bool second_stream(Run& r) {
    if (!r.c->s_time || !r.c->ev_f || !r.c->ev_t) r.check((int)hipErrorInvalidResourceHandle, "second stream");
    return r.err == 0;
}

// rw: the layer's rewrite fused into the second DConv layer's apply pass (bf16 mode, C = 48, 96): returns true when it
// ran there (x then holds the first layer's output only), false when the caller must run the rewrite
bool dconv(Run& r, const EncW& e, void* x, int64_t nb, int64_t L, float* hbuf, uint16_t* hbuf_b,
           const DcRewrite* rw = nullptr) {
    bool fused = false;
    const int ab = r.actbf ? 1 : 0;
    const int C = e.cout, Hh = C / 8;
    for (int dd = 0; dd < 2; ++dd) {
        const int dil = 1 << dd;
        double* st_h = r.stats(nb);
        double* st_y = r.stats(nb);
        // C = 96 in the bf16 mode (the time branch's level 1; the freq level 1 is fused in fenc_row): the MFMA passes
        // of the wide levels below (conv3, GN+GELU with the 1x1's moments, apply), the hidden rows padded to 16
        const bool wide96 = (C == 48 || C == 96) && r.actbf && hbuf_b && e.dc.gram1b[dd] && e.dc.c3[dd].w && L >= 64;
        if (C <= 96 && !wide96) {   // narrow levels: HBM-bound VALU kernels (dconv.hip)
            KSite site(dd == 0 ? "dconv0" : "dconv1");
            r.check(dconv_small_launch(x, ab, hbuf, nb, L, C, dil, e.dc.w3f[dd], e.dc.c3[dd].bias, e.dc.g1w[dd],
                                       e.dc.g1b[dd], e.dc.w1f[dd], e.dc.b1f[dd], e.dc.gram1[dd], e.dc.g2wf[dd], e.dc.g2bf[dd],
                                       e.dc.scale[dd], st_h, st_y, r.s, r.actbf), "dconv_small");
            continue;
        }
        GemmDesc g;
        g.A = x; g.a_bf16 = ab; g.nb = (int)nb; g.H_in = (int)L; g.W = 1; g.C_in = C; g.a_ld = C;
        g.ntaps = 3; g.in_stride = 1; g.in_off = -dil; g.dil = dil; g.H_out = (int)L;
        g.Wp = e.dc.c3[dd].w; g.N = Hh; g.K = e.dc.c3[dd].K; g.Kp = e.dc.c3[dd].Kp; g.bias = e.dc.c3[dd].bias;
        g.C = hbuf; g.H_out_total = (int)L; g.ldo = Hh; g.stats = st_h;
        int rc3 = -1;
        if (r.actbf) {       // bf16 mode: the weights-resident conv3 pass (dconv.hip), else the tiled GEMM
            KSite site("dconv.conv3");
            rc3 = dconv_conv3_launch((const uint16_t*)x, (const uint16_t*)e.dc.c3[dd].w, e.dc.c3[dd].Kp,
                                     e.dc.c3[dd].bias, hbuf, st_h, nb * L, L, C, dil, r.s);
        }
        if (rc3 > 0 || (rc3 != 0 && wide96)) {   // (wide96: the padded hidden rows exist in the MFMA pass only)
            r.check(rc3 > 0 ? rc3 : ATHD_EHIP, "dconv_conv3");
            return fused;
        }
        if (rc3 != 0) r.gemm(g, "dconv.conv3");
        // bf16 mode: GELU(GN(h)) written once as bf16, so both 1x1 passes read half the bytes and run on the bf16
        // MFMA GEMMs (gemm3 / gemm5) instead of converting fp32 A on load
        const bool hb = r.actbf && hbuf_b && (Hh % 8 == 0 || wide96);
        // the 1x1's GroupNorm statistics from its moments, taken by the GN+GELU pass (no statistics GEMM pass)
        bool mom = false;
        {
            KSite site("dconv.gn_gelu");
            if (hb && e.dc.gram1b[dd])
                mom = gn_gelu_mom_launch(hbuf, hbuf_b, (int)nb, L, Hh, st_h, e.dc.g1w[dd], e.dc.g1b[dd], e.dc.gram1b[dd],
                                         st_y, r.s) == 0;
            if (mom) {
                // (statistics of the 1x1 already in st_y)
            } else if (wide96) {
                // the padded-row layout of the narrow MFMA passes (hidden rows of 16) has no other GN+GELU pass
                r.check(ATHD_EHIP, "dconv gn_gelu_mom (C = 48 / 96)");
                return false;
            } else if (hb) {
                gn_gelu_bf16_launch(hbuf, hbuf_b, (int)nb, L * Hh, Hh, st_h, e.dc.g1w[dd], e.dc.g1b[dd], r.s);
            } else {
                gn_gelu_launch(hbuf, (int)nb, L * Hh, Hh, st_h, e.dc.g1w[dd], e.dc.g1b[dd], r.s, r.actbf);
            }
        }
        GemmDesc g2;
        g2.A = hb ? (const void*)hbuf_b : (const void*)hbuf; g2.a_bf16 = hb ? 1 : 0; g2.nb = (int)nb; g2.H_in = (int)L; g2.W = 1; g2.C_in = Hh; g2.a_ld = Hh; g2.H_out = (int)L;
        g2.Wp = e.dc.c1[dd].w; g2.N = 2 * C; g2.K = Hh; g2.Kp = e.dc.c1[dd].Kp; g2.bias = e.dc.c1[dd].bias;
        g2.C = x; g2.c_bf16 = ab; g2.H_out_total = (int)L; g2.ldo = C;
        if (!mom) {
            GemmDesc g1 = g2;
            g1.stats = st_y; g1.store = 0;
            r.gemm(g1, "dconv.conv1x1.stats");
        }
        g2.act = ACT_GLU; g2.gn_stats = st_y; g2.gn_count = L * 2 * C; g2.gn_w = e.dc.g2w[dd]; g2.gn_b = e.dc.g2b[dd];
        g2.res = x; g2.res_bf16 = ab; g2.res_scale = e.dc.scale[dd];
        // bf16 mode: the weights-resident apply pass (dconv.hip dconv_apply_kernel), else the GEMM with its epilogue
        int rc = -1;
        if (hb) {
            KSite site("dconv.conv1x1.apply");
            const DcRewrite* rwd = dd == 1 && wide96 ? rw : nullptr;
            // rc -1: rejected before any launch (fall back); rc > 0: a HIP error after the in-place kernel was issued,
            // so x may already hold the residual update: report it, never run a second apply over it
            rc = dconv_apply_launch(hbuf_b, (const uint16_t*)e.dc.c1[dd].w, e.dc.c1[dd].Kp, e.dc.c1[dd].bias, st_y,
                                    e.dc.g2w[dd], e.dc.g2b[dd], e.dc.scale[dd], (uint16_t*)x, nb * L, L, C, r.s, rwd);
            if (rc == 0 && rwd) fused = true;
            if (rc == -1 && rwd)      // (without the rewrite, then the caller's GEMM)
                rc = dconv_apply_launch(hbuf_b, (const uint16_t*)e.dc.c1[dd].w, e.dc.c1[dd].Kp, e.dc.c1[dd].bias,
                                        st_y, e.dc.g2w[dd], e.dc.g2b[dd], e.dc.scale[dd], (uint16_t*)x, nb * L, L, C, r.s);
            if (rc > 0) { r.check(rc, "dconv_apply"); return fused; }
            if (rc == -1 && wide96) { r.check(ATHD_EHIP, "dconv_apply (C = 48 / 96, padded hidden rows)"); return fused; }
        }
        if (rc != 0) r.gemm(g2, "dconv.conv1x1.apply");
    }
    return fused;
}

// the fused narrow freq level (fenc_row.hip) applies: bf16 mode, C in {48, 96}, T <= 272, padded conv3 packed;
// ATHD_FENC_ROW=0 takes the unfused implicit-GEMM + DConv path instead (parity A/B; read at every forward)
bool br_fused(const EncW& e, int Ts) {
    const char* v = std::getenv("ATHD_FENC_ROW");
    if (v && *v == '0') return false;
    return e.dc.c3p[0].w && e.dc.c3p[1].w && fenc_row_supported(e.cin, e.cout, Ts);
}

void encode(Run& r, const Dims& d, const Bufs& b, const float* wav) {
    athd_ctx* c = r.c;
    KSection sec_enc("encoder");
    const int64_t B = d.B, Ts = d.Tspec;
    // ---- STFT + CaC, input normalisation statistics (ATHTDemucs_v2.py:261-275) ----
    PadPlan pp;
    {
        const int64_t le = d.Tspec, pad = 1536;
        const int64_t pl = pad, pr = pad + le * 1024 - d.T;
        int64_t epl = 0, epr = 0;
        const int64_t maxpad = std::max(pl, pr);
        if (d.T <= maxpad) {
            const int64_t extra = maxpad - d.T + 1;
            epr = std::min(pr, extra);
            epl = extra - epr;
        }
        pp.L = d.T;
        pp.left = pl - epl;
        pp.ext_left = epl;
        pp.Lx = d.T + epl + epr;
    }
    double* st_spec = r.stats(B);
    double* st_wav = r.stats(B);
    stft_launch(wav, (int)B, d.T, pp, (int)Ts, c->tw, r.actbf ? nullptr : c->tw64, c->win, b.specT, st_spec, r.s);
    stats_launch(wav, (int)B, 2 * d.T, st_wav, r.s);
    input_norm_params_launch(st_spec, (int)B, 2048LL * Ts * 4, b.snorm, nullptr, r.s);
    input_norm_params_launch(st_wav, (int)B, 2 * d.T, b.tnorm_div, b.tnorm_std, r.s);

    // ---- encoders (ATHTDemucs_v2.py:197-217; HEncLayer + DConv) ----
    // fork: the time encoder runs on the second stream (own ybuf_t / hbuf_t) beside the frequency encoder; the
    // branches join before the transformer's up-projections.  (The waveform statistics stay before the fork: run as
    // the time stream's first kernels, beside the STFT, they measured 3 % slower per step - the time encoder's
    // kernels then take CUs ahead of the frequency encoder's level-0 rows.)
    if (!second_stream(r)) return;
    hipStream_t const s_enc = r.s, s_tenc = serial_branches(r) ? r.s : c->s_time;
    (void)hipEventRecord(c->ev_f, s_enc);
    (void)hipStreamWaitEvent(s_tenc, c->ev_f, 0);
    const int eab = r.actbf ? 1 : 0;       // encoder activations in bf16 (throughput mode)
    static const char* const kFenc[4] = {"fenc0", "fenc1", "fenc2", "fenc3"};
    static const char* const kTenc[4] = {"tenc0", "tenc1", "tenc2", "tenc3"};
    for (int i = 0; i < 4; ++i) {
        KStage stage(kFenc[i]);
        // freq branch: conv (8,1)/(4,1) along freq rows
        const EncW& e = c->fenc[i];
        const int C = e.cout;
        const int Fi = d.F[i], Fo = d.F[i + 1];
        if (r.actbf && br_fused(e, (int)Ts)) {
            // narrow level: conv + GELU + DConv + rewrite GLU in one kernel per (b, f) row (fenc_row.hip)
            FencRowDesc fr;
            fr.in = i == 0 ? (const void*)b.specT : (const void*)b.saved[i - 1];
            fr.a_norm = i == 0 ? b.snorm : nullptr;
            fr.B = (int)B; fr.Fin = Fi; fr.Fout = Fo; fr.T = (int)Ts;
            fr.wc = (const uint16_t*)e.conv.w; fr.wc_ld = e.conv.Kp; fr.bc = e.conv.bias;
            for (int dd = 0; dd < 2; ++dd) {
                fr.w3[dd] = (const uint16_t*)e.dc.c3p[dd].w; fr.w3_ld = e.dc.c3p[dd].Kp; fr.b3[dd] = e.dc.c3[dd].bias;
                fr.g1w[dd] = e.dc.g1w[dd]; fr.g1b[dd] = e.dc.g1b[dd];
                fr.w1[dd] = (const uint16_t*)e.dc.c1[dd].w; fr.w1_ld = e.dc.c1[dd].Kp; fr.b1[dd] = e.dc.c1[dd].bias;
                fr.g2w[dd] = e.dc.g2w[dd]; fr.g2b[dd] = e.dc.g2b[dd]; fr.scale[dd] = e.dc.scale[dd];
                fr.gram[dd] = e.dc.gram1b[dd];
            }
            fr.wr = (const uint16_t*)e.rewrite.w; fr.wr_ld = e.rewrite.Kp; fr.br = e.rewrite.bias;
            fr.row_add = i == 0 ? c->femb : nullptr;
            fr.out = (uint16_t*)b.saved[i];
            fr.out4 = i == 0 ? (uint16_t*)b.sk4 : nullptr;
            KSite site("fenc_row");
            r.check(fenc_row_launch(fr, e.cin, C, r.s), "fenc_row");
        } else {
        GemmDesc g;
        g.A = i == 0 ? (const void*)b.specT : (const void*)b.saved[i - 1];
        g.a_bf16 = i == 0 ? 0 : eab;
        g.nb = (int)B; g.H_in = Fi; g.W = (int)Ts; g.C_in = e.cin; g.a_ld = e.cin;
        if (i == 0) {   // frame-major spectrogram: the 8 freq taps x 4 channels of a row are 128 contiguous bytes
            g.a_ld = 2048 * 4; g.a_hs = 4; g.a_bs = Ts * 2048 * 4;
        }
        g.ntaps = 8; g.in_stride = 4; g.in_off = -2; g.dil = 1; g.H_out = Fo;
        g.a_norm = i == 0 ? b.snorm : nullptr;
        g.Wp = e.conv.w; g.N = C; g.K = e.conv.K; g.Kp = e.conv.Kp; g.bias = e.conv.bias;
        g.C = b.ybuf; g.c_bf16 = eab; g.H_out_total = Fo; g.ldo = C; g.act = ACT_GELU;
        r.gemm(g, "fenc.conv");
        dconv(r, e, b.ybuf, B * Fo, Ts, b.hbuf, b.hbuf_b);
        GemmDesc gr;
        gr.A = b.ybuf; gr.a_bf16 = eab; gr.nb = (int)B; gr.H_in = Fo; gr.W = (int)Ts; gr.C_in = C; gr.a_ld = C; gr.H_out = Fo;
        gr.Wp = e.rewrite.w; gr.N = 2 * C; gr.K = C; gr.Kp = e.rewrite.Kp; gr.bias = e.rewrite.bias;
        gr.C = b.saved[i]; gr.c_bf16 = eab; gr.H_out_total = Fo; gr.ldo = C; gr.act = ACT_GLU;
        gr.row_add = i == 0 ? c->femb : nullptr;    // + freq_emb_scale * freq_emb(frs) (ATHTDemucs_v2.py:212-215)
        gr.c4 = i == 0 ? b.sk4 : nullptr;
        r.gemm(gr, "fenc.rewrite");
        }

        // time branch: right zero-pad to a multiple of 4 is implicit (rows >= L read as 0)
        r.s = s_tenc;
        KStage tstage(kTenc[i]);
        const EncW& et = c->tenc[i];
        const int64_t Li = d.L[i], Lo = d.L[i + 1];
        if (i == 0) {
            KSite site("tenc.conv");
            tconv0_launch(wav, (int)B, d.T, Lo, et.conv_f32, et.conv.bias, b.tnorm_div, b.ybuf_t, eab, r.s);
        } else {
            GemmDesc gt;
            gt.A = b.saved_t[i - 1]; gt.a_bf16 = eab; gt.a_ld = et.cin;
            gt.nb = (int)B; gt.H_in = (int)Li; gt.W = 1; gt.C_in = et.cin;
            gt.ntaps = 8; gt.in_stride = 4; gt.in_off = -2; gt.dil = 1; gt.H_out = (int)Lo;
            gt.Wp = et.conv.w; gt.N = C; gt.K = et.conv.K; gt.Kp = et.conv.Kp; gt.bias = et.conv.bias;
            gt.C = b.ybuf_t; gt.c_bf16 = eab; gt.H_out_total = (int)Lo; gt.ldo = C; gt.act = ACT_GELU;
            r.gemm(gt, "tenc.conv");
        }
        DcRewrite rwt;
        rwt.w = (const uint16_t*)et.rewrite_perm.w; rwt.kp = et.rewrite_perm.Kp; rwt.bias = et.rewrite_perm.bias;
        rwt.out = (uint16_t*)b.saved_t[i]; rwt.c4 = i == 0 ? (uint16_t*)b.sk4t : nullptr;
        const bool fused_rw = dconv(r, et, b.ybuf_t, B, Lo, b.hbuf_t, b.hbuf_b_t, et.rewrite_perm.w ? &rwt : nullptr);
        if (!fused_rw) {
        GemmDesc grt;
        grt.A = b.ybuf_t; grt.a_bf16 = eab; grt.nb = (int)B; grt.H_in = (int)Lo; grt.W = 1; grt.C_in = C; grt.a_ld = C; grt.H_out = (int)Lo;
        grt.Wp = et.rewrite.w; grt.N = 2 * C; grt.K = C; grt.Kp = et.rewrite.Kp; grt.bias = et.rewrite.bias;
        grt.C = b.saved_t[i]; grt.c_bf16 = eab; grt.H_out_total = (int)Lo; grt.ldo = C; grt.act = ACT_GLU;
        grt.c4 = i == 0 ? b.sk4t : nullptr;
        r.gemm(grt, "tenc.rewrite");
        }
        r.s = s_enc;
    }
    (void)hipEventRecord(c->ev_t, s_tenc);        // join
    (void)hipStreamWaitEvent(s_enc, c->ev_t, 0);

    // ---- cross-transformer (ATHTDemucs_v2.py:219-234) ----
    KStage xstage("transformer");
    KSection sec_x("transformer");
    const int ab = r.actbf ? 1 : 0;
    {
        GemmDesc g = r.lin(c->up, b.saved[3], ab, (int)B, d.Nf, 384);
        g.C = b.X;
        r.gemm(g, "upsampler");
        GemmDesc gt = r.lin(c->up_t, b.saved_t[3], ab, (int)B, d.Nt, 384);
        gt.C = b.XT;
        r.gemm(gt, "upsampler_t");
    }
    pos2d_launch(b.pos2d, 8, (int)Ts, 512, r.s);
    pos1d_launch(b.pos1d, (int)d.Nt, 512, r.s);
    {
        LnDesc l;
        l.x = b.X; l.nb = (int)B; l.N = d.Nf; l.C = 512; l.w = c->nin_w; l.b = c->nin_b; l.pos = b.pos2d; l.out = b.X;
        layernorm_launch(l, r.s);
        LnDesc lt;
        lt.x = b.XT; lt.nb = (int)B; lt.N = d.Nt; lt.C = 512; lt.w = c->nint_w; lt.b = c->nint_b; lt.pos = b.pos1d; lt.out = b.XT;
        layernorm_launch(lt, r.s);
    }
    struct Pending { const double* st = nullptr; const float* w = nullptr; const float* b = nullptr; };
    Pending pf, pt;
    // bf16 mode: the LayerNorm pass that consumes a pending GroupNorm applies it in registers only, without writing
    // X / XT back; the branch's next out_proj applies the same GroupNorm to its residual read (GemmDesc::res_gn_*), the
    // only other reader of those raw rows (the cross layers' second norm of the same rows runs inside the same pass).
    // Saves the 271 MB (freq) / 136 MB (time) write-back per layer.  f32 mode keeps the write-back.
    const bool lazy_gn = r.actbf;
    Pending rf, rt;                              // consumed by the last LayerNorm, due on the next out_proj residual
    auto ln2 = [&](float* x, int64_t N, const float* w, const float* bb, Pending* pend, void* out, const float* w2,
                   const float* b2, void* out2, Pending* resgn) {
        LnDesc l;
        l.x = x; l.nb = (int)B; l.N = N; l.C = 512; l.w = w; l.b = bb; l.out = out; l.out_bf16 = ab;
        if (pend && pend->st) {
            l.gn_stats = pend->st; l.gn_w = pend->w; l.gn_b = pend->b;
            // (the residual epilogue takes it when a 256-row tile spans at most two batches: N >= 256 tokens; the
            // LayerNorm pass has the register-only form only where ln_lazy_gn_ok holds)
            l.out_bf16 = ab; l.out2 = out2;
            if (lazy_gn && resgn && N >= 256 && ln_lazy_gn_ok(l)) { l.gn_writeback = 0; *resgn = *pend; }
            *pend = Pending();
        }
        l.w2 = w2; l.b2 = b2; l.out2 = out2;
        layernorm_launch(l, r.s);
    };
    auto ln = [&](float* x, int64_t N, const float* w, const float* bb, Pending* pend, void* out, Pending* resgn) {
        ln2(x, N, w, bb, pend, out, nullptr, nullptr, nullptr, resgn);
    };
    // attention + FFN of one branch given LN'ed query rows Hq and key/value source (projected inside)
    auto block = [&](const TLayerW& L, float* X, int64_t N, void* Hq, void* Hkv, int64_t Nk, Pending* pend, bool tb,
                     Pending* resgn) {
        void* const sQKV = tb ? b.QKVt : b.QKV;
        void* const sO = tb ? b.Ot : b.O;
        void* const sF1 = tb ? b.F1t : b.F1;
        AttnDesc a;
        a.nb = (int)B; a.Nq = (int)N; a.Nk = (int)Nk; a.heads = 8;
        a.scale = r.actbf ? ATTN_SCALE_PRESCALED : 0.125f;     // bf16: queries prescaled at pack time (attn.h)
        if (!L.cross) {
            GemmDesc g = r.lin(L.qkv, Hq, ab, (int)B, N, 512);
            g.C = sQKV; g.c_bf16 = ab;
            r.gemm(g, "qkv");
            a.Q = sQKV; a.q_bf16 = ab; a.q_bs = N * 1536; a.q_ld = 1536; a.q_off = 0;
            a.K = sQKV; a.k_bf16 = ab; a.k_bs = N * 1536; a.k_ld = 1536; a.k_off = 512;
            a.V = sQKV; a.v_bf16 = ab; a.v_bs = N * 1536; a.v_ld = 1536; a.v_off = 1024;
        } else {
            char* Qb = (char*)sQKV;
            char* KVb = Qb + (size_t)B * d.Nmax * 512 * (ab ? 2 : 4);
            GemmDesc gq = r.lin(L.q, Hq, ab, (int)B, N, 512);
            gq.C = Qb; gq.c_bf16 = ab;
            r.gemm(gq, "q");
            GemmDesc gk = r.lin(L.kv, Hkv, ab, (int)B, Nk, 512);
            gk.C = KVb; gk.c_bf16 = ab;
            r.gemm(gk, "kv");
            a.Q = Qb; a.q_bf16 = ab; a.q_bs = N * 512; a.q_ld = 512; a.q_off = 0;
            a.K = KVb; a.k_bf16 = ab; a.k_bs = Nk * 1024; a.k_ld = 1024; a.k_off = 0;
            a.V = KVb; a.v_bf16 = ab; a.v_bs = Nk * 1024; a.v_ld = 1024; a.v_off = 512;
        }
        a.O = sO; a.o_bf16 = ab; a.o_bs = N * 512; a.o_ld = 512;
        r.check(attn_launch(a, r.mode, r.s), "attention");
        GemmDesc go = r.lin(L.out, sO, ab, (int)B, N, 512);
        go.C = X; go.res = X; go.res_scale = L.g1;
        if (resgn->st) {
            go.res_gn_stats = resgn->st; go.res_gn_count = N * 512; go.res_gn_w = resgn->w; go.res_gn_b = resgn->b;
            *resgn = Pending();
        }
        const float* n2w = L.cross ? L.n3w : L.n2w;
        const float* n2b = L.cross ? L.n3b : L.n2b;
        go.ln_w = n2w; go.ln_b = n2b; go.ln_out = Hq;
        if (r.actbf && rowln_enabled() && rowln_supported(go)) {
            // bf16 mode: out_proj with the FFN's LayerNorm in its epilogue (rowln.hip: whole 512-column rows per
            // workgroup; the LayerNorm pass and its second read of X are gone)
            r.gemm(go, "out_proj.ln");
        } else {
            go.ln_w = go.ln_b = nullptr; go.ln_out = nullptr;
            r.gemm(go, "out_proj");
            ln(X, N, n2w, n2b, nullptr, Hq, nullptr);
        }
        GemmDesc g1 = r.lin(L.l1, Hq, ab, (int)B, N, 512);
        g1.C = sF1; g1.c_bf16 = ab; g1.act = ACT_GELU;
        r.gemm(g1, "linear1");
        double* st = r.stats(B);
        GemmDesc g2 = r.lin(L.l2, sF1, ab, (int)B, N, 2048);
        g2.C = X; g2.res = X; g2.res_scale = L.g2; g2.stats = st;
        g2.sk_ws = r.skws();                     // K = 2048: the last partial round of tiles split along K (gemm5)
        r.gemm(g2, "linear2");
        pend->st = st; pend->w = L.now; pend->b = L.nob;
    };
    // Two streams: the frequency branch on the caller's stream, the time branch on ctx.s_time.  Self-attention
    // layers are independent per branch; a cross layer joins both streams (each waits for the other's previous
    // layer: the key/value norms below overwrite buffers the other branch read), computes its four norms, joins
    // again (each block reads the other branch's kv norm) and runs both blocks side by side.  Buffers: H[0] / H[1]
    // written only on the freq stream, H[2] / H[3] only on the time stream; separate QKV / O / F1 scratch.
    if (!second_stream(r)) return;
    // (while a kernel profile is open the branches run serially on one stream, so per-kernel event times are the
    // kernel's own and not shared with a concurrent one)
    hipStream_t const s_f = r.s, s_t = serial_branches(r) ? r.s : c->s_time;
    auto join = [&]() {
        (void)hipEventRecord(c->ev_f, s_f);
        (void)hipEventRecord(c->ev_t, s_t);
        (void)hipStreamWaitEvent(s_t, c->ev_f, 0);
        (void)hipStreamWaitEvent(s_f, c->ev_t, 0);
    };
    (void)hipEventRecord(c->ev_f, s_f);          // fork: the time stream starts after everything issued so far
    (void)hipStreamWaitEvent(s_t, c->ev_f, 0);
    for (int idx = 0; idx < 5; ++idx) {
        const TLayerW& Lf = c->L[idx];
        const TLayerW& Lt = c->Lt[idx];
        if (!Lf.cross) {
            r.s = s_f;
            ln(b.X, d.Nf, Lf.n1w, Lf.n1b, &pf, b.H[0], &rf);
            block(Lf, b.X, d.Nf, b.H[0], nullptr, d.Nf, &pf, false, &rf);
            r.s = s_t;
            ln(b.XT, d.Nt, Lt.n1w, Lt.n1b, &pt, b.H[2], &rt);
            block(Lt, b.XT, d.Nt, b.H[2], nullptr, d.Nt, &pt, true, &rt);
        } else {
            join();
            // all four norms read the pre-layer X / XT (time branch attends to old_x, demucs transformer.py)
            // (bf16 mode: each pair is one pass over X / XT with two affines, layernorm_launch's out2)
            r.s = s_f;
            ln2(b.X, d.Nf, Lf.n1w, Lf.n1b, &pf, b.H[0], Lt.n2w, Lt.n2b, b.H[1], &rf);   // pending GN applied to X; norm1(x) and
                                                                                // the time branch's kv = norm2_t(old_x)
            r.s = s_t;
            ln2(b.XT, d.Nt, Lt.n1w, Lt.n1b, &pt, b.H[2], Lf.n2w, Lf.n2b, b.H[3], &rt);  // norm1_t(xt) and the freq branch's kv
                                                                                // = norm2(xt)
            join();
            r.s = s_f;
            block(Lf, b.X, d.Nf, b.H[0], b.H[3], d.Nt, &pf, false, &rf);
            r.s = s_t;
            block(Lt, b.XT, d.Nt, b.H[2], b.H[1], d.Nf, &pt, true, &rt);
        }
    }
    // the last layer's pending GroupNorm: in the bf16 mode applied by the downsamplers' A load (gemm2 a_gn; X / XT
    // have no other reader), in the f32 mode written back first
    if (!r.actbf) {
        gn_apply_launch(b.X, (int)B, d.Nf, 512, pf.st, pf.w, pf.b, s_f);
        gn_apply_launch(b.XT, (int)B, d.Nt, 512, pt.st, pt.w, pt.b, s_t);
    }
    {
        r.s = s_t;                               // the time branch's channel downsampler on its own stream
        GemmDesc gt = r.lin(c->down_t, b.XT, 0, (int)B, d.Nt, 512);
        gt.C = b.xt_enc;
        if (r.actbf) { gt.a_gn_stats = pt.st; gt.a_gn_count = d.Nt * 512; gt.a_gn_w = pt.w; gt.a_gn_b = pt.b; }
        r.gemm(gt, "downsampler_t");
        if (b.xt_enc_b) to_bf16_launch(b.xt_enc, b.xt_enc_b, B * d.Nt * 384, s_t);
        r.s = s_f;
        GemmDesc g = r.lin(c->down, b.X, 0, (int)B, d.Nf, 512);
        g.C = b.x_enc;
        if (r.actbf) { g.a_gn_stats = pf.st; g.a_gn_count = d.Nf * 512; g.a_gn_w = pf.w; g.a_gn_b = pf.b; }
        r.gemm(g, "downsampler");
        if (b.x_enc_b) to_bf16_launch(b.x_enc, b.x_enc_b, B * d.Nf * 384, s_f);
    }
    (void)hipEventRecord(c->ev_t, s_t);          // join: the caller's stream continues after the time branch
    (void)hipStreamWaitEvent(s_f, c->ev_t, 0);
}

// ConvTranspose (k8, s4, p2) along H as two GEMMs, one per residue pair: output rows 4u+{0,1} read input rows
// u-1, u; rows 4u+{2,3} read u, u+1.  Each GEMM has N = 2*cout (columns >= cout belong to the odd residue).
// keep < 0: store all rows (4*H_in rows).  keep > 0: store only rows 4u+1, 4u+2 as slots 2u, 2u+1 (the only
// rows the following exact /4 bilinear resize reads); statistics (if st) still cover all four residues.
void conv_t(Run& r, const DecW& w, const void* A, int a_bf16, int nb, int H_in, int W, void* out, int out_bf16,
            double* st, int keep, const char* stage) {
    KStage kst(stage);
    if (w.ct4w && a_bf16 && out_bf16 && convt4_supported(w.cin, w.cout, nb, H_in, W)) {
        // dedicated pass (convt4.hip): weights resident in LDS, barrier-free waves over 32-row units
        ConvT4Desc q;
        q.x = (const uint16_t*)A; q.w = w.ct4w; q.bias = w.ct4b; q.out = (uint16_t*)out; q.stats = st;
        q.nb = nb; q.H = H_in; q.W = W; q.keep = keep < 0 ? 0 : 1;
        r.check(convt4_launch(q, r.s), "convt4");
        return;
    }
    if (w.quad.w) {
        // all four residues in one GEMM (N = 4 cout, K = rows u-1 | u | u+1): the input is read once
        GemmDesc g;
        g.A = A; g.a_bf16 = a_bf16; g.nb = nb; g.H_in = H_in; g.W = W; g.C_in = w.cin; g.a_ld = w.cin;
        g.ntaps = 3; g.in_stride = 1; g.in_off = -1; g.dil = 1; g.H_out = H_in;
        g.Wp = w.quad.w; g.N = w.quad.N; g.K = w.quad.K; g.Kp = w.quad.Kp; g.bias = w.quad.bias;
        g.C = out; g.c_bf16 = out_bf16; g.ldo = w.cout; g.stats = st; g.col_split = w.cout; g.hi_row_off = 1;
        if (w.cin % 32 == 0) g.k_blk = w.cin;       // skip the zero third of K per residue pair (gemm3)
        if (keep < 0) {
            g.H_out_total = 4 * H_in; g.o_stride = 4; g.o_off = 0; g.store_mask = 15;
        } else {                                    // residues 1, 2 -> slots 2u, 2u+1; 0 and 3 feed the statistics
            g.H_out_total = 2 * H_in; g.o_stride = 2; g.o_off = -1; g.store_mask = 6;
        }
        r.gemm(g, "convt.quad");
        return;
    }
    for (int pi = 0; pi < 2; ++pi) {
        GemmDesc g;
        g.A = A; g.a_bf16 = a_bf16; g.nb = nb; g.H_in = H_in; g.W = W; g.C_in = w.cin; g.a_ld = w.cin;
        g.ntaps = 2; g.in_stride = 1; g.in_off = pi == 0 ? -1 : 0; g.dil = 1; g.H_out = H_in;
        g.Wp = w.pair[pi].w; g.N = 2 * w.cout; g.K = w.pair[pi].K; g.Kp = w.pair[pi].Kp; g.bias = w.pair[pi].bias;
        g.C = out; g.c_bf16 = out_bf16; g.ldo = w.cout; g.stats = st; g.col_split = w.cout;
        if (keep < 0) {
            g.H_out_total = 4 * H_in; g.o_stride = 4; g.o_off = 2 * pi; g.hi_row_off = 1; g.store_mask = 3;
        } else {
            g.H_out_total = 2 * H_in; g.o_stride = 2;
            if (pi == 0) { g.o_off = 0; g.hi_row_off = 0; g.store_mask = 2; }   // residue 1 -> slot 2u
            else { g.o_off = 1; g.store_mask = 1; }                              // residue 2 -> slot 2u+1
        }
        r.gemm(g, pi == 0 ? "convt.pair01" : "convt.pair23");
    }
}

void decode_chunk(Run& r, const Dims& d, const Bufs& b, int64_t s0, int64_t Bc, const float* text, bool text_per_item,
                  float* out, float* FO) {
    athd_ctx* c = r.c;
    KSection sec_dec("decoder");
    const int P = d.P;
    const int NI = (int)(Bc * P);
    const int64_t Ts = d.Tspec;
    const int ab = r.actbf ? 1 : 0;
    // Chunk ordering: the previous chunk's time branch (second stream) recorded ev_t after its text cross-attention,
    // i.e. after it read tc0 / tc2 / avec, and - in stream order - after the iSTFT of the chunk before it, the last
    // reader of the FO buffer this chunk's fdec_tail rewrites (FO[c & 1] == FO[(c - 2) & 1]).  Waiting on it here
    // orders both write-after-read pairs; at chunk 0 ev_t is the encoder's join, already waited on.
    if (s0 > 0 && !serial_branches(r)) (void)hipStreamWaitEvent(r.s, c->ev_t, 0);
    // ---- text cross-attention, closed form (ATHTDemucs_v2.py:38-58) ----
    text_vec_launch(text_per_item ? text + s0 * 512 : text, NI, P, text_per_item ? 1 : 0, c->ta_maT, c->ta_ma, c->ta_mcT,
                    c->ta_mc, c->ta_m2b, b.avec, b.tc0, b.tc2, r.s);
    // The prompt enters only through the row vector a = attn_out (one key: softmax == 1), so with u = x + a
    // (ATHTDemucs_v2.py:46-48):  h = GELU(W0 u + b0) = GELU(W0 x + c0),  y = u + W2 h + b2 = x + W2 h + c2  (c0, c2 per
    // prompt, text_vec_kernel).  text.mlp0 multiplies the SEGMENT's x once and its epilogue writes the P prompts' h
    // (F_PB, pfold = P); text.mlp2 adds the segment's x as the residual (res_div = P) and the prompt's c2.
    auto text_attn = [&](const float* enc, const uint16_t* enc_b, int64_t ntok, float* cond, void* Hm, float* Yb) {
        KStage kst(ntok == d.Nf ? "text_attn.freq" : "text_attn.time");
        GemmDesc g = enc_b ? r.lin(c->mlp0, enc_b, 1, (int)Bc, ntok, 384) : r.lin(c->mlp0, enc, 0, (int)Bc, ntok, 384);
        g.bias = nullptr; g.pbias = b.tc0; g.pfold = P;
        g.C = Hm; g.c_bf16 = ab; g.act = ACT_GELU;
        r.gemm(g, "text.mlp0");
        GemmDesc g2 = r.lin(c->mlp2, Hm, ab, NI, ntok, 384);
        g2.bias = nullptr; g2.pbias = b.tc2;
        g2.C = Yb; g2.res = enc; g2.res_div = P; g2.res_bs = ntok * 384;
        if (r.actbf) {
            // bf16 mode: norm_out in the GEMM's epilogue (gemm3 row-LayerNorm variant: 128 x 384 tiles hold whole
            // rows), x_cond written directly; Yb is not used
            g2.C = cond; g2.c_bf16 = 1; g2.ln_w = c->ta_nw; g2.ln_b = c->ta_nb;
            r.gemm(g2, "text.mlp2.ln");
            return;
        }
        r.gemm(g2, "text.mlp2");
        LnDesc l;
        l.x = Yb; l.nb = NI; l.N = ntok; l.C = 384; l.w = c->ta_nw; l.b = c->ta_nb; l.out = cond; l.out_bf16 = ab;
        layernorm_launch(l, r.s);
    };
    // fork after the prompt vectors: the time branch (its text cross-attention with its own U / Hm / Yb scratch, then
    // the time decoder with its own Gt / Dt buffers) runs on the second stream beside the frequency branch and the
    // iSTFT; the branches join before istft_ola_kernel, which reads both
    if (!second_stream(r)) return;
    hipStream_t const s_main = r.s, s_t = serial_branches(r) ? r.s : c->s_time;   // (see encode)
    (void)hipEventRecord(c->ev_f, s_main);
    (void)hipStreamWaitEvent(s_t, c->ev_f, 0);
    text_attn(b.x_enc + s0 * d.Nf * 384, b.x_enc_b ? b.x_enc_b + s0 * d.Nf * 384 : nullptr, d.Nf, b.x_cond, b.Hm, b.Yb);

    // ---- frequency decoder (ATHTDemucs_v2.py:82-104, 293-297) ----
    const int ea = b.ea;
    void* const sv[4] = {eoff(b.saved[0], s0 * 512 * Ts * 48, ea), eoff(b.saved[1], s0 * 128 * Ts * 96, ea),
                         eoff(b.saved[2], s0 * 32 * Ts * 192, ea), eoff(b.saved[3], s0 * 8 * Ts * 384, ea)};
    {
        // level 0: 8 -> 32 rows, GN+GELU (in place, fp32: every source row feeds ~Ts/32 output rows), resize to
        // Tspec rows, + 0.1 * resize(saved[3][:, :192])
        double* st = r.stats(NI);
        // (bf16 mode: the ConvT output G as bf16, its GroupNorm statistics taken by the GEMM epilogue before rounding)
        conv_t(r, c->fdec[0], b.x_cond, ab, NI, 8, (int)Ts, b.G, ab, st, -1, "fdec0");
        KStage kst("fdec0");
        // S = GELU(GN(ConvT0)): in place (fp32 mode) or as a bf16 copy, the A operand of the level-1 tap GEMM
        if (r.actbf)
            gn_gelu_bf16in_launch((const uint16_t*)b.G, (uint16_t*)b.S, NI, 32 * Ts * 192, 192, st, c->fdec[0].gnw,
                                  c->fdec[0].gnb, r.s);
        else gn_gelu_launch(b.G, NI, 32 * Ts * 192, 192, st, c->fdec[0].gnw, c->fdec[0].gnb, r.s, false);
        // level 1 from the 32-row S = GELU(GN(ConvT0)) without materialising the resized 259-row input
        // (fdec_lr.hip): Z = S @ [W_0 .. W_7], Zs = skip3[:, :192] @ [W_0 .. W_7], then stats + merge passes
        KStage kst1("fdec1");
        const DecW& w1 = c->fdec[1];
        GemmDesc gz;
        gz.A = r.actbf ? b.S : (const void*)b.G; gz.a_bf16 = ab; gz.nb = NI; gz.H_in = 32; gz.W = (int)Ts; gz.C_in = w1.cin; gz.a_ld = w1.cin;
        gz.H_out = 32; gz.Wp = w1.taps.w; gz.N = w1.taps.N; gz.K = w1.taps.K; gz.Kp = w1.taps.Kp;
        gz.C = b.Z; gz.c_bf16 = ab; gz.H_out_total = 32; gz.ldo = w1.taps.N;
        LowRankDesc lr;
        lr.steps = b.lrsteps;
        lr.Z = b.Z; lr.Zs = b.Zs; lr.z_bf16 = ab; lr.Hs = 32; lr.Hk = 8; lr.Hd = (int)Ts; lr.W = (int)Ts;
        lr.Co = w1.cout; lr.P = P; lr.NI = NI; lr.bias = w1.bias; lr.stats = r.stats(NI);
        lr.gn_w = w1.gnw; lr.gn_b = w1.gnb; lr.fast_gelu = ab;
        lr.skip = sv[2]; lr.skip_bf16 = ab; lr.H_skip = 32; lr.C_skip = 192;
        lr.out = b.D; lr.out_bf16 = ab;
        lr.S = gz.A; lr.Wt = w1.taps.w; lr.w_ld = w1.taps.Kp; lr.Ci = w1.cin;
        // bf16 mode: the statistics from Gram matrices of Z tiles computed in LDS (fdec1f.hip), which also stores
        // the merge pass's taps 0, 3, 4, 7 of Z (no Z GEMM)
        const bool gram = fdec1_fused_enabled() && b.gram && fdec1_gram_supported(lr);
        if (gram) {
            lr.z_taps = 4;
            lr.z4 = b.Z;                            // written by fdec1_gram_kernel
        } else {
            r.gemm(gz, "fdec1.z");
        }
        GemmDesc gs = gz;
        gs.A = sv[3]; gs.a_bf16 = ab; gs.nb = (int)Bc; gs.H_in = 8; gs.H_out = 8; gs.H_out_total = 8; gs.a_ld = 384;
        gs.Wp = w1.taps.w; gs.N = w1.taps.N; gs.K = w1.taps.K; gs.Kp = w1.taps.Kp; gs.ldo = w1.taps.N;
        gs.C = b.Zs;
        r.gemm(gs, "fdec1.zs");
        r.check(fdec_lr_steps_launch(b.lrsteps, (int)Ts, 32, 8, 32, r.s), "fdec_lr_steps");
        if (gram) r.check(fdec1_gram_launch(lr, b.gram, b.gramq, r.s), "fdec1_gram");
        else r.check(fdec_lr_stats_launch(lr, r.s), "fdec_lr_stats");
        r.check(fdec_lr_merge_launch(lr, r.s), "fdec_lr_merge");
        // levels 1..3: Tspec -> 4 Tspec rows; the /4 bilinear resize reads only rows 4d+1, 4d+2
        const int skH[3] = {32, 128, 512};
        const int skC[3] = {192, 96, 48};
        {
            // level 2 ConvT (only rows 4d+1, 4d+2 stored; statistics over all four residues), then its merge (GN +
            // GELU + resize + skip) fused with level 3 + resize + skip + freq_out 1x1 (4 -> 2) in one pass over the
            // stored ConvT rows (dec_last.hip::fdec_tail_kernel)
            const DecW& w = c->fdec[2];
            double* sti = r.stats(NI);
            conv_t(r, w, b.D, ab, NI, (int)Ts, (int)Ts, b.G, ab, sti, 1, "fdec2");
            KStage kst3("fdec3");
            DecLastDesc dl;
            dl.g = b.G; dl.g_bf16 = ab; dl.stats = sti; dl.gn_count = 4 * Ts * Ts * w.cout; dl.gn_w = w.gnw; dl.gn_b = w.gnb;
            dl.fast_gelu = ab; dl.skip2 = sv[1]; dl.skip2_bf16 = ab; dl.H_skip2 = skH[1]; dl.C_skip2 = skC[1];
            dl.NI = NI; dl.P = P; dl.H = (int)Ts; dl.W = (int)Ts;
            // level-3 skip = saved[0][:, :4]: the compact copy the encoder wrote (4 channels per row)
            dl.fold = c->flast; dl.skip = eoff(b.sk4, s0 * 512 * Ts * 4, ea); dl.skip_bf16 = ab; dl.H_skip = skH[2];
            dl.C_skip = 4;
            dl.out = FO;
            r.check(fdec_tail_launch(dl, r.s), "fdec_tail");
        }
    }

    // ---- time decoder (ATHTDemucs_v2.py:125-139, 313-321) ----
    float* xt2 = nullptr;                            // time_out(time decoder) [NI][T][2]
    r.s = s_t;
    text_attn(b.xt_enc + s0 * d.Nt * 384, b.xt_enc_b ? b.xt_enc_b + s0 * d.Nt * 384 : nullptr, d.Nt, b.xt_cond, b.Hmt, b.Ybt);
    if (!serial_branches(r)) (void)hipEventRecord(c->ev_t, s_t);   // tc0 / tc2 read: the next chunk may rewrite them
    {
        const void* svt[4] = {eoff(b.saved_t[0], s0 * d.L[1] * 48, ea), eoff(b.saved_t[1], s0 * d.L[2] * 96, ea),
                              eoff(b.saved_t[2], s0 * d.L[3] * 192, ea), eoff(b.saved_t[3], s0 * d.L[4] * 384, ea)};
        const void* A = b.xt_cond;
        int64_t Lin = d.Nt;
        static const char* const kT[3] = {"tdec0", "tdec1", "tdec2"};
        for (int i = 0; i < 3; ++i) {
            const DecW& w = c->tdec[i];
            double* st = r.stats(NI);
            conv_t(r, w, A, ab, NI, (int)Lin, 1, b.Gt, ab, st, -1, kT[i]);
            KStage kst(kT[i]);
            const int64_t target = d.L[3 - i];       // lengths_t reversed
            MergeDesc m;
            m.src = b.Gt; m.src_bf16 = ab; m.H_src = (int)(4 * Lin); m.kept = 0; m.C = w.cout; m.fast_gelu = ab;
            m.stats = st; m.gn_count = 4 * Lin * w.cout; m.gn_w = w.gnw; m.gn_b = w.gnb;
            m.skip = svt[3 - i]; m.skip_bf16 = ab; m.H_skip = (int)d.L[4 - i]; m.C_skip = ENC_CH[3 - i]; m.P = P;
            m.out = b.Dt; m.out_bf16 = ab; m.H_out = (int)target; m.W = 1; m.NI = NI;
            if (i == 2) {
                // level 2's merge fused with level 3 + resize + skip + time_out 1x1 (4 -> 2) when 4 L1 == T
                // (dec_last.hip::tdec_tail_kernel): one pass over the ConvT output, xt2 -> D
                DecLastDesc dl;
                dl.g = b.Gt; dl.g_bf16 = ab; dl.Hg = (int)(4 * Lin); dl.stats = st; dl.gn_count = m.gn_count;
                dl.gn_w = w.gnw; dl.gn_b = w.gnb; dl.fast_gelu = ab;
                dl.skip2 = svt[1]; dl.skip2_bf16 = ab; dl.H_skip2 = (int)d.L[2]; dl.C_skip2 = ENC_CH[1];
                dl.NI = NI; dl.P = P; dl.H = (int)target; dl.T = d.T;
                dl.fold = c->tlast; dl.skip = eoff(b.sk4t, s0 * d.L[1] * 4, ea); dl.skip_bf16 = ab; dl.H_skip = (int)d.L[1];
                dl.C_skip = 4;
                dl.out = b.Dt;
                if (tdec_tail_supported(dl)) {
                    KStage kst3("tdec3");
                    r.check(tdec_tail_launch(dl, r.s), "tdec_tail");
                    xt2 = b.Dt;
                    break;
                }
            }
            r.check(dec_merge_launch(m, r.s), "dec_merge");
            A = b.Dt;
            Lin = target;
        }
        if (!xt2) {
            // ragged T: level 3 + resize + skip + time_out 1x1 (4 -> 2) over the merged 48-channel input (dec_last.hip)
            KStage kst("tdec3");
            DecLastDesc dl;
            dl.in = b.Dt; dl.in_bf16 = ab; dl.NI = NI; dl.P = P; dl.H = (int)Lin; dl.T = d.T;
            dl.fold = c->tlast; dl.skip = eoff(b.sk4t, s0 * d.L[1] * 4, ea); dl.skip_bf16 = ab; dl.H_skip = (int)d.L[1];
            dl.C_skip = 4;
            dl.out = b.Gt;
            r.check(tdec_last_launch(dl, r.s), "tdec_last");
            xt2 = b.Gt;
        }
    }
    // join on the SECOND stream: the iSTFT runs there after both branches, so the next chunk's decoder (main stream)
    // overlaps it; its time branch follows it on the second stream in stream order (xt2 is the time decoder's buffer),
    // and forward_impl joins the second stream back into the caller's after the last chunk
    (void)hipEventRecord(c->ev_f, s_main);
    (void)hipStreamWaitEvent(s_t, c->ev_f, 0);
    r.s = s_t;
    // ---- mask + iSTFT + overlap-add + denorm + branch sum (ATHTDemucs_v2.py:297-324), one fused pass ----
    b.xt2 = xt2;
    {
        KStage kst("istft");
        istft_ola_launch(FO, NI, (int)Ts, P, d.T, b.specT + s0 * 2048 * Ts * 4, c->tw, r.actbf ? nullptr : c->tw64,
                         c->win, c->win2, xt2, b.tnorm_std + 2 * s0, out + s0 * P * 2 * d.T, b.ola_part, r.s);
    }
    r.s = s_main;
}

// Debug aid: ATHD_DUMP=<dir> makes the forward synchronise at the end and write the main intermediates of the
// first decode chunk as raw little-endian arrays (<dir>/<name>.f32 / .f64) plus <dir>/index.txt with shapes.
void dump_all(const Dims& d, const Bufs& b, hipStream_t s) {
    const char* dir = std::getenv("ATHD_DUMP");
    if (!dir || !*dir) return;
    if (hipStreamSynchronize(s) != hipSuccess) return;
    const int64_t B = d.B, Ts = d.Tspec, NI = std::min(d.B, d.Bc) * d.P;
    struct E { std::string name; const void* p; int64_t n; std::string shape; };
    std::vector<E> es = {
        {"specT", b.specT, B * Ts * 2048 * 4, "B,Ts,2048,4"},
        {"snorm", b.snorm, 2 * B, "B,2"},
        {"tnorm_std", b.tnorm_std, 2 * B, "B,2"},
        {"x_enc", b.x_enc, B * d.Nf * 384, "B,Nf,384"},
        {"xt_enc", b.xt_enc, B * d.Nt * 384, "B,Nt,384"},
        {"x_cond", b.x_cond, NI * d.Nf * 384, "NI,Nf,384"},
        {"xt_cond", b.xt_cond, NI * d.Nt * 384, "NI,Nt,384"},
        {"FO", b.FO, NI * Ts * Ts * 2, "NI,t,row,2"},
        {"XT2", b.xt2, NI * d.T * 2, "NI,T,2"},
    };
    for (int i = 0; i < 4 && b.ea == 4; ++i) {      // encoder activations are f32 only in parity mode
        es.push_back({"saved" + std::to_string(i), b.saved[i], B * d.F[i + 1] * Ts * ENC_CH[i], "B,F,Ts,C"});
        es.push_back({"saved_t" + std::to_string(i), b.saved_t[i], B * d.L[i + 1] * ENC_CH[i], "B,L,C"});
    }
    for (int i = 0; i < 4 && b.ea == 2; ++i) {      // bf16 mode: the encoder levels as raw bf16 (<name>.bf16)
        for (int tb = 0; tb < 2; ++tb) {            // (freq level, time level)
            const int64_t n = tb ? B * d.L[i + 1] * ENC_CH[i] : B * d.F[i + 1] * Ts * ENC_CH[i];
            std::vector<uint16_t> h((size_t)n);
            if (hipMemcpy(h.data(), tb ? b.saved_t[i] : b.saved[i], (size_t)n * 2, hipMemcpyDeviceToHost) != hipSuccess)
                continue;
            std::string fn = std::string(dir) + (tb ? "/saved_t" : "/saved") + std::to_string(i) + ".bf16";
            FILE* f = std::fopen(fn.c_str(), "wb");
            if (f) { std::fwrite(h.data(), 2, h.size(), f); std::fclose(f); }
        }
    }
    {   // the decoder's scratch buffers as raw bytes (<name>.raw; sizes from the arena order in plan())
        struct Rw { const char* name; const void* p; const void* end; };
        const Rw rws[] = {{"G", b.G, b.D}, {"D", b.D, b.Gt}, {"Gt", b.Gt, b.Dt}, {"Dt", b.Dt, b.S}, {"S", b.S, b.Z},
                          {"Z", b.Z, b.Zs}, {"Zs", b.Zs, b.FO}, {"stats", b.stats, b.specT}};
        for (const auto& e : rws) {
            if (!e.p || !e.end || e.end <= e.p) continue;
            std::vector<char> h((size_t)((const char*)e.end - (const char*)e.p));
            if (hipMemcpy(h.data(), e.p, h.size(), hipMemcpyDeviceToHost) != hipSuccess) continue;
            std::string fn = std::string(dir) + "/" + e.name + ".raw";
            FILE* f = std::fopen(fn.c_str(), "wb");
            if (f) { std::fwrite(h.data(), 1, h.size(), f); std::fclose(f); }
        }
    }
    std::string idx = std::string(dir) + "/index.txt";
    FILE* fi = std::fopen(idx.c_str(), "w");
    for (const auto& e : es) {
        std::vector<float> h((size_t)e.n);
        if (hipMemcpy(h.data(), e.p, (size_t)e.n * 4, hipMemcpyDeviceToHost) != hipSuccess) continue;
        std::string fn = std::string(dir) + "/" + e.name + ".f32";
        FILE* f = std::fopen(fn.c_str(), "wb");
        if (f) { std::fwrite(h.data(), 4, h.size(), f); std::fclose(f); }
        if (fi) std::fprintf(fi, "%s %lld %s\n", e.name.c_str(), (long long)e.n, e.shape.c_str());
    }
    if (fi) std::fclose(fi);
}

int forward_impl(athd_ctx* c, const float* wav, int64_t B, int64_t T, const float* text, bool per_item, int P,
                 float* out, void* ws, size_t ws_bytes, void* stream) {
    if (!c) return ATHD_EINVAL;
    if (!c->finalized) return c->fail(ATHD_ESTATE, "athd_forward before athd_finalize");
    if (!wav || !text || !out || B <= 0 || T <= 0 || P <= 0) return c->fail(ATHD_EINVAL, "bad forward arguments");
    if (P > 256) return c->fail(ATHD_EINVAL, "at most 256 prompts per athd_forward_prompts call");
    if (T > (int64_t)1 << 26) return c->fail(ATHD_EINVAL, "segment too long");
    const Dims d = make_dims(c, B, T, P);
    Bufs b;
    Arena sz;
    const size_t need = plan(sz, d, b, c->mode == 1);
    if (!ws || ws_bytes < need) return c->fail(ATHD_EWORKSPACE, "workspace too small: need " + std::to_string(need));
    Arena ar;
    ar.base = (char*)ws;
    plan(ar, d, b, c->mode == 1);
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(ATHD_EHIP, "hipSetDevice failed");
    Run r;
    r.c = c;
    r.b = &b;
    r.s = (hipStream_t)stream;
    r.mode = c->mode;
    r.actbf = c->mode == 1;
    r.st_next = b.stats;
    if (hipMemsetAsync(b.stats, 0, (size_t)b.nstats * 2 * sizeof(double), r.s) != hipSuccess)
        return c->fail(ATHD_EHIP, "memset failed");
    struct ProfBind {   // route this call's launches into the context's profile window (prof.h)
        KProf* saved;
        explicit ProfBind(KProf* p) : saved(t_kprof) { t_kprof = p; }
        ~ProfBind() { t_kprof = saved; }
    } prof_bind(c->prof);
    encode(r, d, b, wav);
    for (int64_t ch = 0; ch < d.chunks && r.err == 0; ++ch) {
        const int64_t s0 = ch * d.Bc;
        const int64_t bc = std::min(d.Bc, B - s0);
        decode_chunk(r, d, b, s0, bc, text, per_item, out, (ch & 1) && b.FO2 ? b.FO2 : b.FO);
    }
    if (r.err == 0 && !serial_branches(r)) {      // the last chunk's iSTFT (second stream) joins the caller's stream
        (void)hipEventRecord(c->ev_t, c->s_time);
        (void)hipStreamWaitEvent(r.s, c->ev_t, 0);
    }
    if (d.chunks == 1) dump_all(d, b, r.s);
    if (r.err) return c->fail(ATHD_EHIP, "launch failed in " + r.what + " (code " + std::to_string(r.err) + ")");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return c->fail(ATHD_EHIP, std::string("HIP error: ") + hipGetErrorString(e));
    return ATHD_OK;
}

}  // namespace

extern "C" {

size_t athd_workspace_bytes(athd_ctx* c, int64_t B, int64_t T, int P) {
    if (!c || B <= 0 || T <= 0 || P <= 0) return 0;
    Bufs b;
    Arena a;
    return plan(a, make_dims(c, B, T, P), b, c->mode == 1);
}

int athd_forward(athd_ctx* c, const float* wav, int64_t B, int64_t T, const float* text_emb, float* out, void* ws,
                 size_t ws_bytes, void* stream) {
    return forward_impl(c, wav, B, T, text_emb, true, 1, out, ws, ws_bytes, stream);
}

int athd_forward_prompts(athd_ctx* c, const float* wav, int64_t B, int64_t T, const float* text_table, int P,
                         float* out, void* ws, size_t ws_bytes, void* stream) {
    return forward_impl(c, wav, B, T, text_table, false, P, out, ws, ws_bytes, stream);
}

}  // extern "C"
