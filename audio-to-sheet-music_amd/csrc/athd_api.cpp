// athd C-ABI: weight staging/packing and the per-segment forward orchestration.
//
// Data layout in HBM (all channels-last, fp32 unless noted; bf16 mode keeps GEMM-operand intermediates in bf16):
//   spec      [B][2048][Tspec][4]       CaC spectrogram {Re L, Im L, Re R, Im R} (also the complex z for masking)
//   saved[i]  [B][F_i][Tspec][C_i]      freq encoder outputs, F = 512/128/32/8, C = 48/96/192/384
//   saved_t[i][B][L_i][C_i]             time encoder outputs, L = ceil(T/4), ...
//   X / XT    [B][Nf][512] / [B][Nt][512]  transformer tokens; freq tokens kept in (f, t) order (the reference
//                                      uses (t f); attention and GroupNorm are order-free, positions are indexed
//                                      explicitly, so only the summation order differs)
//   decoder   [items][rows][W][C]       items = segments x prompts
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/athd.h"
#include "attn.h"
#include "gemm.h"
#include "kernels.h"
#include "ctx.h"

namespace {


std::vector<std::pair<std::string, std::vector<int64_t>>> required_keys() {
    std::vector<std::pair<std::string, std::vector<int64_t>>> r;
    auto dconv = [&](const std::string& p, int64_t c) {
        int64_t h = c / 8;
        for (int d = 0; d < 2; ++d) {
            std::string q = p + ".dconv.layers." + std::to_string(d);
            r.push_back({q + ".0.weight", {h, c, 3}});
            r.push_back({q + ".0.bias", {h}});
            r.push_back({q + ".1.weight", {h}});
            r.push_back({q + ".1.bias", {h}});
            r.push_back({q + ".3.weight", {2 * c, h, 1}});
            r.push_back({q + ".3.bias", {2 * c}});
            r.push_back({q + ".4.weight", {2 * c}});
            r.push_back({q + ".4.bias", {2 * c}});
            r.push_back({q + ".6.scale", {c}});
        }
    };
    int64_t cf = 4, ct = 2;
    for (int i = 0; i < 4; ++i) {
        int64_t c = ENC_CH[i];
        std::string p = "htdemucs.encoder." + std::to_string(i);
        r.push_back({p + ".conv.weight", {c, cf, 8, 1}});
        r.push_back({p + ".conv.bias", {c}});
        dconv(p, c);
        r.push_back({p + ".rewrite.weight", {2 * c, c, 1, 1}});
        r.push_back({p + ".rewrite.bias", {2 * c}});
        p = "htdemucs.tencoder." + std::to_string(i);
        r.push_back({p + ".conv.weight", {c, ct, 8}});
        r.push_back({p + ".conv.bias", {c}});
        dconv(p, c);
        r.push_back({p + ".rewrite.weight", {2 * c, c, 1}});
        r.push_back({p + ".rewrite.bias", {2 * c}});
        cf = ct = c;
    }
    r.push_back({"htdemucs.freq_emb.embedding.weight", {512, 48}});
    for (const char* s : {"", "_t"}) {
        std::string u = std::string("htdemucs.channel_upsampler") + s, d = std::string("htdemucs.channel_downsampler") + s;
        r.push_back({u + ".weight", {512, 384, 1}});
        r.push_back({u + ".bias", {512}});
        r.push_back({d + ".weight", {384, 512, 1}});
        r.push_back({d + ".bias", {384}});
    }
    const std::string ct_ = "htdemucs.crosstransformer";
    for (const char* s : {".norm_in", ".norm_in_t"}) {
        r.push_back({ct_ + s + ".weight", {512}});
        r.push_back({ct_ + s + ".bias", {512}});
    }
    for (int idx = 0; idx < 5; ++idx) {
        bool cross = idx % 2 == 1;
        for (const char* br : {".layers.", ".layers_t."}) {
            std::string p = ct_ + br + std::to_string(idx);
            std::string a = p + (cross ? ".cross_attn" : ".self_attn");
            r.push_back({a + ".in_proj_weight", {1536, 512}});
            r.push_back({a + ".in_proj_bias", {1536}});
            r.push_back({a + ".out_proj.weight", {512, 512}});
            r.push_back({a + ".out_proj.bias", {512}});
            r.push_back({p + ".linear1.weight", {2048, 512}});
            r.push_back({p + ".linear1.bias", {2048}});
            r.push_back({p + ".linear2.weight", {512, 2048}});
            r.push_back({p + ".linear2.bias", {512}});
            for (const char* n : {".norm1", ".norm2", ".norm3", ".norm_out"}) {
                if (!cross && std::string(n) == ".norm3") continue;
                r.push_back({p + n + ".weight", {512}});
                r.push_back({p + n + ".bias", {512}});
            }
            r.push_back({p + ".gamma_1.scale", {512}});
            r.push_back({p + ".gamma_2.scale", {512}});
        }
    }
    const std::string ta = "text_attn";
    r.push_back({ta + ".v_proj.weight", {384, 512}});
    r.push_back({ta + ".v_proj.bias", {384}});
    r.push_back({ta + ".attn.in_proj_weight", {1152, 384}});
    r.push_back({ta + ".attn.in_proj_bias", {1152}});
    r.push_back({ta + ".attn.out_proj.weight", {384, 384}});
    r.push_back({ta + ".attn.out_proj.bias", {384}});
    r.push_back({ta + ".out_mlp.0.weight", {384, 384}});
    r.push_back({ta + ".out_mlp.0.bias", {384}});
    r.push_back({ta + ".out_mlp.2.weight", {384, 384}});
    r.push_back({ta + ".out_mlp.2.bias", {384}});
    r.push_back({ta + ".norm_out.weight", {384}});
    r.push_back({ta + ".norm_out.bias", {384}});
    for (const char* name : {"freq_decoder", "time_decoder"}) {
        bool fr = std::string(name) == "freq_decoder";
        for (int i = 0; i < 4; ++i) {
            std::string p = std::string(name) + ".layers." + std::to_string(i);
            std::vector<int64_t> ws = {DEC_CH[i], DEC_CH[i + 1], 8};
            if (fr) ws.push_back(1);
            r.push_back({p + ".0.weight", ws});
            r.push_back({p + ".0.bias", {DEC_CH[i + 1]}});
            if (i < 3) {
                r.push_back({p + ".1.weight", {DEC_CH[i + 1]}});
                r.push_back({p + ".1.bias", {DEC_CH[i + 1]}});
            }
        }
    }
    r.push_back({"freq_out.weight", {2, 4, 1, 1}});
    r.push_back({"freq_out.bias", {2}});
    r.push_back({"time_out.weight", {2, 4, 1}});
    r.push_back({"time_out.bias", {2}});
    return r;
}

const std::vector<std::pair<std::string, std::vector<int64_t>>>& keys() {
    static const auto k = required_keys();
    return k;
}


}  // namespace

// =============================================================================================== ABI
extern "C" {

int athd_version(void) { return 101; }

int athd_num_required_keys(void) { return (int)keys().size(); }

const char* athd_required_key(int i) {
    if (i < 0 || i >= (int)keys().size()) return nullptr;
    return keys()[i].first.c_str();
}

int athd_create(athd_ctx** out, int device, int dtype) {
    if (!out || (dtype != ATHD_F32 && dtype != ATHD_BF16)) return ATHD_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return ATHD_EHIP;
    athd_ctx* c = new athd_ctx();
    c->device = device;
    c->mode = dtype;
    *out = c;
    return ATHD_OK;
}

int athd_set_weight(athd_ctx* c, const char* key, const void* host, const int64_t* shape, int ndim, int src_dtype) {
    if (!c || !key || !host || (ndim > 0 && !shape)) return ATHD_EINVAL;
    if (c->finalized) return c->fail(ATHD_ESTATE, "athd_set_weight after finalize");
    if (src_dtype != 0) return c->fail(ATHD_EINVAL, std::string("only fp32 host weights are accepted: ") + key);
    bool needed = false;
    for (const auto& k : keys())
        if (k.first == key) { needed = true; break; }
    if (!needed) return ATHD_OK;   // strict=False: ignore keys outside the hot path
    HostT t;
    int64_t n = 1;
    for (int i = 0; i < ndim; ++i) { t.shape.push_back(shape[i]); n *= shape[i]; }
    t.v.assign((const float*)host, (const float*)host + n);
    c->host[key] = std::move(t);
    return ATHD_OK;
}

int athd_finalize(athd_ctx* c) {
    if (!c) return ATHD_EINVAL;
    if (c->finalized) return c->fail(ATHD_ESTATE, "already finalized");
    for (const auto& k : keys()) {
        auto it = c->host.find(k.first);
        if (it == c->host.end()) return c->fail(ATHD_EKEY, "missing weight: " + k.first);
        if (it->second.shape != k.second) return c->fail(ATHD_EKEY, "shape mismatch for " + k.first);
    }
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(ATHD_EHIP, "hipSetDevice failed");
    // ---- encoders ----
    int cf = 4, ct = 2;
    for (int i = 0; i < 4; ++i) {
        for (int br = 0; br < 2; ++br) {
            EncW& e = br == 0 ? c->fenc[i] : c->tenc[i];
            const int C = ENC_CH[i];
            const std::string p = std::string(br == 0 ? "htdemucs.encoder." : "htdemucs.tencoder.") + std::to_string(i);
            e.cin = br == 0 ? cf : ct;
            e.cout = C;
            e.conv = c->conv_gemm(p + ".conv.weight", p + ".conv.bias", C, e.cin, 8);
            e.rewrite = c->conv_gemm(p + ".rewrite.weight", p + ".rewrite.bias", 2 * C, C, 1, true);
            if (c->mode == 1 && (C == 48 || C == 96)) {
                // K slot 32 ks + 8 g + i <- channel 32 ks + 4 g + i (i < 4) or 32 ks + 16 + 4 g + (i - 4): the order in
                // which the fused DConv apply holds a row's updated channels (dconv.hip dconv_apply_kernel<C, NW, true>)
                const auto& w = c->W(p + ".rewrite.weight").v;     // [2C][C]
                const int K2 = (C + 31) / 32 * 32;
                std::vector<float> q((size_t)2 * C * K2, 0.f);
                for (int n = 0; n < 2 * C; ++n) {
                    const int src = athd_ctx::glu_src(n, 2 * C);
                    for (int k = 0; k < K2; ++k) {
                        const int ks = k / 32, g = (k % 32) / 8, i = k % 8;
                        const int ch = 32 * ks + (i < 4 ? 4 * g + i : 16 + 4 * g + (i - 4));
                        if (ch < C) q[(size_t)n * K2 + k] = w[(size_t)src * C + ch];
                    }
                }
                e.rewrite_perm = c->up_gemm(q, 2 * C, K2, athd_ctx::glu_order(c->W(p + ".rewrite.bias").v));
            }
            if (br == 1 && i == 0) {                      // tconv0_kernel: [C][2][8] -> [C][tap * 2 + ci]
                const auto& w0 = c->W(p + ".conv.weight").v;
                std::vector<float> t0((size_t)C * 16);
                for (int n = 0; n < C; ++n)
                    for (int ci = 0; ci < 2; ++ci)
                        for (int t = 0; t < 8; ++t) t0[(size_t)n * 16 + t * 2 + ci] = w0[((size_t)n * 2 + ci) * 8 + t];
                e.conv_f32 = c->up_f32(t0);
            }
            for (int d = 0; d < 2; ++d) {
                const std::string q = p + ".dconv.layers." + std::to_string(d);
                e.dc.c3[d] = c->conv_gemm(q + ".0.weight", q + ".0.bias", C / 8, C, 3);
                // 1x1 conv in GLU pair order; its GroupNorm affine permuted identically (fused GN->GLU epilogue)
                e.dc.c1[d] = c->conv_gemm(q + ".3.weight", q + ".3.bias", 2 * C, C / 8, 1, true);
                e.dc.g1w[d] = c->up_key(q + ".1.weight");
                e.dc.g1b[d] = c->up_key(q + ".1.bias");
                e.dc.g2w[d] = c->up_f32(athd_ctx::glu_order(c->W(q + ".4.weight").v));
                e.dc.g2b[d] = c->up_f32(athd_ctx::glu_order(c->W(q + ".4.bias").v));
                e.dc.scale[d] = c->up_key(q + ".6.scale");
                if (C <= 96) {
                    const auto& w3 = c->W(q + ".0.weight").v;      // [H][C][3] -> [H][tap*C + c]
                    const int H = C / 8;
                    std::vector<float> t3((size_t)H * 3 * C);
                    for (int j = 0; j < H; ++j)
                        for (int ci = 0; ci < C; ++ci)
                            for (int t = 0; t < 3; ++t) t3[((size_t)j * 3 + t) * C + ci] = w3[((size_t)j * C + ci) * 3 + t];
                    e.dc.w3f[d] = c->up_f32(t3);
                    if (c->mode == 1) {
                        std::vector<float> t16((size_t)16 * 3 * C, 0.f);
                        std::copy(t3.begin(), t3.end(), t16.begin());
                        e.dc.c3p[d] = c->up_gemm(t16, 16, 3 * C, {});
                    }
                    e.dc.w1f[d] = c->up_key(q + ".3.weight");        // [2C][H][1] == [2C][H]
                    e.dc.gram1[d] = c->up_f32(conv1x1_moments(c->W(q + ".3.weight").v, c->W(q + ".3.bias").v, 2 * C, H, false));
                    if (c->mode == 1)
                        e.dc.gram1b[d] = c->up_f32(conv1x1_moments(c->W(q + ".3.weight").v, c->W(q + ".3.bias").v, 2 * C, H, true));
                    e.dc.b1f[d] = c->up_key(q + ".3.bias");
                    e.dc.g2wf[d] = c->up_key(q + ".4.weight");
                    e.dc.g2bf[d] = c->up_key(q + ".4.bias");
                } else if (c->mode == 1) {      // wide levels: the 1x1's statistics from its moments (gn_gelu_mom)
                    e.dc.gram1b[d] = c->up_f32(conv1x1_moments(c->W(q + ".3.weight").v, c->W(q + ".3.bias").v, 2 * C, C / 8, true));
                }
            }
        }
        cf = ct = ENC_CH[i];
    }
    {
        const auto& w = c->W("htdemucs.freq_emb.embedding.weight").v;
        std::vector<float> t(w.size());
        for (size_t i = 0; i < w.size(); ++i) t[i] = (w[i] * 10.0f) * 0.2f;   // ScaledEmbedding * freq_emb_scale
        c->femb = c->up_f32(t);
    }
    {
        auto one = [&](const std::string& s, int N, int K) {
            const auto& w = c->W(s + ".weight").v;
            return c->up_gemm(w, N, K, c->W(s + ".bias").v);
        };
        c->up = one("htdemucs.channel_upsampler", 512, 384);
        c->down = one("htdemucs.channel_downsampler", 384, 512);
        c->up_t = one("htdemucs.channel_upsampler_t", 512, 384);
        c->down_t = one("htdemucs.channel_downsampler_t", 384, 512);
    }
    const std::string ctp = "htdemucs.crosstransformer";
    c->nin_w = c->up_key(ctp + ".norm_in.weight");
    c->nin_b = c->up_key(ctp + ".norm_in.bias");
    c->nint_w = c->up_key(ctp + ".norm_in_t.weight");
    c->nint_b = c->up_key(ctp + ".norm_in_t.bias");
    for (int idx = 0; idx < 5; ++idx) {
        for (int br = 0; br < 2; ++br) {
            TLayerW& l = br == 0 ? c->L[idx] : c->Lt[idx];
            l.cross = idx % 2 == 1;
            const std::string p = ctp + (br == 0 ? ".layers." : ".layers_t.") + std::to_string(idx);
            const std::string a = p + (l.cross ? ".cross_attn" : ".self_attn");
            // bf16 mode: the query projection is prescaled by (1/sqrt(64)) * log2(e) so that the attention kernel's
            // scores come out in log2 units (attn.hip, attn32_kernel); f32 mode keeps the reference weights
            const float qs = c->mode == 1 ? ATTN_Q_PRESCALE : 1.f;
            if (l.cross) {
                l.q = c->lin_gemm(a + ".in_proj_weight", a + ".in_proj_bias", 0, 512, 512, qs);
                l.kv = c->lin_gemm(a + ".in_proj_weight", a + ".in_proj_bias", 512, 1024);
            } else {
                l.qkv = c->lin_gemm(a + ".in_proj_weight", a + ".in_proj_bias", 0, -1, 512, qs);
            }
            l.out = c->lin_gemm(a + ".out_proj.weight", a + ".out_proj.bias");
            l.l1 = c->lin_gemm(p + ".linear1.weight", p + ".linear1.bias");
            l.l2 = c->lin_gemm(p + ".linear2.weight", p + ".linear2.bias");
            l.n1w = c->up_key(p + ".norm1.weight");
            l.n1b = c->up_key(p + ".norm1.bias");
            l.n2w = c->up_key(p + ".norm2.weight");
            l.n2b = c->up_key(p + ".norm2.bias");
            if (l.cross) {
                l.n3w = c->up_key(p + ".norm3.weight");
                l.n3b = c->up_key(p + ".norm3.bias");
            }
            l.now = c->up_key(p + ".norm_out.weight");
            l.nob = c->up_key(p + ".norm_out.bias");
            l.g1 = c->up_key(p + ".gamma_1.scale");
            l.g2 = c->up_key(p + ".gamma_2.scale");
        }
    }
    // ---- text cross-attention (closed form: single key => softmax == 1) ----
    // v = Wv t + bv, vi = Wiv v + biv (the value third of in_proj), a = Wo vi + bo, c0 = W0 a + b0: affine in t, composed
    // in double into a = Ma t + ma and c0 = Mc t + mc (384 x 512), uploaded transposed for text_vec_kernel
    {
        const auto& wv = c->W("text_attn.v_proj.weight").v;          // [384][512]
        const auto& bv = c->W("text_attn.v_proj.bias").v;
        const auto& wi = c->W("text_attn.attn.in_proj_weight").v;     // [1152][384]: rows 768.. = value
        const auto& bi = c->W("text_attn.attn.in_proj_bias").v;
        const auto& wo = c->W("text_attn.attn.out_proj.weight").v;    // [384][384]
        const auto& bo = c->W("text_attn.attn.out_proj.bias").v;
        const auto& w0 = c->W("text_attn.out_mlp.0.weight").v;        // [384][384]
        const auto& b0 = c->W("text_attn.out_mlp.0.bias").v;
        constexpr int D = 384, TD = 512;
        // M' = L . M, m' = L . m + l for L [D][D], M [D][TD]
        auto compose = [&](const float* L, const float* l, const std::vector<double>& M, const std::vector<double>& m,
                           std::vector<double>& Mo, std::vector<double>& mo) {
            Mo.assign((size_t)D * TD, 0.0);
            mo.assign(D, 0.0);
            for (int r = 0; r < D; ++r) {
                double* row = &Mo[(size_t)r * TD];
                double acc = l[r];
                for (int q = 0; q < D; ++q) {
                    const double lv = L[(size_t)r * D + q];
                    const double* mr = &M[(size_t)q * TD];
                    for (int k = 0; k < TD; ++k) row[k] += lv * mr[k];
                    acc += lv * m[q];
                }
                mo[r] = acc;
            }
        };
        std::vector<double> M0((size_t)D * TD), m0(D), M1, m1, Ma, ma, Mc, mc;
        for (size_t i = 0; i < M0.size(); ++i) M0[i] = wv[i];
        for (int r = 0; r < D; ++r) m0[r] = bv[r];
        compose(wi.data() + 768 * 384, bi.data() + 768, M0, m0, M1, m1);
        compose(wo.data(), bo.data(), M1, m1, Ma, ma);
        compose(w0.data(), b0.data(), Ma, ma, Mc, mc);
        auto upT = [&](const std::vector<double>& M) {
            std::vector<float> t((size_t)TD * D);
            for (int r = 0; r < D; ++r)
                for (int k = 0; k < TD; ++k) t[(size_t)k * D + r] = (float)M[(size_t)r * TD + k];
            return c->up_f32(t);
        };
        c->ta_maT = upT(Ma);
        c->ta_mcT = upT(Mc);
        c->ta_ma = c->up_f32(std::vector<float>(ma.begin(), ma.end()));
        c->ta_mc = c->up_f32(std::vector<float>(mc.begin(), mc.end()));
    }
    c->ta_m2b = c->up_key("text_attn.out_mlp.2.bias");
    c->mlp0 = c->lin_gemm("text_attn.out_mlp.0.weight", "text_attn.out_mlp.0.bias");
    c->mlp2 = c->lin_gemm("text_attn.out_mlp.2.weight", "text_attn.out_mlp.2.bias");
    c->ta_nw = c->up_key("text_attn.norm_out.weight");
    c->ta_nb = c->up_key("text_attn.norm_out.bias");
    // ---- decoders: ConvTranspose weight [Cin][Cout][8] -> per residue [Cout][tap*Cin + ci] ----
    for (int br = 0; br < 2; ++br) {
        for (int i = 0; i < 4; ++i) {
            DecW& dw = br == 0 ? c->fdec[i] : c->tdec[i];
            const std::string p = std::string(br == 0 ? "freq_decoder" : "time_decoder") + ".layers." + std::to_string(i);
            dw.cin = DEC_CH[i];
            dw.cout = DEC_CH[i + 1];
            const auto& w = c->W(p + ".0.weight").v;
            const auto& b = c->W(p + ".0.bias").v;
            for (int pi = 0; pi < 2; ++pi) {          // rows [residue 2pi | residue 2pi+1], K = [tap0 | tap1]
                std::vector<float> pk((size_t)2 * dw.cout * 2 * dw.cin);
                std::vector<float> bb(2 * dw.cout);
                for (int h = 0; h < 2; ++h) {
                    const int r = 2 * pi + h;
                    for (int co = 0; co < dw.cout; ++co) {
                        const size_t row = (size_t)(h * dw.cout + co) * 2 * dw.cin;
                        for (int ci = 0; ci < dw.cin; ++ci) {
                            pk[row + ci] = w[((size_t)ci * dw.cout + co) * 8 + RES_K0[r]];
                            pk[row + dw.cin + ci] = w[((size_t)ci * dw.cout + co) * 8 + RES_K1[r]];
                        }
                        bb[h * dw.cout + co] = b[co];
                    }
                }
                dw.pair[pi] = c->up_gemm(pk, 2 * dw.cout, 2 * dw.cin, bb);
            }
            if (i == 2) {                             // one GEMM for all four residues (zero blocks where a
                const int co4 = 4 * dw.cout, K3 = 3 * dw.cin;   // residue does not read that row)
                std::vector<float> q((size_t)co4 * K3, 0.f);
                std::vector<float> qb(co4);
                for (int r = 0; r < 4; ++r) {
                    const int ta = RES_OFF[r] + 1;    // K column block of row u + RES_OFF[r]
                    for (int co = 0; co < dw.cout; ++co) {
                        const size_t row = (size_t)(r * dw.cout + co) * K3;
                        for (int ci = 0; ci < dw.cin; ++ci) {
                            q[row + (size_t)ta * dw.cin + ci] = w[((size_t)ci * dw.cout + co) * 8 + RES_K0[r]];
                            q[row + (size_t)(ta + 1) * dw.cin + ci] = w[((size_t)ci * dw.cout + co) * 8 + RES_K1[r]];
                        }
                        qb[r * dw.cout + co] = b[co];
                    }
                }
                dw.quad = c->up_gemm(q, co4, K3, qb);
                if (c->mode == 1 && convt4_supported(dw.cin, dw.cout, 1, 32, 1)) {
                    // convt4.hip: per row the residue pair's two input rows only (K = 2 cin)
                    const int K2 = 2 * dw.cin;
                    std::vector<uint16_t> q2((size_t)co4 * K2);
                    for (int r = 0; r < 4; ++r) {
                        const int ta = RES_OFF[r] + 1;
                        for (int co = 0; co < dw.cout; ++co)
                            for (int k = 0; k < K2; ++k)
                                q2[(size_t)(r * dw.cout + co) * K2 + k] =
                                    host_f2bf(q[(size_t)(r * dw.cout + co) * K3 + (size_t)ta * dw.cin + k]);
                    }
                    dw.ct4w = c->dalloc<uint16_t>(q2.size());
                    c->h2d(dw.ct4w, q2.data(), q2.size() * 2);
                    dw.ct4b = c->up_f32(b);
                }
            }
            if (br == 0 && i == 1) {                  // [k*cout + co][ci] for the re-associated level 1
                std::vector<float> tk((size_t)8 * dw.cout * dw.cin);
                for (int k = 0; k < 8; ++k)
                    for (int co = 0; co < dw.cout; ++co)
                        for (int ci = 0; ci < dw.cin; ++ci)
                            tk[((size_t)k * dw.cout + co) * dw.cin + ci] = w[((size_t)ci * dw.cout + co) * 8 + k];
                dw.taps = c->up_gemm(tk, 8 * dw.cout, dw.cin, {});
                dw.bias = c->up_f32(b);
            }
            if (i < 3) {
                dw.gnw = c->up_key(p + ".1.weight");
                dw.gnb = c->up_key(p + ".1.bias");
            }
        }
    }
    c->fout_w = c->up_key("freq_out.weight");
    c->fout_b = c->up_key("freq_out.bias");
    c->tout_w = c->up_key("time_out.weight");
    c->tout_b = c->up_key("time_out.bias");
    // ---- last decoder levels folded with their 1x1 output projections (dec_last.hip), in double ----
    for (int br = 0; br < 2; ++br) {
        const std::string p = std::string(br == 0 ? "freq_decoder" : "time_decoder") + ".layers.3.0.";
        const auto& w = c->W(p + "weight").v;      // [48][4][8]
        const auto& b = c->W(p + "bias").v;        // [4]
        const auto& P = c->W(br == 0 ? "freq_out.weight" : "time_out.weight").v;   // [2][4]
        const auto& pb = c->W(br == 0 ? "freq_out.bias" : "time_out.bias").v;      // [2]
        const int cin = DEC_CH[3], co = DEC_CH[4];
        auto pw = [&](int j, int ci, int k) {     // (P W_k)[j][ci]
            double a = 0.0;
            for (int cc = 0; cc < co; ++cc) a += (double)P[j * co + cc] * w[((size_t)ci * co + cc) * 8 + k];
            return a;
        };
        double pbias[2];
        for (int j = 0; j < 2; ++j) {
            pbias[j] = 0.0;
            for (int cc = 0; cc < co; ++cc) pbias[j] += (double)P[j * co + cc] * b[cc];
        }
        std::vector<float> f;
        if (br == 0) {   // Am = P W7 / 2, A0 = P (W3 + W4) / 2, Ap = P W0 / 2; P b + pb; 0.1 P
            for (int m = 0; m < 3; ++m)
                for (int j = 0; j < 2; ++j)
                    for (int ci = 0; ci < cin; ++ci)
                        f.push_back((float)(0.5 * (m == 0 ? pw(j, ci, 7) : m == 1 ? pw(j, ci, 3) + pw(j, ci, 4) : pw(j, ci, 0))));
            for (int j = 0; j < 2; ++j) f.push_back((float)(pbias[j] + pb[j]));
        } else {         // Q_k = P W_k; P b; tb; 0.1 P
            for (int k = 0; k < 8; ++k)
                for (int j = 0; j < 2; ++j)
                    for (int ci = 0; ci < cin; ++ci) f.push_back((float)pw(j, ci, k));
            for (int j = 0; j < 2; ++j) f.push_back((float)pbias[j]);
            for (int j = 0; j < 2; ++j) f.push_back(pb[j]);
        }
        for (int j = 0; j < 2; ++j)
            for (int cc = 0; cc < co; ++cc) f.push_back((float)(0.1 * P[j * co + cc]));
        (br == 0 ? c->flast : c->tlast) = c->up_f32(f);
    }
    // ---- FFT twiddles and the periodic Hann window (torch.hann_window(4096)) ----
    {
        std::vector<float2> tw(4096);
        std::vector<double2> tw64(4096);
        std::vector<float> win(4096), win2(4096);
        for (int k = 0; k < 4096; ++k) {
            const double a = -2.0 * M_PI * (double)k / 4096.0;
            tw[k] = make_float2((float)cos(a), (float)sin(a));
            tw64[k] = make_double2(cos(a), sin(a));
            const float w = (float)(0.5 - 0.5 * cos(2.0 * M_PI * (double)k / 4096.0));
            win[k] = w;
            win2[k] = w * w;
        }
        c->tw = c->dalloc<float2>(4096);
        c->h2d(c->tw, tw.data(), 4096 * sizeof(float2));
        c->tw64 = c->dalloc<double2>(4096);
        c->h2d(c->tw64, tw64.data(), 4096 * sizeof(double2));
        c->win = c->up_f32(win);
        c->win2 = c->up_f32(win2);
    }
    for (void* p : c->allocs)
        if (!p) return c->fail(ATHD_EHIP, "device allocation failed");
    if (c->upload_failed) return c->fail(ATHD_EHIP, "weight upload failed");
    // the time branch's stream and the fork / join events, made here so that athd_forward* create nothing (they
    // can then be captured in a HIP graph from the first call on)
    if (!c->s_time && hipStreamCreateWithFlags(&c->s_time, hipStreamNonBlocking) != hipSuccess)
        return c->fail(ATHD_EHIP, "stream creation failed");
    if (!c->ev_f && hipEventCreateWithFlags(&c->ev_f, hipEventDisableTiming) != hipSuccess)
        return c->fail(ATHD_EHIP, "event creation failed");
    if (!c->ev_t && hipEventCreateWithFlags(&c->ev_t, hipEventDisableTiming) != hipSuccess)
        return c->fail(ATHD_EHIP, "event creation failed");
    if (hipDeviceSynchronize() != hipSuccess) return c->fail(ATHD_EHIP, "upload failed");
    c->host.clear();
    c->finalized = true;
    return ATHD_OK;
}

int athd_set_decode_items(athd_ctx* c, int64_t items) {
    if (!c) return ATHD_EINVAL;
    if (items < 1 || items > 4096) return c->fail(ATHD_EINVAL, "decode_items must be in [1, 4096]");
    c->decode_items = items;
    return ATHD_OK;
}

int64_t athd_num_windows(int64_t length, int64_t chunk_len, int64_t overlap) {
    if (length <= 0 || chunk_len <= 0 || overlap < 0 || overlap >= chunk_len) return 0;
    const int64_t hop = chunk_len - overlap;
    return (length + hop - 1) / hop;
}

int athd_overlap_add(const float* windows, int64_t length, int64_t chunk_len, int64_t overlap, int n_stems,
                     int64_t k0, int64_t k1, float* out, void* stream) {
    const int rc = ola_launch(windows, length, chunk_len, overlap, n_stems, k0, k1, out, (hipStream_t)stream);
    return rc == 0 ? ATHD_OK : (rc == -1 ? ATHD_EINVAL : ATHD_EHIP);
}

int athd_overlap_add_weighted(const float* windows, int64_t length, int64_t chunk_len, int64_t overlap, int n_stems,
                              int64_t k0, int64_t k1, float* out, float* weight, void* stream) {
    const int rc = ola_launch(windows, length, chunk_len, overlap, n_stems, k0, k1, out, (hipStream_t)stream, 1, weight);
    return rc == 0 ? ATHD_OK : (rc == -1 ? ATHD_EINVAL : ATHD_EHIP);
}

int athd_ola_normalize(float* out, const float* weight, int rows, int64_t n, void* stream) {
    const int rc = ola_normalize_launch(out, weight, rows, n, (hipStream_t)stream);
    return rc == 0 ? ATHD_OK : (rc == -1 ? ATHD_EINVAL : ATHD_EHIP);
}

int athd_sdr(const float* est, const float* target, int64_t rows, int64_t n, double* scratch, float* out,
             void* stream) {
    const int rc = sdr_launch(est, target, rows, n, scratch, out, (hipStream_t)stream);
    return rc == 0 ? ATHD_OK : (rc == -1 ? ATHD_EINVAL : ATHD_EHIP);
}

int athd_sisdr(const float* est, const float* target, int64_t rows, int64_t n, double* scratch, float* out,
               void* stream) {
    const int rc = sisdr_launch(est, target, rows, n, scratch, out, (hipStream_t)stream);
    return rc == 0 ? ATHD_OK : (rc == -1 ? ATHD_EINVAL : ATHD_EHIP);
}

int athd_profile_start(athd_ctx* c, const char* kernel) {
    if (!c) return ATHD_EINVAL;
    delete c->prof;
    c->prof = new KProf();
    c->prof->only = kernel ? kernel : "";
    c->prof_done.agg.clear();
    return ATHD_OK;
}

int athd_profile_stop(athd_ctx* c) {
    if (!c || !c->prof) return c ? c->fail(ATHD_ESTATE, "athd_profile_stop without start") : ATHD_EINVAL;
    const int rc = c->prof->collect();
    c->prof_done.agg = c->prof->agg;
    delete c->prof;
    c->prof = nullptr;
    return rc == 0 ? ATHD_OK : c->fail(ATHD_EHIP, "profile event query failed");
}

int athd_profile_count(athd_ctx* c) { return c ? (int)c->prof_done.agg.size() : 0; }

int athd_profile_get(athd_ctx* c, int i, const char** kernel, long long* launches, double* ms, double* flops,
                     double* bytes) {
    if (!c || i < 0 || i >= (int)c->prof_done.agg.size()) return ATHD_EINVAL;
    const auto& g = c->prof_done.agg[i];
    if (kernel) *kernel = g.label.c_str();
    if (launches) *launches = g.n;
    if (ms) *ms = g.ms;
    if (flops) *flops = g.flops;
    if (bytes) *bytes = g.bytes;
    return ATHD_OK;
}

const char* athd_last_error(athd_ctx* c) { return c ? c->err.c_str() : "null context"; }

void athd_destroy(athd_ctx* c) {
    if (!c) return;
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->ev_f) (void)hipEventDestroy(c->ev_f);
    if (c->ev_t) (void)hipEventDestroy(c->ev_t);
    if (c->s_time) (void)hipStreamDestroy(c->s_time);
    delete c->prof;
    delete c;
}

}  // extern "C"
