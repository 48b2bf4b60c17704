// Flash-style multi-head attention for the cross-domain transformer (d_head = 64, 8 heads).
//
// Orientation: each wave computes S^T = K . Q^T for 64 keys x 32 queries, so the MFMA accumulator puts one
// query per lane column and 16 keys per lane in registers.  The column (query) max/sum of the online softmax
// are then in-lane reductions plus two cross-group shuffles, and P^T is already laid out as the B operand of
// O^T += V^T . P^T (the k order inside a step is permuted identically for A and B; see common comments in
// gemm.hip).  K is staged in LDS as [key][d], V transposed as [d][key].  Grid: (ceil(Nq/128), heads, batch).
#include "common.h"
#include "prof.h"
#include "attn.h"

namespace athd {

// Block -> (query block, head, batch), XCD-aware (cdna_hip_programming.md T1): block i runs on XCD i % 8, so the
// tiles (bh-major, the ceil(Nq/128) query blocks of one (b, h) consecutive) are cut into 8 contiguous ranges, one
// per XCD.  All query blocks of a (b, h) then run on one XCD at about the same time and its K / V come from HBM
// once into that XCD's L2, instead of once per XCD they were spread over.
ATHD_DEV void attn_tile(const AttnDesc& d, int& qb, int& h, int64_t& b, int qblock = 128) {
    const int n = (int)gridDim.x, i = (int)blockIdx.x;
    const int q = n / 8, r = n % 8, x = i % 8;
    const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
    const int gq = (d.Nq + qblock - 1) / qblock;
    qb = t % gq;
    const int bh = t / gq;
    h = bh % d.heads;
    b = bh / d.heads;
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16v4;

template <int MODE> struct AT;
template <> struct AT<0> { typedef float T; static constexpr int PAD = 4; };
template <> struct AT<1> { typedef bf16_t T; static constexpr int PAD = 8; };

ATHD_DEV void load8(const void* base, int is_bf16, int64_t off, float* v) {
    if (is_bf16) {
        uint4 q = *reinterpret_cast<const uint4*>((const bf16_t*)base + off);
        const bf16_t* h = reinterpret_cast<const bf16_t*>(&q);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf2f(h[j]);
    } else {
        const float4* p = reinterpret_cast<const float4*>((const float*)base + off);
        float4 a = p[0], b = p[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void attn_kernel(const AttnDesc d) {
    using T = typename AT<MODE>::T;
    constexpr int LDK = 64 + AT<MODE>::PAD;
    __shared__ __attribute__((aligned(16))) T Ks[64 * LDK];
    __shared__ __attribute__((aligned(16))) T Vt[64 * LDK];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    int qblk, h;
    int64_t b;
    attn_tile(d, qblk, h, b);
    const int q0 = qblk * 128 + wave * 32;
    const float sl2 = d.scale * 1.4426950408889634f;

    // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[q][32c + 8g + j]
    float qv[2][2][8];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int q = q0 + 16 * nt + c16;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (q < d.Nq) load8(d.Q, d.q_bf16, b * d.q_bs + (int64_t)q * d.q_ld + d.q_off + h * 64 + 32 * c + 8 * g, qv[nt][c]);
            else {
#pragma unroll
                for (int j = 0; j < 8; ++j) qv[nt][c][j] = 0.f;
            }
        }
    }
    bf16v8 qb[2][2];
    if constexpr (MODE == 1) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int j = 0; j < 8; ++j) qb[nt][c][j] = (__bf16)qv[nt][c][j];
    }

    f32x4_t o[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) o[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    float mrun[2] = {-INFINITY, -INFINITY};
    float lrun[2] = {0.f, 0.f};

    for (int k0 = 0; k0 < d.Nk; k0 += 64) {
        // ---- stage K [key][d] and V^T [d][key] ----
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int gi = tid + 256 * it;
            const int key = gi >> 3, d0 = 8 * (gi & 7);
            float kv[8], vv[8];
            if (k0 + key < d.Nk) {
                load8(d.K, d.k_bf16, b * d.k_bs + (int64_t)(k0 + key) * d.k_ld + d.k_off + h * 64 + d0, kv);
                load8(d.V, d.v_bf16, b * d.v_bs + (int64_t)(k0 + key) * d.v_ld + d.v_off + h * 64 + d0, vv);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) { kv[j] = 0.f; vv[j] = 0.f; }
            }
            if constexpr (MODE == 1) {
                bf16_t tmp[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) tmp[j] = f2bf(kv[j]);
                *reinterpret_cast<uint4*>(&Ks[key * LDK + d0]) = *reinterpret_cast<uint4*>(tmp);
#pragma unroll
                for (int j = 0; j < 8; ++j) Vt[(d0 + j) * LDK + key] = f2bf(vv[j]);
            } else {
                *reinterpret_cast<float4*>(&Ks[key * LDK + d0]) = make_float4(kv[0], kv[1], kv[2], kv[3]);
                *reinterpret_cast<float4*>(&Ks[key * LDK + d0 + 4]) = make_float4(kv[4], kv[5], kv[6], kv[7]);
#pragma unroll
                for (int j = 0; j < 8; ++j) Vt[(d0 + j) * LDK + key] = vv[j];
            }
        }
        __syncthreads();

        // ---- S^T = K Q^T : 4 key tiles x 2 query tiles ----
        f32x4_t s[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) s[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const T* kp = &Ks[(16 * mt + c16) * LDK + 32 * c + 8 * g];
                if constexpr (MODE == 1) {
                    bf16v8 a = *reinterpret_cast<const bf16v8*>(kp);
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt)
                        s[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qb[nt][c], s[mt][nt], 0, 0, 0);
                } else {
                    float4 a0 = reinterpret_cast<const float4*>(kp)[0], a1 = reinterpret_cast<const float4*>(kp)[1];
                    float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
                    for (int ss = 0; ss < 8; ++ss)
#pragma unroll
                        for (int nt = 0; nt < 2; ++nt)
                            s[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ss], qv[nt][c][ss], s[mt][nt], 0, 0, 0);
                }
            }
        }
        // ---- online softmax over keys (per query column) ----
        float p[4][2][4];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            float mx = -INFINITY;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = k0 + 16 * mt + 4 * g + r;
                    float v = (key < d.Nk) ? s[mt][nt][r] * sl2 : -INFINITY;
                    p[mt][nt][r] = v;
                    mx = fmaxf(mx, v);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float mnew = fmaxf(mrun[nt], mx);
            const float alpha = exp2f(mrun[nt] - mnew);
            mrun[nt] = mnew;
            float ls = 0.f;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float e = exp2f(p[mt][nt][r] - mnew);
                    p[mt][nt][r] = e;
                    ls += e;
                }
            lrun[nt] = lrun[nt] * alpha + ls;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 4; ++r) o[dt][nt][r] *= alpha;
        }
        // ---- O^T += V^T P^T ----
        if constexpr (MODE == 1) {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16v8 pb[2];
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        pb[nt][j] = (__bf16)p[2 * kk][nt][j];
                        pb[nt][4 + j] = (__bf16)p[2 * kk + 1][nt][j];
                    }
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const T* vp = &Vt[(16 * dt + c16) * LDK + 32 * kk + 4 * g];
                    bf16v4 lo = *reinterpret_cast<const bf16v4*>(vp);
                    bf16v4 hi = *reinterpret_cast<const bf16v4*>(vp + 16);
                    bf16v8 a;
#pragma unroll
                    for (int j = 0; j < 4; ++j) { a[j] = lo[j]; a[4 + j] = hi[j]; }
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt)
                        o[dt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[nt], o[dt][nt], 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float a = Vt[(16 * dt + c16) * LDK + 16 * mt + 4 * g + r];
#pragma unroll
                        for (int nt = 0; nt < 2; ++nt)
                            o[dt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, p[mt][nt][r], o[dt][nt], 0, 0, 0);
                    }
        }
        __syncthreads();
    }
    // ---- normalise and store O[q][h*64 + d] ----
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        float l = lrun[nt];
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float inv = 1.f / l;
        const int q = q0 + 16 * nt + c16;
        if (q >= d.Nq) continue;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int64_t off = b * d.o_bs + (int64_t)q * d.o_ld + h * 64 + 16 * dt + 4 * g;
            float4 v = make_float4(o[dt][nt][0] * inv, o[dt][nt][1] * inv, o[dt][nt][2] * inv, o[dt][nt][3] * inv);
            if (d.o_bf16) {
                bf16_t t4[4] = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                *reinterpret_cast<uint2*>((bf16_t*)d.O + off) = *reinterpret_cast<uint2*>(t4);
            } else {
                *reinterpret_cast<float4*>((float*)d.O + off) = v;
            }
        }
    }
}

// ----------------------------------------------------------------------------------------------------------------
// bf16 path.  K and V tiles (64 keys x 64 d) are stored row-major [key][d] (144-B rows) in a 2-deep LDS ring with
// 16-B writes; the next tile is prefetched into registers while the current one is computed (T14 split).  The
// PV A-operand V^T[d][keys] is read with ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses row k0+q,
// columns d0+4p..+3 and receives column d0+(lane&15) of rows k0..k0+3, i.e. 4 consecutive keys of one d.
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// defer-max threshold of the bf16 kernel's online softmax (log2 units): P <= 2^8 before the final 1/l
constexpr float ATTN_RESCALE = 8.0f;

#ifdef ATHD_KBENCH      // round-1 16x16x32 kernel: tools/kbench A/B builds only
__global__ __launch_bounds__(256, 3) void attn_bf16_kernel(const AttnDesc d) {
    constexpr int LDK = 72;                        // bf16 per LDS row (64 + 8 pad)
    __shared__ __attribute__((aligned(16))) bf16_t Ks[2][64 * LDK];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[2][64 * LDK];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    int qblk, h;
    int64_t b;
    attn_tile(d, qblk, h, b);
    const int q0 = qblk * 128 + wave * 32;
    const float sl2 = d.scale * 1.4426950408889634f;

    bf16v8 qb[2][2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int q = q0 + 16 * nt + c16;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            float v[8];
            if (q < d.Nq) load8(d.Q, d.q_bf16, b * d.q_bs + (int64_t)q * d.q_ld + d.q_off + h * 64 + 32 * c + 8 * g, v);
            else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = 0.f;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) qb[nt][c][j] = (__bf16)v[j];
        }
    }
    // tile staging: thread -> keys tid/8 and tid/8 + 32, columns 8 (tid % 8) .. +7.  Keys past Nk re-read the
    // last key (finite data; their scores are masked to -inf so P = 0), which keeps the prefetch branch-free.
    const bf16_t* Kb = (const bf16_t*)d.K + b * d.k_bs + d.k_off + h * 64;
    const bf16_t* Vb = (const bf16_t*)d.V + b * d.v_bs + d.v_off + h * 64;
    const int skey = tid >> 3, sd0 = 8 * (tid & 7);          // rows skey and skey + 32
    const int soff = skey * LDK + sd0;
    uint4 k0r, k1r, v0r, v1r;
#define ATHD_FETCH(K0)                                                                                   \
    do {                                                                                                 \
        const int ka = min((K0) + skey, d.Nk - 1), kb = min((K0) + skey + 32, d.Nk - 1);                \
        k0r = *reinterpret_cast<const uint4*>(Kb + (int64_t)ka * d.k_ld + sd0);                          \
        k1r = *reinterpret_cast<const uint4*>(Kb + (int64_t)kb * d.k_ld + sd0);                          \
        v0r = *reinterpret_cast<const uint4*>(Vb + (int64_t)ka * d.v_ld + sd0);                          \
        v1r = *reinterpret_cast<const uint4*>(Vb + (int64_t)kb * d.v_ld + sd0);                          \
    } while (0)
#define ATHD_STASH(ST)                                                                                   \
    do {                                                                                                 \
        *reinterpret_cast<uint4*>(&Ks[ST][soff]) = k0r;                                                  \
        *reinterpret_cast<uint4*>(&Ks[ST][soff + 32 * LDK]) = k1r;                                       \
        *reinterpret_cast<uint4*>(&Vs[ST][soff]) = v0r;                                                  \
        *reinterpret_cast<uint4*>(&Vs[ST][soff + 32 * LDK]) = v1r;                                       \
    } while (0)

    f32x4_t o[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) o[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    float mrun[2] = {-INFINITY, -INFINITY};
    float lrun[2] = {0.f, 0.f};

    ATHD_FETCH(0);
    ATHD_STASH(0);
    __syncthreads();
    int cur = 0;
    for (int k0 = 0; k0 < d.Nk; k0 += 64) {
        const bool more = k0 + 64 < d.Nk;
        if (more) ATHD_FETCH(k0 + 64);
        const bf16_t* K_ = Ks[cur];
        const bf16_t* V_ = Vs[cur];
        // ---- S^T = K Q^T ----
        f32x4_t s[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) s[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const bf16v8 a = *reinterpret_cast<const bf16v8*>(&K_[(16 * mt + c16) * LDK + 32 * c + 8 * g]);
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                    s[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qb[nt][c], s[mt][nt], 0, 0, 0);
            }
        // ---- online softmax (per query column) ----
        // The running max moves only when the tile max exceeds it by more than ATTN_RESCALE (log2 units; T13
        // "defer-max"): P = 2^(s - m) then stays <= 2^ATTN_RESCALE (exact in bf16's range) and the rescale of O and
        // l - an exp and 32 multiplies per lane - runs only on the tiles where some query's max really jumps.
        // Scores are scaled inside the exponent's FMA: the max is taken on the raw scores (scale > 0).
        float p[4][2][4];
        const bool tail = k0 + 64 > d.Nk;
        if (tail) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (k0 + 16 * mt + 4 * g + r >= d.Nk) {
                        s[mt][0][r] = -INFINITY;
                        s[mt][1][r] = -INFINITY;
                    }
        }
        float mnew[2];
        bool jump = false;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            float mx = -INFINITY;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
                mx = fmaxf(fmaxf(fmaxf(mx, s[mt][nt][0]), fmaxf(s[mt][nt][1], s[mt][nt][2])), s[mt][nt][3]);
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            mx *= sl2;
            const bool up = mx > mrun[nt] + ATTN_RESCALE;
            mnew[nt] = up ? mx : mrun[nt];
            jump |= up;
        }
        if (__any(jump)) {
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const float alpha = __builtin_amdgcn_exp2f(mrun[nt] - mnew[nt]);
                mrun[nt] = mnew[nt];
                lrun[nt] *= alpha;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) o[dt][nt][r] *= alpha;
            }
        }
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const float nm = -mrun[nt];
            float ls = 0.f;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float e = __builtin_amdgcn_exp2f(fmaf(s[mt][nt][r], sl2, nm));
                    p[mt][nt][r] = e;
                    ls += e;
                }
            lrun[nt] += ls;
        }
        // ---- O^T += V^T P^T ----
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16v8 pb[2];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const uint32_t w[4] = {pack2bf(p[2 * kk][nt][0], p[2 * kk][nt][1]), pack2bf(p[2 * kk][nt][2], p[2 * kk][nt][3]),
                                       pack2bf(p[2 * kk + 1][nt][0], p[2 * kk + 1][nt][1]),
                                       pack2bf(p[2 * kk + 1][nt][2], p[2 * kk + 1][nt][3])};
                pb[nt] = __builtin_bit_cast(bf16v8, w);
            }
            // tr-read addresses: lane 4q+p of group g -> row (key) k0' + q, columns d0 + 4p
            const int qrow = c16 >> 2, pcol = c16 & 3;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const bf16_t* base = &V_[(32 * kk + 4 * g + qrow) * LDK + 16 * dt + 4 * pcol];
                const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
                const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 16 * LDK));
                const bf16v8 a = __builtin_shufflevector(__builtin_bit_cast(bf16v4, lo), __builtin_bit_cast(bf16v4, hi),
                                                         0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                    o[dt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[nt], o[dt][nt], 0, 0, 0);
            }
        }
        if (more) ATHD_STASH(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        float l = lrun[nt];
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float inv = 1.f / l;
        const int q = q0 + 16 * nt + c16;
        if (q >= d.Nq) continue;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int64_t off = b * d.o_bs + (int64_t)q * d.o_ld + h * 64 + 16 * dt + 4 * g;
            const float4 v = make_float4(o[dt][nt][0] * inv, o[dt][nt][1] * inv, o[dt][nt][2] * inv, o[dt][nt][3] * inv);
            if (d.o_bf16) {
                bf16_t t4[4] = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                *reinterpret_cast<uint2*>((bf16_t*)d.O + off) = *reinterpret_cast<uint2*>(t4);
            } else {
                *reinterpret_cast<float4*>((float*)d.O + off) = v;
            }
        }
    }
}
#endif
#undef ATHD_FETCH
#undef ATHD_STASH

// ----------------------------------------------------------------------------------------------------------------
// bf16 path on v_mfma_f32_32x32x16_bf16 (prescaled queries: scores are log2-unit logits).
//
// Per wave 32 queries, per tile 64 keys.  S^T = K Q^T as two 32x32 blocks (keys x queries): lane l holds query
// r = l & 31 and keys (reg & 3) + 8 (reg >> 2) + 4 (l >> 5) of each block, so the online softmax is in-lane plus one
// exchange between the two 32-lane halves.  The accumulators start at -m (the running max) instead of 0, so the MFMA
// itself subtracts the max: p = exp2(S) is one v_exp_f32 per score.  The max moves only when a tile's scores exceed it
// by more than ATTN_RESCALE (defer-max; the rescale runs before any of the tile's P is formed).
//
// O^T += V^T P^T: for PV k-step kk (16 keys of key block kk >> 1) lane (r, h) feeds its own registers
// 8 (kk & 1) .. +7 as the B operand, i.e. keys 4h + {0..3} and 4h + 8 + {0..3} of the 16 - the k order inside the step
// is permuted, and the A operand (V^T) is read in the same permuted order with two ds_read_b64_tr_b16 (rows
// 4h + q and 4h + 8 + q).  No cross-lane movement of P.  MFMA issue per tile and wave: 8 (QK) + 8 (PV) 32x32x16 =
// 512 cycles; the 32x32 shape blocks vector issue for 8 of every 32 cycles (vs 8 of 16 for 16x16x32), which leaves
// room for the 32 exps, the max and the row sums of each lane.
//
// LDS: K [key][72] (row reads, conflict-free per 8 lanes), V [key][64] with the 16-B chunk XOR-swizzled by
// ((key >> 1) & 1) << 2 so that each 32-lane half of a transposed read (4 keys x 32 d) covers all 64 banks.  2-deep
// ring filled by LDS-DMA for the next tile before the tile's MFMAs (register-staged variant: global loads before, LDS
// writes after), one barrier per tile.  The output tile is staged through LDS and stored as whole 128-B rows.
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;   // (arrays of these stay in registers)

// s_setprio(1) around the QK^T and PV MFMA clusters (cdna_hip_programming.md T5): a wave in its MFMA cluster wins
// issue arbitration over the co-resident waves' softmax VALU; kbench A/B on one box: +3.3 % (N=2072), +4.6 % (N=1034)
#define A32_PRIO(x) __builtin_amdgcn_s_setprio(x)
typedef __attribute__((address_space(3))) void a32_lds_void;
typedef __attribute__((address_space(1))) void a32_gbl_void;

// round-6 form of attn32_kernel (DMA addressing from a uniform tile base, row-sum overflow check instead of a per-tile
// max); 0 builds the round-5 form for A/B libraries
#ifndef ATHD_ATTN_V6
#define ATHD_ATTN_V6 1
#endif
constexpr float A32_SUMCHK = 1024.0f;               // max lane row sum of a tile before the exact-max rescale
// First tile (round 6, late): the exact max is taken over the scores already in registers and subtracted from them in
// place (32 v_sub) instead of running QK^T again from -m (8 MFMAs + 32 v_mov + the K re-read): attention 3.50 ->
// 3.45 ms per forward, whole step +0.5-0.7 % (3 alternating pairs); outputs 57 dB from the recomputed form (bf16 P
// rounding of last-bit score differences).  0 builds the recomputing form for A/B.
#ifndef ATHD_ATTN_T0SUB
#define ATHD_ATTN_T0SUB 1
#endif
#ifndef ATHD_ATTN_KM
#define ATHD_ATTN_KM 0        // 1: the running max subtracted by a fifth QK^T k-step (A/B)
#endif

constexpr int A32_KP = 72;                          // K row pitch (bf16)
constexpr int A32_VP = 64;                          // V row pitch (bf16), swizzled chunks

ATHD_DEV int a32_vchunk(int key, int chunk) { return chunk ^ (((key >> 1) & 1) << 2); }

// value of lane l ^ 32 combined with the lane's own, by v_permlane32_swap (no LDS round trip)
ATHD_DEV float half_swap_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
ATHD_DEV float half_swap_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// v_max3_f32 without the canonicalising v_max(x, x) that fmaxf puts on MFMA results (inputs are never NaN here).
// HAZARD (round 6, tools/hazard/README.md): hipcc inserts no wait states before an inline-asm instruction that reads
// an MFMA result (or a v_exp / v_rcp result): an asm VALU right after v_mfma_f32_32x32x16_bf16 reads the accumulator
// registers before the MFMA has written them, where compiler-emitted VALU reads get s_nop 9.  The round-2..5 kernel's
// per-tile max read the last QK^T MFMA's accumulators this way (a max of partly accumulated scores); the round-6
// kernel's max (tile_max, first tile and rare rescales only) puts explicit wait states before it.
ATHD_DEV float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// exp2 on the FMA pipe (VERDICT r04 #3 experiment; kbench builds with -DATHD_ATTN_POLY=n, the product keeps n = 0):
// x -> n + f with n = rint(x) by the 1.5 * 2^23 magic add (its low mantissa bits hold n), 2^f on [-0.5, 0.5] as a
// degree-3 polynomial fitted to the relative error (max 1.4e-4, below bf16's 2^-9), and n added to the exponent field by
// one v_lshl_add_u32 ((bits(t) << 23) == n << 23 mod 2^32).  Arguments below -126 are clamped (P underflows to ~0).
#ifndef ATHD_ATTN_POLY
#define ATHD_ATTN_POLY 0        // exp2 calls of every 16 per key block evaluated by exp2_poly
#endif
ATHD_DEV float exp2_poly(float x) {
    x = __builtin_fmaxf(x, -126.0f);
    const float t = x + 12582912.0f;
    const float f = x - (t - 12582912.0f);
    const float p = fmaf(fmaf(fmaf(0.05502927f, f, 0.24225698f), f, 0.69325305f), f, 0.99995134f);
    return __uint_as_float((__float_as_uint(t) << 23) + __float_as_uint(p));
}

#define ATHD_A32_QK(INIT)                                                                                      \
    do {                                                                                                       \
        const float init_ = (INIT);                                                                            \
        _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb)                                                    \
            _Pragma("unroll") for (int i = 0; i < 16; ++i) sc[kb][i] = init_;                                  \
        _Pragma("unroll") for (int ks = 0; ks < 4; ++ks)                                                      \
            _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb) {                                              \
                const bf16v8 a_ = *reinterpret_cast<const bf16v8*>(&K_[a32_kidx<DMA>(32 * kb + r, 2 * ks + hh)]); \
                sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_, qf[ks], sc[kb], 0, 0, 0);                 \
            }                                                                                                  \
        if (kt0 + KT > d.Nk) {                                                                                 \
            int lim_ = d.Nk - kt0 - 4 * hh;            /* key index - kt0 - 4 hh vs constants: no per-key adds */ \
            asm volatile("" : "+v"(lim_));             /* (keeps the compares in this branch, not hoisted) */  \
            _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb)                                                \
                _Pragma("unroll") for (int i = 0; i < 16; ++i)                                                 \
                    if (32 * kb + (i & 3) + 8 * (i >> 2) >= lim_) sc[kb][i] = -INFINITY;                       \
        }                                                                                                      \
    } while (0)
// ATHD_ATTN_KM: the running max enters the scores as a fifth k-step of QK^T (K's column 64 is 1, Q's is -mrun, kept
// bf16-exact), so the accumulators start from the inline constant 0 instead of 16 v_mov of -mrun per tile (the
// fifth-step MFMA is the same for both key blocks: one extra MFMA per tile)
#define ATHD_A32_QKM()                                                                                         \
    do {                                                                                                       \
        _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb)                                                    \
            sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k5, q5, (f32x16_t){}, 0, 0, 0);                \
        _Pragma("unroll") for (int ks = 0; ks < 4; ++ks)                                                      \
            _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb) {                                              \
                const bf16v8 a_ = *reinterpret_cast<const bf16v8*>(&K_[a32_kidx<DMA>(32 * kb + r, 2 * ks + hh)]); \
                sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_, qf[ks], sc[kb], 0, 0, 0);                 \
            }                                                                                                  \
        if (kt0 + KT > d.Nk) {                                                                                 \
            int lim_ = d.Nk - kt0 - 4 * hh;                                                                    \
            asm volatile("" : "+v"(lim_));                                                                     \
            _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb)                                                \
                _Pragma("unroll") for (int i = 0; i < 16; ++i)                                                 \
                    if (32 * kb + (i & 3) + 8 * (i >> 2) >= lim_) sc[kb][i] = -INFINITY;                       \
        }                                                                                                      \
    } while (0)
#if ATHD_ATTN_KM
#define ATHD_A32_QKX() ATHD_A32_QKM()
#else
#define ATHD_A32_QKX() ATHD_A32_QK(-mrun)
#endif

// K tile element index of (key, 16-B chunk).  Register-staged: row pitch 72 (padding).  LDS-DMA staged: pitch 64,
// chunk XOR-swizzled by (key >> 1) & 7 - the QK^T fragment reads (lanes = 32 consecutive keys, one chunk) then put the
// 16 lanes of every ds_read_b128 group on 16 distinct 4-bank groups (key & 1 picks the bank half of the 128-B row).
template <bool DMA>
ATHD_DEV int a32_kidx(int key, int chunk) {
    if constexpr (DMA) return key * 64 + 8 * (chunk ^ ((key >> 1) & 7));
    else return key * A32_KP + 8 * chunk;
}

// DMA: K / V tiles staged by global_load_lds_dwordx4 straight into LDS (no VGPR round trip and none of the
// ds_write_b128 transfer cost, which with 4 waves' 16 KB of fragment reads per tile kept the LDS ~90 % busy).  One
// wave instruction fills 1 KB = 8 keys x 128 B, lane -> (key base + lane / 8, physical chunk lane % 8); the lane fetches
// the logical chunk that the tile's swizzle places there.
template <int MINW, int NKB, bool DMA = false>
__global__ __launch_bounds__(256, MINW) void attn32_kernel(const AttnDesc d) {
    constexpr int KT = 32 * NKB;                                  // keys per tile
    constexpr int KSZ = KT * (DMA ? 64 : A32_KP);                 // K slot elements
    // K ring, V ring; the output staging (4 waves x 32 rows x 72) reuses the front
    constexpr int SMEM_E = 2 * KSZ + 2 * KT * A32_VP;
    static_assert(SMEM_E >= 4 * 32 * A32_KP, "output staging fits");
    __shared__ __attribute__((aligned(16))) bf16_t smem_a32[SMEM_E];
    bf16_t (*Ks)[KSZ] = reinterpret_cast<bf16_t (*)[KSZ]>(smem_a32);
    bf16_t (*Vs)[KT * A32_VP] = reinterpret_cast<bf16_t (*)[KT * A32_VP]>(smem_a32 + 2 * KSZ);

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    int qblk, h;
    int64_t b;
    attn_tile(d, qblk, h, b);
    const int qw0 = qblk * 128 + wave * 32;
    const bool active = qw0 < d.Nq;                               // wave-uniform
    const int q = min(qw0 + r, d.Nq - 1);                          // rows past Nq compute on a copy, never stored

    // Q^T fragments (B operand): lane (r, h) holds Q[q][16 ks + 8h .. +7]
    bf16v8 qf[4];
    {
        const bf16_t* Qp = (const bf16_t*)d.Q + b * d.q_bs + (int64_t)q * d.q_ld + d.q_off + h * 64 + 8 * hh;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qf[ks] = *reinterpret_cast<const bf16v8*>(Qp + 16 * ks);
    }
#if ATHD_ATTN_KM
    bf16v8 k5 = {}, q5 = {};                 // the fifth k-step: A row (key) k = 0 is 1, B column (query) k = 0 is -mrun
    if (hh == 0) k5[0] = (__bf16)1.0f;
#endif

    // staging: thread -> keys tid/8 + 32 j, 16-B chunk tid % 8 of the 128-B head row
    const bf16_t* Kb = (const bf16_t*)d.K + b * d.k_bs + d.k_off + h * 64;
    const bf16_t* Vb = (const bf16_t*)d.V + b * d.v_bs + d.v_off + h * 64;
    const int skey = tid >> 3, sch = tid & 7;
    // staging of tile kt0 into registers kr / vr (fetch) and from them into ring slot st (stash)
#define ATHD_A32_FETCH(KT0)                                                                                    \
    _Pragma("unroll") for (int j = 0; j < NKB; ++j) {                                                         \
        const int ka = min((KT0) + skey + 32 * j, d.Nk - 1);                                                   \
        kr[j] = *reinterpret_cast<const u32x4_t*>(Kb + (int64_t)ka * d.k_ld + 8 * sch);                         \
        vr[j] = *reinterpret_cast<const u32x4_t*>(Vb + (int64_t)ka * d.v_ld + 8 * sch);                         \
    }
#define ATHD_A32_STASH(ST)                                                                                     \
    _Pragma("unroll") for (int j = 0; j < NKB; ++j) {                                                         \
        const int key = skey + 32 * j;                                                                         \
        *reinterpret_cast<u32x4_t*>(&Ks[ST][a32_kidx<false>(key, sch)]) = kr[j];                                 \
        *reinterpret_cast<u32x4_t*>(&Vs[ST][key * A32_VP + 8 * a32_vchunk(key, sch)]) = vr[j];                   \
    }
    // LDS-DMA staging of tile KT0 into slot ST: wave w fills keys 8 (w + 4 j) .. +7 of K and of V, j < KT / 32
    const int dkey = lane >> 3, dph = lane & 7;
#if ATHD_ATTN_V6
    // round 6: a tile's sources are a wave-uniform base (the tile's first key row) plus a 32-bit per-lane byte
    // offset (key row in the tile, clamped to the last key, times the row pitch, plus the swizzled chunk), so each
    // piece is one v_min + one v_mad_u32_u24 and the load takes the SGPR-base form; the 64-bit per-piece address
    // arithmetic of the round-2 form (v_mad_i64_i32 + v_lshl_add_u64 per piece) cost ~100 issue cycles per tile.
    // The swizzles depend on key & 15 only, and KT0 is a multiple of 64, so they are tile-invariant.
    const uint32_t kldb = (uint32_t)d.k_ld * 2u, vldb = (uint32_t)d.v_ld * 2u;
    uint32_t kswz[KT / 32], vswz[KT / 32];
#pragma unroll
    for (int j = 0; j < KT / 32; ++j) {
        const int kk = 8 * (wave + 4 * j) + dkey;
        kswz[j] = 16u * (uint32_t)(dph ^ ((kk >> 1) & 7));
        vswz[j] = 16u * (uint32_t)a32_vchunk(kk, dph);
    }
#define ATHD_A32_DMA(KT0, ST)                                                                                  \
    {                                                                                                          \
        const char* kt_ = (const char*)(Kb + (int64_t)(KT0) * d.k_ld);                                         \
        const char* vt_ = (const char*)(Vb + (int64_t)(KT0) * d.v_ld);                                         \
        const int last_ = d.Nk - 1 - (KT0);                                                                    \
        _Pragma("unroll") for (int j = 0; j < KT / 32; ++j) {                                                 \
            const uint32_t kc_ = (uint32_t)min(8 * (wave + 4 * j) + dkey, last_);                              \
            uint32_t ko_ = __umul24(kc_, kldb) + kswz[j];                                     \
            uint32_t vo_ = __umul24(kc_, vldb) + vswz[j];                                     \
            asm volatile("" : "+v"(ko_), "+v"(vo_));     /* opaque: keeps (uniform base, 32-bit offset) */   \
            __builtin_amdgcn_global_load_lds((a32_gbl_void*)(kt_ + ko_),                                       \
                                             (a32_lds_void*)&Ks[ST][8 * (wave + 4 * j) * 64], 16, 0, 0);        \
            __builtin_amdgcn_global_load_lds((a32_gbl_void*)(vt_ + vo_),                                       \
                                             (a32_lds_void*)&Vs[ST][8 * (wave + 4 * j) * A32_VP], 16, 0, 0);   \
        }                                                                                                      \
    }
#else
#define ATHD_A32_DMA(KT0, ST)                                                                                  \
    _Pragma("unroll") for (int j = 0; j < KT / 32; ++j) {                                                     \
        const int kk = 8 * (wave + 4 * j) + dkey;                                                              \
        const int ka = min((KT0) + kk, d.Nk - 1);                                                              \
        __builtin_amdgcn_global_load_lds((a32_gbl_void*)(Kb + (int64_t)ka * d.k_ld + 8 * (dph ^ ((kk >> 1) & 7))), \
                                         (a32_lds_void*)&Ks[ST][8 * (wave + 4 * j) * 64], 16, 0, 0);            \
        __builtin_amdgcn_global_load_lds((a32_gbl_void*)(Vb + (int64_t)ka * d.v_ld + 8 * a32_vchunk(kk, dph)),  \
                                         (a32_lds_void*)&Vs[ST][8 * (wave + 4 * j) * A32_VP], 16, 0, 0);       \
    }
#endif

    // transposed-read addresses (elements): lane 4q'+p of 16-lane group g' -> key row 4h + q' (+8, +16 s2, +32 kb),
    // d columns 32 db + 16 (g' & 1) + 4p
    const int g16 = lane >> 4, i16 = lane & 15, qr = i16 >> 2, pc = i16 & 3;
    const int vrow = 4 * hh + qr;                                  // + 16 s2 + 32 kb (+ 8): same (row >> 1) & 1
    int voff[2];
#pragma unroll
    for (int db = 0; db < 2; ++db) {
        const int col = 32 * db + 16 * (g16 & 1) + 4 * pc;
        voff[db] = vrow * A32_VP + 8 * a32_vchunk(vrow, col >> 3) + (col & 7);
    }

    f32x16_t o0, o1;
#pragma unroll
    for (int i = 0; i < 16; ++i) { o0[i] = 0.f; o1[i] = 0.f; }
    float mrun = 0.f, lrun = 0.f;

    const int ntiles = (d.Nk + KT - 1) / KT;
    if constexpr (DMA) {
        ATHD_A32_DMA(0, 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        u32x4_t kr[NKB], vr[NKB];
        ATHD_A32_FETCH(0)
        ATHD_A32_STASH(0)
    }
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < ntiles; ++t) {
        const int kt0 = t * KT;
        const bool more = t + 1 < ntiles;
        u32x4_t kr[NKB], vr[NKB];
        if (more) {
            // slot cur ^ 1 was last read in iteration t - 1, which ended with a barrier
            if constexpr (DMA) {
                ATHD_A32_DMA(kt0 + KT, cur ^ 1)
            } else {
                ATHD_A32_FETCH(kt0 + KT)
            }
        }
        if (active) {
            const bf16_t* K_ = Ks[cur];
            const bf16_t* V_ = Vs[cur];
            // ---- S^T = K Q^T - m ----
            f32x16_t sc[NKB];
            // (ATHD_A32_QK: key tail -> scores of keys >= Nk are -inf)
            A32_PRIO(1);
#if ATHD_ATTN_V6
            ATHD_A32_QKX();
#else
            ATHD_A32_QK(-mrun);
#endif
            A32_PRIO(0);
#if ATHD_ATTN_V6
            // ---- online softmax (log2 units), round 6: no per-tile max ----
            // The running max is set exactly on the first tile.  Later tiles exponentiate against it at once, and the
            // lane's own row sum (its 32 P values, computed anyway) tells whether any of its P exceeds A32_SUMCHK: only
            // then (rare, __any) are the scores recomputed, their exact max taken, O and l rescaled and the tile
            // re-exponentiated - so P <= A32_SUMCHK always (the defer-max bound; bf16 P keeps its relative precision at
            // any scale).  Saves the 17 v_max3 + swap + compare of every tile (~90 of ~900 issue cycles per tile).
            auto tile_max = [&]() -> float {                      // max over the tile's scores of the lane's query
                // (the vmax3 asm reads MFMA results and hipcc pads nothing before it (see vmax3): the caller's MFMAs
                // are fenced off by sched_barrier and 12 explicit wait states; compiler VALU reads get 10)
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_nop 11" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                float mxk[NKB];
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb) {
                    float m = vmax3(sc[kb][0], sc[kb][1], sc[kb][2]);
#pragma unroll
                    for (int i = 3; i < 15; i += 2) m = vmax3(m, sc[kb][i], sc[kb][i + 1]);
                    mxk[kb] = vmax3(m, sc[kb][15], sc[kb][15]);
                }
                float mx = mxk[0];
#pragma unroll
                for (int kb = 1; kb < NKB; ++kb) mx = vmax3(mx, mxk[kb], mxk[kb]);
                return half_swap_max(mx);
            };
            auto exp_sum = [&]() -> float {                       // P = exp2(S) in place; the lane's row sum
                athd_f2v ls2[NKB];                                 // one chain per key block
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb) {
                    ls2[kb] = (athd_f2v){0.f, 0.f};
#pragma unroll
                    for (int i = 0; i < 16; i += 2) {
                        sc[kb][i] = __builtin_amdgcn_exp2f(sc[kb][i]);
                        sc[kb][i + 1] = __builtin_amdgcn_exp2f(sc[kb][i + 1]);
                        ls2[kb] += (athd_f2v){sc[kb][i], sc[kb][i + 1]};
                    }
                }
#pragma unroll
                for (int kb = 1; kb < NKB; ++kb) ls2[0] += ls2[kb];
                return ls2[0].x + ls2[0].y;
            };
#if ATHD_ATTN_KM
            // (mrun rounded to bf16: the fifth k-step multiplies it exactly; alpha uses the rounded values)
            auto set_max = [&](float m) {
                mrun = (float)(__bf16)m;
                if (hh == 0) q5[0] = (__bf16)(-mrun);
            };
#else
            auto set_max = [&](float m) { mrun = m; };
#endif
            if (t == 0) {                                          // first tile: the exact max (O and l are zero)
                set_max(tile_max());
#if ATHD_ATTN_T0SUB && !ATHD_ATTN_KM
                // the scores already in registers, shifted by the max (instead of QK^T again from -m)
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                    for (int i = 0; i < 16; ++i) sc[kb][i] -= mrun;
#else
                ATHD_A32_QKX();
#endif
            }
            float ls = exp_sum();
            if (__any(!(ls <= A32_SUMCHK))) {                      // some P > A32_SUMCHK (or not finite): rescale
                ATHD_A32_QKX();
                const float m_old = mrun;
                set_max(mrun + fmaxf(tile_max(), 0.f));
                const float alpha = __builtin_amdgcn_exp2f(m_old - mrun);
                lrun *= alpha;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    o0[i] *= alpha;
                    o1[i] *= alpha;
                }
                ATHD_A32_QKX();
                ls = exp_sum();
            }
            lrun += ls;
#else
            // ---- online softmax (log2 units) ----
            float mxk[NKB];
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {                     // independent chains, one per key block
                float m = vmax3(sc[kb][0], sc[kb][1], sc[kb][2]);
#pragma unroll
                for (int i = 3; i < 15; i += 2) m = vmax3(m, sc[kb][i], sc[kb][i + 1]);
                mxk[kb] = vmax3(m, sc[kb][15], sc[kb][15]);
            }
            float mx = mxk[0];
#pragma unroll
            for (int kb = 1; kb < NKB; ++kb) mx = vmax3(mx, mxk[kb], mxk[kb]);
            mx = half_swap_max(mx);
            // first tile: the max is set; later tiles: it moves only past ATTN_RESCALE.  A move rescales O and l
            // and recomputes the tile's scores against the new max (S is never modified in place, which keeps the
            // accumulators in place across the branch)
            const bool jump = t == 0 || mx > ATTN_RESCALE;
            if (__any(jump)) {
                const float dm = jump ? mx : 0.f;
                const float alpha = t == 0 ? 0.f : __builtin_amdgcn_exp2f(-dm);
                mrun += dm;
                lrun *= alpha;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    o0[i] *= alpha;
                    o1[i] *= alpha;
                }
                ATHD_A32_QK(-mrun);
            }
            // row sums on packed adds: 8 v_pk_add_f32 per key block instead of 16 adds
            athd_f2v ls2[NKB];                                     // one chain per key block
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
                ls2[kb] = (athd_f2v){0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    // (ATHD_ATTN_POLY of the 16 on the FMA pipe, spread over the block: pairs i with i % 8 >= 8 - n/2)
                    const bool poly = ATHD_ATTN_POLY > 0 && (i & 7) >= 8 - ATHD_ATTN_POLY / 2;
                    sc[kb][i] = poly ? exp2_poly(sc[kb][i]) : __builtin_amdgcn_exp2f(sc[kb][i]);
                    sc[kb][i + 1] = poly ? exp2_poly(sc[kb][i + 1]) : __builtin_amdgcn_exp2f(sc[kb][i + 1]);
                    ls2[kb] += (athd_f2v){sc[kb][i], sc[kb][i + 1]};
                }
            }
#pragma unroll
            for (int kb = 1; kb < NKB; ++kb) ls2[0] += ls2[kb];
            lrun += ls2[0].x + ls2[0].y;
#endif
            // ---- O^T += V^T P^T ----
            A32_PRIO(1);
#pragma unroll
            for (int kk = 0; kk < 2 * NKB; ++kk) {
                const f32x16_t& sp = sc[kk >> 1];
                const int j0 = 8 * (kk & 1);
                const uint32_t w[4] = {pack2bf(sp[j0 + 0], sp[j0 + 1]), pack2bf(sp[j0 + 2], sp[j0 + 3]),
                                       pack2bf(sp[j0 + 4], sp[j0 + 5]), pack2bf(sp[j0 + 6], sp[j0 + 7])};
                const bf16v8 pb = __builtin_bit_cast(bf16v8, w);
                const int rb = (32 * (kk >> 1) + 16 * (kk & 1)) * A32_VP;
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const bf16_t* base = &V_[rb + voff[db]];
                    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
                    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 8 * A32_VP));
                    const bf16v8 a = __builtin_shufflevector(__builtin_bit_cast(bf16v4, lo),
                                                             __builtin_bit_cast(bf16v4, hi), 0, 1, 2, 3, 4, 5, 6, 7);
                    if (db == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, o0, 0, 0, 0);
                    else o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, o1, 0, 0, 0);
                }
            }
            A32_PRIO(0);
        }
        if constexpr (DMA) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // this wave's DMA into slot cur ^ 1 landed
        } else if (more) {
            ATHD_A32_STASH(cur ^ 1)
        }
        __syncthreads();
        cur ^= 1;
    }
    // ---- normalise; stage the wave's 32 x 64 output tile in LDS; store whole 128-B rows ----
    const float l = half_swap_sum(lrun);
    const float inv = 1.f / l;
    bf16_t* stage = smem_a32 + wave * 32 * A32_KP;                 // 4 waves x 32 rows x 72 (static_assert above)
    if (active) {
#pragma unroll
        for (int db = 0; db < 2; ++db) {
            const f32x16_t& oo = db ? o1 : o0;
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int dcol = 32 * db + 8 * g4 + 4 * hh;
                *reinterpret_cast<uint2*>(&stage[r * A32_KP + dcol]) =
                    make_uint2(pack2bf(oo[4 * g4] * inv, oo[4 * g4 + 1] * inv),
                               pack2bf(oo[4 * g4 + 2] * inv, oo[4 * g4 + 3] * inv));
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);                         // lgkmcnt(0): the wave's own LDS writes landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int id = it * 64 + lane, row = id >> 3, ch = id & 7;
            const int qq = qw0 + row;
            if (qq < d.Nq) {
                const uint4 v = *reinterpret_cast<const uint4*>(&stage[row * A32_KP + 8 * ch]);
                *reinterpret_cast<uint4*>((bf16_t*)d.O + b * d.o_bs + (int64_t)qq * d.o_ld + h * 64 + 8 * ch) = v;
            }
        }
    }
}

#undef ATHD_A32_FETCH
#undef ATHD_A32_STASH
#undef ATHD_A32_DMA

// ----------------------------------------------------------------------------------------------------------------
// Ping-pong form (ATHD_ATTN_PP=1): 8 waves in two groups of 4, G0 = waves 0-3 and G1 = waves 4-7
// (one wave of each per SIMD), 32 queries per wave, 256 per workgroup, 64-key tiles.  A group spends a tile in two
// sections separated by workgroup barriers:
//   M(t)  MFMA section: QK^T of tile t into fresh score accumulators (started at -m, as attn32_kernel) and PV of tile
//         t - 1 with the P packed in the group's previous section - 16 v_mfma_f32_32x32x16_bf16 at s_setprio 1;
//   V(t)  softmax section: key-tail mask, exp2 + row sums, the A32_SUMCHK check (rare rescale: O and l scaled, the
//         tile's scores recomputed), P -> bf16, this wave's LDS-DMA pieces of K(t + 3) and V(t + 2), and the K(t + 1)
//         fragments for the next M.
// G1 runs one section behind G0, so in every section one wave of each SIMD issues MFMAs while the other runs the
// softmax: matrix beside VALU by construction (attn32_kernel gets it from the chance alignment of three independent
// workgroups per CU; MFMA busy 0.44, profiles/pmc_sq_r05.txt).
// LDS: rings of 4 K slots and 4 V slots (8 KB each; attn32_kernel's swizzles).  K(t) is read in sections 2t - 1 (G0)
// and 2t (G1), V(t) in 2t + 2 and 2t + 3; V(t) issues K(t + 3) into the slot of K(t - 1) and V(t + 2) into that of
// V(t - 2), both free by then.  Before every barrier a wave waits (counted vmcnt) for all of its pieces except those
// of its latest softmax section: every piece has >= 2 sections in flight and a barrier between landing and first read.
// The fragment reads are inline asm with explicit lgkmcnt waits: the compiler cannot tell the ring slots apart and
// would put a vmcnt(0) before every LDS read while DMAs are in flight.
// Same arithmetic in the same order as attn32_kernel<3, 2, true>: the outputs are bit-identical (test_gpu_parity).
constexpr int PP_KT = 64;                          // keys per tile
constexpr int PP_SLOT_B = PP_KT * 64 * 2;          // bytes per K or V slot
constexpr int PP_NS = 4;                           // slots per ring
typedef __attribute__((ext_vector_type(2))) unsigned int pp_u32x2;

ATHD_DEV void pp_vm_wait(int n) {                  // n wave-uniform, 0..4
    if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// PRIO: 1 = s_setprio 1 around each MFMA section (as attn32_kernel); 0 = none; 2 = the static form for G1 only
// (cdna_hip_programming.md T5; MI355X_MICROARCH.md §Two waves per SIMD item 2: a prio-1 MFMA wave delays the other
// wave's v_exp by hundreds of cycles per section)
template <int PRIO>
__global__ __launch_bounds__(512, 1) void attn_pp_kernel(const AttnDesc d) {
    constexpr int KT = PP_KT, NKB = 2;
    __shared__ __attribute__((aligned(1024))) char smem_pp[2 * PP_NS * PP_SLOT_B];    // K ring | V ring (64 KB)
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem_pp;
    const uint32_t vring = lds0 + PP_NS * PP_SLOT_B;

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;
    const int r = lane & 31, hh = lane >> 5;
    int qblk, h;
    int64_t b;
    attn_tile(d, qblk, h, b, 256);
    const int qw0 = qblk * 256 + wave * 32;
    const bool active = qw0 < d.Nq;                               // wave-uniform
    const int q = min(qw0 + r, d.Nq - 1);                          // rows past Nq compute on a copy, never stored
    bf16v8 qf[4];
    {
        const bf16_t* Qp = (const bf16_t*)d.Q + b * d.q_bs + (int64_t)q * d.q_ld + d.q_off + h * 64 + 8 * hh;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qf[ks] = *reinterpret_cast<const bf16v8*>(Qp + 16 * ks);
    }
    const bf16_t* Kb = (const bf16_t*)d.K + b * d.k_bs + d.k_off + h * 64;
    const bf16_t* Vb = (const bf16_t*)d.V + b * d.v_bs + d.v_off + h * 64;
    const int T = (d.Nk + KT - 1) / KT;

    // LDS-DMA: wave w fills keys 8w .. 8w + 7 of every K and V tile (one 1-KB piece each); the lane fetches the logical
    // 16-B chunk that the slot's swizzle puts at its physical chunk (attn32_kernel's images)
    const int dkey = lane >> 3, dph = lane & 7, kk8 = 8 * wave + dkey;
    const uint32_t kswz = 16u * (uint32_t)(dph ^ ((kk8 >> 1) & 7));
    const uint32_t vswz = 16u * (uint32_t)a32_vchunk(kk8, dph);
    const uint32_t kldb = (uint32_t)d.k_ld * 2u, vldb = (uint32_t)d.v_ld * 2u;
    auto dma_k = [&](int t) {
        const char* base = (const char*)(Kb + (int64_t)t * KT * d.k_ld);
        uint32_t off = __umul24((uint32_t)min(kk8, d.Nk - 1 - t * KT), kldb) + kswz;
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_global_load_lds((a32_gbl_void*)(base + off),
                                         (a32_lds_void*)(smem_pp + (t & (PP_NS - 1)) * PP_SLOT_B + wave * 1024), 16, 0, 0);
    };
    auto dma_v = [&](int t) {
        const char* base = (const char*)(Vb + (int64_t)t * KT * d.v_ld);
        uint32_t off = __umul24((uint32_t)min(kk8, d.Nk - 1 - t * KT), vldb) + vswz;
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_global_load_lds((a32_gbl_void*)(base + off),
                                         (a32_lds_void*)(smem_pp + (PP_NS + (t & (PP_NS - 1))) * PP_SLOT_B + wave * 1024),
                                         16, 0, 0);
    };

    // K fragment (key 32 kb + r, 16-B chunk 2 ks + hh) byte offsets in a slot: 128 r + 16 ((2 ks + hh) ^ ((r >> 1) & 7))
    // + 4096 kb (the kb part is the immediate)
    uint32_t koff[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) koff[ks] = 128u * r + 16u * (uint32_t)((2 * ks + hh) ^ ((r >> 1) & 7));
    // V transposed-read byte offsets (attn32_kernel's voff), + 2048 kk + 1024 for the upper 8 keys as immediates
    const int g16 = lane >> 4, i16 = lane & 15, qr = i16 >> 2, pc = i16 & 3;
    const int vrow = 4 * hh + qr;
    uint32_t voffb[2];
#pragma unroll
    for (int db = 0; db < 2; ++db) {
        const int col = 32 * db + 16 * (g16 & 1) + 4 * pc;
        voffb[db] = 2u * (uint32_t)(vrow * A32_VP + 8 * a32_vchunk(vrow, col >> 3) + (col & 7));
    }

    bf16v8 kf[4][NKB];                          // K fragments of the tile the next QK^T uses
    auto read_k = [&](int t) {
        const uint32_t sb = lds0 + (uint32_t)(t & (PP_NS - 1)) * PP_SLOT_B;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const uint32_t a = sb + koff[ks];
            asm volatile("ds_read_b128 %0, %1" : "=v"(kf[ks][0]) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(kf[ks][1]) : "v"(a));
        }
    };
    auto pin_k = [&]() {                         // after an lgkmcnt(0): the fragments are used no earlier
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[ks][0]), "+v"(kf[ks][1]));
    };

    f32x16_t o0, o1, sc[NKB];
#pragma unroll
    for (int i = 0; i < 16; ++i) { o0[i] = 0.f; o1[i] = 0.f; }
    float mrun = 0.f, lrun = 0.f;
    bf16v8 pb[4];                               // P of the group's last softmax section, bf16, per PV k-step

    auto qk = [&](float init) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) sc[kb][i] = init;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks][kb], qf[ks], sc[kb], 0, 0, 0);
    };
    auto mask_tail = [&](int kt0) {             // keys >= Nk -> -inf (last tile only)
        if (kt0 + KT > d.Nk) {
            int lim = d.Nk - kt0 - 4 * hh;
            asm volatile("" : "+v"(lim));
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (32 * kb + (i & 3) + 8 * (i >> 2) >= lim) sc[kb][i] = -INFINITY;
        }
    };
    auto tile_max = [&]() -> float {            // (explicit pad before the vmax3 asm: see vmax3)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 11" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        float mxk[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            float m = vmax3(sc[kb][0], sc[kb][1], sc[kb][2]);
#pragma unroll
            for (int i = 3; i < 15; i += 2) m = vmax3(m, sc[kb][i], sc[kb][i + 1]);
            mxk[kb] = vmax3(m, sc[kb][15], sc[kb][15]);
        }
        return half_swap_max(vmax3(mxk[0], mxk[1], mxk[1]));
    };
    auto exp_sum = [&]() -> float {
        athd_f2v ls2[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            ls2[kb] = (athd_f2v){0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                sc[kb][i] = __builtin_amdgcn_exp2f(sc[kb][i]);
                sc[kb][i + 1] = __builtin_amdgcn_exp2f(sc[kb][i + 1]);
                ls2[kb] += (athd_f2v){sc[kb][i], sc[kb][i + 1]};
            }
        }
        ls2[0] += ls2[1];
        return ls2[0].x + ls2[0].y;
    };

    // ---- prologue: K(0), K(1), V(0), K(2), V(1) (those that exist) ----
    dma_k(0);
    if (T > 1) dma_k(1);
    dma_v(0);
    if (T > 2) dma_k(2);
    if (T > 1) dma_v(1);
    const int npro = 2 + (T > 1 ? 2 : 0) + (T > 2 ? 1 : 0);
    pp_vm_wait(npro - 1);                       // K(0) landed ...
    __builtin_amdgcn_s_barrier();               // ... in every wave's pieces
    __builtin_amdgcn_sched_barrier(0);
    if (active) read_k(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pin_k();
    int nlast = (T > 2 ? 1 : 0) + (T > 1 ? 1 : 0);   // pieces of the latest issuing section (the prologue's K(2), V(1))

    // one section boundary: this wave's LDS reads retired, its pieces older than its latest softmax section landed
    // (the first boundary after B0: K(1), which G0's V(0) reads), then the workgroup barrier
    int nbar = 0;
    auto boundary = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pin_k();
        if (nbar++ == 0) pp_vm_wait(T > 1 ? npro - 2 : npro - 1);
        else pp_vm_wait(nlast);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    if (grp == 1) boundary();                   // the stagger: G1 runs one section behind G0
    if constexpr (PRIO == 2) {
        if (grp == 1) __builtin_amdgcn_s_setprio(1);
    }
    for (int t = 0; t <= T; ++t) {
        // ---- M(t): QK^T of tile t, PV of tile t - 1 ----
        if (active) {
            pp_u32x2 vlo[4][2], vhi[4][2];
            if (t >= 1) {
                const uint32_t sb = vring + (uint32_t)((t - 1) & (PP_NS - 1)) * PP_SLOT_B;
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const uint32_t a = sb + voffb[db];
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(vlo[0][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(vhi[0][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(vlo[1][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:3072" : "=v"(vhi[1][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:4096" : "=v"(vlo[2][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:5120" : "=v"(vhi[2][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:6144" : "=v"(vlo[3][db]) : "v"(a));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:7168" : "=v"(vhi[3][db]) : "v"(a));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PRIO == 1) A32_PRIO(1);
            if (t < T) qk(-mrun);
            if (t >= 1) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int db = 0; db < 2; ++db) asm volatile("" : "+v"(vlo[kk][db]), "+v"(vhi[kk][db]));
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const pp_u32x2 l0 = vlo[kk][0], h0 = vhi[kk][0], l1 = vlo[kk][1], h1 = vhi[kk][1];
                    const bf16v8 a0 = __builtin_bit_cast(bf16v8, (u32x4_t){l0.x, l0.y, h0.x, h0.y});
                    const bf16v8 a1 = __builtin_bit_cast(bf16v8, (u32x4_t){l1.x, l1.y, h1.x, h1.y});
                    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, pb[kk], o0, 0, 0, 0);
                    o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, pb[kk], o1, 0, 0, 0);
                }
            }
            if constexpr (PRIO == 1) A32_PRIO(0);
            __builtin_amdgcn_sched_barrier(0);
        }
        boundary();
        if (t == T) break;
        // ---- V(t): DMA, the next K fragments (their latency under the softmax), softmax of tile t ----
        const int kt0 = t * KT;
        nlast = 0;
        if (t + 3 < T) { dma_k(t + 3); ++nlast; }
        if (t + 2 < T) { dma_v(t + 2); ++nlast; }
        if (active) {
            if (t + 1 < T) read_k(t + 1);
            // the recomputations of this tile's scores (first tile; rare rescale) re-read K(t) (its slot is rewritten
            // only by V(t + 1)'s DMA) and then K(t + 1) again
            auto with_kt = [&](auto&& fn) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                pin_k();
                read_k(t);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                pin_k();
                fn();
                if (t + 1 < T) read_k(t + 1);
            };
            mask_tail(kt0);
            if (t == 0) {                                      // first tile: the exact max (O and l are zero)
#if ATHD_ATTN_T0SUB
                mrun = tile_max();                             // (attn32_kernel's form: the scores shifted in place)
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int i = 0; i < 16; ++i) sc[kb][i] -= mrun;
#else
                with_kt([&]() {
                    mrun = tile_max();
                    qk(-mrun);
                    mask_tail(kt0);
                });
#endif
            }
            float ls = exp_sum();
            if (__any(!(ls <= A32_SUMCHK))) {                  // some P > A32_SUMCHK (or not finite): rescale
                with_kt([&]() {
                    qk(-mrun);
                    mask_tail(kt0);
                    const float m_old = mrun;
                    mrun = mrun + fmaxf(tile_max(), 0.f);
                    const float alpha = __builtin_amdgcn_exp2f(m_old - mrun);
                    lrun *= alpha;
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        o0[i] *= alpha;
                        o1[i] *= alpha;
                    }
                    qk(-mrun);
                    mask_tail(kt0);
                    ls = exp_sum();
                });
            }
            lrun += ls;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const f32x16_t& sp = sc[kk >> 1];
                const int j0 = 8 * (kk & 1);
                const uint32_t w[4] = {pack2bf(sp[j0 + 0], sp[j0 + 1]), pack2bf(sp[j0 + 2], sp[j0 + 3]),
                                       pack2bf(sp[j0 + 4], sp[j0 + 5]), pack2bf(sp[j0 + 6], sp[j0 + 7])};
                pb[kk] = __builtin_bit_cast(bf16v8, w);
            }
        }
        boundary();
    }
    if (grp == 0) boundary();                   // equal barrier counts

    // ---- normalise; stage the wave's 32 x 64 output tile in LDS (the ring is free); store whole 128-B rows ----
    const float l = half_swap_sum(lrun);
    const float inv = 1.f / l;
    bf16_t* stage = reinterpret_cast<bf16_t*>(smem_pp) + wave * 32 * A32_KP;    // 8 x 32 x 72 x 2 B = 36 KB
    if (active) {
#pragma unroll
        for (int db = 0; db < 2; ++db) {
            const f32x16_t& oo = db ? o1 : o0;
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int dcol = 32 * db + 8 * g4 + 4 * hh;
                *reinterpret_cast<uint2*>(&stage[r * A32_KP + dcol]) =
                    make_uint2(pack2bf(oo[4 * g4] * inv, oo[4 * g4 + 1] * inv),
                               pack2bf(oo[4 * g4 + 2] * inv, oo[4 * g4 + 3] * inv));
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);                         // lgkmcnt(0): the wave's own LDS writes landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int id = it * 64 + lane, row = id >> 3, ch = id & 7;
            const int qq = qw0 + row;
            if (qq < d.Nq) {
                const uint4 v = *reinterpret_cast<const uint4*>(&stage[row * A32_KP + 8 * ch]);
                *reinterpret_cast<uint4*>((bf16_t*)d.O + b * d.o_bs + (int64_t)qq * d.o_ld + h * 64 + 8 * ch) = v;
            }
        }
    }
}

#undef ATHD_A32_QK
#undef ATHD_A32_QKM
#undef ATHD_A32_QKX

// kernel choice for the bf16 path (tools/kbench builds, -DATHD_KBENCH; the product always takes 0): 0 =
// attn32_kernel<3, 2, true> (3 waves per SIMD, 64-key tiles, LDS-DMA staging), 1 = attn_bf16_kernel (16x16x32), 2 = attn32_kernel<2, 2>, 3 = attn32_kernel<2, 4> (128-key
// tiles), 4 = attn32_kernel<3, 2, false> (register staging), 5 / 6 = attn32_kernel<2, 4> / <4, 2> with LDS-DMA staging;
// set by tools/kbench.hip for A/B timing.  kbench (B=64, N=2072 / 1034, same box): register staging 722 / 730 TFLOP/s,
// LDS-DMA staging 849 / 777.  Tried and dropped: a software-pipelined form (QK^T of tile t+1 issued before the
// softmax of tile t, 3-deep K/V ring: 761 vs 804 TFLOP/s), 64 queries per wave on register staging (256 VGPRs with
// spills: 757) and on LDS-DMA staging (two 32-query blocks sharing every K / V fragment read, 2 waves per workgroup,
// 2 waves per SIMD at 255 VGPRs: 765 / 648 vs 845 / 776), and 192-query workgroups (6 waves; 2 % tail waste at
// N = 2072 instead of 5 %, DMA pieces shared by 6 waves): 729-739 / 614-630 vs 853 / 781 on one box.
#ifdef ATHD_KBENCH
int g_attn_variant = 0;       // set by tools/kbench.hip
static int attn_variant() { return g_attn_variant; }
#else
static constexpr int attn_variant() { return 0; }
#endif

static bool attn32_ok(const AttnDesc& d, int mode) {
    return attn_variant() != 1 && mode == 1 && d.q_bf16 && d.k_bf16 && d.v_bf16 && d.o_bf16 &&
           fabsf(d.scale * 1.4426950408889634f - 1.f) < 1e-6f && d.q_ld % 8 == 0 && d.k_ld % 8 == 0 &&
           d.v_ld % 8 == 0 && d.o_ld % 8 == 0 && d.q_off % 8 == 0 && d.k_off % 8 == 0 && d.v_off % 8 == 0 &&
           d.Nq > 0 && d.Nk > 0;
}

// ATHD_ATTN_PP=1/2/3: the bf16 path on attn_pp_kernel<1/0/2> (A/B; read at every launch)
static int attn_pp_mode() {
    const char* e = std::getenv("ATHD_ATTN_PP");
    return e && e[0] >= '1' && e[0] <= '3' ? e[0] - '0' : 0;
}

int attn_launch(const AttnDesc& d, int mode, hipStream_t s) {
    if (d.heads * 64 > d.o_ld && d.o_ld != 0) return -2;
    const bool a32 = attn32_ok(d, mode);
    const int ppm = attn_pp_mode();
    if (a32 && attn_variant() == 0 && ppm) {
        dim3 grid((unsigned)((d.Nq + 255) / 256) * (unsigned)d.heads * (unsigned)d.nb);
        KScope ks(s);
        if (ks.on()) {
            const double nh = (double)d.nb * d.heads;
            ks.begin("attn_pp_kernel", 4.0 * nh * d.Nq * d.Nk * 64, nh * 64 * 2.0 * (2.0 * d.Nq + 2.0 * d.Nk));
        }
        if (ppm == 1) hipLaunchKernelGGL(attn_pp_kernel<1>, grid, dim3(512), 0, s, d);
        else if (ppm == 2) hipLaunchKernelGGL(attn_pp_kernel<0>, grid, dim3(512), 0, s, d);
        else hipLaunchKernelGGL(attn_pp_kernel<2>, grid, dim3(512), 0, s, d);
        return (int)hipGetLastError();
    }
    const int qblock = 128;
    dim3 grid((unsigned)((d.Nq + qblock - 1) / qblock) * (unsigned)d.heads * (unsigned)d.nb);   // attn_tile decodes it
    KScope ks(s);
    if (ks.on()) {
        const bool v2 = mode == 1 && d.q_bf16 && d.k_bf16 && d.v_bf16;
        const double nh = (double)d.nb * d.heads;
        const double fl = 4.0 * nh * d.Nq * d.Nk * 64;
        const double by = nh * 64 * (d.Nq * (d.q_bf16 ? 2 : 4) + d.Nk * ((d.k_bf16 ? 2 : 4) + (d.v_bf16 ? 2 : 4)) +
                                     d.Nq * (d.o_bf16 ? 2 : 4));
        ks.begin(a32 ? std::string("attn32_kernel<3,2,true>") : v2 ? std::string("attn_bf16_kernel") : klabel("attn_kernel<%d>", mode),
                 fl, by);
    }
#ifdef ATHD_KBENCH
    if (a32 && attn_variant() == 4) hipLaunchKernelGGL((attn32_kernel<3, 2, false>), grid, dim3(256), 0, s, d);
    else if (a32 && attn_variant() == 5) hipLaunchKernelGGL((attn32_kernel<2, 4, true>), grid, dim3(256), 0, s, d);
    else if (a32 && attn_variant() == 6) hipLaunchKernelGGL((attn32_kernel<4, 2, true>), grid, dim3(256), 0, s, d);
    else if (a32 && attn_variant() == 2) hipLaunchKernelGGL((attn32_kernel<2, 2>), grid, dim3(256), 0, s, d);
    else if (a32 && attn_variant() == 3) hipLaunchKernelGGL((attn32_kernel<2, 4>), grid, dim3(256), 0, s, d);
    else if (a32) hipLaunchKernelGGL((attn32_kernel<3, 2, true>), grid, dim3(256), 0, s, d);
    else if (mode == 1 && d.q_bf16 && d.k_bf16 && d.v_bf16) hipLaunchKernelGGL(attn_bf16_kernel, grid, dim3(256), 0, s, d);
    else if (mode == 1) hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL(attn_kernel<0>, grid, dim3(256), 0, s, d);
#else
    // product: bf16 mode -> attn32_kernel (the forward's Q/K/V/O are bf16, 8-element aligned, Q prescaled);
    // f32 parity mode -> attn_kernel<0> (fp32 MFMA)
    if (a32) hipLaunchKernelGGL((attn32_kernel<3, 2, true>), grid, dim3(256), 0, s, d);
    else if (mode == 0) hipLaunchKernelGGL(attn_kernel<0>, grid, dim3(256), 0, s, d);
    else return -3;                                // bf16 mode operands attn32_kernel does not take
#endif
    return (int)hipGetLastError();
}

}  // namespace athd
