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
ATHD_DEV void attn_tile(const AttnDesc& d, int& qb, int& h, int64_t& b) {
    const int n = (int)gridDim.x, i = (int)blockIdx.x;
    const int q = n / 8, r = n % 8, x = i % 8;
    const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i / 8;
    const int gq = (d.Nq + 127) / 128;
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
#undef ATHD_FETCH
#undef ATHD_STASH

int attn_launch(const AttnDesc& d, int mode, hipStream_t s) {
    if (d.heads * 64 > d.o_ld && d.o_ld != 0) return -2;
    dim3 grid((unsigned)((d.Nq + 127) / 128) * (unsigned)d.heads * (unsigned)d.nb);   // attn_tile decodes it
    KScope ks(s);
    if (ks.on()) {
        const bool v2 = mode == 1 && d.q_bf16 && d.k_bf16 && d.v_bf16;
        const double nh = (double)d.nb * d.heads;
        const double fl = 4.0 * nh * d.Nq * d.Nk * 64;
        const double by = nh * 64 * (d.Nq * (d.q_bf16 ? 2 : 4) + d.Nk * ((d.k_bf16 ? 2 : 4) + (d.v_bf16 ? 2 : 4)) +
                                     d.Nq * (d.o_bf16 ? 2 : 4));
        ks.begin(v2 ? std::string("attn_bf16_kernel") : klabel("attn_kernel<%d>", mode), fl, by);
    }
    if (mode == 1 && d.q_bf16 && d.k_bf16 && d.v_bf16) hipLaunchKernelGGL(attn_bf16_kernel, grid, dim3(256), 0, s, d);
    else if (mode == 1) hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL(attn_kernel<0>, grid, dim3(256), 0, s, d);
    return (int)hipGetLastError();
}

}  // namespace athd
