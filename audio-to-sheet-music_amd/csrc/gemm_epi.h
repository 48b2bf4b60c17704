// Shared GEMM epilogue (both MFMA GEMM kernels).  The kernels compute C^T tiles (weights as the MFMA A operand),
// so with the v_mfma_f32_16x16x{32,4} C/D map (col = l&15, row = 4(l>>4)+r) each lane owns one output row and
// four consecutive output columns: vector bias/residual loads and 8-B (bf16) / 16-B (f32) stores.
//   v = acc + bias[n]; [GroupNorm(v) with per-batch stats]; act (GELU | GLU over packed column pairs);
//   + row_add[ho][n]; out = res + res_scale[n] * v; {sum, sumsq} of out per batch -> stats; store f32/bf16.
// The feature set is a compile-time bitmask F so that each instantiation only carries the code it runs (a fully
// general epilogue unrolled over 16 rows x 4 column tiles is ~25k instructions and thrashes the I-cache).
#pragma once
#include "common.h"
#include "gemm.h"

namespace athd {

constexpr int EPI_MAXG = 32;   // GroupNorm groups tracked per block in LDS

#ifndef ATHD_EPI_MARK
#define ATHD_EPI_MARK(i)           // measurement hook (tools/kbench build of gemm4 only)
#endif

enum EpiFlag : unsigned {
    F_GELU = 1u, F_GLU = 2u, F_RES = 4u, F_STATS = 8u, F_GN = 16u, F_ROWADD = 32u, F_SPLIT = 64u, F_CBF16 = 128u,
    F_NOSTORE = 256u, F_PB = 512u, F_LN = 1024u, F_RGN = 2048u,
    F_ALL = 0xFFFFu
};

inline unsigned epi_flags(const GemmDesc& d) {
    unsigned f = 0;
    if (d.act == ACT_GELU) f |= F_GELU;
    if (d.act == ACT_GLU) f |= F_GLU;
    if (d.res) f |= F_RES;
    if (d.stats) f |= F_STATS;
    if (d.gn_stats) f |= F_GN;
    if (d.row_add) f |= F_ROWADD;
    if (d.col_split) f |= F_SPLIT;
    if (d.c_bf16 && d.store) f |= F_CBF16;     // the output dtype is irrelevant when nothing is stored
    if (!d.store) f |= F_NOSTORE;
    if (d.pbias) f |= F_PB;
    if (d.ln_w) f |= F_LN;
    if (d.res_gn_stats) f |= F_RGN;
    return f;
}

// The combinations the forward uses; anything else runs the general (F_ALL) instantiation.
#define ATHD_EPI_LIST(X)                                                                                         \
    X(0u) X(F_CBF16) X(F_GELU) X(F_GELU | F_CBF16) X(F_RES) X(F_RES | F_STATS) X(F_GLU) X(F_GLU | F_ROWADD)    \
    X(F_STATS | F_NOSTORE) X(F_GN | F_GLU | F_RES) X(F_STATS) X(F_SPLIT | F_STATS) X(F_SPLIT)                  \
    X(F_SPLIT | F_STATS | F_CBF16) X(F_SPLIT | F_CBF16) X(F_GLU | F_CBF16) X(F_GLU | F_ROWADD | F_CBF16)         \
    X(F_GN | F_GLU | F_RES | F_CBF16) X(F_GELU | F_CBF16 | F_PB) X(F_GELU | F_PB) X(F_RES | F_PB) X(F_RES | F_RGN)

// Publishes the LDS statistics partials before the per-block flush: the LDS atomics retired (lgkmcnt) + s_barrier.
// Not __syncthreads(): that also waits vmcnt(0), i.e. for every output store of the tile to be acknowledged,
// which holds the block (and, at one block per CU, the CU) for the store latency.
ATHD_DEV void stats_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <unsigned F>
ATHD_DEV bool on(unsigned flag) { return (F & flag) != 0; }

// 4 consecutive residual values (f32 or bf16 storage)
ATHD_DEV void ld_res4(const GemmDesc& d, int64_t off, float* r) {
    if (d.res_bf16) {
        const uint2 q = *reinterpret_cast<const uint2*>((const bf16_t*)d.res + off);
        r[0] = __uint_as_float(q.x << 16);
        r[1] = __uint_as_float(q.x & 0xFFFF0000u);
        r[2] = __uint_as_float(q.y << 16);
        r[3] = __uint_as_float(q.y & 0xFFFF0000u);
    } else {
        const float4 v = *reinterpret_cast<const float4*>((const float*)d.res + off);
        r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    }
}

// Per-column bias of the lane's TN 4-column groups (the epilogue's only loads besides the residual).
template <int TN>
ATHD_DEV void load_bias4(const GemmDesc& d, int n0, int wn0, int lane, float4 (&bj)[TN]) {
    const int fg = lane >> 4;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nb = n0 + wn0 + 16 * j + 4 * fg;
        bj[j] = (d.bias && nb + 3 < d.N) ? *reinterpret_cast<const float4*>(d.bias + nb) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (d.bias && nb < d.N && nb + 3 >= d.N) {   // ragged N (N % 4 != 0 never occurs; keep it exact anyway)
            float t[4] = {0.f, 0.f, 0.f, 0.f};
            for (int q = 0; q < 4 && nb + q < d.N; ++q) t[q] = d.bias[nb + q];
            bj[j] = make_float4(t[0], t[1], t[2], t[3]);
        }
    }
}

// bpre: the bias already loaded by the kernel (load_bias4 before its main loop).  Loaded here instead, its
// vmcnt wait lands inside the per-store branches, where the compiler can only use vmcnt(0): every store then
// waits for all earlier stores to retire (measured: 16-18k cycles for 32 stores per lane on gemm4).
template <int TM, int TN, unsigned F, bool FASTG>
ATHD_DEV void gemm_epilogue(const GemmDesc& d, const f32x4_t (&acc)[TM][TN], int64_t m0, int n0, int wm0, int wn0,
                            int lane, double* st_lds, int BM, const float4* bpre = nullptr) {
    // Transposed accumulators (the kernels issue mfma(W_frag, A_frag)): lane l holds, for tile (i, j), output row
    // m = m0 + wm0 + 16 i + (l & 15) and the 4 consecutive columns n = n0 + wn0 + 16 j + 4 (l >> 4) + {0..3}.
    constexpr bool GEN = F == F_ALL;
    const bool f_gelu = GEN ? d.act == ACT_GELU : on<F>(F_GELU);
    const bool f_glu = GEN ? d.act == ACT_GLU : on<F>(F_GLU);
    const bool f_res = GEN ? d.res != nullptr : on<F>(F_RES);
    const bool f_stats = GEN ? d.stats != nullptr : on<F>(F_STATS);
    const bool f_gn = GEN ? d.gn_stats != nullptr : on<F>(F_GN);
    const bool f_row = GEN ? d.row_add != nullptr : on<F>(F_ROWADD);
    const bool f_split = GEN ? d.col_split != 0 : on<F>(F_SPLIT);
    const bool f_cbf = GEN ? d.c_bf16 != 0 : on<F>(F_CBF16);
    const bool f_store = GEN ? d.store != 0 : !on<F>(F_NOSTORE);
    const bool f_pb = GEN ? d.pbias != nullptr : on<F>(F_PB);

    const int fr = lane & 15, fg = lane >> 4;
    const uint32_t M = (uint32_t)d.nb * d.H_out * d.W;       // < 2^31 on every use
    const int64_t c_bs = d.c_bs >= 0 ? d.c_bs : (int64_t)d.H_out_total * d.W * d.ldo;
    const int Nout = f_glu ? d.N / 2 : d.N;
    const uint32_t g0 = fdiv((uint32_t)m0, d.fd_hw);                  // first GroupNorm group touched by this block
    uint32_t mlast = (uint32_t)m0 + (uint32_t)BM - 1;
    if (mlast >= M) mlast = M - 1;
    const bool one_group = fdiv(mlast, d.fd_hw) == g0;                // fast path: the whole tile in one group
    const int64_t hi_off = f_split ? (int64_t)d.hi_row_off * d.W * d.ldo - d.col_split : 0;
    // one batch of W = 1 rows (the transformer / linear layers): row m is (b, ho, w) = (0, m, 0), no divisions
    const bool linear = d.W == 1 && d.nb == 1;
    // paired 16-B bf16 stores (T21): whole 32-column pairs (N % 32 == 0, pair starts 32-aligned), no column split
    const bool f_wide = TN % 2 == 0 && f_cbf && !f_split && !f_glu && f_store && d.N % 32 == 0 && (n0 + wn0) % 32 == 0;
    float q1 = 0.f, q2 = 0.f;

    ATHD_EPI_MARK(12);
    // per-column constants (hoisted out of the row loop): columns n = nb_j + {0..3}
    float4 bj[TN];
    int grp[TN];     // ConvT residue group of the lane's 4 columns (col_split % 4 == 0: a 4-group never straddles)
    if (bpre) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bj[j] = bpre[j];
    } else {
        load_bias4<TN>(d, n0, wn0, lane, bj);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nb = n0 + wn0 + 16 * j + 4 * fg;
        grp[j] = f_split ? nb / d.col_split : 0;
    }
    ATHD_EPI_MARK(13);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        if (i == 1) ATHD_EPI_MARK(14);
        const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
        float p1 = 0.f, p2 = 0.f;
        if (m < M) {
            uint32_t w = 0, ho = m, b = 0;
            if (!linear) {
                const uint32_t t = fdiv(m, d.fd_w);
                w = m - t * (uint32_t)d.W;
                b = fdiv(t, d.fd_h);
                ho = t - b * (uint32_t)d.H_out;
            }
            // signed row arithmetic: o_off may be negative (its row is then masked out by store_mask / hi_row_off)
            const int64_t orow = (int64_t)(int)ho * d.o_stride + d.o_off;
            const int64_t obase = (int64_t)b * c_bs + (orow * d.W + w) * d.ldo + d.col_off;
            float gm = 0.f, gr = 1.f;
            if (f_gn) {
                const double mm = d.gn_stats[2 * b] / (double)d.gn_count;
                double var = d.gn_stats[2 * b + 1] / (double)d.gn_count - mm * mm;
                if (var < 0) var = 0;
                gm = (float)mm;
                gr = (float)(1.0 / sqrt(var + 1e-5));
            }
            if (f_glu) {
#pragma unroll
                for (int j = 0; j + 1 < TN; j += 2) {
                    const int na = n0 + wn0 + 16 * j + 4 * fg;        // packed columns of the 'a' half
                    const int oc = (n0 + wn0 + 16 * j) / 2 + 4 * fg;  // output channels oc..oc+3
                    if (oc >= Nout) continue;
                    const float bav[4] = {bj[j].x, bj[j].y, bj[j].z, bj[j].w};
                    const float bgv[4] = {bj[j + 1].x, bj[j + 1].y, bj[j + 1].z, bj[j + 1].w};
                    float o[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float a = acc[i][j][q] + bav[q], g = acc[i][j + 1][q] + bgv[q];
                        if (f_gn) {
                            a = (a - gm) * gr * d.gn_w[na + q] + d.gn_b[na + q];
                            g = (g - gm) * gr * d.gn_w[na + 16 + q] + d.gn_b[na + 16 + q];
                        }
                        float v = a * sigmoid<FASTG>(g);
                        if (f_row) v += d.row_add[(int64_t)ho * Nout + oc + q];
                        o[q] = v;
                    }
                    if (f_res) {
                        float rr[4];
                        ld_res4(d, obase + oc, rr);
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] = rr[q] + (d.res_scale ? d.res_scale[oc + q] : 1.f) * o[q];
                    }
                    if (f_store) {
                        if (f_cbf) {
                            *reinterpret_cast<uint2*>((bf16_t*)d.C + obase + oc) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
                        } else {
                            *reinterpret_cast<float4*>((float*)d.C + obase + oc) = make_float4(o[0], o[1], o[2], o[3]);
                        }
                        if (d.c4 && oc == 0) {        // compact copy of channels 0..3 (row index of the dense C)
                            const int64_t ri = (obase - d.col_off) / d.ldo;
                            if (f_cbf) *reinterpret_cast<uint2*>((bf16_t*)d.c4 + 4 * ri) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
                            else *reinterpret_cast<float4*>((float*)d.c4 + 4 * ri) = make_float4(o[0], o[1], o[2], o[3]);
                        }
                    }
                }
            } else {
                // F_PB: per-batch bias; pfold output batches per input batch; residual batch = output batch / res_div
                const int np = f_pb && d.pfold > 1 ? d.pfold : 1;
                const int64_t inb = obase - (int64_t)b * c_bs;          // offset within the batch
                for (int pp = 0; pp < np; ++pp) {
                const int64_t bo = f_pb && d.pfold > 1 ? (int64_t)b * d.pfold + pp : (int64_t)b;   // output batch
                const int64_t ob = bo * c_bs + inb;
                const int64_t rbase = f_pb && d.res_div > 1 ? (bo / d.res_div) * d.res_bs + inb : ob;
                uint2 pk_even = make_uint2(0u, 0u);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = n0 + wn0 + 16 * j + 4 * fg;
                    if (n >= d.N) continue;
                    float bv[4] = {bj[j].x, bj[j].y, bj[j].z, bj[j].w};
                    if (f_pb) {
                        const float4 pq = *reinterpret_cast<const float4*>(d.pbias + bo * d.N + n);
                        bv[0] += pq.x; bv[1] += pq.y; bv[2] += pq.z; bv[3] += pq.w;
                    }
                    float o[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float v = acc[i][j][q] + bv[q];
                        if (f_gn) v = (v - gm) * gr * d.gn_w[n + q] + d.gn_b[n + q];
                        o[q] = v;
                    }
                    if (f_gelu) {
                        if constexpr (FASTG) {      // bf16 mode: the polynomial and scaling on packed pairs
                            const athd_f2v g01 = gelu_fast_pk((athd_f2v){o[0], o[1]});
                            const athd_f2v g23 = gelu_fast_pk((athd_f2v){o[2], o[3]});
                            o[0] = g01.x; o[1] = g01.y; o[2] = g23.x; o[3] = g23.y;
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q) o[q] = gelu<FASTG>(o[q]);
                        }
                    }
                    if (f_row) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] += d.row_add[(int64_t)ho * Nout + n + q];
                    }
                    if (f_res) {
                        float rr[4];
                        ld_res4(d, rbase + n, rr);
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] = rr[q] + (d.res_scale ? d.res_scale[n + q] : 1.f) * o[q];
                    }
                    if (f_stats) {            // statistics of the final value (GroupNorm input)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            p1 += o[q];
                            p2 += o[q] * o[q];
                        }
                    }
                    if (f_store) {
                        int64_t off = ob + n;
                        bool st = true;
                        if (f_split) {
                            st = (d.store_mask >> grp[j]) & 1;
                            off += grp[j] * hi_off;
                        }
                        if (st) {
                            if (f_wide) {
                                // T21 (cdna_hip_programming.md): tiles j, j+1 of one row are trade halves between lane
                                // groups fg and fg^1 with v_permlane16_swap, so each lane stores 8 consecutive
                                // columns (16 B) instead of 4: half the store instructions, same bytes
                                const uint2 pk = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
                                if ((j & 1) == 0) {
                                    pk_even = pk;
                                } else {
                                    const auto rx = __builtin_amdgcn_permlane16_swap(pk_even.x, pk.x, false, false);
                                    const auto ry = __builtin_amdgcn_permlane16_swap(pk_even.y, pk.y, false, false);
                                    const int col = n0 + wn0 + 16 * (j - 1) + 16 * (fg & 1) + 8 * (fg >> 1);
                                    *reinterpret_cast<uint4*>((bf16_t*)d.C + ob + col) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
                                }
                            } else if (f_cbf) {
                                *reinterpret_cast<uint2*>((bf16_t*)d.C + off) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
                            } else {
                                *reinterpret_cast<float4*>((float*)d.C + off) = make_float4(o[0], o[1], o[2], o[3]);
                            }
                        }
                    }
                }
                }  // pp
            }
        }  // m < M
        if (f_stats && one_group) {
            q1 += p1;
            q2 += p2;
        } else if (f_stats) {
            // the 4 lane groups (lane >> 4) hold the same row m: reduce across them, one LDS add per row
            p1 += __shfl_xor(p1, 16, 64);
            p2 += __shfl_xor(p2, 16, 64);
            p1 += __shfl_xor(p1, 32, 64);
            p2 += __shfl_xor(p2, 32, 64);
            if (fg == 0 && m < M) {
                const uint32_t gi = fdiv(m, d.fd_hw) - g0;
                if (gi < (uint32_t)EPI_MAXG) {
                    atomicAdd(&st_lds[2 * gi], (double)p1);
                    atomicAdd(&st_lds[2 * gi + 1], (double)p2);
                } else {
                    atomicAdd(&d.stats[2 * (g0 + gi)], (double)p1);
                    atomicAdd(&d.stats[2 * (g0 + gi) + 1], (double)p2);
                }
            }
        }
    }
    ATHD_EPI_MARK(15);
    if (f_stats && one_group) {
        const double t1 = wave_sum_d((double)q1), t2 = wave_sum_d((double)q2);
        if (lane == 0) {
            atomicAdd(&st_lds[0], t1);
            atomicAdd(&st_lds[1], t2);
        }
    }
    if (f_stats) {
        stats_barrier();
        if (threadIdx.x < EPI_MAXG) {
            const double a = st_lds[2 * threadIdx.x], q = st_lds[2 * threadIdx.x + 1];
            st_lds[2 * threadIdx.x] = 0.0;          // ready for the next tile of a persistent kernel
            st_lds[2 * threadIdx.x + 1] = 0.0;
            if (a != 0.0 || q != 0.0) {
                atomicAdd(&d.stats[2 * (g0 + threadIdx.x)], a);
                atomicAdd(&d.stats[2 * (g0 + threadIdx.x) + 1], q);
            }
        }
    }
}

// DConv 1x1 apply epilogue (F_GN | F_GLU | F_RES | F_CBF16 with a bf16 residual, dense rows: row m at m*ldo; the
// wide encoder levels, forward.cpp dconv): out = res + scale * GLU(GN(acc + bias)).  Branch-free: every residual
// value of the wave's rows is loaded before the first store (rows past M read the last row and store into a sink),
// so the tile pays one load latency, not one per row fragment behind the previous fragment's stores as in
// gemm_epilogue's guarded form.
__device__ __attribute__((weak)) uint2 g_epi_sink2[64];

ATHD_HD bool epi_glures_ok(const GemmDesc& d) {
    return d.act == ACT_GLU && d.res && d.res_bf16 && d.c_bf16 && d.store && d.gn_stats && !d.row_add && !d.pbias &&
           !d.col_split && !d.stats && !d.c4 && d.o_stride == 1 && d.o_off == 0 && d.H_out_total == d.H_out &&
           d.c_bs < 0 && d.col_off == 0 && d.N % 32 == 0;
}

template <int TM, int TN>
ATHD_DEV void gemm_epilogue_glures(const GemmDesc& d, f32x4_t (&acc)[TM][TN], int64_t m0, int n0, int wm0, int wn0,
                                   int lane, const float4 (&bj)[TN]) {
    static_assert(TN % 2 == 0, "GLU column pairs");
    constexpr int TP = TN / 2;
    const int fr = lane & 15, fg = lane >> 4;
    const uint32_t M = (uint32_t)d.nb * d.H_out * d.W;
    const int Nout = d.N / 2;
    const bf16_t* X = (const bf16_t*)d.res;
    uint2 rr[TM][TP];
    int64_t ro[TM];
    bool ok[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
        ok[i] = m < M;
        ro[i] = (int64_t)(ok[i] ? m : M - 1) * d.ldo;
#pragma unroll
        for (int p = 0; p < TP; ++p) {
            const int oc = (n0 + wn0 + 32 * p) / 2 + 4 * fg;
            rr[i][p] = *reinterpret_cast<const uint2*>(X + ro[i] + (oc < Nout ? oc : 0));
        }
    }
    float gm[TM], gr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const uint32_t b = fdiv((uint32_t)(ro[i] / d.ldo), d.fd_hw);
        const double mm = d.gn_stats[2 * b] / (double)d.gn_count;
        double var = d.gn_stats[2 * b + 1] / (double)d.gn_count - mm * mm;
        if (var < 0) var = 0;
        gm[i] = (float)mm;
        gr[i] = (float)(1.0 / sqrt(var + 1e-5));
    }
#pragma unroll
    for (int p = 0; p < TP; ++p) {
        const int na = n0 + wn0 + 32 * p + 4 * fg;            // packed columns of the 'a' half (gate: na + 16)
        const int oc = (n0 + wn0 + 32 * p) / 2 + 4 * fg;      // output channels oc .. oc + 3
        if (oc >= Nout) continue;
        const float4 wa = *reinterpret_cast<const float4*>(d.gn_w + na), ba = *reinterpret_cast<const float4*>(d.gn_b + na);
        const float4 wg = *reinterpret_cast<const float4*>(d.gn_w + na + 16), bg = *reinterpret_cast<const float4*>(d.gn_b + na + 16);
        const float4 sc = d.res_scale ? *reinterpret_cast<const float4*>(d.res_scale + oc) : make_float4(1.f, 1.f, 1.f, 1.f);
        const float wav[4] = {wa.x, wa.y, wa.z, wa.w}, bav[4] = {ba.x, ba.y, ba.z, ba.w};
        const float wgv[4] = {wg.x, wg.y, wg.z, wg.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
        const float scv[4] = {sc.x, sc.y, sc.z, sc.w};
        const float b0[4] = {bj[2 * p].x, bj[2 * p].y, bj[2 * p].z, bj[2 * p].w};
        const float b1[4] = {bj[2 * p + 1].x, bj[2 * p + 1].y, bj[2 * p + 1].z, bj[2 * p + 1].w};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const uint2 q = rr[i][p];
            const float r4[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                                 __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u)};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = (acc[i][2 * p][e] + b0[e] - gm[i]) * gr[i] * wav[e] + bav[e];
                const float g = (acc[i][2 * p + 1][e] + b1[e] - gm[i]) * gr[i] * wgv[e] + bgv[e];
                o[e] = r4[e] + scv[e] * (a * sigmoid_fast(g));
            }
            uint2* dst = ok[i] ? reinterpret_cast<uint2*>((bf16_t*)d.C + ro[i] + oc) : g_epi_sink2 + lane;
            *dst = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
        }
    }
}

// Residual-stream epilogue (F_RES [+ F_STATS], f32 output and residual, dense rows: row m at m*ldo): out = res +
// res_scale * (acc + bias), GroupNorm statistics of out.  Written branch-free - rows past M read a clamped row and
// store into a sink line - with the residual loads of row tile i+1 issued before the stores of tile i.  The compiler
// then counts vmcnt exactly (straight-line code): a residual load waits only for the stores issued before it, two
// tiles back, instead of vmcnt(0) behind every store (gemm_epilogue's branch-guarded loads).
__device__ __attribute__((weak)) float4 g_epi_sink[64];

ATHD_HD bool epi_res_fast_ok(const GemmDesc& d) {
    return d.res && !d.res_bf16 && !d.c_bf16 && d.store && d.act == ACT_NONE && !d.gn_stats && !d.row_add && !d.pbias &&
           !d.col_split && d.o_stride == 1 && d.o_off == 0 && d.H_out_total == d.H_out && d.c_bs < 0 && d.N % 4 == 0 &&
           (!d.res_gn_stats || (d.res_gn_w && d.res_gn_b && d.res_gn_count > 0 && d.col_off == 0 &&
                                 (int64_t)d.H_out * d.W >= 256));
}

// F_RGN: gn_lds holds the residual GroupNorm affine of the tile's columns, w at [n - n0], b at [256 + n - n0], and
// the residual scale at [512 + n - n0] (staged by the kernel; registers for them would spill the residual ring)
template <int TM, int TN, unsigned F>
ATHD_DEV void gemm_epilogue_res(const GemmDesc& d, const f32x4_t (&acc)[TM][TN], int64_t m0, int n0, int wm0, int wn0,
                                int lane, double* st_lds, int BM, const float4* bj, const float* gn_lds = nullptr) {
    constexpr bool f_stats = (F & F_STATS) != 0;
    constexpr bool f_rgn = (F & F_RGN) != 0;
    const int fr = lane & 15, fg = lane >> 4;
    const uint32_t M = (uint32_t)d.nb * d.H_out * d.W;
    const uint32_t g0 = fdiv((uint32_t)m0, d.fd_hw);
    uint32_t mlast = (uint32_t)m0 + (uint32_t)BM - 1;
    if (mlast >= M) mlast = M - 1;
    const bool one_group = fdiv(mlast, d.fd_hw) == g0;
    int ncol[TN];
    float4 sc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        ncol[j] = n0 + wn0 + 16 * j + 4 * fg;
        const int nc = ncol[j] < d.N ? ncol[j] : d.N - 4;
        ncol[j] = nc;
        if constexpr (!f_rgn)   // (F_RGN: the scale is read from gn_lds per fragment, its registers go to the affine)
            sc[j] = d.res_scale ? *reinterpret_cast<const float4*>(d.res_scale + nc) : make_float4(1.f, 1.f, 1.f, 1.f);
    }
    bool colok[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) colok[j] = n0 + wn0 + 16 * j + 4 * fg < d.N;
    int64_t rb[TM];
    bool ok[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
        ok[i] = m < M;
        rb[i] = (int64_t)(ok[i] ? m : M - 1) * d.ldo + d.col_off;
    }
    // F_RGN: (mean, rstd) of the tile's first batch g0 and of g0 + 1 (a BM-row tile spans at most two batches: every
    // caller has H_out * W >= BM rows per batch, epi_res_fast_ok)
    float rgn[4] = {0.f, 1.f, 0.f, 1.f};
    if constexpr (f_rgn) {
        const uint32_t glast = fdiv(M - 1, d.fd_hw);
        gn_params(d.res_gn_stats, g0, d.res_gn_count, rgn[0], rgn[1]);
        gn_params(d.res_gn_stats, g0 + 1 <= glast ? g0 + 1 : glast, d.res_gn_count, rgn[2], rgn[3]);
    }
    const float* res = (const float*)d.res;
    float* C = (float*)d.C;
    float* sink = reinterpret_cast<float*>(g_epi_sink + lane);
    // residual ring: the loads of row fragment i + RD - 1 are issued before the stores of fragment i, so RD - 1
    // fragments of loads are in flight across the stores (round 2: one; the epilogue then streamed at ~20 GB/s per
    // CU, an HBM round trip per fragment).  The K-loop's operand fragments are dead here, so the ring's registers
    // do not raise the kernel's VGPR count.
#ifndef ATHD_RES_RD
#define ATHD_RES_RD 3      // 3: two fragments ahead (244-246 VGPRs; 4 spills in the K-loop kernels)
#endif
    constexpr int RD0 = f_rgn ? 2 : ATHD_RES_RD;     // (F_RGN: its per-fragment affine needs the ring's registers)
    constexpr int RD = TM < RD0 ? TM : RD0;
    float4 rr[RD][TN];
#pragma unroll
    for (int i = 0; i + 1 < RD; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) rr[i][j] = *reinterpret_cast<const float4*>(res + rb[i] + ncol[j]);
    float p1[TM], p2[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        if (i + RD - 1 < TM) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
                rr[(i + RD - 1) % RD][j] = *reinterpret_cast<const float4*>(res + rb[i + RD - 1] + ncol[j]);
        }
        float s1 = 0.f, s2 = 0.f;
        float rgm = 0.f, rgr = 1.f;            // F_RGN: the residual row's GroupNorm (mean, rstd)
        if constexpr (f_rgn) {
            const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
            const bool second = fdiv(ok[i] ? m : M - 1, d.fd_hw) != g0;
            rgm = second ? rgn[2] : rgn[0];
            rgr = second ? rgn[3] : rgn[1];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            float4 rc = rr[i % RD][j];
            if constexpr (f_rgn) {
                const int cl = ncol[j] - n0;
                const float4 gw = *reinterpret_cast<const float4*>(gn_lds + cl);
                const float4 gb = *reinterpret_cast<const float4*>(gn_lds + 256 + cl);
                sc[j] = *reinterpret_cast<const float4*>(gn_lds + 512 + cl);
                rc.x = (rc.x - rgm) * rgr * gw.x + gb.x;
                rc.y = (rc.y - rgm) * rgr * gw.y + gb.y;
                rc.z = (rc.z - rgm) * rgr * gw.z + gb.z;
                rc.w = (rc.w - rgm) * rgr * gw.w + gb.w;
            }
            const float4 o = make_float4(rc.x + sc[j].x * (acc[i][j][0] + bj[j].x), rc.y + sc[j].y * (acc[i][j][1] + bj[j].y),
                                         rc.z + sc[j].z * (acc[i][j][2] + bj[j].z), rc.w + sc[j].w * (acc[i][j][3] + bj[j].w));
            const bool st = ok[i] && colok[j];
            if (f_stats && st) {
                s1 += (o.x + o.y) + (o.z + o.w);
                s2 += (o.x * o.x + o.y * o.y) + (o.z * o.z + o.w * o.w);
            }
            *reinterpret_cast<float4*>(st ? C + rb[i] + ncol[j] : sink) = o;
        }
        p1[i] = s1;
        p2[i] = s2;
    }
    if constexpr (f_stats) {
        if (one_group) {
            float q1 = 0.f, q2 = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                q1 += p1[i];
                q2 += p2[i];
            }
            const double t1 = wave_sum_d((double)q1), t2 = wave_sum_d((double)q2);
            if (lane == 0) {
                atomicAdd(&st_lds[0], t1);
                atomicAdd(&st_lds[1], t2);
            }
        } else {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                float a = p1[i], b = p2[i];
                a += __shfl_xor(a, 16, 64);
                b += __shfl_xor(b, 16, 64);
                a += __shfl_xor(a, 32, 64);
                b += __shfl_xor(b, 32, 64);
                const uint32_t m = (uint32_t)m0 + wm0 + 16 * i + fr;
                if (fg == 0 && ok[i]) {
                    const uint32_t gi = fdiv(m, d.fd_hw) - g0;
                    if (gi < (uint32_t)EPI_MAXG) {
                        atomicAdd(&st_lds[2 * gi], (double)a);
                        atomicAdd(&st_lds[2 * gi + 1], (double)b);
                    } else {
                        atomicAdd(&d.stats[2 * (g0 + gi)], (double)a);
                        atomicAdd(&d.stats[2 * (g0 + gi) + 1], (double)b);
                    }
                }
            }
        }
        stats_barrier();
        if (threadIdx.x < EPI_MAXG) {
            const double a = st_lds[2 * threadIdx.x], q = st_lds[2 * threadIdx.x + 1];
            st_lds[2 * threadIdx.x] = 0.0;
            st_lds[2 * threadIdx.x + 1] = 0.0;
            if (a != 0.0 || q != 0.0) {
                atomicAdd(&d.stats[2 * (g0 + threadIdx.x)], a);
                atomicAdd(&d.stats[2 * (g0 + threadIdx.x) + 1], q);
            }
        }
    }
}

}  // namespace athd
