// Multi-head attention (d_head 64) on MFMA.  Q/K/V/O are token-major: X[b][token][ld] with head h at columns
// off + 64h .. off + 64h + 63.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace athd {

// Queries prescaled by 1/sqrt(d_head) * log2(e) (bf16 mode, folded into the in-projection weights at pack time):
// the kernel's logits are then base-2 exponents.  AttnDesc::scale is always the factor that turns q.k into a
// natural-log logit, so prescaled queries are described by scale = ln 2.
constexpr float ATTN_Q_PRESCALE = 0.125f * 1.4426950408889634f;
constexpr float ATTN_SCALE_PRESCALED = 0.6931471805599453f;

struct AttnDesc {
    const void* Q = nullptr; int q_bf16 = 0; int64_t q_bs = 0; int q_ld = 0; int q_off = 0;
    const void* K = nullptr; int k_bf16 = 0; int64_t k_bs = 0; int k_ld = 0; int k_off = 0;
    const void* V = nullptr; int v_bf16 = 0; int64_t v_bs = 0; int v_ld = 0; int v_off = 0;
    void* O = nullptr; int o_bf16 = 0; int64_t o_bs = 0; int o_ld = 0;
    int nb = 1, Nq = 0, Nk = 0, heads = 8;
    float scale = 0.125f;
};

int attn_launch(const AttnDesc& d, int mode, hipStream_t s);

}  // namespace athd
