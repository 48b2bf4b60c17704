"""CPU check of the identity behind fdec1f.hip (the level-1 frequency decoder's GroupNorm statistics as quadratic
forms of per-item Gram matrices): for random Z (32 rows x 8 taps), Zs (8 rows x 8 taps) and bias, the sum and sum of
squares of the level-1 ConvT output rows computed the direct way (fdec_lr.hip's step formula: row 4v+rho =
b + T_v[rho+2] + (rho < 2 ? T_{v-1}[rho+6] : T_{v+1}[rho-2]), T_s = lerp of the Z rows + 0.1 lerp of the Zs rows,
ATHTDemucs_v2.py:90-103 re-associated) equal 4 Hd W sum b + sum_q c1_q . u_q and
4 Hd W sum b^2 + 2 sum_q c1_q . ub_q + sum_q <Q_q, G_q> with fdec1_gram_q_kernel's coefficients (g_coef, restated
here).  The lerp weights are PyTorch's (F.interpolate, bilinear, align_corners=False), checked against
torch.nn.functional.interpolate itself.  Float64 throughout: this pins the algebra, not the rounding."""
import numpy as np
import pytest
import torch

HS, HK = 32, 8


def lin_index(dst, n_in, n_out):
    """common.h::lin_index (ATen area_pixel_compute_source_index, align_corners=False), in fp32 like the kernels."""
    if n_in == n_out:
        return dst, dst, 0.0
    scale = np.float32(n_in) / np.float32(n_out)
    src = np.float32(scale * (np.float32(dst) + np.float32(0.5)) - np.float32(0.5))
    if src < 0:
        src = np.float32(0.0)
    i0 = min(int(np.floor(src)), n_in - 1)
    lam = float(min(max(src - np.float32(i0), 0.0), 1.0))
    i1 = i0 + (1 if i0 < n_in - 1 else 0)
    return i0, i1, lam


def lerp_row(v, n_in, n_out):
    i0, i1, l = lin_index(v, n_in, n_out)
    r = np.zeros(n_in)
    r[i0] += 1.0 - l
    r[i1] += l
    return r


def g_coef(q, v, a, hd):
    """fdec1f.hip::g_coef: coefficient of x_q entry a in ConvT output row 4v + rho, rho = (q + 2) % 4."""
    rho = (q + 2) & 3
    t_main = q if rho < 2 else q + 4
    v_oth = v - 1 if rho < 2 else v + 1
    zs = a >= 64
    idx = (a - 64) & 7 if zs else a & 31
    tap = (q if a < 72 else q + 4) if zs else (q if a < 32 else q + 4)
    s = v if tap == t_main else v_oth
    if s < 0 or s >= hd:
        return 0.0
    cf = lerp_row(s, HK if zs else HS, hd)[idx]
    return cf * float(np.float32(0.1)) if zs else cf


@pytest.mark.parametrize("hd", [33, 49, 259])
def test_lerp_matches_torch_interpolate(hd):
    for n_in in (HS, HK):
        eye = torch.eye(n_in, dtype=torch.float32).reshape(1, 1, n_in, n_in)   # fp32: fp32 index math, as the kernels
        m = torch.nn.functional.interpolate(eye, size=(hd, n_in), mode="bilinear", align_corners=False)[0, 0]
        ours = np.stack([lerp_row(v, n_in, hd) for v in range(hd)])
        assert np.allclose(ours, m.numpy(), atol=1e-6)


@pytest.mark.parametrize("hd,W,C", [(33, 3, 4), (49, 5, 6), (259, 2, 3)])
def test_stats_quadratic_form_identity(hd, W, C):
    rng = np.random.default_rng(hd * 100 + W)
    Z = rng.standard_normal((HS, 8, W, C))          # [j][tap][w][c]
    Zs = rng.standard_normal((HK, 8, W, C))
    b = rng.standard_normal(C)

    # direct: every ConvT output row of the level (fdec_lr.hip)
    Lz = np.stack([lerp_row(v, HS, hd) for v in range(hd)])       # [hd][32]
    Lk = np.stack([lerp_row(v, HK, hd) for v in range(hd)])       # [hd][8]
    T = np.einsum("vj,jkwc->vkwc", Lz, Z) + float(np.float32(0.1)) * np.einsum("vm,mkwc->vkwc", Lk, Zs)   # 0.1f as the kernels
    zero = np.zeros_like(T[0])
    rows = []
    for v in range(hd):
        prev = T[v - 1] if v >= 1 else zero
        nxt = T[v + 1] if v + 1 < hd else zero
        for rho in range(4):
            other = prev[rho + 6] if rho < 2 else nxt[rho - 2]
            rows.append(b + T[v][rho + 2] + other)
    Y = np.stack(rows)
    s1_direct, s2_direct = Y.sum(), (Y ** 2).sum()

    # quadratic forms: per class q, x_q = (Z_q, Z_{q+4}, Zs_q, Zs_{q+4}) at each (w, c)
    s1 = 4.0 * hd * W * b.sum()
    s2 = 4.0 * hd * W * (b ** 2).sum()
    for q in range(4):
        X = np.concatenate([Z[:, q], Z[:, q + 4], Zs[:, q], Zs[:, q + 4]]).reshape(80, W * C)   # [a][(w, c)]
        coef = np.array([[g_coef(q, v, a, hd) for a in range(80)] for v in range(hd)])       # [row][a]
        Q = coef.T @ coef
        c1 = coef.sum(axis=0)
        G = X @ X.T
        bw = np.tile(b, W)                                  # b_c at each (w, c)
        u, ub = X.sum(axis=1), X @ bw
        s1 += c1 @ u
        s2 += 2.0 * c1 @ ub + (Q * G).sum()
    assert np.isclose(s1, s1_direct, rtol=1e-10, atol=1e-8), (s1, s1_direct)
    assert np.isclose(s2, s2_direct, rtol=1e-10), (s2, s2_direct)
