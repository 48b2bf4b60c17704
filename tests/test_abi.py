"""C-ABI contract checks that need no GPU: the library loads, exports every function include/athd.h declares,
and its weight contract is the hot-path subset of the reference state dict."""
import os
import re

from conftest import REPO


def _header_functions():
    src = open(os.path.join(REPO, "include", "athd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(athd_[a-z_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from athd import native
    names = _header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(native.lib, n), n
    assert set(names) == set(native.EXPORTED)
    assert native.lib.athd_version() >= 100


def test_required_keys_are_reference_keys():
    from athd import native
    from athd.weights import hot_path_spec
    spec = {k for k, _, _ in hot_path_spec()}
    req = set(native.required_keys())
    assert req <= spec
    # only the dead query branch of TextCrossAttention (softmax over one key == 1) is unused
    assert spec - req == {f"text_attn.{m}.{p}" for m in ("q_proj", "k_proj", "norm_q") for p in ("weight", "bias")}


def test_create_without_device_fails_cleanly():
    import ctypes
    import torch
    from athd import native
    if torch.cuda.is_available():
        return
    h = ctypes.c_void_p()
    assert native.lib.athd_create(ctypes.byref(h), 0, 1) != 0


def test_text_closed_form_equals_attention(state_dict, text_table):
    """The native path replaces MHA over ONE text token by its closed form out_proj(W_v v_proj(t) + b_v);
    check the identity on the oracle side (CPU)."""
    import torch
    import torch.nn.functional as F
    from oracle.athtdemucs_ref import TextCrossAttentionRef
    ta = TextCrossAttentionRef(state_dict)
    s = ta.sd
    q = torch.randn(2, 50, 384)
    te = torch.as_tensor(text_table[:2])
    out = ta.forward_attend(q, te)
    v = F.linear(te, s["v_proj.weight"], s["v_proj.bias"])
    vi = F.linear(v, s["attn.in_proj_weight"][768:], s["attn.in_proj_bias"][768:])
    a = F.linear(vi, s["attn.out_proj.weight"], s["attn.out_proj.bias"])
    u = q + a[:, None, :]
    y = u + F.linear(F.gelu(F.linear(u, s["out_mlp.0.weight"], s["out_mlp.0.bias"])), s["out_mlp.2.weight"],
                     s["out_mlp.2.bias"])
    ref = F.layer_norm(y, (384,), s["norm_out.weight"], s["norm_out.bias"], 1e-5)
    assert torch.allclose(out, ref, atol=2e-6)
