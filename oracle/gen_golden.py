"""ORACLE tooling - generates tests/golden/*.npz by running the REFERENCE module itself.

Runs only where /root/reference exists (the survey/build container), never on the GPU box.  Steps (SURVEY.md
§8(c) "Golden vectors"):
  1. a `sys.modules` stub for `demucs.htdemucs` (the reference only uses `HTDemucs` as a type hint,
     `ATHTDemucs_v2.py:18,153`); demucs==4.0.1 is not installed and is never fetched;
  2. seeded weights from `athd.weights.synthetic_state_dict(seed=0)`;
  3. the htdemucs stand-in = oracle/htdemucs_ref.HTDemucsHot (parity with demucs itself unpinned);
  4. a fake tokenizer + CLAP text tower returning rows of a seeded L2-normalised (4, 512) table through the
     non-ClapModel branch of `_get_clap_embeddings` (`ATHTDemucs_v2.py:245-248`);
  5. the reference `AudioTextHTDemucs.forward` (`ATHTDemucs_v2.py:250-326`) on seeded synthetic audio, with
     forward hooks capturing intermediates.
The fixtures are data only (inputs and the reference's outputs); no reference source is copied.

    python oracle/gen_golden.py          # rewrites tests/golden/*.npz
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "audio-to-sheet-music_amd"))

from athd.weights import STEMS, synthetic_state_dict, synthetic_text_table, weights_checksum  # noqa: E402
from athd.synth import synthetic_mixture  # noqa: E402
from oracle.htdemucs_ref import load_hot  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")


def import_reference():
    demucs = types.ModuleType("demucs")
    htd = types.ModuleType("demucs.htdemucs")

    class HTDemucs(nn.Module):   # type-hint placeholder only
        pass

    htd.HTDemucs = HTDemucs
    demucs.htdemucs = htd
    sys.modules.setdefault("demucs", demucs)
    sys.modules.setdefault("demucs.htdemucs", htd)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import importlib
    return importlib.import_module("src.models.stem_separation.ATHTDemucs_v2")


class FakeTokenizer:
    """tokenizer(text, padding=True, return_tensors='pt') -> {'input_ids': (B,1) prompt index}."""

    def __call__(self, text, padding=True, return_tensors="pt"):
        if isinstance(text, str):
            text = [text]
        return {"input_ids": torch.tensor([[STEMS.index(t)] for t in text], dtype=torch.long)}


class FakeClapText(nn.Module):
    def __init__(self, table: np.ndarray):
        super().__init__()
        self.table = nn.Parameter(torch.as_tensor(table), requires_grad=False)

    def forward(self, input_ids=None, **kw):
        return types.SimpleNamespace(text_embeds=self.table[input_ids[:, 0]])


def build_reference_model(sd, table):
    ref = import_reference()
    htd = load_hot(sd)
    model = ref.AudioTextHTDemucs(htd, FakeClapText(table), FakeTokenizer())
    own = {k: torch.as_tensor(v) for k, v in sd.items() if not k.startswith("htdemucs.")}
    missing, unexpected = model.load_state_dict(own, strict=False)
    assert not unexpected, unexpected
    bad = [k for k in missing if not (k.startswith("htdemucs.") or k.startswith("clap."))]
    assert not bad, bad
    return model.eval()


CASES = [
    # name, B, T, prompts, full-intermediates
    ("b1_t44100_vocals", 1, 44100, ["vocals"], True),
    ("b2_t30000_drums_bass", 2, 30000, ["drums", "bass"], False),
    ("b1_t1500_other", 1, 1500, ["other"], False),
    ("b1_t264600_vocals", 1, 264600, ["vocals"], False),
]


def run_case(model, name, B, T, prompts, full):
    wav = torch.stack([torch.as_tensor(synthetic_mixture(T, seed=1234 + i)) for i in range(B)])
    cap = {}
    hooks = [
        model.text_attn.register_forward_hook(lambda m, i, o: cap.update(x_enc=i[0], xt_enc=i[1],
                                                                          x_cond=o[0], xt_cond=o[1])),
        model.freq_decoder.register_forward_hook(lambda m, i, o: cap.update(x_fdec=o)),
        model.time_decoder.register_forward_hook(lambda m, i, o: cap.update(xt_tdec=o)),
    ]
    with torch.no_grad():
        out = model(wav, prompts[0] if B == 1 else prompts)
    for h in hooks:
        h.remove()
    rec = {"wav": wav.numpy(), "prompt_idx": np.array([STEMS.index(p) for p in prompts]), "out_shape": np.array(out.shape)}
    if T <= 44100:
        rec["out"] = out.numpy()
    else:
        rec["out_stride97"] = out[..., ::97].numpy().copy()
        rec["out_absmean"] = np.array(out.abs().mean().item())
    if full:
        for k in ("x_enc", "xt_enc", "x_cond", "xt_cond", "x_fdec", "xt_tdec"):
            rec[k] = cap[k].numpy()
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.manual_seed(0)
    sd = synthetic_state_dict(seed=0)
    table = synthetic_text_table(4, seed=7)
    model = build_reference_model(sd, table)
    np.savez_compressed(os.path.join(OUT, "meta.npz"), text_table=table, weights_checksum=weights_checksum(sd),
                        torch_version=np.array(torch.__version__))
    for case in CASES:
        out = run_case(model, *case)
        print(case[0], tuple(out.shape), float(out.abs().mean()))


if __name__ == "__main__":
    main()
