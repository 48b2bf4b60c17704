"""Prompt -> 512-d text embedding (the CLAP side of `ATHTDemucs_v2.py:238-248`).

The CLAP text tower is frozen and its output depends only on the prompt string, so it is evaluated once per
distinct prompt and cached; the per-segment hot path only sees embedding rows.  Sources, in order:
  1. an explicit table {prompt: (512,) vector} (used when no CLAP weights exist offline - synthetic runs);
  2. a real CLAP model + tokenizer passed like the reference (`ClapModel.get_text_features` for ClapModel,
     `.forward(...).text_embeds` otherwise, exactly the branch logic of `_get_clap_embeddings`).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Union

import numpy as np
import torch

from .weights import STEMS, synthetic_text_table


CLAP_NAME = "laion/clap-htsat-unfused"     # test_inference.py:27-28


def load_clap(name: str = CLAP_NAME):
    """The reference's `ClapModel.from_pretrained(name)` + `AutoTokenizer.from_pretrained(name)`
    (`test_inference.py:26-28`), from the local Hugging Face cache only (`local_files_only=True`: there is no
    network on the target nodes).  Raises a RuntimeError naming the missing model and the `text_table=` alternative
    when the cache lacks its files."""
    try:
        from transformers import AutoTokenizer, ClapModel
    except ImportError as e:   # pragma: no cover - transformers is in the image
        raise RuntimeError(f"CLAP '{name}' needs transformers ({e}); pass text_table={{prompt: 512-vector}} "
                           f"instead") from e
    try:
        clap = ClapModel.from_pretrained(name, local_files_only=True)
        tokenizer = AutoTokenizer.from_pretrained(name, local_files_only=True)
    except (OSError, ValueError) as e:
        raise RuntimeError(
            f"CLAP model '{name}' is not in the local Hugging Face cache ({type(e).__name__}: {e}). The reference "
            f"downloads it (test_inference.py:27-28); offline, either place its files in the cache (HF_HOME) or pass "
            f"text_table={{prompt: 512-vector}} (e.g. precomputed ClapModel.get_text_features rows) or "
            f"clap=/tokenizer=") from e
    clap.eval()
    for p in clap.parameters():          # frozen, as ATHTDemucs_v2.py:174-176
        p.requires_grad = False
    return clap, tokenizer


class PromptEmbedder:
    def __init__(self, clap=None, tokenizer=None, table: Optional[Dict[str, np.ndarray]] = None):
        self.clap = clap
        self.tokenizer = tokenizer
        self.table: Dict[str, torch.Tensor] = {}
        self._from_clap: set = set()      # table entries computed by the CLAP model (invalidated on weight loads)
        if table:
            for k, v in table.items():
                self.table[k] = torch.as_tensor(np.asarray(v, dtype=np.float32)).reshape(-1)

    def load_clap_state(self, state: Dict[str, torch.Tensor]):
        """The `clap.*` part of a reference checkpoint, loaded into the CLAP model non-strictly as the reference's
        `model.load_state_dict(..., strict=False)` does for its `self.clap` submodule (`test_inference.py:34-35`).
        Embeddings computed with the previous weights are dropped.  Returns the number of tensors loaded."""
        if not state or self.clap is None or not hasattr(self.clap, "load_state_dict"):
            return 0
        own = self.clap.state_dict() if hasattr(self.clap, "state_dict") else {}
        sub = {k: v for k, v in state.items() if k in own}    # a shape mismatch raises, as in torch's strict=False
        if sub:
            self.clap.load_state_dict(sub, strict=False)
            for p in self._from_clap:
                self.table.pop(p, None)
            self._from_clap.clear()
        return len(sub)

    @classmethod
    def synthetic(cls, seed: int = 7) -> "PromptEmbedder":
        t = synthetic_text_table(len(STEMS), seed=seed)
        return cls(table={s: t[i] for i, s in enumerate(STEMS)})

    def _clap_embed(self, prompts: List[str]) -> torch.Tensor:
        if self.clap is None or self.tokenizer is None:
            raise KeyError(f"no embedding for prompts {prompts} and no CLAP model/tokenizer to compute one")
        inputs = self.tokenizer(prompts, padding=True, return_tensors="pt")
        params = getattr(self.clap, "parameters", None)
        dev = next(params()).device if params is not None else "cpu"
        inputs = {k: v.to(dev) for k, v in inputs.items()}
        with torch.no_grad():
            if _is_clap_model(self.clap):
                out = _text_features(self.clap.get_text_features(**inputs))
            else:                                             # ClapTextModelWithProjection (:245-248)
                out = self.clap.forward(**inputs).text_embeds
        if not isinstance(out, torch.Tensor) or out.dim() != 2 or out.shape[0] != len(prompts):
            raise ValueError(f"CLAP returned {type(out).__name__} {tuple(getattr(out, 'shape', ()))}, expected "
                             f"({len(prompts)}, {TEXT_DIM})")
        return out.float().cpu()

    def rows(self, text: Union[str, List[str]], batch: int) -> torch.Tensor:
        """(batch, 512) f32 CPU tensor for the reference's `text` argument (str broadcast or list of B)."""
        prompts = [text] * batch if isinstance(text, str) else list(text)
        if len(prompts) != batch:
            raise ValueError(f"{len(prompts)} prompts for a batch of {batch}")
        missing = sorted({p for p in prompts if p not in self.table})
        if missing:
            emb = self._clap_embed(missing)
            for p, e in zip(missing, emb):
                self.table[p] = e
                self._from_clap.add(p)
        out = torch.stack([self.table[p] for p in prompts])
        if out.shape != (batch, TEXT_DIM):
            raise ValueError(f"prompt embeddings must be {TEXT_DIM}-d (text_dim, config.yaml:16), got "
                             f"{tuple(out.shape[1:])}")
        return out


TEXT_DIM = 512


def _is_clap_model(m) -> bool:
    """`isinstance(self.clap, ClapModel)` of ATHTDemucs_v2.py:241 (by class name when transformers is absent)."""
    try:
        from transformers import ClapModel
        if isinstance(m, ClapModel):
            return True
    except ImportError:
        pass
    return any(c.__name__ == "ClapModel" for c in type(m).__mro__)


def _text_features(out) -> torch.Tensor:
    """`ClapModel.get_text_features` result -> (P, 512) projected, L2-normalised text features.  transformers 4.x
    (the reference's pin, requirements.txt:14) returns that tensor directly; transformers >= 5 returns a
    BaseModelOutputWithPooling whose `pooler_output` holds it (its `last_hidden_state` is the 768-d RoBERTa
    output, not an embedding)."""
    if isinstance(out, torch.Tensor):
        return out
    pooled = getattr(out, "pooler_output", None)
    if isinstance(pooled, torch.Tensor):
        return pooled
    emb = getattr(out, "text_embeds", None)
    if isinstance(emb, torch.Tensor):
        return emb
    raise TypeError(f"unrecognised get_text_features output {type(out).__name__}")
