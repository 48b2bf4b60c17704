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


class PromptEmbedder:
    def __init__(self, clap=None, tokenizer=None, table: Optional[Dict[str, np.ndarray]] = None):
        self.clap = clap
        self.tokenizer = tokenizer
        self.table: Dict[str, torch.Tensor] = {}
        if table:
            for k, v in table.items():
                self.table[k] = torch.as_tensor(np.asarray(v, dtype=np.float32)).reshape(-1)

    @classmethod
    def synthetic(cls, seed: int = 7) -> "PromptEmbedder":
        t = synthetic_text_table(len(STEMS), seed=seed)
        return cls(table={s: t[i] for i, s in enumerate(STEMS)})

    def _clap_embed(self, prompts: List[str]) -> torch.Tensor:
        if self.clap is None or self.tokenizer is None:
            raise KeyError(f"no embedding for prompts {prompts} and no CLAP model/tokenizer to compute one")
        inputs = self.tokenizer(prompts, padding=True, return_tensors="pt")
        dev = next(self.clap.parameters()).device if hasattr(self.clap, "parameters") else "cpu"
        inputs = {k: v.to(dev) for k, v in inputs.items()}
        with torch.no_grad():
            cls_name = type(self.clap).__name__
            if cls_name == "ClapModel":
                out = self.clap.get_text_features(**inputs)
                if not isinstance(out, torch.Tensor):       # transformers >= 5 returns a ModelOutput
                    out = getattr(out, "text_embeds", None) or out[0]
            else:
                out = self.clap.forward(**inputs).text_embeds
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
        return torch.stack([self.table[p] for p in prompts])
