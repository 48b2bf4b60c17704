"""Prompt -> embedding (athd/text.py) against both branches of `_get_clap_embeddings` (ATHTDemucs_v2.py:238-248),
with tiny randomly initialised CLAP text towers built offline from configs (no pretrained weights exist here).

  * ClapModel: `get_text_features` = L2-normalised `text_projection(text_model(...).pooler_output)`.  The reference
    pins transformers 4.51.1, where that call returns the tensor; the installed 5.x returns a ModelOutput whose
    `pooler_output` holds it - both must give the same (P, 512) rows.
  * ClapTextModelWithProjection: `forward(...).text_embeds` (un-normalised).
"""
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")

TEXT_CFG = dict(vocab_size=64, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64,
                max_position_embeddings=40, projection_dim=512)


class FakeTokenizer:
    """RoBERTa-shaped: <s>=0, </s>=2, pad=1, one id per word; padding=True pads to the longest prompt."""

    def __call__(self, prompts, padding=True, return_tensors="pt"):
        assert padding is True and return_tensors == "pt"
        seqs = [[0] + [3 + (sum(map(ord, w)) % 60) for w in p.split()] + [2] for p in prompts]
        n = max(map(len, seqs))
        ids = torch.tensor([s + [1] * (n - len(s)) for s in seqs])
        return {"input_ids": ids, "attention_mask": (ids != 1).long()}


def _clap_model():
    from transformers import ClapConfig, ClapModel
    torch.manual_seed(0)
    audio = dict(hidden_size=32, depths=[1, 1], num_attention_heads=[2, 2], patch_embeds_hidden_size=16,
                 window_size=4, spec_size=64, num_mel_bins=16, projection_dim=512, patch_stride=[4, 4], patch_size=4)
    return ClapModel(ClapConfig(text_config=TEXT_CFG, audio_config=audio, projection_dim=512)).eval()


def test_clap_model_branch_uses_projected_normalised_features():
    from athd.text import PromptEmbedder
    m, tok = _clap_model(), FakeTokenizer()
    prompts = ["drums", "bass", "other instruments", "vocals"]
    got = PromptEmbedder(clap=m, tokenizer=tok).rows(prompts, 4)
    with torch.no_grad():
        inp = tok(sorted(set(prompts)))
        pooled = m.text_model(**inp).pooler_output
        ref = F.normalize(m.text_projection(pooled), dim=-1)            # transformers 4.51 get_text_features
    ref = dict(zip(sorted(set(prompts)), ref))
    assert got.shape == (4, 512) and got.dtype == torch.float32
    for i, p in enumerate(prompts):
        assert torch.allclose(got[i], ref[p], atol=1e-6), p
    assert torch.allclose(got.norm(dim=-1), torch.ones(4), atol=1e-5)


def test_text_model_with_projection_branch():
    from transformers import ClapTextConfig, ClapTextModelWithProjection
    from athd.text import PromptEmbedder
    torch.manual_seed(1)
    m, tok = ClapTextModelWithProjection(ClapTextConfig(**TEXT_CFG)).eval(), FakeTokenizer()
    got = PromptEmbedder(clap=m, tokenizer=tok).rows("vocals", 3)        # bare str broadcast over the batch
    with torch.no_grad():
        ref = m(**tok(["vocals"])).text_embeds[0]
    assert got.shape == (3, 512)
    for r in got:
        assert torch.allclose(r, ref, atol=1e-6)


def test_embeddings_are_cached_per_prompt():
    from athd.text import PromptEmbedder

    class Counting(FakeTokenizer):
        calls = 0

        def __call__(self, prompts, **kw):
            Counting.calls += 1
            return super().__call__(prompts, **kw)

    e = PromptEmbedder(clap=_clap_model(), tokenizer=Counting())
    a = e.rows(["drums", "bass"], 2)
    b = e.rows(["bass", "drums", "drums"], 3)
    assert Counting.calls == 1
    assert torch.equal(a[0], b[1]) and torch.equal(a[1], b[0])


def test_bad_embeddings_are_rejected():
    import numpy as np
    from athd.text import PromptEmbedder, _text_features
    with pytest.raises(ValueError):
        PromptEmbedder(table={"vocals": np.zeros(768, np.float32)}).rows("vocals", 1)
    with pytest.raises(KeyError):
        PromptEmbedder(table={"vocals": np.zeros(512, np.float32)}).rows("drums", 1)
    with pytest.raises(ValueError):
        PromptEmbedder(table={}).rows(["a", "b"], 3)
    with pytest.raises(TypeError):
        _text_features(object())
