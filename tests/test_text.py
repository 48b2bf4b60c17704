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


def _patch_from_pretrained(monkeypatch, clap, seen):
    """ClapModel / AutoTokenizer.from_pretrained replaced by offline stand-ins (the HF cache has no CLAP here);
    records the names and flags the library asked for."""
    from transformers import AutoTokenizer, ClapModel

    def clap_fp(name, **kw):
        seen.append(("clap", name, kw))
        return clap

    def tok_fp(name, **kw):
        seen.append(("tok", name, kw))
        return FakeTokenizer()

    monkeypatch.setattr(ClapModel, "from_pretrained", staticmethod(clap_fp))
    monkeypatch.setattr(AutoTokenizer, "from_pretrained", staticmethod(tok_fp))


def test_test_inference_default_clap_reaches_window_loop(tmp_path, monkeypatch, state_dict):
    """the reference's own call `test_inference(checkpoint_path, data_dir)` (no keyword arguments)
    builds CLAP + tokenizer like `test_inference.py:26-28` (here from the local cache: local_files_only=True),
    loads the checkpoint's `clap.*` keys into it (`:34-35`) and embeds the stem prompts through
    `get_text_features` (`ATHTDemucs_v2.py:241-244`).  The device parts (forward, OLA, sdr) are stubbed on this
    CPU-only host; the GPU twin is tests/test_gpu_track.py::test_test_inference_default_clap."""
    import numpy as np
    import athd.inference as inf
    from athd.model import AudioTextHTDemucs
    from athd.musdb import HQ_FILES, write_wav
    from athd.weights import STEMS

    clap = _clap_model()
    trained = _clap_model()
    with torch.no_grad():                               # the checkpoint's CLAP differs from the "pretrained" one
        trained.text_projection.linear1.weight.mul_(-2.0)
    seen = []
    _patch_from_pretrained(monkeypatch, clap, seen)
    sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}
    sd.update({"clap." + k: v.clone() for k, v in trained.state_dict().items()})
    ckpt = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": sd, "epoch": 1}, ckpt)
    L = 300000
    d = tmp_path / "quick_train" / "A - B"
    d.mkdir(parents=True)
    rng = np.random.default_rng(0)
    for f in HQ_FILES:
        write_wav(d / f"{f}.wav", (0.1 * rng.standard_normal((L, 2))).astype(np.float32), 44100, "FLOAT")

    calls = []

    def fake_to(self, device):                          # no HIP device here: keep the model on the host
        self.device = torch.device("cpu")
        return self

    def fake_forward_prompts(self, wav, prompts, out=None):
        calls.append((tuple(wav.shape), list(prompts), self.embedder.rows(list(prompts), len(prompts)).clone()))
        o = torch.zeros((wav.shape[0], len(prompts), 2, wav.shape[2]))
        if out is not None:
            out.copy_(o)
            return out
        return o

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(AudioTextHTDemucs, "to", fake_to)
    monkeypatch.setattr(AudioTextHTDemucs, "forward_prompts", fake_forward_prompts)
    monkeypatch.setattr(inf, "overlap_add", lambda win, length, *a, **k: torch.zeros((win.shape[1], 2, length)))
    monkeypatch.setattr(inf, "sdr_loss", lambda e, t: torch.tensor(1.5))
    monkeypatch.chdir(tmp_path)

    scores = inf.test_inference(str(ckpt), str(tmp_path / "quick_train"))

    assert [(k, n, kw.get("local_files_only")) for k, n, kw in seen] == [
        ("clap", "laion/clap-htsat-unfused", True), ("tok", "laion/clap-htsat-unfused", True)]
    assert scores == {s: -1.5 for s in STEMS}
    assert calls and all(p == list(STEMS) for _, p, _ in calls)
    assert [c[0] for c in calls] == [(1, 2, 264600), (1, 2, 300000 - 260190)]   # a full window, the tail
    # the rows the window loop saw are the get_text_features rows of the CHECKPOINT's CLAP weights
    with torch.no_grad():
        inp = FakeTokenizer()(list(STEMS))
        want = F.normalize(trained.text_projection(trained.text_model(**inp).pooler_output), dim=-1)
    for _, _, rows in calls:
        assert torch.allclose(rows, want, atol=1e-6)
    assert (tmp_path / "results" / "A__B" / "extracted_vocals.wav").exists()


def test_load_model_without_cached_clap_names_the_alternative(tmp_path, monkeypatch, state_dict):
    import numpy as np
    from transformers import ClapModel
    from athd.inference import load_model

    def missing(name, **kw):
        raise OSError(f"We couldn't connect to 'https://huggingface.co' to load the files of {name}")

    monkeypatch.setattr(ClapModel, "from_pretrained", staticmethod(missing))
    ckpt = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}}, ckpt)
    with pytest.raises(RuntimeError, match="laion/clap-htsat-unfused.*text_table="):
        load_model(str(ckpt), "cuda")


def test_checkpoint_clap_keys_invalidate_cached_embeddings():
    from athd.model import AudioTextHTDemucs
    clap = _clap_model()
    m = AudioTextHTDemucs(None, clap, FakeTokenizer(), dtype="f32")
    before = m.embedder.rows("vocals", 1).clone()
    new = {"clap." + k: (-v if k.startswith("text_projection") else v) for k, v in clap.state_dict().items()}
    missing, unexpected = m.load_state_dict(new)
    assert not any(k.startswith("clap.") for k in unexpected)
    after = m.embedder.rows("vocals", 1)
    assert not torch.allclose(before, after)
