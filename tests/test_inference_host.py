"""Host-side pieces of athd/inference.py and athd/model.py that need no GPU: checkpoint ingestion
(test_inference.py:21-40 semantics with weights_only loading), non-strict state-dict filtering, prompt resolution."""
import numpy as np
import pytest
import torch


def test_load_model_reads_checkpoint(tmp_path, state_dict):
    from athd.inference import load_model
    from athd.weights import hot_path_spec
    sd = {("module." + k if i % 3 == 0 else k): torch.as_tensor(np.asarray(v)) for i, (k, v) in enumerate(state_dict.items())}
    sd["clap.text_model.embeddings.word_embeddings.weight"] = torch.zeros(4, 8)     # ignored (strict=False)
    sd["htdemucs.decoder.0.conv_tr.weight"] = torch.zeros(2, 2)                     # unused by the reference forward
    path = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": sd, "epoch": 7, "optimizer_state_dict": {}}, path)
    m = load_model(str(path), device="cuda", dtype="f32", text_table={"vocals": np.ones(512, np.float32)})
    needed = {k for k, _, _ in hot_path_spec()}
    assert needed <= set(m._weights)
    assert "clap.text_model.embeddings.word_embeddings.weight" not in m._weights
    k0 = next(iter(state_dict))
    np.testing.assert_array_equal(m._weights[k0], np.asarray(state_dict[k0], np.float32))
    assert m.device == torch.device("cuda", 0) and not m.training


def test_load_model_rejects_lone_tokenizer_or_clap(tmp_path):
    """a caller-given tokenizer without a CLAP model (or the reverse) is an error, not silently replaced
    by the cached pair (the reference builds the two together, test_inference.py:26-28)."""
    from athd.inference import load_model
    path = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": {}}, path)
    with pytest.raises(ValueError, match="both clap= and tokenizer="):
        load_model(str(path), device="cuda", tokenizer=object())
    with pytest.raises(ValueError, match="both clap= and tokenizer="):
        load_model(str(path), device="cuda", clap=object())


def test_load_state_dict_reports_missing_and_strict():
    from athd.model import AudioTextHTDemucs
    m = AudioTextHTDemucs(dtype="bf16")
    missing, unexpected = m.load_state_dict({"foo": torch.zeros(1)})
    assert unexpected == ["foo"] and len(missing) > 400
    with pytest.raises(RuntimeError):
        m.load_state_dict({"foo": torch.zeros(1)}, strict=True)


def test_prompt_rows_broadcast_and_list():
    from athd.text import PromptEmbedder
    e = PromptEmbedder.synthetic()
    r1 = e.rows("vocals", 3)
    assert r1.shape == (3, 512) and torch.equal(r1[0], r1[2])
    r2 = e.rows(["drums", "bass"], 2)
    assert not torch.equal(r2[0], r2[1])
    with pytest.raises(ValueError):
        e.rows(["drums"], 2)
    with pytest.raises(KeyError):
        e.rows("piano", 1)          # no table row and no CLAP model to compute one


def test_model_rejects_cpu_device():
    from athd.model import AudioTextHTDemucs
    with pytest.raises(RuntimeError):
        AudioTextHTDemucs().to("cpu")


def test_test_inference_signature_matches_reference():
    """test_inference.py:44-52: same positional parameters and defaults (the build adds keyword-only ones)."""
    import inspect
    from athd.inference import test_inference as ti
    ps = [p for p in inspect.signature(ti).parameters.values() if p.kind == p.POSITIONAL_OR_KEYWORD]
    assert [(p.name, p.default) for p in ps] == [
        ("checkpoint_path", "checkpoints/best_model.pt"), ("data_dir", "data/quick_train"), ("output_dir", "results"),
        ("sample_rate", 44100), ("segment_seconds", 6.0), ("overlap", 0.1), ("device", None)]


@pytest.mark.parametrize("name,want", [("Al James - Schoolboy Facination.stem.mp4", "Al_James__Schoolboy_Facination"),
                                       ("/x/y/Mu's Band - Track-1.stem.npy", "Mus_Band__Track1"),
                                       ("Dr. Who - Theme.stem.mp4", "Dr._Who__Theme")])
def test_cleaned_track_name(name, want):
    """test_inference.py:159-162."""
    from athd.inference import cleaned_track_name
    assert cleaned_track_name(name) == want


def test_main_reads_config_keys(tmp_path, monkeypatch):
    """test_inference.py:208-218: checkpoint_dir/best_model.pt, data.test_dir, wandb.output_dir, sample_rate and
    segment_seconds come from config.yaml (utils.load_config = yaml.safe_load)."""
    import athd.inference as inf
    cfg = tmp_path / "config.yaml"
    cfg.write_text("data:\n  test_dir: /d/test\n  segment_seconds: 6.0\n  sample_rate: 44100\n"
                   "wandb:\n  checkpoint_dir: ck/2025/\n  output_dir: res/2025\n")
    seen = {}
    monkeypatch.setattr(inf, "test_inference", lambda **kw: seen.update(kw) or {"ok": 1})
    assert inf.main(str(cfg)) == {"ok": 1}
    assert seen == {"checkpoint_path": "ck/2025/best_model.pt", "data_dir": "/d/test", "output_dir": "res/2025",
                    "sample_rate": 44100, "segment_seconds": 6.0}
