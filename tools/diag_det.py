"""Diagnostics (tooling, not a test): bf16 forward run-to-run determinism and agreement between kernel variants
selected by environment switches (each variant in its own process: the switches are read once)."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-to-sheet-music_amd"))


def run(out):
    import torch
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS, synthetic_state_dict, synthetic_text_table
    t = synthetic_text_table(4, seed=7)
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: t[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(synthetic_state_dict(seed=0))
    m = m.to("cuda").eval()
    wav = torch.as_tensor(synthetic_batch(2, 264600, seed0=31)).cuda()
    a = m.forward_prompts(wav, list(STEMS)).cpu().numpy()
    b = m.forward_prompts(wav, list(STEMS)).cpu().numpy()
    np.save(out, np.stack([a, b]))


def sdr(r, o):
    return 10 * np.log10(np.sum(r.astype(np.float64) ** 2) / max(np.sum((r.astype(np.float64) - o) ** 2), 1e-300))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        run(sys.argv[2])
        sys.exit(0)
    res = {}
    # arguments: KEY=VALUE (an environment variant) or a library path (an ATHD_LIB variant)
    variants = [("new", {})]
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=", 1)
            variants.append((a, {k: v}))
        else:
            variants.append((os.path.basename(a), {"ATHD_LIB": os.path.realpath(a)}))
    for name, env in variants:
        f = f"/tmp/diag_{name}.npy"
        subprocess.check_call([sys.executable, __file__, "run", f], env={**os.environ, **env})
        res[name] = np.load(f)
        print(f"{name}: run-to-run SDR {sdr(res[name][0], res[name][1]):.1f} dB", flush=True)
    for name, _ in variants[1:]:
        print(f"{name} vs new: {sdr(res['new'][0], res[name][0]):.1f} dB", flush=True)
