"""Tooling: is the bf16 forward (bench shape, 4 segments x 4 prompts) bit-identical under two environment settings?
usage: python tools/r6/same_env.py "ENV=A" "ENV=B" (each applied to a fresh subprocess)"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "audio-to-sheet-music_amd"))


def run(path):
    import torch
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS, synthetic_state_dict, synthetic_text_table
    t = synthetic_text_table(4, seed=7)
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: t[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(synthetic_state_dict(seed=0))
    m = m.to("cuda").eval()
    wav = torch.as_tensor(synthetic_batch(4, 264600, seed0=57)).cuda()
    np.save(path, m.forward_prompts(wav, list(STEMS)).cpu().numpy())


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
        sys.exit(0)
    outs = []
    for k, e in enumerate(sys.argv[1:3]):
        env = dict(os.environ)
        for kv in e.split():
            a, b = kv.split("=", 1)
            env[a] = b
        p = f"/tmp/same_env_{k}.npy"
        subprocess.check_call([sys.executable, __file__, "run", p], env=env)
        outs.append(np.load(p))
    a, b = outs[0].astype(np.float64), outs[1].astype(np.float64)
    sdr = 10 * np.log10(np.sum(a ** 2) / max(np.sum((a - b) ** 2), 1e-300))
    print(sys.argv[1], "vs", sys.argv[2], ":", int((outs[0] != outs[1]).sum()), "differing of", outs[0].size,
          f"SDR {sdr:.1f} dB")
