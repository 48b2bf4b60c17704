"""Diagnostics (tooling, not a test): run the bf16 forward twice with ATHD_DUMP and report where the encoder level
outputs (saved0..3, bf16) differ between the two runs."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-to-sheet-music_amd"))


def main():
    import torch
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS, synthetic_state_dict, synthetic_text_table
    if len(sys.argv) > 1:
        os.environ["ATHD_LIB"] = os.path.realpath(sys.argv[1])
    t = synthetic_text_table(4, seed=7)
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: t[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(synthetic_state_dict(seed=0))
    m = m.to("cuda").eval()
    # DIAG_B / DIAG_SEED / DIAG_RUNS: batch, synthetic seed, forwards compared against the first
    nb, seed, runs = (int(os.environ.get(k, v)) for k, v in (("DIAG_B", 2), ("DIAG_SEED", 31), ("DIAG_RUNS", 2)))
    wav = torch.as_tensor(synthetic_batch(nb, 264600, seed0=seed)).cuda()
    outs = []
    for k in range(runs):
        d = tempfile.mkdtemp()
        os.environ["ATHD_DUMP"] = d
        y = m.forward_prompts(wav, list(STEMS))
        torch.cuda.synchronize()
        o = {n: np.fromfile(os.path.join(d, n), np.uint8) for n in sorted(os.listdir(d)) if n != "index.txt"}
        o["output"] = y.cpu().numpy().view(np.uint8).ravel()
        outs.append(o)
    del os.environ["ATHD_DUMP"]
    for k in range(1, runs):
        print(f"-- run 0 vs run {k}", flush=True)
        for n in outs[0]:
            a, b = outs[0][n], outs[k][n]
            if (a != b).any() or k == 1:
                print(f"{n}: {int((a != b).sum())} of {a.size} bytes differ", flush=True)
            if n == "stats.raw" and (a != b).any():
                da, db = a.view(np.float64), b.view(np.float64)
                for i in np.nonzero(da != db)[0][:40]:
                    print(f"   stats[{i}]: {da[i]!r} vs {db[i]!r}", flush=True)

if __name__ == "__main__":
    main()
