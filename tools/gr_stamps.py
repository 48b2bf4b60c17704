"""Phase timing of fdec1_gram_kernel from in-kernel s_memtime stamps (measurement build: ATHD_GR_STAMP, e.g.
`make -C audio-to-sheet-music_amd/csrc EXTRA=-DATHD_GR_STAMP OUT=$PWD/ablibs/libathd_grstamp.so OBJDIR=/tmp/obj_gr`).
Runs the bench configuration's forward with ATHD_LIB = that build and prints the cycles per tile of each phase."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-to-sheet-music_amd"))

from athd.model import AudioTextHTDemucs  # noqa: E402
from athd.synth import synthetic_batch  # noqa: E402
from athd.weights import STEMS, synthetic_state_dict, synthetic_text_table  # noqa: E402

PH = ["4-tap stores + flush + Z MFMA", "barrier 1", "ZT/Zs stores + barrier 2", "Zs prefetch", "Gram MFMA"]


def main():
    table = synthetic_text_table(4, seed=7)
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: table[i] for i, s in enumerate(STEMS)}, decode_items=256)
    m.load_state_dict(synthetic_state_dict(seed=0))
    m = m.to("cuda").eval()
    wav = torch.as_tensor(synthetic_batch(64, 264600, seed0=1000)).cuda()
    for _ in range(2):
        m.forward_prompts(wav, STEMS)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["ATHD_LIB"])
    buf = np.zeros((1024, 8, 8), dtype=np.uint64)
    assert lib.athd_gr_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    st = buf[buf[:, 0, 7] == 1].astype(np.int64)
    nt = st[:, :, 5]
    print(f"blocks {len(st)}, tiles per block {nt[:, 0].mean():.1f}, span per tile {(st[:, :, 6] / nt).mean():.0f}")
    for k, name in enumerate(PH):
        v = st[:, :, k] / nt
        print(f"  {name:26s} per tile mean {v.mean():7.0f}  waves 0..7: " + " ".join(f"{v[:, w].mean():6.0f}" for w in range(8)))


if __name__ == "__main__":
    main()
