"""Phase timing of fenc_row0_kernel from in-kernel s_memtime stamps (measurement build: ATHD_FR_STAMP, see
tools/build notes).  Runs the bench configuration's forward twice with ATHD_LIB = that build and prints, per phase,
the mean / median cycles over all workgroups, plus the launch span."""
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

PH = ["gather+xin", "conv+gelu", "dc0 conv3", "dc0 sum1", "dc0 gelu+gram+sum2", "dc0 apply", "dc1 conv3", "dc1 sum1",
      "dc1 gelu+gram+sum2", "dc1 apply", "rewrite", "store"]


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
    blocks = 64 * 512
    buf = np.zeros((blocks, 16), dtype=np.uint64)
    rc = lib.athd_fr_stamps(buf.ctypes.data_as(ctypes.c_void_p), blocks)
    assert rc == 0, rc
    # level 1 (fenc_row_kernel<48, 96>, 64 x 128 rows) runs after level 0 and overwrites blocks 0 .. 8191
    lvl = int(os.environ.get("FR_LEVEL", "0"))
    buf = buf[8192:] if lvl == 0 else buf[:8192]
    print(f"level {lvl}")
    st = buf[:, :13].astype(np.int64)
    ok = (st[:, 12] > st[:, 0]) & (st[:, 0] > 0)
    st = st[ok]
    d = np.diff(st, axis=1)
    print(f"workgroups {len(st)}, launch span {(st[:, 12].max() - st[:, 0].min())} cycles, per-workgroup total "
          f"mean {np.mean(st[:, 12] - st[:, 0]):.0f} median {np.median(st[:, 12] - st[:, 0]):.0f}")
    for k, name in enumerate(PH):
        print(f"  {name:22s} mean {d[:, k].mean():8.0f}  median {np.median(d[:, k]):8.0f}  p90 {np.percentile(d[:, k], 90):8.0f}")


if __name__ == "__main__":
    main()
