"""MUSDB18 tracks and the dataset segment index, feeding the sharded runner (athd/dist.py).

Mirrors `src/dataloader.py`:
  * `STEM_PROMPTS`, `PROMPT_TO_STEM`, `STEM_NAME_TO_INDEX`   <- `:21-34`
  * `segment_index`                                          <- the index map of `MusDBStemDataset.__init__`
                                                                (`:60-72`): (file_idx, stem_idx, segment_idx) for
                                                                every stem and ceil(total / segment) segments
  * `extract_segment`                                        <- `_extract_segment` (`:104-121`), deterministic
                                                                mode: [seg * S, (seg + 1) * S), the last one
                                                                zero-padded
  * `MusDBTracks.load_stems`                                 <- `_load_stems` (`:79-84`): (5, T, 2) =
                                                                [mixture, drums, bass, other, vocals]
The reference decodes `.stem.mp4` with stempeg/ffmpeg (`:79-84`, `benchmark.py:591-615`); neither is installed
here, so tracks are read from the decoded forms: a MUSDB18-HQ directory per track (`mixture.wav drums.wav bass.wav
other.wav vocals.wav`), or one `<name>.stem.npy` array (5, T, 2).  `.stem.mp4` is used only if stempeg imports.
The WAV reader/writer is plain RIFF (PCM 16/24/32-bit and IEEE float 32), numpy only.
"""
from __future__ import annotations

import math
import struct
from pathlib import Path
from typing import Dict, Iterator, List, Sequence, Tuple

import numpy as np
import torch

STEM_PROMPTS: Dict[str, List[str]] = {
    "drums": ["drums", "drum kit", "percussion", "the drums"],
    "bass": ["bass", "bass guitar", "the bass", "bass line"],
    "other": ["other instruments", "accompaniment", "instruments"],
    "vocals": ["vocals", "voice", "singing", "the vocals"],
}
PROMPT_TO_STEM: Dict[str, str] = {p: s for s, ps in STEM_PROMPTS.items() for p in ps}
STEM_NAME_TO_INDEX = {"drums": 0, "bass": 1, "other": 2, "vocals": 3}
STEM_NAMES = ["drums", "bass", "other", "vocals"]
HQ_FILES = ["mixture", "drums", "bass", "other", "vocals"]


# ----------------------------------------------------------------------------------------------------- WAV I/O
def read_wav(path) -> Tuple[np.ndarray, int]:
    """RIFF/WAVE -> (frames, channels) float32 in [-1, 1) for PCM (x / 2^(bits-1)), as stored for IEEE float."""
    data = Path(path).read_bytes()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, rate, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:           # WAVE_FORMAT_EXTENSIBLE: sub-format's first 2 bytes
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, rate, bits)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, rate, bits = fmt
    if tag == 3 and bits == 32:
        x = np.frombuffer(pcm, dtype="<f4").astype(np.float32)
    elif tag == 1 and bits == 16:
        x = np.frombuffer(pcm, dtype="<i2").astype(np.float32) / 32768.0
    elif tag == 1 and bits == 32:
        x = (np.frombuffer(pcm, dtype="<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    elif tag == 1 and bits == 24:
        b = np.frombuffer(pcm[:len(pcm) // 3 * 3], dtype=np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = (v / 8388608.0).astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported WAV format tag {tag} / {bits} bits")
    return x[:len(x) // ch * ch].reshape(-1, ch), rate


def wav_info(path) -> Tuple[int, int, int]:
    """(frames, channels, sample rate) of a RIFF/WAVE file from its chunk headers only (no sample data read)."""
    with open(path, "rb") as f:
        head = f.read(12)
        if head[:4] != b"RIFF" or head[8:12] != b"WAVE":
            raise ValueError(f"{path}: not a RIFF/WAVE file")
        ch = rate = align = None
        while True:
            h = f.read(8)
            if len(h) < 8:
                raise ValueError(f"{path}: missing fmt or data chunk")
            cid, size = h[:4], struct.unpack("<I", h[4:8])[0]
            if cid == b"fmt ":
                body = f.read(size)
                _, ch, rate, _, align, _ = struct.unpack("<HHIIHH", body[:16])
                f.seek(size & 1, 1)
            elif cid == b"data":
                if align is None:
                    raise ValueError(f"{path}: data chunk before fmt chunk")
                return size // align, ch, rate
            else:
                f.seek(size + (size & 1), 1)


def write_wav(path, audio: np.ndarray, sample_rate: int = 44100, subtype: str = "PCM_16") -> None:
    """(frames, channels) or (channels, frames) with channels <= 8 -> WAV.  PCM_16 (soundfile's default for WAV,
    as test_inference.py:157-175 writes) scales by 32767 and clips; FLOAT writes the values."""
    a = np.asarray(audio, dtype=np.float32)
    if a.ndim == 1:
        a = a[:, None]
    if a.shape[0] <= 8 and a.shape[1] > 8:
        a = a.T
    ch = a.shape[1]
    if subtype == "PCM_16":
        body = np.clip(np.rint(a * 32767.0), -32768, 32767).astype("<i2").tobytes()
        tag, bits = 1, 16
    elif subtype == "FLOAT":
        body = a.astype("<f4").tobytes()
        tag, bits = 3, 32
    else:
        raise ValueError(f"unsupported subtype {subtype}")
    fmt = struct.pack("<HHIIHH", tag, ch, sample_rate, sample_rate * ch * bits // 8, ch * bits // 8, bits)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(body)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt)) + fmt)
        f.write(b"data" + struct.pack("<I", len(body)) + body)


# ----------------------------------------------------------------------------------------------- dataset
def num_segments(total_samples: int, segment_samples: int) -> int:
    """`math.ceil(total_samples / segment_samples)` (dataloader.py:67)."""
    return math.ceil(total_samples / segment_samples)


def segment_index(track_lengths: Sequence[int], segment_samples: int,
                  n_stems: int = 4) -> List[Tuple[int, int, int]]:
    """The reference's index map (dataloader.py:61-72): for each file, each stem, each segment."""
    out = []
    for fi, n in enumerate(track_lengths):
        for si in range(n_stems):
            for seg in range(num_segments(n, segment_samples)):
                out.append((fi, si, seg))
    return out


def extract_segment(stems: np.ndarray, seg_idx: int, segment_samples: int) -> np.ndarray:
    """`_extract_segment` with random_segments=False (dataloader.py:104-121): stems (S, T, C) -> (S, seg, C)."""
    start = seg_idx * segment_samples
    end = start + segment_samples
    if end <= stems.shape[1]:
        return stems[:, start:end, :]
    seg = stems[:, start:, :]
    return np.pad(seg, ((0, 0), (0, end - stems.shape[1]), (0, 0)), mode="constant")


class MusDBTracks:
    """Tracks of one MUSDB18 split directory (`root/*.stem.mp4` in the reference; here the decoded forms)."""

    def __init__(self, root, sample_rate: int = 44100):
        self.root = Path(root)
        self.sample_rate = sample_rate
        hq = sorted(p for p in self.root.iterdir() if p.is_dir() and (p / "mixture.wav").exists())
        npy = sorted(self.root.glob("*.stem.npy"))
        mp4 = sorted(self.root.glob("*.stem.mp4"))
        self.files: List[Path] = hq + npy
        if mp4:
            try:
                import stempeg  # noqa: F401
                self.files += mp4
            except ImportError:
                pass
        if not self.files:
            raise ValueError(f"no MUSDB18 tracks (HQ wav directories, *.stem.npy or decodable *.stem.mp4) in {root}")

    def __len__(self) -> int:
        return len(self.files)

    def name(self, i: int) -> str:
        p = self.files[i]
        return p.name if p.is_dir() else p.name.replace(".stem.npy", "").replace(".stem.mp4", "")

    def load_stems(self, i: int) -> np.ndarray:
        """(5, T, 2) float32 = [mixture, drums, bass, other, vocals] (dataloader.py:79-84)."""
        p = self.files[i]
        if p.is_dir():
            parts = []
            for f in HQ_FILES:
                x, rate = read_wav(p / f"{f}.wav")
                if rate != self.sample_rate:
                    raise ValueError(f"{p / f}.wav: {rate} Hz, expected {self.sample_rate}")
                parts.append(x)
            n = min(x.shape[0] for x in parts)
            st = np.stack([x[:n] for x in parts])
        elif p.suffix == ".npy":
            st = np.load(p, allow_pickle=False)
        else:
            import stempeg
            st, rate = stempeg.read_stems(str(p))
        st = np.asarray(st, dtype=np.float32)
        if st.ndim != 3 or st.shape[0] != 5:
            raise ValueError(f"{p}: expected (5, T, C) stems, got {st.shape}")
        if st.shape[2] == 1:                                   # ensure stereo (dataloader.py:155-158)
            st = np.repeat(st, 2, axis=2)
        return st

    def track(self, i: int) -> Tuple[str, torch.Tensor, Dict[str, torch.Tensor]]:
        """(name, mixture (2, T), {stem: (2, T)}) in benchmark.load_track_stems' form (benchmark.py:591-615)."""
        st = torch.from_numpy(self.load_stems(i)).permute(0, 2, 1).contiguous()
        return self.name(i), st[0], {s: st[j + 1] for j, s in enumerate(STEM_NAMES)}

    def tracks(self) -> Iterator[Tuple[str, torch.Tensor, Dict[str, torch.Tensor]]]:
        for i in range(len(self)):
            yield self.track(i)

    def length(self, i: int) -> int:
        """Samples of track i as load_stems returns it, read from the file headers (HQ: the shortest of the five
        WAVs; .stem.npy: memory-mapped shape)."""
        p = self.files[i]
        if p.is_dir():
            return min(wav_info(p / f"{f}.wav")[0] for f in HQ_FILES)
        if p.suffix == ".npy":
            return int(np.load(p, mmap_mode="r", allow_pickle=False).shape[1])
        return self.load_stems(i).shape[1]

    def lengths(self) -> List[int]:
        return [self.length(i) for i in range(len(self))]

    def mixture(self, i: int) -> torch.Tensor:
        """(2, T) float32 mixture of track i (the first row of load_stems) without decoding the other stems when
        the storage allows it."""
        p = self.files[i]
        if p.is_dir():
            x, rate = read_wav(p / "mixture.wav")
            if rate != self.sample_rate:
                raise ValueError(f"{p}/mixture.wav: {rate} Hz, expected {self.sample_rate}")
            x = x[:self.length(i)]
            if x.shape[1] == 1:
                x = np.repeat(x, 2, axis=1)
            return torch.from_numpy(np.ascontiguousarray(x.T, dtype=np.float32))
        return torch.from_numpy(self.load_stems(i)[0].T.copy())

    def mixture_segments(self, segment_samples: int) -> Tuple[torch.Tensor, List[Tuple[int, int]]]:
        """Every (track, segment) mixture of the split as (N, 2, segment) plus its (file_idx, segment_idx) list:
        the units of the sharded runner (one forward_prompts per segment serves all 4 stems of the index map)."""
        segs, keys = [], []
        for fi in range(len(self)):
            st = self.load_stems(fi)
            for seg in range(num_segments(st.shape[1], segment_samples)):
                segs.append(extract_segment(st[:1], seg, segment_samples)[0].T)
                keys.append((fi, seg))
        return torch.from_numpy(np.stack(segs).astype(np.float32)), keys
