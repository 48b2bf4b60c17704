"""`AudioTextHTDemucs` - drop-in for the reference model class (`ATHTDemucs_v2.py:141-326`) on MI355X.

Same construction and call surface that `test_inference.load_model` / `benchmark.OurModel` use
(`test_inference.py:21-40`, `benchmark.py:125-153,175`):

    model = AudioTextHTDemucs(htdemucs, clap, tokenizer)      # htdemucs: nn.Module with demucs key names, or None
    model.load_state_dict(checkpoint["model_state_dict"], strict=False)
    model = model.to("cuda").eval()
    out = model(wav, "vocals")  /  model(wav, ["drums", "bass"])  # (B,2,T) f32 cuda -> (B,2,T) f32 cuda

`forward` runs entirely in libathd.so (HIP kernels on the current torch stream).  PyTorch only provides device
memory and the stream.  Additionally `forward_prompts(wav, prompts)` encodes once and decodes once per prompt.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Union

import numpy as np
import torch

from .text import PromptEmbedder
from .weights import hot_path_spec


def _to_numpy(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        return v.detach().to("cpu", torch.float32).numpy()
    return np.asarray(v, dtype=np.float32)


class AudioTextHTDemucs:
    def __init__(self, htdemucs_model=None, clap_encoder=None, clap_tokenizer=None, model_dim: int = 384,
                 text_dim: int = 512, num_heads: int = 8, sample_rate: int = 44100, segment: float = 7.8,
                 dtype: str = "bf16", text_table: Optional[Dict[str, np.ndarray]] = None,
                 decode_items: Optional[int] = None):
        if (model_dim, text_dim, num_heads) != (384, 512, 8):
            raise ValueError("the native path is built for model_dim=384, text_dim=512, num_heads=8 "
                             "(config.yaml:15-17)")
        if dtype not in ("bf16", "f32"):
            raise ValueError("dtype must be 'bf16' or 'f32'")
        self.sample_rate = sample_rate
        self.segment = segment
        self.dtype = dtype
        # (segment, prompt) items per decode chunk (athd_set_decode_items; None = the library default, 64).  256 puts
        # a 64-segment x 4-prompt batch in one chunk (≈49 GB at round 3: athd_workspace_bytes, reported by bench.py as workspace_gb).
        self.decode_items = decode_items
        self.embedder = PromptEmbedder(clap_encoder, clap_tokenizer, text_table)
        self._weights: Dict[str, np.ndarray] = {}
        if htdemucs_model is not None:
            for k, v in htdemucs_model.state_dict().items():
                self._weights["htdemucs." + k] = _to_numpy(v)
        self.device: Optional[torch.device] = None
        self._ctx = None
        self._ws: Optional[torch.Tensor] = None
        self.training = False

    # ------------------------------------------------------------------ nn.Module-like surface
    def load_state_dict(self, state_dict, strict: bool = False):
        """Reference key names; like `load_state_dict(strict=False)` unknown keys (htdemucs.decoder.*, ...) are
        ignored.  `clap.*` keys are loaded into the attached CLAP model (non-strictly, as the reference's submodule)
        when there is one, and ignored otherwise.  Returns (missing_keys, unexpected_keys) restricted to the hot-path
        contract."""
        needed = {k for k, _, _ in hot_path_spec()}
        unexpected = []
        clap_state = {}
        for k, v in state_dict.items():
            if k.startswith("module."):
                k = k[len("module."):]        # DataParallel prefix (benchmark.py:398-404)
            if k in needed:
                self._weights[k] = _to_numpy(v)
            else:
                if k.startswith("clap."):     # the reference's self.clap submodule (ATHTDemucs_v2.py:165)
                    clap_state[k[len("clap."):]] = v
                unexpected.append(k)
        if self.embedder.load_clap_state(clap_state):
            loaded = set(self.embedder.clap.state_dict())
            unexpected = [k for k in unexpected
                          if not (k.startswith("clap.") and k[len("clap."):] in loaded)]
        missing = sorted(needed - set(self._weights))
        if strict and (missing or unexpected):
            raise RuntimeError(f"missing {missing[:5]}..., unexpected {unexpected[:5]}...")
        self._ctx = None
        return missing, unexpected

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("athd runs on a HIP device only (there is no CPU path)")
        if device.index is None:     # torch's current device (0 until torch.cuda is initialised; no init here)
            device = torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_initialized() else 0)
        if self.device != device:
            self._ctx = None
        self.device = device
        return self

    def cuda(self, index: int = 0):
        return self.to(torch.device("cuda", index))

    def eval(self):
        self.training = False
        return self

    def train(self, mode: bool = True):
        if mode:
            raise RuntimeError("athd is inference-only")
        return self

    def parameters(self):
        return iter(())

    # ------------------------------------------------------------------ native context
    def _ensure_ctx(self):
        if self._ctx is not None:
            return self._ctx
        from . import native   # raises if libathd.so is missing
        if self.device is None:
            self.to("cuda")
        ctx = native.Context(self.device.index, native.BF16 if self.dtype == "bf16" else native.F32)
        missing = [k for k in native.required_keys() if k not in self._weights]
        if missing:
            raise RuntimeError(f"{len(missing)} hot-path weights missing, e.g. {missing[:3]}")
        for k in native.required_keys():
            ctx.set_weight(k, self._weights[k])
        ctx.finalize()
        if self.decode_items is not None:
            ctx.set_decode_items(self.decode_items)
        self._ctx = ctx
        return ctx

    def set_decode_items(self, items: Optional[int]):
        self.decode_items = items
        if self._ctx is not None:
            self._ctx.set_decode_items(64 if items is None else items)

    def profile_start(self, kernel: Optional[str] = None):
        """Measurement aid (bench.py): HIP-event timing of one kernel (or all) in the following forwards."""
        self._ensure_ctx().profile_start(kernel)

    def profile_stop(self) -> list:
        return self._ensure_ctx().profile_stop()

    def _workspace(self, nbytes: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < nbytes or self._ws.device != self.device:
            self._ws = None
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self._ws

    def _check_wav(self, wav: torch.Tensor):
        if wav.dim() != 3 or wav.shape[1] != 2:
            raise ValueError(f"expected (B, 2, T) stereo, got {tuple(wav.shape)}")
        if self.device is None:
            self.to(wav.device)
        if wav.device != self.device:
            raise ValueError(f"wav on {wav.device}, model on {self.device}")
        return wav.contiguous().float()

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, wav: torch.Tensor, text: Union[str, List[str]]) -> torch.Tensor:
        """`ATHTDemucs_v2.py:250-326`: (B,2,T) mixture + prompt(s) -> (B,2,T) separated stem."""
        wav = self._check_wav(wav)
        B, _, T = wav.shape
        ctx = self._ensure_ctx()
        emb = self.embedder.rows(text, B).to(self.device).contiguous()
        out = torch.empty_like(wav)
        nbytes = ctx.workspace_bytes(B, T, 1)
        ws = self._workspace(nbytes)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        ctx.forward(wav.data_ptr(), B, T, emb.data_ptr(), out.data_ptr(), ws.data_ptr(), ws.numel(), stream)
        return out

    __call__ = forward

    @torch.no_grad()
    def forward_prompts(self, wav: torch.Tensor, prompts: List[str], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Encode once, decode once per prompt: (B,2,T) -> (B,P,2,T) (written into `out` when given)."""
        wav = self._check_wav(wav)
        B, _, T = wav.shape
        ctx = self._ensure_ctx()
        table = self.embedder.rows(list(prompts), len(prompts)).to(self.device).contiguous()
        P = table.shape[0]
        if out is None:
            out = torch.empty((B, P, 2, T), dtype=torch.float32, device=self.device)
        elif (tuple(out.shape) != (B, P, 2, T) or out.dtype != torch.float32 or out.device != self.device
              or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous float32 {(B, P, 2, T)} tensor on {self.device}")
        nbytes = ctx.workspace_bytes(B, T, P)
        ws = self._workspace(nbytes)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        ctx.forward_prompts(wav.data_ptr(), B, T, table.data_ptr(), P, out.data_ptr(), ws.data_ptr(), ws.numel(),
                            stream)
        return out

    @torch.no_grad()
    def capture_prompts(self, wav: torch.Tensor, prompts: List[str], out: Optional[torch.Tensor] = None,
                        workspace: Optional[torch.Tensor] = None):
        """`forward_prompts` on these exact buffers captured into one HIP graph (torch.cuda.CUDAGraph over the
        library's launches: both branch streams, their event fork / joins and the statistics memset).  Returns
        (graph, out): `graph.replay()` re-runs every kernel of the forward on the same device buffers, so the caller
        refreshes `wav` in place between replays; the prompt rows, the workspace and `out` stay bound to the graph.
        The graph owns its workspace (not the model's cached one), so replays may overlap eager calls on other streams;
        graphs replayed only in order on ONE stream may share a caller-given `workspace` (e.g. ping-pong outputs).
        Memory: without `workspace` every captured graph holds a full `athd_workspace_bytes(B, T, P)` arena (≈ 49 GB
        at B = 64, T = 264600, P = 4), so capturing k graphs costs k arenas.
        `wav` must already be a contiguous float32 (B, 2, T) tensor on the model's device (no copy is captured)."""
        if wav.dtype != torch.float32 or not wav.is_contiguous():
            raise ValueError("capture_prompts needs a contiguous float32 wav (B, 2, T)")
        wav = self._check_wav(wav)
        B, _, T = wav.shape
        ctx = self._ensure_ctx()
        table = self.embedder.rows(list(prompts), len(prompts)).to(self.device).contiguous()
        P = table.shape[0]
        if out is None:
            out = torch.empty((B, P, 2, T), dtype=torch.float32, device=self.device)
        # a workspace of the graph's own: an eager forward on this model (self._ws) may run on another stream while
        # the graph replays, and the two must not share scratch memory
        nbytes = ctx.workspace_bytes(B, T, P)
        if workspace is None:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        elif workspace.dtype != torch.uint8 or workspace.numel() < nbytes or workspace.device != self.device:
            raise ValueError(f"workspace must be a uint8 tensor of >= {nbytes} bytes on {self.device}")
        else:
            ws = workspace
        run = lambda: ctx.forward_prompts(wav.data_ptr(), B, T, table.data_ptr(), P, out.data_ptr(), ws.data_ptr(),
                                          ws.numel(), torch.cuda.current_stream(self.device).cuda_stream)
        run()                                   # eager once: one-time launch-configuration queries happen outside
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        # thread_local: only this thread's calls are checked during capture (a process-group watchdog thread may
        # query its events meanwhile); the library issues all of its HIP calls on this thread
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            run()
        g._athd_keep = (wav, table, out, ws)    # the graph's device pointers stay valid while it lives
        return g, out
