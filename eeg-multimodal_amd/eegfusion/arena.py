"""Flat parameter arena: every parameter of the path is a view into ONE fp32 master buffer, with a
matching fp32 gradient buffer and (bf16 mode) a bf16 compute shadow at the same element offsets.

Why: the fused Adam (eegf_adam) updates a whole optimizer group in one launch, the DDP gradient
all-reduce moves one contiguous buffer in a few large buckets, and the BERT Q/K/V weights (and
biases) are laid out back-to-back so the fused QKV projection reads them as one [2304, 768]
matrix with no copy.  Offsets are 64-element (256 B) aligned.
"""
from __future__ import annotations

import weakref
from collections import OrderedDict

import torch

ALIGN = 64
_LIVE: "weakref.WeakSet[ParamArena]" = weakref.WeakSet()


class ParamArena:
    def __init__(self, specs: list[tuple[str, tuple[int, ...]]], device, dp_names=("DP",)):
        # model parameters first (one contiguous optimizer range), DP-group parameters last
        model = [(n, s) for n, s in specs if n not in dp_names]
        dp = [(n, s) for n, s in specs if n in dp_names]
        self.offsets: "OrderedDict[str, tuple[int, tuple[int, ...]]]" = OrderedDict()
        off = 0
        for n, s in model:
            self.offsets[n] = (off, tuple(s))
            off += self._numel(s)
            off = (off + ALIGN - 1) // ALIGN * ALIGN
        self.model_range = (0, off)
        dp_start = off
        for n, s in dp:
            self.offsets[n] = (off, tuple(s))
            off += self._numel(s)
            off = (off + ALIGN - 1) // ALIGN * ALIGN
        self.dp_range = (dp_start, off)
        self.numel = off
        self.device = torch.device(device)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.shadow = None              # bf16 copy (allocated on demand)
        self.shadow_version = -1
        _LIVE.add(self)

    @staticmethod
    def owner(t: torch.Tensor) -> "ParamArena | None":
        """The live arena whose master buffer holds tensor t (a parameter view), if any."""
        p = t.untyped_storage().data_ptr()
        for a in list(_LIVE):
            if a.master.untyped_storage().data_ptr() == p:
                return a
        return None

    def invalidate_shadow(self) -> None:
        """The master was written outside torch's version counter (a raw-pointer optimizer step): the
        bf16 compute shadow is re-cast before the next forward."""
        self.shadow_version = -1

    @staticmethod
    def _numel(s):
        n = 1
        for d in s:
            n *= d
        return n

    def view(self, name: str, buf: torch.Tensor | None = None) -> torch.Tensor:
        off, s = self.offsets[name]
        buf = self.master if buf is None else buf
        return buf[off: off + self._numel(s)].view(s)

    def gview(self, name: str) -> torch.Tensor:
        return self.view(name, self.grad)

    def span(self, first: str, n_params: int, buf: torch.Tensor | None = None) -> torch.Tensor:
        """Contiguous view covering `n_params` consecutive parameters starting at `first`
        (used for the fused Q|K|V weight / bias)."""
        names = list(self.offsets)
        i = names.index(first)
        off0 = self.offsets[first][0]
        last = names[i + n_params - 1]
        off1 = self.offsets[last][0] + self._numel(self.offsets[last][1])
        buf = self.master if buf is None else buf
        return buf[off0:off1]

    def ranges(self, names) -> list[tuple[int, int]]:
        """Coalesced [lo, hi) element ranges covering `names` (gaps of pure alignment padding merge)."""
        spans = sorted((self.offsets[n][0], self.offsets[n][0] + self._numel(self.offsets[n][1])) for n in names)
        out: list[list[int]] = []
        for lo, hi in spans:
            if out and lo - out[-1][1] < ALIGN:
                out[-1][1] = max(out[-1][1], hi)
            else:
                out.append([lo, hi])
        return [(lo, hi) for lo, hi in out]

    def offset(self, name: str) -> int:
        return self.offsets[name][0]

    def to(self, device) -> "ParamArena":
        device = torch.device(device)
        if device != self.device:
            self.master = self.master.to(device)
            self.grad = self.grad.to(device)
            self.shadow = None
            self.shadow_version = -1
            self.device = device
        return self
