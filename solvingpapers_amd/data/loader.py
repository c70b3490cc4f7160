"""Python face of the native token loader (csrc/runtime/token_loader.cpp).

``NativeTokenLoader(source, batch, seq, ...)`` produces (x, y) int64 batches from a flat
token stream — an mmap'ed binary file of uint16/int32 ids or an in-memory tensor — with
C++ worker threads filling a prefetch ring (pinned host memory when a GPU is present,
so ``.to(device, non_blocking=True)`` is an async DMA). Batch ``i`` is a pure function
of (seed, rank, i): ``loader(i)`` matches the Trainer's ``train_batch(i)`` interface
and resuming at step ``i`` is ``seek(i)`` — no data-loader state to checkpoint.
"""
from __future__ import annotations

import os
from typing import Optional, Union

import torch

from ..ops import _ext


class NativeTokenLoader:
    def __init__(self, source: Union[str, torch.Tensor], batch_size: int, seq_len: int, seed: int = 0,
                 rank: int = 0, world: int = 1, threads: int = 2, depth: int = 4, device=None,
                 file_dtype: torch.dtype = torch.uint16, sequential: bool = False, pin: Optional[bool] = None):
        _ext.load()
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        if pin is None:
            pin = self.device.type == "cuda"
        if isinstance(source, (str, os.PathLike)):
            elem = {torch.uint16: 2, torch.int32: 4}[file_dtype]
            self._h = torch.classes.spa.TokenLoader(str(source), elem, torch.empty(0, dtype=torch.int32), batch_size,
                                                    seq_len, seed, rank, world, threads, depth, pin, sequential)
        else:
            t = source.detach().cpu().contiguous()
            if t.dtype not in (torch.int16, torch.uint16, torch.int32, torch.int64):
                t = t.to(torch.int32)
            self._h = torch.classes.spa.TokenLoader("", 0, t, batch_size, seq_len, seed, rank, world, threads, depth,
                                                    pin, sequential)
        self.B, self.T = batch_size, seq_len

    def __len__(self):
        return int(self._h.num_tokens())

    def _out(self, t):
        if self.device.type != "cpu":
            t = t.to(self.device, non_blocking=True)
        return t[0], t[1]

    def __call__(self, i: int):
        if self._h.position() != i:
            self._h.seek(i)
        return self._out(self._h.next())

    def __iter__(self):
        while True:
            yield self._out(self._h.next())

    def seek(self, i: int):
        self._h.seek(i)

    def batch_at(self, i: int):
        return self._out(self._h.batch_at(i))


def write_token_file(path: str, tokens: torch.Tensor, dtype: torch.dtype = torch.uint16):
    """Write a flat id stream (the format NativeTokenLoader mmaps)."""
    import numpy as np
    arr = tokens.detach().cpu().numpy().astype(np.uint16 if dtype == torch.uint16 else np.int32)
    tmp = path + ".tmp"
    arr.tofile(tmp)
    os.replace(tmp, path)
