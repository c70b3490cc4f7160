"""Byte-level BPE tokenizer (the GPT-2 scheme the reference's LLaMA and DeepSeek slices use).

The reference tokenizes with ``tiktoken.get_encoding("gpt2")`` (llama3/LLaMA-jax.ipynb:196,260)
and ``AutoTokenizer.from_pretrained("gpt2")`` (deepseekv3/deepseekv3.ipynb:524-527). Neither is
reachable here (no tiktoken, no network, no HF cache), so this wraps the installed HF
``tokenizers`` package, whose BPE encoder is native code:

* ``BPETokenizer.from_gpt2_files(vocab.json, merges.txt)`` builds the exact GPT-2 encoder from
  the published files, if the user has them (50257 ids, ``<|endoftext|>`` = 50256);
* ``BPETokenizer.train(texts, vocab_size)`` learns a byte-level BPE offline, with the same
  pre-tokenizer and byte alphabet, so every string round-trips;
* ``encode_to_token_file`` streams a corpus into the uint16/int32 file the native
  ``TokenLoader`` (csrc/runtime/token_loader.cpp) memory-maps.
"""
from __future__ import annotations

import json
import os
from typing import Iterable, List, Optional

import numpy as np

EOT = "<|endoftext|>"


def _require():
    try:
        import tokenizers  # noqa: F401
    except ImportError as e:  # pragma: no cover - the image ships it
        raise RuntimeError("the HF 'tokenizers' package is required for BPE tokenization") from e


class BPETokenizer:
    """encode / decode / vocab_size / eot_token, as the reference uses tiktoken's gpt2 encoding."""

    def __init__(self, tok):
        self._tok = tok
        self.eot_token = tok.token_to_id(EOT)

    # ------------------------------------------------------------------ builders
    @staticmethod
    def _byte_level(model):
        from tokenizers import Tokenizer, decoders, pre_tokenizers
        t = Tokenizer(model)
        t.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
        t.decoder = decoders.ByteLevel()
        return t

    @classmethod
    def from_gpt2_files(cls, vocab_json: str, merges_txt: str) -> "BPETokenizer":
        """The GPT-2 encoder from its published vocab.json / merges.txt."""
        _require()
        from tokenizers import models
        t = cls._byte_level(models.BPE.from_file(vocab_json, merges_txt))
        return cls(t)

    @classmethod
    def train(cls, texts: Iterable[str], vocab_size: int = 8192, min_frequency: int = 2) -> "BPETokenizer":
        """Learn a byte-level BPE of ``vocab_size`` ids (256 byte symbols + merges + EOT)."""
        _require()
        from tokenizers import models, pre_tokenizers, trainers
        t = cls._byte_level(models.BPE())
        tr = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=min_frequency, special_tokens=[EOT],
                                 initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
        t.train_from_iterator(texts, trainer=tr)
        return cls(t)

    @classmethod
    def load(cls, path: str) -> "BPETokenizer":
        _require()
        from tokenizers import Tokenizer
        return cls(Tokenizer.from_file(path))

    def save(self, path: str):
        self._tok.save(path)

    # ------------------------------------------------------------------ API
    @property
    def vocab_size(self) -> int:
        return self._tok.get_vocab_size()

    @property
    def n_vocab(self) -> int:  # tiktoken's name
        return self.vocab_size

    def encode(self, s: str) -> List[int]:
        return self._tok.encode(s, add_special_tokens=False).ids

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(texts, add_special_tokens=False)]

    def decode(self, ids) -> str:
        return self._tok.decode([int(i) for i in ids], skip_special_tokens=False)


def encode_to_token_file(tok: BPETokenizer, texts: Iterable[str], path: str, append_eot: bool = True,
                         batch: int = 256) -> int:
    """Tokenize ``texts`` (documents) into a flat id file for ``NativeTokenLoader``: uint16 when
    the vocabulary fits (GPT-2's 50257 does), else int32. Streams in batches; returns the count.
    A JSON sidecar (``path + '.json'``) records dtype, vocab size and token count."""
    dtype = np.uint16 if tok.vocab_size <= 65536 else np.int32
    n = 0
    buf: List[str] = []

    def flush(f):
        nonlocal n
        for ids in tok.encode_batch(buf):
            if append_eot and tok.eot_token is not None:
                ids = ids + [tok.eot_token]
            a = np.asarray(ids, dtype=dtype)
            f.write(a.tobytes())
            n += a.size
        buf.clear()

    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        for t in texts:
            buf.append(t)
            if len(buf) >= batch:
                flush(f)
        if buf:
            flush(f)
    os.replace(tmp, path)
    with open(path + ".json", "w") as f:
        json.dump({"dtype": np.dtype(dtype).name, "vocab_size": tok.vocab_size, "tokens": n}, f)
    return n


def token_file_dtype(path: str) -> Optional[str]:
    """dtype name recorded by ``encode_to_token_file`` (None if there is no sidecar)."""
    side = path + ".json"
    if not os.path.exists(side):
        return None
    with open(side) as f:
        return json.load(f)["dtype"]
