"""Byte-level BPE tokenizer (data/bpe.py): the GPT-2 scheme of the reference's LLaMA
(tiktoken gpt2, llama3/LLaMA-jax.ipynb:196,260) and DeepSeek (AutoTokenizer gpt2,
deepseekv3/deepseekv3.ipynb:524-527) slices. The real GPT-2 vocab files are not available
offline, so GPT-2-format loading is checked on a hand-written vocab/merges pair (parity with
tiktoken's ids: unpinned)."""
import json

import numpy as np
import torch

from solvingpapers_amd.data import synthetic_corpus
from solvingpapers_amd.data.bpe import EOT, BPETokenizer, encode_to_token_file, token_file_dtype
from solvingpapers_amd.data.loader import NativeTokenLoader


def _docs():
    text = synthetic_corpus(40_000, seed=1)
    return [text[i:i + 400] for i in range(0, len(text), 400)]


def test_trained_bpe_round_trips_any_string():
    tok = BPETokenizer.train(_docs(), vocab_size=600)
    assert 300 < tok.vocab_size <= 600 and tok.eot_token is not None
    for s in ["the king and queen", "  spaced\tout\nlines  ", "unicode: é ü 中文 🙂", ""]:
        assert tok.decode(tok.encode(s)) == s
    ids = tok.encode("the king and queen of rome")
    assert len(ids) < len("the king and queen of rome") / 2      # merges learnt from the corpus
    assert max(ids) < tok.vocab_size


def test_save_load_identical(tmp_path):
    tok = BPETokenizer.train(_docs(), vocab_size=400)
    p = str(tmp_path / "tok.json")
    tok.save(p)
    t2 = BPETokenizer.load(p)
    s = "noble heart and fair mind"
    assert t2.encode(s) == tok.encode(s) and t2.eot_token == tok.eot_token


def test_gpt2_format_files(tmp_path):
    # GPT-2 byte-level alphabet: space is 'Ġ' (U+0120); a merge list in merges.txt order
    from tokenizers import pre_tokenizers
    alphabet = sorted(pre_tokenizers.ByteLevel.alphabet())
    vocab = {c: i for i, c in enumerate(alphabet)}
    merges = [("t", "h"), ("th", "e"), ("Ġ", "k"), ("Ġk", "i")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    vocab[EOT] = len(vocab)
    vp, mp = tmp_path / "vocab.json", tmp_path / "merges.txt"
    vp.write_text(json.dumps(vocab))
    mp.write_text("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n")
    tok = BPETokenizer.from_gpt2_files(str(vp), str(mp))
    ids = tok.encode("the kin")
    assert [tok._tok.id_to_token(i) for i in ids] == ["the", "Ġki", "n"]
    assert tok.eot_token == len(vocab) - 1 and tok.n_vocab == len(vocab)
    assert tok.decode(ids) == "the kin"


def test_token_file_feeds_native_loader(tmp_path):
    docs = _docs()[:20]
    tok = BPETokenizer.train(docs, vocab_size=500)
    p = str(tmp_path / "corpus.bin")
    n = encode_to_token_file(tok, docs, p, batch=7)
    assert token_file_dtype(p) == "uint16"
    flat = np.fromfile(p, dtype=np.uint16)
    assert flat.size == n == sum(len(tok.encode(d)) + 1 for d in docs)
    assert flat[-1] == tok.eot_token
    assert tok.decode(flat[:len(tok.encode(docs[0]))]) == docs[0]
    ld = NativeTokenLoader(p, 2, 32, sequential=True)
    x, y = ld(0)
    assert torch.equal(x[0], torch.from_numpy(flat[:32].astype(np.int64)))
    assert torch.equal(x[0, 1:], y[0, :-1])


def test_cli_trains_from_text_and_token_file(tmp_path):
    from solvingpapers_amd.train.__main__ import main
    docs = _docs()
    txt = tmp_path / "corpus.txt"
    txt.write_text("".join(docs), encoding="utf-8")
    tjson = str(tmp_path / "tok.json")
    tok = BPETokenizer.train(docs, vocab_size=512)
    tok.save(tjson)
    common = ["llama3", "--preset", "llama3_ref", "--set", "n_layers=1", "--steps", "2", "--batch", "2",
              "--seq", "32", "--device", "cpu"]
    tr = main(common + ["--text", str(txt), "--tokenizer", tjson])
    assert tr.model.tok_embeddings.shape[0] == tok.vocab_size if hasattr(tr.model, "tok_embeddings") else True
    binp = str(tmp_path / "train.bin")
    encode_to_token_file(tok, docs, binp)
    tr2 = main(common + ["--data", binp, "--set", f"vocab_size={tok.vocab_size}"])
    assert tr2 is not None
