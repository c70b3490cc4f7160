"""Native C++ token loader (csrc/runtime/token_loader.cpp): correctness of windows,
determinism / seek-resume, rank streams, mmap file source, prefetch threads."""
import torch

from solvingpapers_amd.data.loader import NativeTokenLoader, write_token_file


def test_windows_are_shifted_slices_and_deterministic():
    toks = torch.arange(10_000, dtype=torch.int32) * 7 % 50257
    ld = NativeTokenLoader(toks, 4, 32, seed=3, threads=3, depth=3)
    seen = [ld(i) for i in range(6)]
    for x, y in seen:
        assert x.shape == (4, 32) and x.dtype == torch.int64
        assert torch.equal(x[:, 1:], y[:, :-1])
        for r in range(4):                      # x row is a contiguous window of the stream
            s = int((toks == x[r, 0]).nonzero()[0])
            assert torch.equal(x[r], toks[s:s + 32].long())
    again = NativeTokenLoader(toks, 4, 32, seed=3, threads=1)
    x3, _ = again(3)                            # seek straight to batch 3
    assert torch.equal(x3, seen[3][0])
    assert torch.equal(again.batch_at(5)[1], seen[5][1])
    other = NativeTokenLoader(toks, 4, 32, seed=3, rank=1, world=2)
    assert not torch.equal(other(0)[0], seen[0][0])


def test_mmap_file_source_and_sequential(tmp_path):
    toks = torch.randint(0, 60000, (5000,))
    p = str(tmp_path / "tok.bin")
    write_token_file(p, toks)
    ld = NativeTokenLoader(p, 2, 16, sequential=True)
    assert len(ld) == 5000
    x, y = ld(0)
    assert torch.equal(x[0], toks[:16]) and torch.equal(x[1], toks[16:32]) and torch.equal(y[0], toks[1:17])
    x1, _ = ld(1)
    assert torch.equal(x1[0], toks[32:48])
    it = iter(ld)
    assert next(it)[0].shape == (2, 16)
