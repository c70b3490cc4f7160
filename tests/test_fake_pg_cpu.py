"""8-way layouts without 8 processes (shape-only): one process joins a
``FakeProcessGroup`` as rank r of 8 (collectives are no-ops that keep shapes), builds the
sharded model exactly as that rank of an 8-GPU job would, and checks every local shard,
the ZeRO-1 partition and that a forward + backward runs through the sharded code paths.
Values are meaningless under the fake group; numerics are covered by the gloo tests."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


PRELUDE = """
    import torch, torch.distributed as dist
    from torch.testing._internal.distributed.fake_pg import FakeStore
    RANK, WORLD = {rank}, 8
    dist.init_process_group("fake", store=FakeStore(), rank=RANK, world_size=WORLD)
"""


@pytest.mark.parametrize("rank", [0, 5])
def test_gemma_7b_tp8_shards(rank):
    """Gemma-7B-shape (D3072, 16 heads x hd256, 1 KV head, GeGLU 24576, V 256000), TP=8, one
    layer: rank-local shards + a forward/backward through the vocab-parallel and
    column/row-parallel paths."""
    out = _run(PRELUDE.format(rank=rank) + """
    from solvingpapers_amd.models import gemma
    c = gemma.config("gemma_7b_mqa", n_layers=1, max_seq_len=16)
    m = gemma.Gemma(c, dtype=torch.float32, tp_group=dist.group.WORLD)
    l = m.layers[0]
    assert m.embed.shape == (256000 // 8, 3072)
    assert l.wq.shape == (2 * 256, 3072)            # 2 of 16 query heads
    assert l.wkv.shape == (2 * 256, 3072)           # MQA K/V replicated
    assert l.wo.shape == (3072, 2 * 256)
    assert l.w13.shape == (2 * 24576 // 8, 3072)
    assert l.w2.shape == (3072, 24576 // 8)
    ids = torch.randint(0, 256000, (1, 9))
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    assert loss.dim() == 0 and l.w13.grad is not None and l.w13.grad.shape == l.w13.shape
    print("ok", sum(p.numel() for p in m.parameters()))
    """)
    assert out.startswith("ok")


def test_llama_8b_zero1_dp8_partition():
    """LLaMA3-8B-shape DP=8 with ZeRO-1: every flat-buffer bucket splits into 8 equal
    contiguous shards and the 8 ranks' shards tile the buffer exactly (2 layers, meta-free
    CPU build at the real widths)."""
    out = _run(PRELUDE.format(rank=3) + """
    from solvingpapers_amd.models import llama3
    from solvingpapers_amd.parallel.data_parallel import DataParallel
    from solvingpapers_amd.utils.flat import FlatParams
    c = llama3.config("llama3_8b", n_layers=2, vocab_size=4096)
    m = llama3.Llama3(c, dtype=torch.bfloat16)
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16, align=64 * 8)
    dp = DataParallel(m, flat, zero1=True)
    ranges = dp.shard_ranges()
    assert len(ranges) == len(flat.buckets)
    for b, (s, e) in zip(flat.buckets, ranges):
        n = b.numel // 8
        assert b.numel % 8 == 0 and e - s == n and s == b.start + 3 * n
    per_layer = sum(p.numel() for p in m.layers[0].parameters())
    assert per_layer == 4096 * 6144 + 4096 * 4096 + 3 * 4096 * 14336 + 2 * 4096   # 218.1M params / layer
    print("ok")
    """)
    assert out.startswith("ok")


@pytest.mark.parametrize("rank", [0, 7])
def test_dsv3_v3_ep8_expert_shards(rank):
    """DeepSeek-V3 layout (256 routed experts top-8, MLA qk 128+64 / v 128 heads), EP=8 at a
    CPU-sized width: each rank holds 32 of the 256 routed experts and every other weight
    (layout only; the routed forward is covered by the gloo EP test)."""
    out = _run(PRELUDE.format(rank=rank) + """
    from solvingpapers_amd.models import deepseekv3 as ds
    c = ds.config("dsv3_v3", vocab_size=512, dim=256, n_heads=8, q_lora_rank=64, kv_lora_rank=32,
                  expert_hidden=64, dense_hidden=128, n_layers=2, n_dense_layers=1, block_size=16)
    assert (c.n_experts, c.top_k, c.qk_nope_dim, c.qk_rope_dim, c.v_head_dim) == (256, 8, 128, 64, 128)
    m = ds.DeepSeekV3(c, ep_group=dist.group.WORLD)
    moe = m.moe_layers()
    assert moe and all(l.w13.shape[0] == 256 // WORLD for l in moe), [l.w13.shape for l in moe]
    # shape-only: the fake group's all-to-all leaves the exchanged token counts uninitialised,
    # so the routed forward is covered by the gloo EP test instead
    n_local = sum(p.numel() for p in m.parameters())
    full = ds.DeepSeekV3(ds.config("dsv3_v3", vocab_size=512, dim=256, n_heads=8, q_lora_rank=64,
                                   kv_lora_rank=32, expert_hidden=64, dense_hidden=128, n_layers=2,
                                   n_dense_layers=1, block_size=16))
    per_expert = 3 * 64 * 256
    assert sum(p.numel() for p in full.parameters()) - n_local == len(moe) * (256 - 32) * per_expert
    print("ok", tuple(moe[0].w13.shape))
    """)
    assert "ok (32," in out
