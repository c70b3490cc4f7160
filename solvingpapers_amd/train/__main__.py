"""Command-line training entry point for every model family.

    python -m solvingpapers_amd.train gpt     --preset gpt_ref --steps 1000
    python -m solvingpapers_amd.train llama3  --preset llama3_ref --steps 200
    python -m solvingpapers_amd.train gemma   --preset gemma_ref
    python -m solvingpapers_amd.train dsv3    --preset dsv3_ref --ckpt-dir ck/
    python -m solvingpapers_amd.train vit | ae | vae | kd
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m solvingpapers_amd.train llama3 --preset llama3_8b ...
    torchrun --nproc-per-node 8 ... -m solvingpapers_amd.train gemma --preset gemma_7b_mqa --tp 8 --sp
    torchrun --nproc-per-node 8 ... -m solvingpapers_amd.train dsv3 --preset dsv3_style --ep 8

Model hyper-parameters can be overridden with ``--set key=value`` (config dataclass
fields). Language models train through train/trainer.py (data parallel over RCCL when
launched under torchrun, checkpoint/auto-resume, JSONL metrics); char-level presets
(gpt_ref, gemma_ref) use the synthetic Shakespeare-like corpus + char tokenizer, the
token-level ones a synthetic id stream served by the native C++ loader. Image models
run their reference-style epoch loops (ViT / AE / VAE / KD) on MNIST IDX files when
``--mnist-root`` is given, else synthetic MNIST-like digits.
"""
from __future__ import annotations

import argparse
import ast
import dataclasses
import json
import os

import torch


def _parse_sets(items):
    out = {}
    for it in items or []:
        k, v = it.split("=", 1)
        try:
            out[k] = ast.literal_eval(v)
        except (ValueError, SyntaxError):
            out[k] = v
    return out


def _tokenizer(spec: str, text: str):
    """char | bpe:<vocab> (train a byte-level BPE on the text) | gpt2:<dir with vocab.json +
    merges.txt> | <path to a saved tokenizer.json>."""
    from ..data.bpe import BPETokenizer
    from ..data.text import CharTokenizer
    if spec == "char":
        return CharTokenizer(text)
    if spec.startswith("bpe:"):
        chunk = 1 << 16
        return BPETokenizer.train((text[i:i + chunk] for i in range(0, len(text), chunk)), int(spec[4:]))
    if spec.startswith("gpt2:"):
        d = spec[5:]
        return BPETokenizer.from_gpt2_files(os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt"))
    return BPETokenizer.load(spec)


def _lm(args, info):
    from ..data.loader import NativeTokenLoader
    from ..data.text import synthetic_corpus
    from ..models import deepseekv3, gemma, gpt, llama3
    from ..parallel.groups import build_groups
    from .trainer import TrainConfig, Trainer
    dev = info.device if args.device is None else torch.device(args.device)
    # world = tp x data, data = ep x expert-dp (parallel/groups.py); the data loader shards by the
    # DATA coordinate: TP peers read the same batch, DP/EP ranks different ones
    pg = build_groups(args.tp, args.ep)
    if args.tp > 1 and args.model != "gemma":
        raise SystemExit("--tp is implemented for gemma (Megatron column/row-parallel + vocab-parallel CE)")
    if args.ep > 1 and args.model != "dsv3":
        raise SystemExit("--ep is implemented for dsv3 (MoE all-to-all dispatch)")
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype or ("bf16" if dev.type == "cuda" else "fp32")]
    sets = _parse_sets(args.set)
    char = args.preset in ("gpt_ref", "gpt_tiny_cpu", "gemma_ref")
    stream = files = None
    if args.data:
        files = args.data.split(",")
    elif args.text or char:
        text = open(args.text, encoding="utf-8").read() if args.text else synthetic_corpus(400_000, seed=args.seed)
        tok = _tokenizer(args.tokenizer or ("char" if char else "bpe:8192"), text)
        stream = torch.tensor(tok.encode(text), dtype=torch.int32)
        sets.setdefault("vocab_size", tok.vocab_size)
        char = True
    fam = args.model
    if fam == "gpt":
        c = gpt.config(args.preset or "gpt_ref", **sets)
        model = gpt.GPT(c, device=dev, dtype=dtype, seed=args.seed)
        V, T, B = c.vocab_size, c.block_size, c.batch_size
    elif fam == "llama3":
        c = llama3.config(args.preset or "llama3_ref", **sets)
        model = llama3.Llama3(c, device=dev, dtype=dtype, seed=args.seed)
        V, T, B = c.vocab_size, args.seq or min(c.max_seq_len or 128, 128), c.batch_size
    elif fam == "gemma":
        pre = args.preset or "gemma_ref"
        c = gemma.config(pre, **sets)
        if pre == "gemma_ref":
            if args.tp > 1:
                raise SystemExit("gemma_ref (reference-parity model) runs unsharded; use gemma_tiny / gemma_7b_mqa")
            model = gemma.GemmaRef(c).to(device=dev, dtype=dtype)
            V, T, B = c.vocab_size, c.block_size, c.batch_size
        else:
            model = gemma.Gemma(c, device=dev, dtype=dtype, seed=args.seed, tp_group=pg.tp_group,
                                sequence_parallel=args.sp, tp_pipeline=args.pipeline)
            V, T, B = c.vocab_size, args.seq or c.max_seq_len, c.batch_size
    elif fam == "dsv3":
        c = deepseekv3.config(args.preset or "dsv3_ref", **sets)
        model = deepseekv3.DeepSeekV3(c, device=dev, dtype=dtype, seed=args.seed, ep_group=pg.ep_group)
        V, T, B = c.vocab_size, c.block_size, c.batch_size
    else:
        raise SystemExit(f"unknown model {fam}")
    T = args.seq or T
    B = args.batch or B
    if files:
        # token files (data/bpe.encode_to_token_file) memory-mapped by the native loader; without a
        # second file the eval batches are drawn from the training file with another seed
        from ..data.bpe import token_file_dtype
        fd = [torch.int32 if token_file_dtype(f) == "int32" else torch.uint16 for f in files]
        tr = NativeTokenLoader(files[0], B, T, seed=args.seed, rank=pg.dp_rank, world=pg.dp, device=dev,
                               file_dtype=fd[0])
        ev = NativeTokenLoader(files[-1], B, T, seed=args.seed + 1, rank=pg.dp_rank, world=pg.dp,
                               device=dev, file_dtype=fd[-1])
    else:
        if not char:
            stream = torch.randint(0, V, (max(200_000, 4 * B * (T + 1)),),
                                   generator=torch.Generator().manual_seed(args.seed), dtype=torch.int32)
        n = int(stream.numel() * 0.9)
        tr = NativeTokenLoader(stream[:n], B, T, seed=args.seed, rank=pg.dp_rank, world=pg.dp, device=dev)
        ev = NativeTokenLoader(stream[n:], B, T, seed=args.seed + 1, rank=pg.dp_rank, world=pg.dp, device=dev)
    tc = TrainConfig(steps=args.steps, lr=args.lr, min_lr=args.min_lr, warmup=args.warmup,
                     weight_decay=args.weight_decay, clip=args.clip, eval_every=args.eval_every,
                     eval_iters=args.eval_iters, ckpt_dir=args.ckpt_dir, ckpt_every=args.ckpt_every,
                     log_path=args.log, grad_accum=args.accum, zero1=args.zero1, optimizer=args.optimizer,
                     grad_dtype=dtype, log_every=args.log_every,
                     pair_microbatches=args.pipeline)
    hooks = [lambda r: print(json.dumps(r), flush=True)] if info.rank == 0 else []
    if info.rank == 0 and args.wandb:
        from .metrics import WandbHook
        hooks.append(WandbHook(args.wandb, config=vars(args), tokens_per_step=B * T * args.accum * pg.dp))
    trainer = Trainer(model, tc, tr, ev.batch_at, hooks=hooks, groups=pg)
    trainer.fit()
    return trainer


def _images(args, info):
    from ..models import autoencoder, kd, vit
    sets = _parse_sets(args.set)
    dev = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    if args.model == "vit":
        c = vit.config(args.preset or "vit_mnist_ref", **sets)
        return vit.train(c, epochs=args.epochs, device=dev, mnist_root=args.mnist_root, seed=args.seed)
    if args.model in ("ae", "vae"):
        c = autoencoder.AEConfig(kind=args.model, device=dev, mnist_root=args.mnist_root, seed=args.seed, **sets)
        if args.epochs:
            c.epochs = args.epochs
        return autoencoder.train(c)
    if args.model == "kd":
        c = kd.KDConfig(device=dev, mnist_root=args.mnist_root, seed=args.seed, **sets)
        if args.epochs:
            c.epochs = args.epochs
        return kd.train(c)
    raise SystemExit(f"unknown model {args.model}")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m solvingpapers_amd.train")
    ap.add_argument("model", choices=["gpt", "llama3", "gemma", "dsv3", "vit", "ae", "vae", "kd"])
    ap.add_argument("--preset", default=None)
    ap.add_argument("--set", action="append", help="config override key=value")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--seq", type=int, default=None)
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--optimizer", default="adamw", choices=["adamw", "adam", "sgd"])
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--min-lr", type=float, default=None)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--weight-decay", type=float, default=0.1)
    ap.add_argument("--clip", type=float, default=1.0)
    ap.add_argument("--eval-every", type=int, default=0)
    ap.add_argument("--eval-iters", type=int, default=10)
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--log", default=None)
    ap.add_argument("--zero1", action="store_true")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (gemma)")
    ap.add_argument("--sp", action="store_true", default=None,
                    help="Megatron sequence parallelism with --tp (the default; --no-sp: plain TP)")
    ap.add_argument("--no-sp", dest="sp", action="store_false")
    ap.add_argument("--ep", type=int, default=1, help="expert-parallel degree (dsv3)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="with --tp / --ep: no two-chunk comm/compute overlap (TP: sequence-parallel chunk "
                         "pair; EP: micro-batch pairs)")
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--device", default=None)
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"])
    ap.add_argument("--mnist-root", default=None)
    ap.add_argument("--data", default=None, help="token file(s) TRAIN[,EVAL] written by data.bpe.encode_to_token_file")
    ap.add_argument("--text", default=None, help="UTF-8 text file to tokenize (LM models)")
    ap.add_argument("--tokenizer", default=None, help="char | bpe:<vocab> | gpt2:<dir> | <tokenizer.json>")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--wandb", default=None, help="W&B project (reference metric names; needs the wandb package)")
    args = ap.parse_args(argv)
    from ..parallel import dist as sdist
    from ..utils.tuning import load_gemm_tuning
    info = sdist.init_distributed()
    load_gemm_tuning()  # tuned hipBLASLt/rocBLAS solutions for the shapes in tuning/*.csv
    try:
        if args.model in ("vit", "ae", "vae", "kd"):
            return _images(args, info)
        return _lm(args, info)
    finally:
        sdist.cleanup()


if __name__ == "__main__":
    main()
