"""Data layer: char tokenizer, synthetic corpora/token streams,
sliding-window causal datasets with rank sharding, byte-level BPE (GPT-2 scheme) + token files for the native loader, MNIST IDX reader + synthetic
MNIST-like images (torchvision is not installed; there is no network)."""
from .text import CharTokenizer, TokenWindowDataset, get_batch, synthetic_corpus, synthetic_tokens
from .bpe import BPETokenizer, encode_to_token_file
from .images import load_mnist_idx, synthetic_images, synthetic_mnist, ImageBatches

__all__ = ["BPETokenizer", "encode_to_token_file", "CharTokenizer", "TokenWindowDataset", "get_batch", "synthetic_corpus", "synthetic_tokens",
           "load_mnist_idx", "synthetic_images", "synthetic_mnist", "ImageBatches"]
