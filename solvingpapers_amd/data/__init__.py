"""Data layer: char tokenizer, synthetic corpora/token streams,
sliding-window causal datasets with rank sharding, MNIST IDX reader + synthetic
MNIST-like images (torchvision is not installed; there is no network)."""
from .text import CharTokenizer, TokenWindowDataset, get_batch, synthetic_corpus, synthetic_tokens
from .images import load_mnist_idx, synthetic_images, synthetic_mnist, ImageBatches

__all__ = ["CharTokenizer", "TokenWindowDataset", "get_batch", "synthetic_corpus", "synthetic_tokens",
           "load_mnist_idx", "synthetic_images", "synthetic_mnist", "ImageBatches"]
