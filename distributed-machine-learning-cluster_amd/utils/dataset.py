"""ImageNet-1k layout helpers.

The reference serves ``test_files/imagenet_1k/train/<wnid>/<one JPEG>`` with
labels from ``synset_words.txt`` (``<wnid> <label text>``, same order as the
class indices; src/services.rs:170-184,475-497). There is no network here,
so tests and benchmarks build synthetic datasets of the same layout.
"""
from __future__ import annotations

import os

import numpy as np


def read_labels(path: str) -> list[tuple[str, str]]:
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            wnid, _, text = line.partition(" ")
            out.append((wnid, text.strip()))
    return out


def write_labels(path: str, entries: list[tuple[str, str]]) -> str:
    with open(path, "w") as f:
        for wnid, text in entries:
            f.write(f"{wnid} {text}\n")
    return path


def synthetic_labels(n: int = 1000) -> list[tuple[str, str]]:
    return [(f"n{10000000 + i:08d}", f"class {i}") for i in range(n)]


def make_synthetic_dataset(root: str, labels: list[tuple[str, str]], size=(375, 500), seed: int = 0,
                           quality: int = 90) -> str:
    """One smooth random JPEG per wnid (PIL encoder, baseline JPEG). `size`
    is (h, w) or a list of (h, w) used in turn (ragged, like the reference's
    imagenet_1k with its 344 distinct sizes)."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    sizes = size if isinstance(size, list) else [size]
    for i, (wnid, _) in enumerate(labels):
        h, w = sizes[i % len(sizes)]
        d = os.path.join(root, wnid)
        os.makedirs(d, exist_ok=True)
        base = rng.integers(0, 256, (h // 16 + 1, w // 16 + 1, 3), dtype=np.uint8)
        img = Image.fromarray(base).resize((w, h), Image.BILINEAR)
        img.save(os.path.join(d, f"img_{i:05d}.JPEG"), quality=quality)
    return root


def synthetic_u8_batch(n: int, size: int = 224, seed: int = 0) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, (n, size, size, 3), dtype=np.uint8)
