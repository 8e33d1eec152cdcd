"""u8 image shards for the SDFS-staged data-parallel path (format:
csrc/serve/shard.h): 32-byte header (b"DMLCU8S1", u32 n, h, w, label0,
flags, zeros) then n decoded and resized images u8 [h, w, 3]. With flags
bit 0 set the shard is labelled: image i is class label0 + i. A shard `put`
into the SDFS is kept resident in HBM by every member that holds a replica
(one slice per GPU); `predict-shard` classifies it there, and `predict
<shard> ...` runs the jobs over labelled shards."""
from __future__ import annotations

import os
import struct

import numpy as np

MAGIC = b"DMLCU8S1"
HEADER = 32


def write_shard(path: str, images: np.ndarray, label0: int | None = None) -> str:
    """label0: the class of the first image (image i is class label0 + i);
    None writes an unlabelled shard."""
    images = np.ascontiguousarray(images, dtype=np.uint8)
    if images.ndim != 4 or images.shape[-1] != 3:
        raise ValueError("images must be u8 [n, h, w, 3]")
    n, h, w, _ = images.shape
    flags = 0 if label0 is None else 1
    with open(path, "wb") as f:
        f.write(MAGIC + struct.pack("<IIIII", n, h, w, label0 or 0, flags) + b"\0" * 4)
        f.write(images.tobytes())
    return path


def read_shard(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        hdr = f.read(HEADER)
        if hdr[:8] != MAGIC:
            raise ValueError("not a dmlc u8 shard")
        n, h, w = struct.unpack("<III", hdr[8:20])
        return np.frombuffer(f.read(), dtype=np.uint8).reshape(n, h, w, 3)


def shard_info(path: str) -> dict:
    with open(path, "rb") as f:
        hdr = f.read(HEADER)
    if hdr[:8] != MAGIC:
        raise ValueError("not a dmlc u8 shard")
    n, h, w, label0, flags = struct.unpack("<IIIII", hdr[8:28])
    return {"n": n, "h": h, "w": w, "label0": label0 if flags & 1 else None}


def decode_resize(files: list[str], size: int = 224) -> np.ndarray:
    """Decode JPEGs (the native decoder) and resize them the way the engine
    does (short side -> size, centre crop, bilinear, u8): [n, size, size, 3]."""
    import torch
    import torch.nn.functional as F
    from .. import native
    C = native()
    out = np.empty((len(files), size, size, 3), dtype=np.uint8)
    for i, p in enumerate(files):
        img = C.decode_jpeg(open(p, "rb").read())
        h, w, _ = img.shape
        if h <= w:
            rh, rw = size, size * w // h
        else:
            rh, rw = size * h // w, size
        t = torch.from_numpy(img).permute(2, 0, 1)[None].float()
        r = F.interpolate(t, size=(rh, rw), mode="bilinear", align_corners=False)
        oy, ox = (rh - size) // 2, (rw - size) // 2
        out[i] = r[0, :, oy:oy + size, ox:ox + size].round().clamp(0, 255).byte().permute(1, 2, 0).numpy()
    return out


def shard_from_jpegs(path: str, files: list[str], size: int = 224, label0: int | None = None) -> str:
    return write_shard(path, decode_resize(files, size), label0)


def synthetic_shard(path: str, n: int, size: int = 224, seed: int = 0) -> str:
    rng = np.random.default_rng(seed)
    return write_shard(path, rng.integers(0, 256, (n, size, size, 3), dtype=np.uint8))


__all__ = ["write_shard", "read_shard", "shard_info", "decode_resize", "shard_from_jpegs", "synthetic_shard", "HEADER",
           "MAGIC"]
