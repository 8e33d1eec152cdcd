#!/usr/bin/env python3
"""Cut an imagenet_1k-layout dataset (<root>/<wnid>/<first JPEG>, one image
per class, as the reference's test_files/imagenet_1k/train) into labelled u8
shards for the SDFS (BASELINE config 3: "SDFS-staged imagenet_1k shards").

The classes are taken in sorted wnid order, which is synset_words.txt's
order, so the i-th image of the dataset is class i; shard k holds images
[k*per, (k+1)*per) and records label0 = k*per (csrc/serve/shard.h). Each
image is decoded (native decoder) and resized the way the engine does
(short side 224, centre crop, bilinear, u8), so a shard replica is served
from HBM with no host work.

    python tools/make_shards.py --src /root/reference/test_files/imagenet_1k/train \
        --out data/shards --per 250
    # then on a node:  put data/shards/imagenet_1k.0.u8s imagenet_1k.0.u8s  (x4)
    #                  predict imagenet_1k.0.u8s imagenet_1k.1.u8s ...
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="/root/reference/test_files/imagenet_1k/train")
    ap.add_argument("--out", default=os.path.join(ROOT, "data", "shards"))
    ap.add_argument("--per", type=int, default=250, help="images per shard")
    ap.add_argument("--limit", type=int, default=0, help="only the first N classes")
    ap.add_argument("--name", default="imagenet_1k")
    ap.add_argument("--synthetic", type=int, default=0,
                    help="N random 224x224 images (labels 0..N-1) instead of a dataset (throughput runs on a box "
                         "without the reference's JPEGs)")
    a = ap.parse_args()
    from dmlc.utils.shards import decode_resize, write_shard
    if a.synthetic:
        import numpy as np
        os.makedirs(a.out, exist_ok=True)
        rng = np.random.default_rng(0)
        for k, s in enumerate(range(0, a.synthetic, a.per)):
            n = min(a.per, a.synthetic - s)
            imgs = rng.integers(0, 256, size=(n, 224, 224, 3), dtype=np.uint8)
            p = write_shard(os.path.join(a.out, f"{a.name}.{k}.u8s"), imgs, label0=s)
            print(f"{p}: synthetic images {s}..{s + n - 1}", flush=True)
        return
    wnids = sorted(os.listdir(a.src))
    if a.limit:
        wnids = wnids[:a.limit]
    files = []
    for w in wnids:
        d = os.path.join(a.src, w)
        files.append(os.path.join(d, sorted(os.listdir(d))[0]))  # the first file, as src/services.rs:485-490
    os.makedirs(a.out, exist_ok=True)
    for k, s in enumerate(range(0, len(files), a.per)):
        imgs = decode_resize(files[s:s + a.per])
        p = write_shard(os.path.join(a.out, f"{a.name}.{k}.u8s"), imgs, label0=s)
        print(f"{p}: images {s}..{s + len(imgs) - 1} ({os.path.getsize(p) / 1e6:.1f} MB)", flush=True)


if __name__ == "__main__":
    main()
