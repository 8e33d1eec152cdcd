#!/usr/bin/env python3
"""Copy the first N classes of the reference's real dataset
(test_files/imagenet_1k/train/<wnid>/<one JPEG>, 1000 JPEGs in 344 distinct
sizes) and its synset_words.txt into data/, so GPU-box benchmarks
(tools/bench_jobs.py --dataset data/imagenet_1k_subset/train --labels
data/synset_words.txt) run on real images. The files are data, not source:
data/imagenet_1k_subset/ is git-ignored.

usage: python tools/make_subset.py [--n 256] [--ref /root/reference]"""
import argparse
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    src = os.path.join(a.ref, "test_files", "imagenet_1k", "train")
    dst = os.path.join(ROOT, "data", "imagenet_1k_subset", "train")
    total = 0
    wnids = sorted(os.listdir(src))[:a.n]
    for w in wnids:
        os.makedirs(os.path.join(dst, w), exist_ok=True)
        f = sorted(os.listdir(os.path.join(src, w)))[0]
        shutil.copy(os.path.join(src, w, f), os.path.join(dst, w, f))
        total += os.path.getsize(os.path.join(src, w, f))
    shutil.copy(os.path.join(a.ref, "synset_words.txt"), os.path.join(ROOT, "data", "synset_words.txt"))
    print(f"{len(wnids)} JPEGs, {total / 1e6:.1f} MB -> {dst}")


if __name__ == "__main__":
    main()
