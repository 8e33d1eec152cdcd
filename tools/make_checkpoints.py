#!/usr/bin/env python3
"""Write random-init `.ot` checkpoints (tch-rs VarStore format) for the model
zoo. The reference's pretrained_models/{alexnet,resnet18}.ot are git-LFS
pointer stubs (pretrained_models/alexnet.ot:1-3), so real weights do not
exist here; every node/bench uses random weights of the right architecture.

usage: python tools/make_checkpoints.py OUT_DIR [--models resnet18,alexnet] [--seed 0]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dmlc.utils.ot import write_random_checkpoint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--models", default="resnet18,alexnet")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for m in a.models.split(","):
        p = write_random_checkpoint(m, os.path.join(a.out, f"{m}.ot"), seed=a.seed)
        print(p, os.path.getsize(p))


if __name__ == "__main__":
    main()
