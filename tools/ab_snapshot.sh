#!/bin/bash
# Save the current in-tree libdmlc_gpu.so as A/B variant <name>
# (build/ab/<name>/libdmlc_gpu.so, shipped to the GPU box with the tree).
#   python tools/build.py && tools/ab_snapshot.sh <name>
cd "$(dirname "$0")/.."
mkdir -p "build/ab/$1"
cp distributed-machine-learning-cluster_amd/libdmlc_gpu.so "build/ab/$1/libdmlc_gpu.so"
echo "saved build/ab/$1"
