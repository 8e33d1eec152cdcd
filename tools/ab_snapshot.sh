#!/bin/bash
# Save the current in-tree libdmlc_gpu.so and _C*.so (bindings) as A/B
# variant <name> (build/ab/<name>/, shipped to the GPU box with the tree).
#   python tools/build.py && tools/ab_snapshot.sh <name>
cd "$(dirname "$0")/.."
mkdir -p "build/ab/$1"
cp distributed-machine-learning-cluster_amd/libdmlc_gpu.so distributed-machine-learning-cluster_amd/_C*.so "build/ab/$1/"
echo "saved build/ab/$1"
