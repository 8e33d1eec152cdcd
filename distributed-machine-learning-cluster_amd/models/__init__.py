"""Model zoo: reference ``torch.nn`` definitions + GPU-engine architectures.

The GPU engine (``dmlc.runtime.InferenceEngine``) builds the same graphs in
C++ (csrc/runtime/engine.cpp) from the same parameter names.
"""
from .reference import ARCHS, AlexNet, BasicBlock, Bottleneck, ResNet, build, state_dict_f32  # noqa: F401

SUPPORTED = tuple(sorted(ARCHS))
