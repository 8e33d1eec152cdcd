"""Host-only audit of the packed weight arena (csrc/runtime/engine.cpp
pack_host), no GPU needed.

Every write of the weight packer goes through a bounds-checked region of the
layout pass (RegionRef), so packing a model whose layout gives some layer too
small a region raises instead of spilling into the next layer's weights (the
round-5 advisor finding: the bf16 fragment-order copy of an e4m3
conv3x3_stream8 layer wrote 2x its region). Here every model and the
kernel-path option sets the GPU tests use are packed on the host and the
regions are checked to be disjoint and inside the arena.
"""
import pytest

from dmlc import native
from dmlc.models import build, state_dict_f32

CASES = [
    ("resnet18", {}),
    ("resnet18", {"ds_into_conv2": False, "fused_block": False}),
    ("resnet34", {}),
    ("resnet50", {}),
    ("resnet50_fp8", {}),
    ("resnet50_fp8", {"fp8_3x3_in": False}),
    ("resnet50_fp8", {"fp8_3x3_out": False, "fp8_3x3_in": False}),
    ("resnet50_fp8", {"ds_into_expand": False, "fused_bottleneck": False}),
    ("alexnet", {}),
]


@pytest.fixture(scope="module")
def weights():
    cache = {}

    def get(arch):
        base = arch.replace("_fp8", "")
        if base not in cache:
            sd = state_dict_f32(build(base, seed=0))
            cache[base] = {k: v.detach().cpu().float().numpy() for k, v in sd.items()}
        return cache[base]
    return get


@pytest.mark.parametrize("arch,opts", CASES, ids=[f"{a}-{'-'.join(o) or 'default'}" for a, o in CASES])
def test_pack_regions_disjoint_and_bounded(weights, arch, opts):
    C = native()
    regions, total = C.pack_audit(arch, weights(arch), opts)
    assert total > 0 and regions
    spans = sorted((off, off + n, layer, kind) for layer, kind, off, n in regions)
    for (a0, a1, la, ka), (b0, b1, lb, kb) in zip(spans, spans[1:]):
        assert a1 <= b0, f"{la}.{ka} [{a0},{a1}) overlaps {lb}.{kb} [{b0},{b1})"
    assert spans[-1][1] <= total
    kinds = {k for _, k, _, _ in regions}
    assert {"w", "b"} <= kinds
    if arch == "resnet50_fp8":
        # e4m3 layers: alpha region, and the stream8 fragment copies are e4m3 (1 B / weight)
        assert "alpha" in kinds
        wf8 = [(layer, n) for layer, kind, _, n in regions if kind == "wf" and "conv2" in layer
               and not layer.startswith("layer1")]
        w8 = {layer: n for layer, kind, _, n in regions if kind == "w"}
        if opts.get("fp8_3x3_in", True):
            assert wf8, "expected stream8 fragment-order regions for layer2-4 3x3 convs"
            for layer, n in wf8:
                assert n <= w8[layer], (layer, n, w8[layer])
