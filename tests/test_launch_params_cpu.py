"""Host-side launch-parameter choices of the GPU kernels (no GPU needed: the
native module's host functions run on the CPU)."""
import pytest

import dmlc

C = dmlc.native()
CUS = 256  # MI355X


@pytest.mark.parametrize("B,ns", [(1, 16), (16, 16), (64, 16), (256, 16), (512, 8), (1024, 4)])
def test_head_pooled_splits(B, ns):
    """head_pooled's class-split count for 1000 classes: 16 splits while the
    grid (16 images per workgroup x splits) stays within one workgroup per CU
    (ResNet18 / ResNet50 at B = 256: 256 workgroups; profiles/r5_head_splits.txt),
    fewer once the image groups alone fill the CUs."""
    got = C.head_pooled_splits(B, 1000, CUS)
    assert got == ns
    groups = (B + 15) // 16
    assert groups * got <= max(CUS, groups)  # never more than one round of workgroups
    # the workspace sized for the largest split count holds the partials and counters
    assert C.head_ws_bytes(B) >= B * got * 16 + groups * 4


def test_kernel_stagger_defaults_and_lanes():
    """Workgroup start stagger (csrc/kernels/stagger.hip): off for every
    kernel family by default (two compute lanes: profiles/r6_stagger.txt),
    4 on the stream convs in one-lane processes, restored by lanes > 1; the
    A/B hook's -1 restores the default and out-of-range values are refused."""
    families = 8
    try:
        assert [C.kernel_stagger(k) for k in range(families)] == [0] * families
        C.kernel_stagger_for_lanes(1)
        assert C.kernel_stagger(0) == 4 and [C.kernel_stagger(k) for k in range(1, families)] == [0] * (families - 1)
        C.kernel_stagger_for_lanes(2)
        assert C.kernel_stagger(0) == 0
        C.kernel_stagger_set(3, 2)
        assert C.kernel_stagger(3) == 2
        C.kernel_stagger_set(3, -1)
        assert C.kernel_stagger(3) == 0
        with pytest.raises(Exception):
            C.kernel_stagger_set(families, 1)
        with pytest.raises(Exception):
            C.kernel_stagger_set(0, 64)
    finally:
        for k in range(families):
            C.kernel_stagger_set(k, -1)
