"""`.ot` checkpoint format (libtorch archive, '|' keys) — CPU only."""
import torch

from dmlc.models import build, state_dict_f32
from dmlc.utils.ot import load_ot, load_ot_jit, save_ot, write_random_checkpoint


def test_roundtrip_native(tmp_path):
    sd = state_dict_f32(build("resnet18", seed=1))
    p = str(tmp_path / "r18.ot")
    save_ot(p, sd)
    back = load_ot(p)
    assert set(back) == set(sd)
    for k in sd:
        assert torch.equal(back[k], sd[k]), k


def test_archive_readable_by_torchscript_loader(tmp_path):
    """Cross-check with an independent reader: the file is a TorchScript
    archive whose parameter names use '|' (tch-rs VarStore convention)."""
    p = write_random_checkpoint("alexnet", str(tmp_path / "alexnet.ot"), seed=2)
    m = torch.jit.load(p)
    names = [n for n, _ in m.named_parameters()]
    assert "features|0|weight" in names and "classifier|6|bias" in names
    a, b = load_ot(p), load_ot_jit(p)
    assert set(a) == set(b)
    for k in a:
        assert torch.equal(a[k], b[k])


def test_param_counts_match_reference_sizes():
    """The reference's LFS stubs record the fp32 file sizes
    (pretrained_models/alexnet.ot:3 -> 244,408,272 B; resnet18.ot:3 ->
    46,831,783 B); our architectures have the matching parameter counts."""
    n_alex = sum(v.numel() for v in state_dict_f32(build("alexnet")).values())
    n_r18 = sum(v.numel() for k, v in state_dict_f32(build("resnet18")).items())
    assert abs(n_alex * 4 - 244_408_272) / 244_408_272 < 0.001
    assert abs(n_r18 * 4 - 46_831_783) / 46_831_783 < 0.01
