"""Whole-model numerics: GPU engine (HIP kernels, BN folded, bf16) vs the
fp32 torch.nn reference on CPU, for every architecture in the zoo."""
import pytest
import torch

from dmlc.models import build, state_dict_f32
from dmlc.models.calibrated import calibrated, discrimination, e4m3_emulated_logits, mixed_images, normalize
from dmlc.runtime import InferenceEngine

pytestmark = pytest.mark.gpu

MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


def _ref_logits(model, img_u8):
    x = (img_u8.permute(0, 3, 1, 2).float() / 255 - MEAN) / STD
    with torch.no_grad():
        return model(x)


def _ref_logits_chunked(model, img_u8, chunk=64):
    with torch.no_grad():
        return torch.cat([model(normalize(c)) for c in img_u8.split(chunk)])


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _assert_discriminating(logits, ref, bar, min_classes, idx=None, prob=None, what="", agree=0.9):
    """The whole-model check on a calibrated model (dmlc.models.calibrated):
    the fp32 reference itself discriminates (>= min_classes distinct top-1
    classes, per-image part >= 20% of the logit norm), the engine's logits are
    within `bar` (relative L2), and two negative controls exceed that bar: the
    engine's logits paired with another image's reference (a rolled batch),
    and the batch-mean logits for every image. top-1 may differ from fp32 only
    where the fp32 top-2 gap is within 4x that image's rms logit error."""
    logits, ref = logits.float().cpu(), ref.float().cpu()
    n_cls, share = discrimination(ref)
    rel = _rel(logits, ref)
    rel_roll = _rel(logits.roll(1, 0), ref)
    rel_mean = _rel(logits.mean(0, keepdim=True).expand_as(logits), ref)
    print(f"{what}: fp32 top-1 classes {n_cls}, per-image share {share:.3f}, rel {rel:.4f} "
          f"(rolled {rel_roll:.3f}, batch-mean {rel_mean:.3f}, bar {bar})")
    assert n_cls >= min_classes, (what, n_cls)
    assert share >= 0.2, (what, share)
    assert rel < bar, (what, rel)
    assert rel_roll > bar and rel_mean > bar, (what, rel_roll, rel_mean)
    if idx is not None:
        idx = torch.as_tensor(idx).long().cpu()
        gap = ref.topk(2, -1).values
        rms = (logits - ref).pow(2).mean(-1).sqrt()
        near = (gap[:, 0] - gap[:, 1]) < 4 * rms
        mism = idx != ref.argmax(-1)
        assert torch.all(~mism | near), (what, mism.sum().item(), (mism & ~near).sum().item())
        assert (~mism).float().mean().item() > agree, (what, mism.sum().item())
    if prob is not None:
        # the top-1 probability of the same forward: |log p - log p_fp32| is
        # at most twice the image's largest logit error (the top logit and the
        # log-sum-exp each move by at most that much)
        ref_p = torch.softmax(ref, -1).max(-1).values
        got_p = torch.as_tensor(prob).float().cpu()
        tol = 2 * (logits - ref).abs().amax(-1) + 2e-3
        assert torch.all((got_p.log() - ref_p.log()).abs() <= tol), (what, (got_p.log() - ref_p.log()).abs().max())


def _fp8_bar(model, img, n=32):
    """The e4m3 engine's bars on a discriminating model, from an ideal e4m3
    rounding of the same network (calibrated.e4m3_emulated_logits) on the
    same images: relative L2 within 1.25x its error (never below 6%), top-1
    agreement with fp32 at most 0.15 below its agreement."""
    ref = _ref_logits_chunked(model, img[:n])
    emu = e4m3_emulated_logits(model, img[:n])
    floor = _rel(emu, ref)
    agree = (emu.argmax(-1) == ref.argmax(-1)).float().mean().item()
    print(f"ideal e4m3 rounding of this model: rel {floor:.4f} vs fp32, top-1 agreement {agree:.3f}")
    return max(6e-2, 1.25 * floor), max(0.3, agree - 0.15)


@pytest.mark.parametrize("arch", ["resnet18", "alexnet", "resnet50", "resnet34"])
def test_engine_matches_reference(gpu, arch):
    """Eager forward at B = 32 of a calibrated model (discriminating: per-image
    logits, many top-1 classes) vs fp32 torch.nn."""
    model = calibrated(arch, seed=11)
    eng = InferenceEngine(arch, state_dict_f32(model), max_batch=32)
    img = mixed_images(32, seed=12)
    ref = _ref_logits(model, img)
    idx, prob, logits = eng.predict(img.to(gpu), return_logits=True, use_graph=False)
    torch.cuda.synchronize()
    _assert_discriminating(logits, ref, 3e-2, 12, idx=idx, prob=prob, what=arch)


@pytest.mark.parametrize("arch,small_m,small_conv,B", [
    ("resnet18", 1, 1, 1), ("resnet18", 1, 0, 1), ("resnet18", 0, 0, 1), ("resnet18", 1, 1, 3),
    ("resnet34", 1, 1, 2), ("alexnet", 1, 1, 1), ("alexnet", 0, 1, 1)])
def test_engine_batch1_matches_reference(gpu, arch, small_m, small_conv, B):
    """The query path: one image per forward (the reference's batch of one,
    src/services.rs:421,493) on the query-batch kernels (conv_small.hip, fused
    head) graph-replayed, vs fp32 torch.nn; also with the query-batch conv off
    (row convs, split-K implicit GEMMs with and without the small-M tile/split
    policy, engine option igemm_small_m) and at batches 2-3."""
    model = build(arch, seed=17, randomize_bn=True)
    eng = InferenceEngine(arch, state_dict_f32(model), max_batch=B,
                          options={"igemm_small_m": bool(small_m), "small_conv": bool(small_conv)})
    g = torch.Generator().manual_seed(18)
    for _ in range(3):
        img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8)
        ref = _ref_logits(model, img)
        idx, prob, logits = eng.predict(img.to(gpu), return_logits=True)
        torch.cuda.synchronize()
        rel = ((logits.cpu() - ref).norm() / ref.norm()).item()
        assert rel < 3e-2, rel
        top2 = torch.softmax(ref, -1).topk(2, -1).values
        ok = (idx.cpu().long() == ref.argmax(-1)) | ((top2[:, 0] - top2[:, 1]) < 1e-2)
        assert torch.all(ok)


def test_engine_resnet50_fp8(gpu):
    """ResNet50 with layers 2-4 on the block-scaled e4m3 MFMA (per-channel
    weight scales, per-tensor activation scales calibrated at load) vs the
    fp32 reference on a calibrated (discriminating) model: e4m3 keeps 3
    mantissa bits, so the bar is looser than the bf16 engine's: logits within
    6% (relative L2) and top-1 agreement on all but near-ties."""
    model = calibrated("resnet50", seed=11)
    sd = state_dict_f32(model)
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=32)
    img = mixed_images(32, seed=12)
    ref = _ref_logits(model, img)
    idx, prob, logits = eng.predict(img.to(gpu), return_logits=True, use_graph=False)
    torch.cuda.synchronize()
    bar, agree = _fp8_bar(model, img)
    _assert_discriminating(logits, ref, bar, 12, idx=idx, prob=prob, what="resnet50_fp8 B=32", agree=agree)
    # graph replay gives the same answer
    i2, p2 = eng.predict(img.to(gpu), use_graph=True)
    assert torch.equal(i2.cpu(), idx.cpu())


@pytest.mark.parametrize("B,s2", [(16, False), (256, False), (256, True)])
def test_resnet50_fp8_3x3_e4m3_out(gpu, B, s2):
    """fp8_3x3_out: the bottleneck 3x3 convs write e4m3 (a calibrated
    per-tensor scale; the row / stream kernels' e4m3 epilogue at B = 256, the
    implicit GEMM at B = 16; s2: the strided ones too, on the implicit GEMM)
    and the expand convs read it on the e4m3 MFMA. Against fp32 on (up to)
    the first 32 images with the e4m3 bars of test_engine_resnet50_fp8, and at
    B = 256 against the engine with bf16 3x3 outputs: both within those bars
    of fp32, so within twice the bar of each other."""
    model = calibrated("resnet50", seed=11)
    sd = state_dict_f32(model)
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"fp8_3x3_out": True, "fp8_3x3_out_s2": s2})
    img = mixed_images(B, seed=31 + B)
    n = min(B, 32)
    idx, prob, logits = eng.predict(img.to(gpu), return_logits=True, use_graph=False)
    torch.cuda.synchronize()
    bar, agree = _fp8_bar(model, img, n)
    _assert_discriminating(logits[:n], _ref_logits(model, img[:n]), bar, 8, idx=idx[:n], prob=prob[:n],
                           what=f"fp8_3x3_out B={B} s2={s2} vs fp32", agree=agree)
    if B > 16:
        base = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"fp8_3x3_out": False})
        _, _, ref = base.predict(img.to(gpu), return_logits=True, use_graph=False)
        _assert_discriminating(logits, ref.cpu(), 2 * bar, 8, what=f"fp8_3x3_out B={B} s2={s2} vs bf16 3x3 out")
    i2, _ = eng.predict(img.to(gpu), use_graph=True)
    assert torch.equal(i2.cpu(), idx.cpu())


@pytest.mark.parametrize("B", [16, 64])
def test_resnet50_fp8_fused_head_matches_unfused(gpu, B):
    """The fused head reads ResNet50 e4m3's last activation directly (pool
    from e4m3 + dequantisation scale, fc, softmax/top-1) instead of three
    launches (fp8 avgpool, fc, softmax): pooled vectors bit-identical to the
    fp8 avgpool kernel's, the fc summed in another order, so logits agree to
    fp32 rounding; replayed twice (the combine tickets re-arm)."""
    model = build("resnet50", seed=13, randomize_bn=True)
    sd = state_dict_f32(model)
    ref_eng = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"fused_head": False})
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"fused_head": True})
    g = torch.Generator().manual_seed(70 + B)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    ri, rp, rl = ref_eng.predict(img, return_logits=True)
    for _ in range(2):
        i, p, lg = eng.predict(img, return_logits=True)
        torch.cuda.synchronize()
        assert torch.allclose(lg, rl, rtol=1e-4, atol=1e-4), (lg - rl).abs().max().item()
        top2 = torch.softmax(rl, -1).topk(2, -1).values
        assert torch.all((i == ri) | ((top2[:, 0] - top2[:, 1]) < 1e-5))
        assert torch.allclose(p, rp, rtol=1e-4, atol=1e-6)


def test_graph_replay_matches_eager(gpu):
    eng = InferenceEngine("resnet18", max_batch=32)
    img = torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=gpu)
    i0, p0 = eng.predict(img, use_graph=False)
    i1, p1 = eng.predict(img, use_graph=True)
    i2, p2 = eng.predict(img, use_graph=True)  # replay
    torch.cuda.synchronize()
    assert torch.equal(i0, i1) and torch.equal(i1, i2)
    assert torch.equal(p1, p2)


def test_batch_independence(gpu):
    """A sample's result does not depend on the batch it is in (no cross-
    sample leakage through tiling / split-K)."""
    eng = InferenceEngine("resnet18", max_batch=64)
    img = torch.randint(0, 256, (64, 224, 224, 3), dtype=torch.uint8, device=gpu)
    _, _, l_all = eng.predict(img, return_logits=True)
    _, _, l_one = eng.predict(img[5:6].contiguous(), return_logits=True)
    torch.cuda.synchronize()
    assert torch.allclose(l_all[5], l_one[0], rtol=2e-2, atol=2e-2)


def test_ot_checkpoint_engine(gpu, tmp_path):
    from dmlc.utils.ot import write_random_checkpoint
    p = write_random_checkpoint("alexnet", str(tmp_path / "alexnet.ot"), seed=3)
    e1 = InferenceEngine("alexnet", p, max_batch=4)
    e2 = InferenceEngine("alexnet", state_dict_f32(build("alexnet", seed=3)), max_batch=4)
    img = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device=gpu)
    a = e1.predict(img, return_logits=True)[2]
    b = e2.predict(img, return_logits=True)[2]
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("B", [1, 3, 6, 64, 256])
def test_fused_head_and_side_stream_match_unfused(gpu, B):
    """head.hip (avgpool+fc+softmax/top-1, split over classes with a ticketed
    last-arriver combine) and the downsample side-stream branch against the
    three-kernel single-stream path: pooled vectors are bit-identical, the fc
    sums in a different order, so logits agree to fp32 rounding; replayed
    twice to check the tickets re-arm."""
    model = build("resnet18", seed=21, randomize_bn=True)
    sd = state_dict_f32(model)
    ref_eng = InferenceEngine("resnet18", sd, max_batch=B, options={"fused_head": False, "fork_ds": False})
    eng = InferenceEngine("resnet18", sd, max_batch=B, options={"fused_head": True, "fork_ds": True})
    g = torch.Generator().manual_seed(B)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    ri, rp, rl = ref_eng.predict(img, return_logits=True)
    for _ in range(2):
        i, p, lg = eng.predict(img, return_logits=True)
        torch.cuda.synchronize()
        assert torch.allclose(lg, rl, rtol=1e-4, atol=1e-4), (lg - rl).abs().max().item()
        top2 = torch.softmax(rl, -1).topk(2, -1).values
        near_tie = (top2[:, 0] - top2[:, 1]) < 1e-5
        assert torch.all((i == ri) | near_tie)
        assert torch.allclose(p, rp, rtol=1e-4, atol=1e-6)


def test_engine_stream_path_matches_reference(gpu):
    """B=64 fills the CUs, so the engine takes the stream convs (fused
    downsample, register-weight layer4) that B=16 does not: vs fp32 torch."""
    model = build("resnet18", seed=13, randomize_bn=True)
    eng = InferenceEngine("resnet18", state_dict_f32(model), max_batch=64)
    g = torch.Generator().manual_seed(14)
    img = torch.randint(0, 256, (64, 224, 224, 3), generator=g, dtype=torch.uint8)
    ref = _ref_logits(model, img)
    idx, prob, logits = eng.predict(img.to(gpu), return_logits=True)
    torch.cuda.synchronize()
    rel = ((logits.cpu() - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel


def test_graph_replay_on_two_streams_is_ordered(gpu):
    """Direct graph replays share the activation arena: a replay on a second
    stream right after one on the first must not overlap it."""
    model = build("resnet18", seed=31)
    eng = InferenceEngine("resnet18", state_dict_f32(model), max_batch=8)
    g = torch.Generator().manual_seed(32)
    a = torch.randint(0, 256, (8, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    b = torch.randint(0, 256, (8, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    _, _, la = eng.predict(a, return_logits=True)
    _, _, lb = eng.predict(b, return_logits=True)
    torch.cuda.synchronize()
    la, lb = la.clone(), lb.clone()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(s1):
            _, _, xa = eng.predict(a, return_logits=True)
        with torch.cuda.stream(s2):
            _, _, xb = eng.predict(b, return_logits=True)
        torch.cuda.synchronize()
        assert torch.equal(xa, la) and torch.equal(xb, lb)


@pytest.mark.parametrize("B", [37, 100, 255])
def test_fast_paths_match_plain_paths_odd_batches(gpu, B):
    """Every fast path at odd batch sizes (partial image groups, partial head
    groups, row-conv strips that do not fill the CUs evenly) against the
    plain paths: register weights off, downsample unfused, three-kernel head."""
    model = build("resnet18", seed=41, randomize_bn=True)
    sd = state_dict_f32(model)
    plain = {k: False for k in ("stream_wreg", "rows_wreg", "fuse_ds", "fused_head", "fused_block", "fused_pool")}
    ref_eng = InferenceEngine("resnet18", sd, max_batch=B, options=plain)
    eng = InferenceEngine("resnet18", sd, max_batch=B)
    g = torch.Generator().manual_seed(B + 1)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    _, _, rl = ref_eng.predict(img, return_logits=True)
    i, p, lg = eng.predict(img, return_logits=True)
    torch.cuda.synchronize()
    rel = ((lg - rl).norm() / rl.norm()).item()
    # (accumulation order and bf16 activation rounding differ path by path:
    # 0.7-1e-3 in round 4, 2.0e-3 at B = 255 since the fused block and the row
    # convs start their accumulators from the bias; bf16's own step is 7.8e-3)
    assert rel < 5e-3, rel


@pytest.mark.parametrize("B", [3, 64, 256])
def test_alexnet_fused_stem_matches_unfused(gpu, B):
    """alex_stem.hip (u8 -> normalise -> conv 11x11/s4 + ReLU -> maxpool in
    one kernel) against the three-kernel path it replaces (preprocess_u8, the
    packed-RGB implicit GEMM, maxpool2d): the same bf16 math, so logits agree
    to accumulation-order rounding and top-1 is identical but for near-ties;
    and against fp32 torch.nn at B=3."""
    model = build("alexnet", seed=31)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(B)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8)
    x = img.to(gpu)
    ref_eng = InferenceEngine("alexnet", sd, max_batch=B, options={"fused_stem": False})
    eng = InferenceEngine("alexnet", sd, max_batch=B)
    ri, _, rl = ref_eng.predict(x, return_logits=True, use_graph=False)
    fi, _, fl = eng.predict(x, return_logits=True)
    torch.cuda.synchronize()
    rel = ((fl - rl).norm() / rl.norm()).item()
    assert rel < 1e-2, rel
    p = torch.softmax(rl.float().cpu(), -1)
    top2 = p.topk(2, -1).values
    near = (top2[:, 0] - top2[:, 1]) < 1e-2
    assert torch.all((fi.cpu() == ri.cpu()) | near)
    if B == 3:
        ref = _ref_logits(model, img)
        assert ((fl.cpu() - ref).norm() / ref.norm()).item() < 3e-2


@pytest.mark.parametrize("arch", ["resnet18", "alexnet", "resnet50_fp8"])
def test_bench_config_b256_matches_fp32(gpu, arch):
    """The exact bench.py configuration of each benchmarked model — B = 256,
    default kernel selection, hipGraph replay, two compute lanes (the second a
    copied engine on its own stream), primed pipeline, driven by the native DP
    runner (csrc/comm/runner.cpp) — on a calibrated (discriminating) model
    against fp32 torch.nn over all 256 images of a step on each lane: top-1
    and probabilities (the runner's answers) and the logits of the same
    graph-replayed forward, relative L2 within 3% (bf16) / 1.25x an ideal e4m3
    rounding of the same network (e4m3), with the rolled-batch and batch-mean
    negative controls failing that bar."""
    import dmlc
    model = calibrated(arch, seed=21)
    eng = InferenceEngine(arch, state_dict_f32(model), max_batch=256)
    img = mixed_images(512, seed=22)
    pool = img.to(gpu)
    torch.cuda.synchronize()
    r = dmlc.native().DpRunner(eng._e, 1, 0, b"", b"", 256, lanes=2)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    refs = [_ref_logits_chunked(model, img[k * 256:(k + 1) * 256]) for k in range(2)]
    bar, agree = _fp8_bar(model, img) if arch.endswith("_fp8") else (3e-2, 0.9)
    idx0, prob0, logits = eng.predict(pool[:256], return_logits=True)  # graph replay, same kernel paths
    torch.cuda.synchronize()
    _assert_discriminating(logits, refs[0], bar, 16, idx=idx0, prob=prob0, what=f"{arch} b256 logits", agree=agree)
    # prime as bench.py does (every slot's graph captured, both lanes used)
    r.run(pool.data_ptr(), 512, 0, 9)
    for first, batch in ((9, 1), (10, 0)):  # step 9: lane 1 on batch 1; step 10: lane 0 on batch 0
        r.run(pool.data_ptr(), 512, first, 1)
        r.sync()
        idx, prob = r.last_results()
        ref = refs[batch]
        n_cls, _ = discrimination(ref)
        assert n_cls >= 16, n_cls
        gap = ref.topk(2, -1).values
        idx = torch.tensor(idx).long()
        mism = idx != ref.argmax(-1)
        # (the logits of this batch are not returned by the runner: the near-tie
        # scale is the bar times the image's rms logit)
        near = (gap[:, 0] - gap[:, 1]) < 4 * bar * ref.pow(2).mean(-1).sqrt()
        print(f"{arch} step {first} (lane {first % 2}): top-1 mismatches {mism.sum().item()} "
              f"(near-ties {near.sum().item()})")
        assert torch.all(~mism | near), (first, mism.sum().item())
        assert (~mism).float().mean().item() > agree, (first, mism.sum().item())
        # the answers belong to their own images: against the other batch's reference they fail
        other = refs[1 - batch].argmax(-1)
        assert (idx == other).float().mean().item() < 0.5


def test_fused_pool_head_matches_unfused(gpu):
    """The last conv's fused global average pool + the pooled head (graph
    path: the layer4 activation is never stored) against the unfused
    avgpool+fc+softmax head: identical top-1, logits equal within bf16
    rounding of the pooled vector."""
    model = build("resnet18", seed=41, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(42)
    img = torch.randint(0, 256, (96, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    ref_eng = InferenceEngine("resnet18", sd, max_batch=96, options={"fused_pool": False})
    eng = InferenceEngine("resnet18", sd, max_batch=96)
    ri, rp, rl = ref_eng.predict(img, return_logits=True)
    fi, fp, fl = eng.predict(img, return_logits=True)  # graph replay: activation not stored
    i2, p2 = eng.predict(img)                           # the bench's graph (no logits output)
    torch.cuda.synchronize()
    rel = ((fl - rl).norm() / rl.norm()).item()
    assert rel < 1e-2, rel
    assert torch.equal(fi, ri) and torch.equal(i2, ri)
    assert torch.allclose(fp, rp, rtol=1e-2, atol=1e-4) and torch.allclose(p2, rp, rtol=1e-2, atol=1e-4)


def test_fused_block_matches_unfused(gpu):
    """ResNet18's layer1 blocks as one kernel each (conv3x3_block.hip) vs two
    row convs per block (options fused_block=False): same MFMA order and bf16
    intermediate; the fused block starts its accumulators from the bias and
    adds the residual by v_dot2c_f32_bf16 (rounding differently from the row
    convs' bias-after / unpacked-residual epilogue, which the kernel test pins
    bit for bit as variant 32), so the logits agree to bf16 rounding."""
    model = build("resnet18", seed=43, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(44)
    # (fused only once the batch fills >= 70% of the CUs: one image per workgroup)
    img = torch.randint(0, 256, (192, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    ref_eng = InferenceEngine("resnet18", sd, max_batch=192, options={"fused_block": False})
    eng = InferenceEngine("resnet18", sd, max_batch=192)
    ri, rp, rl = ref_eng.predict(img, return_logits=True)
    fi, fp, fl = eng.predict(img, return_logits=True)
    torch.cuda.synchronize()
    rel = ((fl.float() - rl.float()).norm() / rl.float().norm()).item()
    assert rel < 1e-2, rel
    assert (fi == ri).float().mean().item() > 0.95


@pytest.mark.parametrize("option", ["s2rows", "rows28", "ds_into_conv2"])
def test_weight_stationary_rows_match_stream(gpu, option):
    """ResNet18's layer2 convs as weight-stationary row-streaming kernels
    (s2rows: layer2.0 conv1 + downsample, conv3x3_s2rows.hip; rows28: the
    stride-1 convs, conv3x3_rows28.hip; ds_into_conv2: layer2.0's downsample
    as 2 more K steps of its conv2 instead of an s2rows output read back as
    the residual) vs the path with the option off: different accumulation
    order (and no bf16 rounding of the downsample output), so logits agree to
    bf16 rounding, not bit for bit."""
    model = build("resnet18", seed=45, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(46)
    img = torch.randint(0, 256, (192, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    ref_eng = InferenceEngine("resnet18", sd, max_batch=192, options={option: False})
    eng = InferenceEngine("resnet18", sd, max_batch=192)
    ri, _, rl = ref_eng.predict(img, return_logits=True)
    fi, _, fl = eng.predict(img, return_logits=True)
    torch.cuda.synchronize()
    rel = ((fl.float() - rl.float()).norm() / rl.float().norm()).item()
    assert rel < 2e-2, rel
    assert (fi == ri).float().mean().item() > 0.95


@pytest.mark.parametrize("B", [1, 5, 16])
def test_alexnet_small_batch_fc_matches_reference(gpu, B):
    """Query-sized AlexNet batches run the classifier on the weight-streaming
    split-K GEMV (fc_small.hip): vs fp32 torch.nn, and vs the throughput
    path (options fc_small=False: the implicit GEMM) on the same inputs."""
    model = build("alexnet", seed=51, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(52 + B)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8)
    eng = InferenceEngine("alexnet", sd, max_batch=B)
    idx, prob, logits = eng.predict(img.to(gpu), return_logits=True)
    i2, p2 = eng.predict(img.to(gpu))  # graph replay, no logits output
    ref_eng = InferenceEngine("alexnet", sd, max_batch=B, options={"fc_small": False})
    _, _, ref_gemm = ref_eng.predict(img.to(gpu), return_logits=True)
    torch.cuda.synchronize()
    ref = _ref_logits(model, img)
    rel = ((logits.cpu() - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    rel2 = ((logits - ref_gemm).norm() / ref_gemm.norm()).item()
    assert rel2 < 5e-3, rel2
    assert torch.equal(idx, i2) and torch.allclose(prob, p2)


@pytest.mark.parametrize("B", [5, 256])
def test_alexnet_direct13_matches_igemm(gpu, B):
    """AlexNet's 13x13 convs (features.6/.8/.10) and its 5x5 conv (features.3)
    on the LDS-resident direct convs (conv3x3_13.hip, conv5x5_27.hip) vs the
    implicit GEMM (direct13 / direct27 off): both bf16 MFMA
    with fp32 accumulation, different K order, so logits agree to bf16
    rounding; and vs fp32 torch.nn on a few images. The direct kernel is the
    one that ran: features.8 takes well under the implicit GEMM's time."""
    model = build("alexnet", seed=57, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(58 + B)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8)
    x = img.to(gpu)
    eng = InferenceEngine("alexnet", sd, max_batch=B)
    ref_eng = InferenceEngine("alexnet", sd, max_batch=B, options={"direct13": False, "direct27": False})
    fi, _, fl = eng.predict(x, return_logits=True)
    ri, _, rl = ref_eng.predict(x, return_logits=True)
    torch.cuda.synchronize()
    rel = ((fl - rl).norm() / rl.norm()).item()
    assert rel < 1e-2, rel
    p = torch.softmax(rl.float().cpu(), -1)
    top2 = p.topk(2, -1).values
    near = (top2[:, 0] - top2[:, 1]) < 1e-2
    assert torch.all((fi.cpu() == ri.cpu()) | near)
    n = min(B, 8)
    ref = _ref_logits(model, img[:n])
    assert ((fl[:n].cpu() - ref).norm() / ref.norm()).item() < 3e-2
    if B == 256:
        prof = dict(eng._e.profile(x.data_ptr(), B, 224, 224, 0))
        rprof = dict(ref_eng._e.profile(x.data_ptr(), B, 224, 224, 0))
        print("direct vs igemm (ms):",
              {k: (prof[k], rprof[k]) for k in ("features.3", "features.6", "features.8", "features.10")})
        assert prof["features.8"] < rprof["features.8"], (prof, rprof)
        assert prof["features.3"] < rprof["features.3"], (prof, rprof)


@pytest.mark.parametrize("arch", ["resnet50", "resnet50_fp8"])
def test_resnet50_downsample_in_expand_matches_separate(gpu, arch):
    """layer1.0's 1x1 downsample folded into its expand conv (one conv1x1
    GEMM over K = [conv2 output | block input] with weights [W3 | Wd], bias
    b3 + bd) vs the two convs + residual add (ds_into_expand off): the same
    products, the residual no longer rounded to the activation dtype first, so
    logits agree to that rounding; and the fused engine is the faster one on
    layer1.0."""
    model = build("resnet50", seed=63, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(64)
    img = torch.randint(0, 256, (64, 224, 224, 3), generator=g, dtype=torch.uint8)
    x = img.to(gpu)
    eng = InferenceEngine(arch, sd, max_batch=64)
    ref_eng = InferenceEngine(arch, sd, max_batch=64, options={"ds_into_expand": False})
    fi, _, fl = eng.predict(x, return_logits=True)
    ri, _, rl = ref_eng.predict(x, return_logits=True)
    torch.cuda.synchronize()
    # both against fp32 (the fp8 engine's activation scales are calibrated with
    # every activation materialised, whichever paths it runs), then each other
    ref = _ref_logits(model, img[:16])
    for lg in (fl, rl):
        r = ((lg[:16].float().cpu() - ref).norm() / ref.norm()).item()
        assert r < (0.15 if arch.endswith("fp8") else 3e-2), r
    rel = ((fl - rl).norm() / rl.norm()).item()
    assert rel < (5e-2 if arch.endswith("fp8") else 1e-2), rel
    p = torch.softmax(rl.float().cpu(), -1)
    top2 = p.topk(2, -1).values
    near = (top2[:, 0] - top2[:, 1]) < 5e-2
    if arch.endswith("fp8"):
        # e4m3 paths that differ in rounding points: a top-1 may flip where the
        # two leading logits are within a few times the per-image rms logit
        # difference of the two engines (large-logit random models make the
        # probability gap a poor tie measure)
        lg = rl.float().cpu()
        gap = lg.topk(2, -1).values
        rms = (fl.float().cpu() - lg).pow(2).mean(-1).sqrt()
        near = near | ((gap[:, 0] - gap[:, 1]) < 4 * rms)
    assert torch.all((fi.cpu() == ri.cpu()) | near)
    prof = dict(eng._e.profile(x.data_ptr(), 64, 224, 224, 0))
    rprof = dict(ref_eng._e.profile(x.data_ptr(), 64, 224, 224, 0))
    fused = prof["layer1.0.downsample.0"] + prof["layer1.0.conv3"]
    sep = rprof["layer1.0.downsample.0"] + rprof["layer1.0.conv3"]
    print(arch, "layer1.0 ds + conv3 (ms): fused", fused, "separate", sep)
    assert fused < 0.8 * sep  # (the skipped downsample op profiles at the ~5 us empty-op floor)


def test_resnet50_fp8_fused_bottleneck_matches_unfused(gpu):
    """resnet50_fp8's layer1 identity blocks (layer1.1, layer1.2) as one kernel
    each (bottleneck56.hip: conv1 e4m3 MFMA -> t1 in LDS -> conv2 -> t2 in LDS
    -> conv3 + residual -> e4m3) vs the three-kernel path (fused_bottleneck
    off): the same e4m3 / bf16 roundings, different accumulation order in
    conv2, so logits agree to a few e4m3 ulps, top-1 on all but near-ties; and
    the fused kernel is the one that ran (its conv2/conv3 ops take no time of
    their own in the per-op profile)."""
    model = build("resnet50", seed=61, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(62)
    img = torch.randint(0, 256, (32, 224, 224, 3), generator=g, dtype=torch.uint8)
    x = img.to(gpu)
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=32, options={"fused_bottleneck": True})
    ref_eng = InferenceEngine("resnet50_fp8", sd, max_batch=32, options={"fused_bottleneck": False})
    fi, fp, fl = eng.predict(x, return_logits=True, use_graph=False)
    gi, gp = eng.predict(x)
    ri, rp, rl = ref_eng.predict(x, return_logits=True, use_graph=False)
    torch.cuda.synchronize()
    rel = ((fl - rl).norm() / rl.norm()).item()
    assert rel < 5e-2, rel
    p = torch.softmax(rl.float().cpu(), -1)
    top2 = p.topk(2, -1).values
    near = (top2[:, 0] - top2[:, 1]) < 5e-2
    assert torch.all((fi.cpu() == ri.cpu()) | near)
    assert torch.equal(fi, gi)
    ref = _ref_logits(model, img[:8])
    assert ((fl[:8].cpu() - ref).norm() / ref.norm()).item() < 0.15
    prof = dict(eng._e.profile(x.data_ptr(), 32, 224, 224, 0))
    rprof = dict(ref_eng._e.profile(x.data_ptr(), 32, 224, 224, 0))
    # layer1.0's reduce + 3x3 run as one bottleneck56_head kernel in its conv1 op
    assert prof["layer1.0.conv2"] < 0.6 * rprof["layer1.0.conv2"], (prof, rprof)
    for blk in ("layer1.1", "layer1.2"):
        # (the fused path's conv3 op is an empty op at the ~5-7 us launch
        # floor; the unfused expand conv takes ~17 us at B = 32)
        assert prof[blk + ".conv3"] < 0.6 * rprof[blk + ".conv3"], (blk, prof, rprof)


@pytest.mark.parametrize("B", [4, 12, 32, 256])
def test_resnet50_fp8_chain_1x1_matches_unchained(gpu, B):
    """resnet50_fp8 layer2: each expand conv with the next bottleneck's reduce
    conv on its output in one launch (conv1x1_chain: the reduce reads the
    output blocks from LDS) vs two launches. Same MFMA instruction per 128-K
    step, same K order, same epilogue arithmetic: the logits are bit-identical;
    and the chained path is the one that ran (the reduce ops it absorbs take
    no kernel time of their own)."""
    model = build("resnet50", seed=71, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(72)
    x = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"chain_1x1": True})
    ref_eng = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"chain_1x1": False})
    ci, cp, cl = eng.predict(x, return_logits=True, use_graph=False)
    gi, gp = eng.predict(x)
    ri, rp, rl = ref_eng.predict(x, return_logits=True, use_graph=False)
    torch.cuda.synchronize()
    assert torch.equal(cl, rl), ((cl - rl).abs().max().item(), (rl.norm()).item())
    assert torch.equal(ci, ri) and torch.equal(ci, gi)
    if B < 32:  # (ragged persistent grids: workgroups with one block or none; timing is launch-bound)
        return
    prof = dict(eng._e.profile(x.data_ptr(), B, 224, 224, 0))
    rprof = dict(ref_eng._e.profile(x.data_ptr(), B, 224, 224, 0))
    for blk in ("layer2.1", "layer2.2", "layer2.3"):
        assert prof[blk + ".conv1"] < 0.6 * rprof[blk + ".conv1"], (blk, prof, rprof)


def test_unknown_engine_option_is_an_error(gpu):
    with pytest.raises(Exception, match="unknown engine option"):
        InferenceEngine("resnet18", max_batch=1, options={"no_such_path": True})


@pytest.mark.parametrize("B", [64, 256])
def test_resnet50_fp8_3x3_in_matches_bf16_in(gpu, B):
    """fp8_3x3_in: layer3/4's stride-1 bottleneck 3x3 convs read e4m3 t1
    (per-channel scales, written by the reduce 1x1) on conv3x3_stream8 vs the
    same engine with those convs on bf16 inputs (conv3x3_stream): one more
    e4m3 rounding per block, so the logits differ by a few percent and top-1
    agrees except on near-ties."""
    model = build("resnet50", seed=15, randomize_bn=True)
    sd = state_dict_f32(model)
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=B)
    base = InferenceEngine("resnet50_fp8", sd, max_batch=B, options={"fp8_3x3_in": False})
    g = torch.Generator().manual_seed(93 + B)
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    i, _, lg = eng.predict(img, return_logits=True)
    ri, _, rl = base.predict(img, return_logits=True)
    torch.cuda.synchronize()
    rel = ((lg - rl).norm() / rl.norm()).item()
    print(f"fp8_3x3_in B={B}: rel {rel:.4f} vs bf16 3x3 inputs")
    assert rel < 0.05, rel
    top2 = torch.softmax(rl.float(), -1).topk(2, -1).values
    assert torch.all((i == ri) | ((top2[:, 0] - top2[:, 1]) < 5e-2))
