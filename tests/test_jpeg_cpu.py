"""Host JPEG decoder (csrc/runtime/jpeg.cpp) against PIL (libjpeg-turbo) on
images encoded with every chroma layout the fast colour path handles (4:4:4,
4:2:2, 4:2:0) and widths that leave AVX2 tails and odd chroma edges. The
reference decodes its query images with tch's imagenet loader (a libjpeg
decode, src/services.rs:485-490); PIL is the libjpeg decode available here."""
import io

import numpy as np
import pytest

import dmlc

PIL = pytest.importorskip("PIL.Image")


def _jpeg(w, h, subsampling, seed):
    rng = np.random.default_rng(seed)
    # smooth colour gradients + noise: realistic chroma, every code path busy
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([128 + 100 * np.sin(xx / 17 + c) * np.cos(yy / 23 - c) for c in range(3)], -1)
    img = np.clip(img + rng.normal(0, 12, img.shape), 0, 255).astype(np.uint8)
    buf = io.BytesIO()
    PIL.fromarray(img).save(buf, "JPEG", quality=90, subsampling=subsampling)
    return buf.getvalue()


# (tiny images with subsampled chroma differ more: libjpeg blends the bottom
# chroma edge with its padded rows, this decoder clamps to the valid ones)
@pytest.mark.parametrize("w,h", [(500, 375), (17, 9), (33, 34), (224, 224), (7, 19), (2, 2)])
@pytest.mark.parametrize("subsampling", [0, 1, 2])  # 4:4:4, 4:2:2, 4:2:0
def test_decode_matches_pil(w, h, subsampling):
    data = _jpeg(w, h, subsampling, seed=w * 7 + h)
    ours = np.asarray(dmlc.native().decode_jpeg(data)).astype(np.int32)
    ref = np.asarray(PIL.open(io.BytesIO(data)).convert("RGB")).astype(np.int32)
    assert ours.shape == ref.shape == (h, w, 3)
    diff = np.abs(ours - ref)
    # float AAN IDCT vs libjpeg's integer IDCT: +-1-2 LSB here and there
    assert diff.mean() < 0.6, diff.mean()
    assert diff.max() <= 8, diff.max()
