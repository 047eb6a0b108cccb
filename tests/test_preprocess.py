"""On-GPU eval preprocessing: the CPU restatement (oracle/preprocess.py) is
pinned against Pillow itself (the library torchvision's Resize calls for PIL inputs; importable
here and on the GPU box), the host geometry against the oracle, and the HIP kernels against the
oracle - bit-exact (uint8 resampling, fp32 normalisation with the same correctly-rounded ops)."""
import numpy as np
import pytest
import torch

from oracle import preprocess as P

SHAPES = [(375, 500), (500, 375), (224, 224), (256, 300), (100, 80), (1000, 37), (257, 256), (256, 256),
          (640, 480), (333, 1111), (50, 50), (37, 1000), (480, 640)]


def _images(shapes, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i, (h, w) in enumerate(shapes):
        if i % 2:
            out.append(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
        else:  # smooth gradients + noise: exercises the rounding of nearly-equal taps
            y, x = np.mgrid[0:h, 0:w]
            base = np.stack([x * 255.0 / max(w - 1, 1), y * 255.0 / max(h - 1, 1), (x + y) % 256], -1)
            out.append(np.clip(base + rng.normal(0, 3, base.shape), 0, 255).astype(np.uint8))
    return out


def _pil_transform(img, mode):
    """The reference pipeline with Pillow doing the resize (scripts/_io.py restates torchvision)."""
    from PIL import Image

    from scripts import _io

    im = Image.fromarray(img)
    im = _io.center_crop(_io.resize_shorter(im, 256), 224) if mode == "crop" else im.resize((224, 224), Image.BILINEAR)
    return _io.to_normalized_tensor(im).numpy()


@pytest.mark.parametrize("mode", ["crop", "square"])
def test_oracle_matches_pillow(mode):
    pytest.importorskip("PIL")
    for img in _images(SHAPES):
        assert np.array_equal(P.preprocess(img, mode), _pil_transform(img, mode)), img.shape


def test_host_geometry_matches_oracle():
    from image_caption_amd.preprocess import geometry

    for h, w in SHAPES:
        g = geometry(h, w, "crop")
        assert (g[2], g[3]) == P.resized_size(h, w, 256)
        assert (g[4], g[5]) == P.crop_offsets(g[2], g[3], 224)
        if g[2] != h:  # the source-row window covers exactly the taps of the kept rows
            xmin, n, _ = P.resample_coeffs(h, g[2])
            rows = slice(g[4], g[4] + 224)
            assert g[6] == xmin[rows].min() and g[6] + g[7] == (xmin + n)[rows].max()
        gs = geometry(h, w, "square")
        assert gs[:6] == [h, w, 224, 224, 0, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["crop", "square"])
def test_gpu_preprocess_bit_exact_ragged_batch(mode):
    from image_caption_amd.preprocess import preprocess_batch

    imgs = _images(SHAPES, seed=3)
    got = preprocess_batch(imgs, mode, device="cuda").cpu().numpy()
    ref = P.preprocess_batch(imgs, mode)
    assert got.shape == (len(imgs), 3, 224, 224)
    assert np.array_equal(got, ref)
    one = preprocess_batch(imgs[5:6], mode, device="cuda").cpu().numpy()  # batch independence
    assert np.array_equal(one[0], ref[5])


@pytest.mark.gpu
def test_gpu_preprocess_feeds_encoder(cuda):
    """uint8 images -> HIP preprocessing -> HIP ViT encoder == oracle preprocessing -> oracle encoder."""
    from image_caption_amd import weights as W
    from image_caption_amd.engine import Engine
    from image_caption_amd.preprocess import preprocess_batch
    from oracle import captioner as O

    sd = W.to_torch(W.vit_state_dict(0))
    imgs = _images([(375, 500), (480, 640)], seed=5)
    x = preprocess_batch(imgs, "crop", device=cuda)
    mem = Engine(sd, "vit", {}, device=cuda).encode(x)
    ref = O.vit_encode(sd, torch.from_numpy(P.preprocess_batch(imgs, "crop")))
    assert (mem.cpu() - ref).abs().max().item() < 4e-3  # f16 encoder (default): fp16 operands
