"""Drop-in `scripts/inference_vit_transformer.py`: load a ViT+Transformer checkpoint and caption
images (reference: scripts/inference_vit_transformer.py).  Images on a GPU run the HIP engine.
`batch_generate_captions` batches all images into one `generate` call (the reference loops one
image at a time, :175); captions are identical because each image's tokens up to its first
<end> do not depend on the rest of the batch.  COCO metric evaluation (pycocoevalcap / Java
METEOR) is outside the hot path and not provided.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from models.vit_transformer_model import build_model  # noqa: E402
from models._common import decode_ids  # noqa: E402
from scripts._io import default_vocab_path, load_checkpoint, load_vocab, preprocess, preprocess_to_device  # noqa: E402


def load_model(checkpoint_path, device="cuda"):
    """Checkpoint dict {model_state_dict, config, ...} -> (model, vocab, config) (ref :20-62)."""
    ckpt = load_checkpoint(checkpoint_path, device)
    config = dict(ckpt.get("config", {}))
    vocab = load_vocab(config.get("vocab_path", default_vocab_path()))
    model = build_model(len(vocab), dict(config, pretrained_vit=False))
    model.load_state_dict(ckpt["model_state_dict"])
    model = model.to(device)
    model.eval()
    return model, vocab, config


def preprocess_image(image_path, image_size=224):
    """Resize(256) + CenterCrop(224) + ToTensor + Normalize -> (1,3,224,224) (ref :65-85)."""
    return preprocess(image_path, "crop", image_size).unsqueeze(0)


def _captions(model, images, vocab, method, max_len):
    with torch.no_grad():
        ids = model.generate(images, start_token=vocab["<start>"], end_token=vocab["<end>"], max_len=max_len,
                             method=method)
    idx2word = {i: w for w, i in vocab.items()}
    return decode_ids(ids.cpu(), idx2word, vocab["<end>"], vocab["<pad>"], vocab["<start>"]), ids.cpu().tolist()


def generate_caption(model, image_path, vocab, device="cuda", method="greedy", max_len=50):
    """One image -> (caption, ids) (ref :88-129)."""
    caps, ids = _captions(model, preprocess_image(image_path).to(device), vocab, method, max_len)
    return caps[0], ids[0]


def batch_generate_captions(model, image_paths, vocab, device="cuda", method="greedy", max_len=50):
    """Many images -> captions, batched into one generate call for greedy (ref :158-180)."""
    if method != "greedy":
        return [generate_caption(model, p, vocab, device, method, max_len)[0] for p in image_paths]
    imgs = preprocess_to_device(image_paths, "crop", device)
    caps, _ = _captions(model, imgs, vocab, method, max_len)
    for p, c in zip(image_paths, caps):
        print(f"  {os.path.basename(p)}: {c}")
    return caps


def main():
    ap = argparse.ArgumentParser(description="ViT+Transformer captioning (MI355X HIP path on GPU)")
    ap.add_argument("images", nargs="+")
    ap.add_argument("--checkpoint", default="checkpoints/vit_transformer/best_model.pth")
    ap.add_argument("--method", default="greedy", choices=["greedy", "beam_search"])
    ap.add_argument("--max-len", type=int, default=50)
    args = ap.parse_args()
    device = "cuda" if torch.cuda.is_available() else "cpu"
    model, vocab, _ = load_model(args.checkpoint, device)
    batch_generate_captions(model, args.images, vocab, device, args.method, args.max_len)


if __name__ == "__main__":
    main()
