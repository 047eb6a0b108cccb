"""Drop-in `scripts/inference_grid_transformer.py` (reference of the same path): Grid+Transformer
checkpoint loading and captioning; Resize((224,224)) preprocessing (ref :41-49), beam_size
passed through (ref :52-76).  COCO metric evaluation is outside the hot path."""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from models.grid_transformer_model import build_model  # noqa: E402
from models._common import decode_ids  # noqa: E402
from scripts._io import default_vocab_path, load_checkpoint, load_vocab, preprocess, preprocess_to_device  # noqa: E402


def load_model(checkpoint_path, device="cuda"):
    ckpt = load_checkpoint(checkpoint_path, device)
    config = dict(ckpt.get("config", {}))
    vocab = load_vocab(config.get("vocab_path", default_vocab_path()))
    model = build_model(len(vocab), dict(config, pretrained_cnn=False))
    model.load_state_dict(ckpt["model_state_dict"])
    model = model.to(device)
    model.eval()
    return model, vocab, config


def preprocess_image(image_path, image_size=224):
    return preprocess(image_path, "square", image_size).unsqueeze(0)


def generate_caption(model, image_path, vocab, device="cuda", method="greedy", max_len=50, beam_size=5):
    image = preprocess_to_device([image_path], "square", device)
    with torch.no_grad():
        ids = model.generate(image, start_token=vocab["<start>"], end_token=vocab["<end>"], max_len=max_len,
                             method=method, beam_size=beam_size)
    idx2word = {i: w for w, i in vocab.items()}
    row = ids[0].cpu().tolist()
    return decode_ids([row], idx2word, vocab["<end>"], vocab["<pad>"], vocab["<start>"])[0], row


def main():
    ap = argparse.ArgumentParser(description="Grid+Transformer captioning (MI355X HIP path on GPU)")
    ap.add_argument("images", nargs="+")
    ap.add_argument("--checkpoint", default="checkpoints/grid_transformer/best_model.pth")
    ap.add_argument("--method", default="greedy", choices=["greedy", "beam_search"])
    ap.add_argument("--beam-size", type=int, default=5)
    args = ap.parse_args()
    device = "cuda" if torch.cuda.is_available() else "cpu"
    model, vocab, _ = load_model(args.checkpoint, device)
    for p in args.images:
        print(f"{os.path.basename(p)}: {generate_caption(model, p, vocab, device, args.method, beam_size=args.beam_size)[0]}")


if __name__ == "__main__":
    main()
