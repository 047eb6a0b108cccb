"""Drop-in `scripts/inference.py`: single-image CLI with its own greedy loop (reference
scripts/inference.py:60-101).  Semantics kept: NO causal mask (the prefix attends
bidirectionally, :79), at most max_len steps, stop at <end> without emitting it, one host sync
per step.  On a GPU each `model.decoder(inputs, features)` call runs the HIP full-prefix
decoder (icap_decoder_forward with causal=0)."""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from models.vit_transformer_model import build_model  # noqa: E402
from scripts._io import load_checkpoint, load_vocab, preprocess  # noqa: E402


def load_model(checkpoint_path, vocab_path, device):
    ckpt = load_checkpoint(checkpoint_path, device)
    config = dict(ckpt["config"])
    vocab = load_vocab(vocab_path)
    model = build_model(len(vocab), dict(config, pretrained_vit=False))
    model.load_state_dict(ckpt["model_state_dict"])
    model = model.to(device)
    model.eval()
    return model, vocab, config


def preprocess_image(image_path):
    return preprocess(image_path, "square", 224)


def generate_caption(model, image, vocab, device, max_len=50):
    idx2word = {v: k for k, v in vocab.items()}
    image = image.unsqueeze(0).to(device)
    words = []
    with torch.no_grad():
        features = model.encoder(image)
        inputs = torch.tensor([[vocab["<start>"]]], device=device)
        for _ in range(max_len):
            pid = int(model.decoder(inputs, features)[:, -1, :].max(1)[1].item())
            if pid == vocab["<end>"]:
                break
            w = idx2word.get(pid, "<unk>")
            if w not in ("<start>", "<pad>"):
                words.append(w)
            inputs = torch.cat([inputs, torch.tensor([[pid]], device=device)], dim=1)
    return " ".join(words)


def main():
    ap = argparse.ArgumentParser(description="Image Captioning Inference")
    ap.add_argument("--image", type=str, required=True)
    ap.add_argument("--model", type=str, default="checkpoints/vit_transformer/best_model.pth")
    ap.add_argument("--vocab", type=str, default="data/vocab.json")
    args = ap.parse_args()
    if not os.path.exists(args.image):
        print(f"image not found: {args.image}")
        return
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model, vocab, _ = load_model(args.model, args.vocab, device)
    print(generate_caption(model, preprocess_image(args.image), vocab, device))


if __name__ == "__main__":
    main()
