"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own code.

Runs in the build container only (needs /root/reference, read-only); the fixtures it writes are
plain data (npz: inputs' seeds + outputs) and are what travels.  Weights and images come from the
seeded generator image_caption_amd/weights.py, so any machine can regenerate the inputs.

What is the reference's own code here (imported by file path from /root/reference):
  * models/vit_transformer_model.py: TransformerDecoder (vit:103-182), VisionTransformerEncoder
    .forward (vit:71-100), ViTTransformerCaptioning.generate/_greedy_search (vit:276-325).
What is restated because its module cannot import here:
  * torchvision's ViT-B/16 trunk (absent) -> models/_vision.VisionTransformer, pinned against
    HF transformers.ViTModel by tests/test_oracle.py;
  * models/grid_transformer_model.py imports torchvision at module top (grid:8): the Grid golden
    uses the reference decoder + greedy loop (grid:230-251 is the same algorithm as vit:296-325)
    over GridFeatureEncoder from models/ (torch path), whose ResNet-101 is pinned against HF
    ResNetModel;
  * scripts/inference.py (imports torchvision.transforms) and utils/scst_loss.py (imports
    pycocoevalcap): their decode loops (inference.py:75-99, scst_loss:220-249) are restated here
    around the reference decoder module, with torch.multinomial replaced by inverse-CDF sampling
    on fixed uniforms.

Usage: python tests/golden/make_golden.py [beam_vit|forward]   (writes tests/golden/*.npz, ~2 min on
       8 cores; with beam_vit / forward only that fixture)
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from image_caption_amd import weights as W  # noqa: E402

REF = "/root/reference"
END_BIAS = 1.4  # <end> logit offset of the beam-search fixtures (makes beams finish early)


def load_ref_vit_module():
    spec = importlib.util.spec_from_file_location("ref_vit_transformer_model",
                                                  os.path.join(REF, "models", "vit_transformer_model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ref_decoder(ref, sd, max_len=100):
    dec = ref.TransformerDecoder(W.VOCAB_SIZE, max_len=max_len)
    dec.load_state_dict({k[len("decoder."):]: v for k, v in sd.items() if k.startswith("decoder.")}, strict=True)
    return dec.eval()


def ref_vit_model(ref, sd):
    """The reference ViTTransformerCaptioning with its own encoder/decoder classes; only the
    torchvision trunk object inside VisionTransformerEncoder is the build's restatement."""
    from models._vision import VisionTransformer

    enc = ref.VisionTransformerEncoder.__new__(ref.VisionTransformerEncoder)
    nn.Module.__init__(enc)
    enc.vit = VisionTransformer()
    enc.vit.heads = nn.Identity()
    enc.projection = nn.Linear(768, 512)
    model = ref.ViTTransformerCaptioning.__new__(ref.ViTTransformerCaptioning)
    nn.Module.__init__(model)
    model.vocab_size, model.d_model = W.VOCAB_SIZE, 512
    model.encoder = enc
    model.decoder = ref.TransformerDecoder(W.VOCAB_SIZE, max_len=100)
    model.load_state_dict(sd, strict=True)
    return model.eval()


def teacher_forced(dec, memory, ids):
    T = ids.shape[1] - 1
    with torch.no_grad():
        return dec(ids[:, :-1], memory, tgt_mask=dec.generate_square_subsequent_mask(T, "cpu"))


def decoder_ops_memory() -> np.ndarray:
    """The (3,196,512) memory of decoder_ops.npz, regenerated from its seed (not stored)."""
    return np.random.Generator(np.random.PCG64(8)).standard_normal((3, 196, 512)).astype(np.float32)


def top2(logits):
    t = logits.topk(2, dim=-1).values
    return (t[..., 0] - t[..., 1]).numpy()


def make_beam(ref, sd, imgs, out):
    # (vi) beam search through the reference's OWN ViTTransformerCaptioning._beam_search (vit:327-420),
    # one image per call as the reference loops: default weights (beam 3, images 0-1, no beam ever
    # ends) and the same weights with the <end> logit raised by END_BIAS (beam 5, images 0-3: beams
    # finish, are collected and pruned).  The oracle's selection margin is stored with each case.
    from oracle import captioner as O

    cases = [(0.0, 3, i) for i in range(2)] + [(END_BIAS, 5, i) for i in range(4)]
    rows, lens, margins = [], [], []
    for delta, k, i in cases:
        sdb = dict(sd)
        fb = sdb["decoder.fc_out.bias"].clone()
        fb[W.END_TOKEN] += delta
        sdb["decoder.fc_out.bias"] = fb
        mb = ref_vit_model(ref, sdb)
        with torch.no_grad():
            seq = mb.generate(imgs[i:i + 1], W.START_TOKEN, W.END_TOKEN, max_len=30, method="beam_search")
            if k != 5:  # generate() fixes beam_size=5 for the ViT model (vit:292); other widths go direct
                seq = mb._beam_search(imgs[i:i + 1], W.START_TOKEN, W.END_TOKEN, 30, k)
            _, margin = O.beam_from_memory(sdb, mb.encoder(imgs[i:i + 1]), W.START_TOKEN, W.END_TOKEN, 30, k,
                                           False, return_margins=True)
        row = np.full(30, -1, dtype=np.int64)
        row[: seq.shape[1]] = seq[0].numpy()
        rows.append(row)
        lens.append(seq.shape[1])
        margins.append(margin)
    np.savez_compressed(os.path.join(HERE, "beam_vit.npz"), end_bias=np.array([c[0] for c in cases]),
                        beam=np.array([c[1] for c in cases]), image=np.array([c[2] for c in cases]),
                        ids=np.stack(rows), lengths=np.array(lens), margins=np.array(margins))
    out["beam_vit"] = (len(cases),)


def make_forward(ref, out):
    # (vii) teacher-forced training forward with padding masks: the reference's OWN
    # ViTTransformerCaptioning.forward (vit:216-255, padding from caption_lengths) and the Grid form
    # (grid:185-207: padding from caption_lengths - 1, restated around the reference decoder and its
    # own _generate_padding_mask, since grid_transformer_model.py imports torchvision).  Lengths cover
    # a full row, a partial one, 1, 0 (every key masked) and, for Grid, -1 (mask[i, -1:] slicing).
    from models.grid_transformer_model import GridFeatureEncoder

    imgs = torch.from_numpy(W.synthetic_images(4, seed=0))
    rng = np.random.Generator(np.random.PCG64(11))
    caps = rng.integers(0, W.VOCAB_SIZE, size=(4, 17)).astype(np.int64)
    caps[:, 0] = W.START_TOKEN
    captions = torch.from_numpy(caps)
    vit_len = [17, 9, 1, 0]
    model = ref_vit_model(ref, W.to_torch(W.vit_state_dict(0)))
    with torch.no_grad():
        vit_logits = model(imgs, captions, vit_len)
    gsd = W.to_torch(W.grid_state_dict(0))
    genc = GridFeatureEncoder(pretrained_cnn=False)
    genc.load_state_dict({k[len("encoder."):]: v for k, v in gsd.items() if k.startswith("encoder.")}, strict=True)
    gdec = ref_decoder(ref, gsd)
    grid_len = [17, 9, 2, 0]
    with torch.no_grad():
        gmem = genc.eval()(imgs)
        tgt = captions[:, :-1]
        pad = ref.ViTTransformerCaptioning._generate_padding_mask(None, tgt, [l - 1 for l in grid_len])
        grid_logits = gdec(tgt, gmem, tgt_mask=gdec.generate_square_subsequent_mask(tgt.size(1), "cpu"),
                           tgt_key_padding_mask=pad)
    np.savez_compressed(os.path.join(HERE, "forward_b4.npz"), captions=caps, vit_lengths=np.array(vit_len),
                        grid_lengths=np.array(grid_len), vit_logits=vit_logits.numpy(),
                        grid_logits=grid_logits.numpy())
    out["forward_b4"] = vit_logits.shape


def main():
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count() or 8)
    ref = load_ref_vit_module()
    out = {}
    if sys.argv[1:] == ["forward"]:  # regenerate only the training-forward fixture
        make_forward(ref, out)
        print(out)
        return
    if sys.argv[1:] == ["beam_vit"]:  # regenerate only the beam fixture
        make_beam(ref, W.to_torch(W.vit_state_dict(0)), torch.from_numpy(W.synthetic_images(4, seed=0)), out)
        print(out)
        return

    # (i)/(ii) ViT config-1: B=4, greedy max_len=30 through the reference generate()
    sd = W.to_torch(W.vit_state_dict(0))
    model = ref_vit_model(ref, sd)
    imgs = torch.from_numpy(W.synthetic_images(4, seed=0))
    with torch.no_grad():
        mem = model.encoder(imgs)
        ids = model.generate(imgs, W.START_TOKEN, W.END_TOKEN, max_len=30, method="greedy")
    tf = teacher_forced(model.decoder, mem, ids)
    np.savez_compressed(os.path.join(HERE, "vit_b4.npz"), weights_seed=0, image_seed=0, max_len=30,
                        ids=ids.numpy().astype(np.int64), memory_head=mem[:, :4, :16].numpy(),
                        memory_sum=mem.double().sum(dim=(1, 2)).numpy(), logits_tf=tf.numpy(),
                        margins=top2(tf))
    out["vit_b4"] = ids.shape

    # (iii) decoder forward on fixed tokens: causal and unmasked (inference.py:79 form)
    rng = np.random.Generator(np.random.PCG64(7))
    tgt = torch.from_numpy(rng.integers(0, W.VOCAB_SIZE, size=(3, 9)).astype(np.int64))
    memx = torch.from_numpy(decoder_ops_memory())
    dec = ref_decoder(ref, sd)
    with torch.no_grad():
        causal = dec(tgt, memx, tgt_mask=dec.generate_square_subsequent_mask(9, "cpu"))
        nomask = dec(tgt, memx)
    np.savez_compressed(os.path.join(HERE, "decoder_ops.npz"), tgt=tgt.numpy(), memory_seed=8,
                        logits_causal=causal.numpy(), logits_nomask=nomask.numpy())
    out["decoder_ops"] = causal.shape

    # scripts/inference.py loop (no causal mask, B=1, max_len=20) around the reference decoder
    nm_ids = []
    with torch.no_grad():
        inputs = torch.tensor([[W.START_TOKEN]])
        for _ in range(20):
            pid = int(dec(inputs, mem[:1])[:, -1, :].max(1)[1].item())
            if pid == W.END_TOKEN:
                break
            nm_ids.append(pid)
            inputs = torch.cat([inputs, torch.tensor([[pid]])], dim=1)
    np.savez_compressed(os.path.join(HERE, "nomask_b1.npz"), ids=np.array(nm_ids, dtype=np.int64))
    out["nomask_b1"] = len(nm_ids)

    # (v) sampled decode with fixed uniforms (scst_loss:220-249 loop, inverse-CDF draw)
    u = torch.from_numpy(np.random.Generator(np.random.PCG64(11)).random((29, 4)).astype(np.float32))
    B = 4
    generated = torch.full((B, 1), W.START_TOKEN, dtype=torch.long)
    finished = torch.zeros(B, dtype=torch.bool)
    lps = []
    with torch.no_grad():
        for step in range(29):
            logits = dec(generated, mem, tgt_mask=dec.generate_square_subsequent_mask(generated.size(1), "cpu"))[:, -1]
            probs = torch.softmax(logits, -1)
            cdf = probs.cumsum(-1)
            nxt = (cdf <= u[step].unsqueeze(-1) * cdf[:, -1:]).sum(-1).clamp_max(W.VOCAB_SIZE - 1)
            lps.append(torch.log_softmax(logits, -1).gather(1, nxt.unsqueeze(1)).squeeze(1).masked_fill(finished, 0.0))
            generated = torch.cat([generated, nxt.unsqueeze(1)], dim=1)
            finished = finished | (nxt == W.END_TOKEN)
            if bool(finished.all()):
                break
    np.savez_compressed(os.path.join(HERE, "sample_b4.npz"), uniforms=u.numpy(), ids=generated.numpy(),
                        log_probs=torch.stack(lps, 1).numpy())
    out["sample_b4"] = generated.shape

    # (iv) Grid: reference greedy loop + decoder over the build's GridFeatureEncoder (torch path)
    from models.grid_transformer_model import GridFeatureEncoder

    gsd = W.to_torch(W.grid_state_dict(0))
    genc = GridFeatureEncoder(pretrained_cnn=False)
    genc.load_state_dict({k[len("encoder."):]: v for k, v in gsd.items() if k.startswith("encoder.")}, strict=True)
    genc.eval()
    gmodel = ref.ViTTransformerCaptioning.__new__(ref.ViTTransformerCaptioning)
    nn.Module.__init__(gmodel)
    gmodel.vocab_size, gmodel.d_model = W.VOCAB_SIZE, 512
    gmodel.encoder = genc
    gmodel.decoder = ref_decoder(ref, gsd)
    with torch.no_grad():
        gmem = genc(imgs)
        gids = gmodel.generate(imgs, W.START_TOKEN, W.END_TOKEN, max_len=30, method="greedy")
    gtf = teacher_forced(gmodel.decoder, gmem, gids)
    np.savez_compressed(os.path.join(HERE, "grid_b4.npz"), weights_seed=0, image_seed=0, max_len=30,
                        ids=gids.numpy(), memory_sum=gmem.double().sum(dim=(1, 2)).numpy(),
                        memory_head=gmem[:, :4, :16].numpy(), logits_tf=gtf.numpy(), margins=top2(gtf))
    out["grid_b4"] = gids.shape
    make_beam(ref, sd, imgs, out)
    make_forward(ref, out)
    for k, v in out.items():
        print(k, tuple(v) if hasattr(v, "__len__") else v)


if __name__ == "__main__":
    main()
