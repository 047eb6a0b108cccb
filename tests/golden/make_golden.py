"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own code.

Runs in the build container only (needs /root/reference, read-only); the fixtures it writes are
plain data (npz: inputs' seeds + outputs) and are what travels.  Weights and images come from the
seeded generator image_caption_amd/weights.py, so any machine can regenerate the inputs.

Every loop below is the reference's own code, imported by file path from /root/reference:
  * models/vit_transformer_model.py: TransformerDecoder (vit:103-182), VisionTransformerEncoder
    .forward (vit:71-100), ViTTransformerCaptioning.generate / _greedy_search / _beam_search / forward
    (vit:216-420);
  * models/grid_transformer_model.py: GridTransformerCaptioning with its GridFeatureEncoder.forward
    (grid:86-110), generate / _greedy_search / _beam_search (grid:222-322) and forward (grid:185-210);
  * utils/scst_loss.py: SCSTLoss._sample_with_log_probs (scst_loss:202-254), with torch.multinomial
    replaced by an inverse-CDF draw on fixed uniforms for the duration of the call;
  * scripts/inference.py: generate_caption (inference.py:60-101, the no-mask loop).
Third-party modules absent from this image are replaced by import-only stand-ins, visible only while
the reference module executes (sys.modules is restored afterwards):
  * torchvision.models (grid:8, vit:8): resnet101 / vit_b_16 / *_Weights from models/_vision.py, the
    build's restatement of the torchvision architectures (pinned against HF transformers' ViTModel /
    ResNetModel by tests/test_oracle.py);
  * torchvision.transforms (inference.py:6): names only, never called (generate_caption takes a tensor);
  * pycocoevalcap.cider / .bleu (scst_loss:16-17): classes whose construction is a no-op and whose
    compute_score raises - the sampler never scores.

Usage: python tests/golden/make_golden.py [beam_vit|forward|grid|sample]   (writes tests/golden/*.npz,
       ~3 min on 8 cores; with an argument only that fixture)
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from image_caption_amd import weights as W  # noqa: E402
from tests.golden.inputs import decoder_ops_memory  # noqa: E402,F401

REF = "/root/reference"
END_BIAS = 1.4  # <end> logit offset of the beam-search fixtures (makes beams finish early)


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    return m


def _shims():
    """Import-only stand-ins for the third-party modules the reference imports at module top."""
    from models import _vision

    class _Scorer:  # pycocoevalcap Cider / Bleu: constructible, never used by the sampler
        def __init__(self, *a, **k):
            pass

        def compute_score(self, *a, **k):
            raise RuntimeError("pycocoevalcap is absent: the golden script never scores")

    class _T:  # torchvision.transforms names (inference.py:6), never called by generate_caption
        def __init__(self, *a, **k):
            raise RuntimeError("torchvision.transforms is absent")

    tv_models = _module("torchvision.models", resnet101=_vision.resnet101, ResNet101_Weights=_vision.ResNet101_Weights,
                        vit_b_16=_vision.vit_b_16, ViT_B_16_Weights=_vision.ViT_B_16_Weights)
    tv_transforms = _module("torchvision.transforms", Compose=_T, Resize=_T, ToTensor=_T, Normalize=_T,
                            CenterCrop=_T)
    cider = _module("pycocoevalcap.cider.cider", Cider=_Scorer)
    bleu = _module("pycocoevalcap.bleu.bleu", Bleu=_Scorer)
    return {
        "torchvision": _module("torchvision", models=tv_models, transforms=tv_transforms),
        "torchvision.models": tv_models, "torchvision.transforms": tv_transforms,
        "pycocoevalcap": _module("pycocoevalcap"), "pycocoevalcap.cider": _module("pycocoevalcap.cider", cider=cider),
        "pycocoevalcap.cider.cider": cider, "pycocoevalcap.bleu": _module("pycocoevalcap.bleu", bleu=bleu),
        "pycocoevalcap.bleu.bleu": bleu,
    }


def load_ref(relpath, name, extra_modules=None):
    """Execute the reference file /root/reference/<relpath> as module `name`, with the shims (and
    `extra_modules`) in sys.modules only while it executes."""
    inject = dict(_shims(), **(extra_modules or {}))
    saved = {k: sys.modules.get(k) for k in inject}
    saved_path = list(sys.path)
    sys.modules.update(inject)
    try:
        spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
        sys.path[:] = saved_path
    return mod


def load_ref_vit_module():
    return load_ref("models/vit_transformer_model.py", "ref_vit_transformer_model")


def ref_grid_model(sd):
    """The reference GridTransformerCaptioning (grid:161-322), random-init trunk, our weights."""
    mod = load_ref("models/grid_transformer_model.py", "ref_grid_transformer_model")
    model = mod.GridTransformerCaptioning(W.VOCAB_SIZE, pretrained_cnn=False)
    model.load_state_dict(sd, strict=True)
    return model.eval()


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
    # ViTTransformerCaptioning.forward (vit:216-255, padding from caption_lengths) and
    # GridTransformerCaptioning.forward (grid:185-210: padding from caption_lengths - 1).  Lengths cover
    # a full row, a partial one, 1, 0 (every key masked) and, for Grid, -1 (mask[i, -1:] slicing).
    imgs = torch.from_numpy(W.synthetic_images(4, seed=0))
    rng = np.random.Generator(np.random.PCG64(11))
    caps = rng.integers(0, W.VOCAB_SIZE, size=(4, 17)).astype(np.int64)
    caps[:, 0] = W.START_TOKEN
    captions = torch.from_numpy(caps)
    vit_len = [17, 9, 1, 0]
    model = ref_vit_model(ref, W.to_torch(W.vit_state_dict(0)))
    with torch.no_grad():
        vit_logits = model(imgs, captions, vit_len)
    gmodel = ref_grid_model(W.to_torch(W.grid_state_dict(0)))
    grid_len = [17, 9, 2, 0]
    with torch.no_grad():
        grid_logits = gmodel(imgs, captions, grid_len)
    np.savez_compressed(os.path.join(HERE, "forward_b4.npz"), captions=caps, vit_lengths=np.array(vit_len),
                        grid_lengths=np.array(grid_len), vit_logits=vit_logits.numpy(),
                        grid_logits=grid_logits.numpy())
    out["forward_b4"] = vit_logits.shape


def make_sample(ref, out):
    # (v) sampled decode: the reference's OWN SCSTLoss._sample_with_log_probs (scst_loss:202-254) on the
    # reference ViT model in eval mode (dropout off), torch.multinomial replaced during the call by an
    # inverse-CDF draw on fixed uniforms (one row of uniforms per call = per decode step)
    scst = load_ref("utils/scst_loss.py", "ref_scst_loss")
    model = ref_vit_model(ref, W.to_torch(W.vit_state_dict(0)))
    imgs = torch.from_numpy(W.synthetic_images(4, seed=0))
    u = torch.from_numpy(np.random.Generator(np.random.PCG64(11)).random((29, 4)).astype(np.float32))
    step = [0]
    real = torch.multinomial

    def inverse_cdf(probs, num_samples=1, *a, **k):
        assert num_samples == 1
        cdf = probs.cumsum(-1)
        nxt = (cdf <= u[step[0]].unsqueeze(-1) * cdf[:, -1:]).sum(-1).clamp_max(probs.shape[-1] - 1)
        step[0] += 1
        return nxt.unsqueeze(1)

    torch.multinomial = inverse_cdf
    try:
        with torch.no_grad():
            generated, lps = scst.SCSTLoss()._sample_with_log_probs(model, imgs, W.START_TOKEN, W.END_TOKEN, 30,
                                                                   torch.device("cpu"))
    finally:
        torch.multinomial = real
    np.savez_compressed(os.path.join(HERE, "sample_b4.npz"), uniforms=u.numpy(), ids=generated.numpy(),
                        log_probs=lps.numpy())
    out["sample_b4"] = generated.shape


def make_nomask(ref, out):
    # scripts/inference.py's OWN generate_caption (inference.py:60-101: no causal mask, B = 1, stops at
    # <end>, max_len 20 here) on the reference ViT model; words are "w<id>" so the caption maps back to ids
    import models  # noqa: F401  (the package the reference's `from models.vit_transformer_model` resolves in)

    inf = load_ref("scripts/inference.py", "ref_inference", {"models.vit_transformer_model": ref})
    model = ref_vit_model(ref, W.to_torch(W.vit_state_dict(0)))
    vocab = {f"w{i}": i for i in range(W.VOCAB_SIZE)}
    vocab.update({"<pad>": W.PAD_TOKEN, "<unk>": 106, "<start>": W.START_TOKEN, "<end>": W.END_TOKEN})
    img = torch.from_numpy(W.synthetic_images(4, seed=0))[0]
    cap = inf.generate_caption(model, img, vocab, torch.device("cpu"), max_len=20)
    ids = [vocab[w] for w in cap.split()]
    np.savez_compressed(os.path.join(HERE, "nomask_b1.npz"), ids=np.array(ids, dtype=np.int64), caption=np.array(cap))
    out["nomask_b1"] = len(ids)


SCRIPT_END_BIAS = {"vit": 1.6, "grid": 1.9}  # <end> logit offsets of the entry-script fixtures (varied lengths)


def make_scripts(ref, out):
    # The drop-in entry scripts, run through the reference's OWN script functions on PNG files:
    #  * scripts/inference_vit_transformer.py: generate_caption (:88-129, greedy and beam_search, max_len 50)
    #    and batch_generate_captions (:158-180, one generate_caption per image);
    #  * scripts/inference_grid_transformer.py: generate_caption (:52-76, greedy and beam_search, beam 5);
    #  * scripts/inference.py: generate_caption (:60-101, the no-mask loop) with the real vocabulary;
    #  * utils/scst_loss.py: SCSTLoss._decode_captions (:256-269) and get_reference_captions (:328-354) on a
    #    crafted id matrix (<end> mid-row, <pad> / <start> inside, unknown-free).
    # The scripts' preprocess_image is torchvision (absent): for the call it is replaced by the oracle's
    # Pillow-pinned restatement (oracle/preprocess.py) of the same transforms, applied to the decoded PNG.
    # Images: tests/golden/inputs.script_images (seeded uint8 arrays of several sizes, PNG is lossless).
    # Vocabulary: data/vocab.json (identical to the reference's data/vocab.json).  Weights: the seed-0
    # state dicts with the <end> logit raised by SCRIPT_END_BIAS.
    import json
    import tempfile

    from oracle import captioner as O
    from oracle import preprocess as OP
    from tests.golden.inputs import script_images, write_pngs

    vocab = json.load(open(os.path.join(ROOT, "data", "vocab.json"), encoding="utf-8"))
    arrays = script_images()
    tmp = tempfile.mkdtemp()
    paths = write_pngs(arrays, tmp)

    def patched(mod, mode):
        def preprocess_image(image_path, image_size=224):
            i = paths.index(image_path)
            return torch.from_numpy(OP.preprocess(arrays[i], mode, image_size))[None]
        mod.preprocess_image = preprocess_image
        return mod

    def biased(sd, kind):
        sd = dict(sd)
        b = sd["decoder.fc_out.bias"].clone()
        b[W.END_TOKEN] += SCRIPT_END_BIAS[kind]
        sd["decoder.fc_out.bias"] = b
        return sd

    evalm = _module("utils.eval_metrics", COCOScoreEvaluator=object)
    vsd = biased(W.to_torch(W.vit_state_dict(0)), "vit")
    vmodel = ref_vit_model(ref, vsd)
    vit_s = patched(load_ref("scripts/inference_vit_transformer.py", "ref_inference_vit",
                             {"models.vit_transformer_model": ref, "utils.eval_metrics": evalm}), "crop")
    res = {}
    with torch.no_grad():
        greedy = [vit_s.generate_caption(vmodel, p, vocab, "cpu", "greedy") for p in paths]
        res["vit_batch"] = vit_s.batch_generate_captions(vmodel, paths, vocab, "cpu", "greedy")
        beam = vit_s.generate_caption(vmodel, paths[0], vocab, "cpu", "beam_search")
    res["vit_greedy_caps"] = [c for c, _ in greedy]
    res["vit_greedy_ids"] = [i for _, i in greedy]
    res["vit_beam_cap"], res["vit_beam_ids"] = beam
    # the oracle's top-2 margin along each greedy caption (teacher-forced on the reference's ids)
    imgs = torch.stack([torch.from_numpy(OP.preprocess(a, "crop")) for a in arrays])
    with torch.no_grad():
        vmem = O.vit_encode(vsd, imgs)
    res["vit_greedy_margin"] = [float(O.top2_margin(O.teacher_forced_logits(vsd, vmem[i:i + 1],
                                      torch.tensor([ids]))).min()) for i, ids in enumerate(res["vit_greedy_ids"])]
    res["vit_beam_margin"] = O.beam_from_memory(vsd, vmem[:1], W.START_TOKEN, W.END_TOKEN, 50, 5, False,
                                                return_margins=True)[1]

    gmod = load_ref("models/grid_transformer_model.py", "ref_grid_transformer_model")
    gsd = biased(W.to_torch(W.grid_state_dict(0)), "grid")
    gmodel = gmod.GridTransformerCaptioning(W.VOCAB_SIZE, pretrained_cnn=False)
    gmodel.load_state_dict(gsd, strict=True)
    gmodel.eval()
    grid_s = patched(load_ref("scripts/inference_grid_transformer.py", "ref_inference_grid",
                              {"models.grid_transformer_model": gmod, "utils.eval_metrics": evalm}), "square")
    with torch.no_grad():
        gg = [grid_s.generate_caption(gmodel, p, vocab, "cpu", "greedy") for p in paths]
        gb = grid_s.generate_caption(gmodel, paths[1], vocab, "cpu", "beam_search", beam_size=5)
    res["grid_greedy_caps"] = [c for c, _ in gg]
    res["grid_greedy_ids"] = [i for _, i in gg]
    res["grid_beam_cap"], res["grid_beam_ids"] = gb
    gimgs = torch.stack([torch.from_numpy(OP.preprocess(a, "square")) for a in arrays])
    with torch.no_grad():
        gmem = O.grid_encode(gsd, gimgs)
    res["grid_greedy_margin"] = [float(O.top2_margin(O.teacher_forced_logits(gsd, gmem[i:i + 1],
                                       torch.tensor([ids]))).min()) for i, ids in enumerate(res["grid_greedy_ids"])]
    res["grid_beam_margin"] = O.beam_from_memory(gsd, gmem[1:2], W.START_TOKEN, W.END_TOKEN, 50, 5, True,
                                                 return_margins=True)[1]

    inf = load_ref("scripts/inference.py", "ref_inference", {"models.vit_transformer_model": ref})
    sq = torch.stack([torch.from_numpy(OP.preprocess(a, "square")) for a in arrays])
    with torch.no_grad():
        res["nomask_caps"] = [inf.generate_caption(vmodel, sq[i], vocab, torch.device("cpu")) for i in range(len(arrays))]
        # the oracle's top-2 margin at every step of the no-mask loop, along the reference's words
        smem = O.vit_encode(vsd, sq)
        res["nomask_margin"] = []
        for i, cap in enumerate(res["nomask_caps"]):
            ids, m = [W.START_TOKEN], float("inf")
            for w in cap.split() + [None]:
                lg = O.decoder_forward(vsd, torch.tensor([ids]), smem[i:i + 1], causal=False)[:, -1, :]
                m = min(m, float(O.top2_margin(lg)))
                if w is not None:
                    ids.append(vocab[w])
            res["nomask_margin"].append(m)

    # detokenize on a crafted id matrix: rows with <end> mid-row, <pad> and <start> inside, no <end> at all
    rng = np.random.Generator(np.random.PCG64(5))
    crafted = rng.integers(1, 106, size=(6, 12)).astype(np.int64)
    crafted[0, 5] = W.END_TOKEN
    crafted[1, 0], crafted[1, 3], crafted[1, 7] = W.START_TOKEN, W.PAD_TOKEN, W.END_TOKEN
    crafted[2, 0] = W.END_TOKEN
    crafted[3, :] = W.PAD_TOKEN
    crafted[4, 2], crafted[4, 4] = W.START_TOKEN, W.PAD_TOKEN  # row 4: no <end>
    crafted[5, 11] = W.END_TOKEN
    scst = load_ref("utils/scst_loss.py", "ref_scst_loss")
    idx2word = {i: w for w, i in vocab.items()}
    res["detok_ids"] = crafted.tolist()
    res["detok_scst"] = scst.SCSTLoss()._decode_captions(torch.from_numpy(crafted), idx2word, W.END_TOKEN,
                                                         W.PAD_TOKEN, W.START_TOKEN)
    res["detok_refs"] = scst.get_reference_captions(torch.from_numpy(crafted), vocab)
    res["end_bias"] = SCRIPT_END_BIAS
    with open(os.path.join(HERE, "scripts.json"), "w", encoding="utf-8") as f:
        json.dump(res, f, ensure_ascii=False, indent=1)
    for p in paths:
        os.remove(p)
    os.rmdir(tmp)
    out["scripts"] = (len(paths), [len(i) for i in res["vit_greedy_ids"]], [len(i) for i in res["grid_greedy_ids"]],
                      [round(m, 5) for m in res["vit_greedy_margin"] + res["grid_greedy_margin"]])


def make_grid(out):
    # (iv) Grid: the reference's OWN GridTransformerCaptioning (trunk = the torchvision-named restatement)
    # generate(greedy) at B = 4, its trunk features (B, 2048, 7, 7) and memory, teacher-forced logits of
    # its ids; then _beam_search (grid:253-322) one image per call as the reference loops, with the
    # <end> logit raised by END_BIAS so beams finish and the Grid stop tests (completed >= live) fire
    from oracle import captioner as O

    gsd = W.to_torch(W.grid_state_dict(0))
    gmodel = ref_grid_model(gsd)
    imgs = torch.from_numpy(W.synthetic_images(4, seed=0))
    with torch.no_grad():
        feats = gmodel.encoder.cnn(imgs)
        gmem = gmodel.encoder(imgs)
        gids = gmodel.generate(imgs, W.START_TOKEN, W.END_TOKEN, max_len=30, method="greedy")
    gtf = teacher_forced(gmodel.decoder, gmem, gids)
    np.savez_compressed(os.path.join(HERE, "grid_b4.npz"), weights_seed=0, image_seed=0, max_len=30,
                        ids=gids.numpy(), memory_sum=gmem.double().sum(dim=(1, 2)).numpy(),
                        memory_head=gmem[:, :4, :16].numpy(), logits_tf=gtf.numpy(), margins=top2(gtf),
                        trunk_sum=feats.double().sum(dim=(2, 3)).numpy(), trunk_head=feats[:, :8, :, :].numpy())
    out["grid_b4"] = gids.shape
    # <end> offsets for the Grid weights: 2.0 / 2.2 end every beam after 9 / 7 tokens (pruning on the way),
    # 2.8 ends at the first step (the completed-count stop with one token)
    cases = [(0.0, 3, 0), (0.0, 3, 1), (2.0, 5, 0), (2.0, 5, 1), (2.2, 5, 2), (2.2, 5, 3), (2.8, 5, 0)]
    rows, lens, margins = [], [], []
    for delta, k, i in cases:
        sdb = dict(gsd)
        fb = sdb["decoder.fc_out.bias"].clone()
        fb[W.END_TOKEN] += delta
        sdb["decoder.fc_out.bias"] = fb
        gmodel.load_state_dict(sdb, strict=True)
        with torch.no_grad():
            seq = gmodel.generate(imgs[i:i + 1], W.START_TOKEN, W.END_TOKEN, max_len=30, method="beam_search",
                                  beam_size=k)
            _, margin = O.beam_from_memory(sdb, gmodel.encoder(imgs[i:i + 1]), W.START_TOKEN, W.END_TOKEN, 30, k,
                                           True, return_margins=True)
        row = np.full(30, -1, dtype=np.int64)
        row[: seq.shape[1]] = seq[0].numpy()
        rows.append(row)
        lens.append(seq.shape[1])
        margins.append(margin)
    np.savez_compressed(os.path.join(HERE, "beam_grid.npz"), end_bias=np.array([c[0] for c in cases]),
                        beam=np.array([c[1] for c in cases]), image=np.array([c[2] for c in cases]),
                        ids=np.stack(rows), lengths=np.array(lens), margins=np.array(margins))
    out["beam_grid"] = (len(cases),)


def main():
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count() or 8)
    ref = load_ref_vit_module()
    out = {}
    only = sys.argv[1] if len(sys.argv) > 1 else None
    if only == "forward":
        make_forward(ref, out)
    elif only == "beam_vit":
        make_beam(ref, W.to_torch(W.vit_state_dict(0)), torch.from_numpy(W.synthetic_images(4, seed=0)), out)
    elif only == "grid":
        make_grid(out)
    elif only == "sample":
        make_sample(ref, out)
    elif only == "nomask":
        make_nomask(ref, out)
    elif only == "scripts":
        make_scripts(ref, out)
    elif only is not None:
        raise SystemExit(f"unknown fixture {only!r}")
    if only is not None:
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

    make_nomask(ref, out)
    make_sample(ref, out)
    make_grid(out)
    make_beam(ref, sd, imgs, out)
    make_forward(ref, out)
    make_scripts(ref, out)
    for k, v in out.items():
        print(k, tuple(v) if hasattr(v, "__len__") else v)


if __name__ == "__main__":
    main()
