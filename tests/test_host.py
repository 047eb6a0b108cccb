"""Host-side logic on CPU: drop-in modules (PyTorch path) vs the oracle, the C-ABI library's
exports, stop rules, CIDEr-D, preprocessing, and the data-parallel gather over gloo (world 2)."""
import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from image_caption_amd import weights as W
from image_caption_amd.engine import apply_stop_rule
from oracle import captioner as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch.set_num_threads(min(8, os.cpu_count() or 1))


def test_header_symbols_exported():
    from image_caption_amd import _lib

    decl = re.findall(r"\b(icap_\w+)\s*\(", open(os.path.join(ROOT, "include", "icap.h")).read())
    assert len(set(decl)) >= 14
    lib = _lib.load()
    for name in set(decl):
        assert hasattr(lib, name), name
    assert set(decl) == set(_lib.SIGNATURES), set(decl) ^ set(_lib.SIGNATURES)
    assert lib.icap_abi_version() == _lib.ABI_VERSION


def test_dropout_hash_oracle_matches_library():
    """oracle/dropout.py's numpy hash is the library's icap_drop_hash (common.h), bit for bit, and the
    masks keep 1 - p of the elements."""
    from image_caption_amd import _lib
    from oracle import dropout as D

    lib = _lib.load()
    g = np.random.Generator(np.random.PCG64(0))
    args = g.integers(0, 2**32, size=(500, 6), dtype=np.uint64)
    args[:, 1] %= 7
    args[:, 2] %= 6
    args[:250, 3:] %= 300  # small rows / positions / indices as the decoder uses them
    want = [lib.icap_drop_hash_host(*(int(v) for v in a)) for a in args]
    for a, w in zip(args, want):
        assert int(D.drop_hash(int(a[0]), int(a[1]), int(a[2]), int(a[3]), int(a[4]), int(a[5]))) == w
    m = D.decoder_masks(0.1, 7, 4, 29, 196)
    frac = np.mean([float((v == 0).float().mean()) for v in m.values()])
    assert abs(frac - 0.1) < 0.005, frac
    assert set(torch.unique(m["ff_h.3"]).tolist()) == {0.0, float(np.float32(1) / np.float32(0.9))}


def test_library_refuses_without_gpu_inputs():
    from image_caption_amd import _lib

    lib = _lib.load()
    assert lib.icap_encode_vit(None, None, 1, None, None) != 0
    assert b"bad arguments" in lib.icap_last_error()


def test_product_build_refuses_measurement_knobs(monkeypatch):
    """The product library compiles every ICAP_* measurement knob to its default and icap_create refuses
    to run while one is set, so no environment can change what it computes (the check precedes any GPU
    call, so it runs on CPU)."""
    import ctypes

    from image_caption_amd import _lib

    lib = _lib.load()
    if lib.icap_tools_build():
        pytest.skip("tools build")
    monkeypatch.setenv("ICAP_I8_NOMFMA", "1")
    h = ctypes.c_void_p()
    desc = _lib.ModelDesc()
    assert lib.icap_create(ctypes.byref(desc), None, ctypes.byref(h)) != 0
    assert b"ICAP_I8_NOMFMA" in lib.icap_last_error() and b"tools build" in lib.icap_last_error()


def test_product_build_ships_only_shipped_forms():
    """The measured-and-rejected kernel forms (gemm_tools.hip, the persistent decode steps decstep.hip / xdec.hip, the
    key-split and wave-owned cross-attentions, the LayerNorm-folding decode blocks) are compiled into the tools build only: the product source list does not hold them and the product library's code
    object has none of their kernels."""
    from image_caption_amd import _lib, build

    for src in ("gemm_tools.hip", "decstep.hip", "xdec.hip"):
        assert src not in build.SOURCES and src in build.TOOLS_SOURCES
    lib = _lib.load()
    if lib.icap_tools_build():
        pytest.skip("tools build")
    blob = build.LIB.read_bytes()
    for kernel in (b"dec_step_kernel", b"xdec_kernel", b"gemm_f16q_kernel", b"gemm_8ph_kernel",
                   b"cross_attn_f16s_kernel", b"cross_attn_wk_kernel", b"cross_attn_f16_kernelILi2E",
                   b"dec_chain_kernelILb1ELi2ELi8E", b"dec_ffn_kernelILb1ELi2ELi8E"):
        assert kernel not in blob, kernel


def test_dropin_vit_model_state_dict_and_greedy():
    from models.vit_transformer_model import build_model

    m = build_model(W.VOCAB_SIZE, {"pretrained_vit": False})
    sd = W.to_torch(W.vit_state_dict(0))
    m.load_state_dict(sd, strict=True)
    assert set(m.state_dict()) == set(sd)
    imgs = torch.from_numpy(W.synthetic_images(2, seed=9))
    ids = m.generate(imgs, W.START_TOKEN, W.END_TOKEN, max_len=10)
    assert not m.training
    assert torch.equal(ids, O.greedy_search(sd, imgs, W.START_TOKEN, W.END_TOKEN, 10))
    with pytest.raises(ValueError):
        m.generate(imgs, W.START_TOKEN, W.END_TOKEN, method="nope")


def test_dropin_grid_model_state_dict():
    from models.grid_transformer_model import build_model

    m = build_model(W.VOCAB_SIZE, {"pretrained_cnn": False})
    sd = W.to_torch(W.grid_state_dict(0))
    m.load_state_dict(sd, strict=True)
    assert set(m.state_dict()) == set(sd)


def test_every_knob_is_refused_by_the_product_build():
    """Every ICAP_* measurement knob the sources read (icap_knob) is in icap_knobs_set's list, so a product
    build refuses to run with any of them set (no environment can change what the library computes)."""
    import re

    csrc = os.path.join(ROOT, "image_caption_amd", "csrc")
    read = set()
    for f in os.listdir(csrc):
        with open(os.path.join(csrc, f)) as fh:
            read |= set(re.findall(r'icap_knob\("(ICAP_[A-Z0-9_]+)"', fh.read()))
    with open(os.path.join(csrc, "icap.cpp")) as fh:
        src = fh.read()
    lst = src[src.index("const char* icap_knobs_set()"):]
    refused = set(re.findall(r'"(ICAP_[A-Z0-9_]+)"', lst[:lst.index("};")]))
    assert read and read <= refused, sorted(read - refused)


def test_deepcopy_routes_to_the_copy():
    """copy.deepcopy of a drop-in model: the copy's encoder / decoder route to the copy (not the original's
    engine), and a packed engine (a device handle) is never copied or shared."""
    import copy

    from models._hip import owner_of
    from models.vit_transformer_model import build_model

    m = build_model(W.VOCAB_SIZE, {"pretrained_vit": False})
    object.__setattr__(m, "_hip_cache", ("sentinel",))  # stands in for a packed engine
    twin = copy.deepcopy(m)
    assert owner_of(twin.encoder) is twin and owner_of(twin.decoder) is twin
    assert owner_of(m.encoder) is m
    assert twin._hip_cache is None and m._hip_cache == ("sentinel",)
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), twin.state_dict().values()))


def test_forced_hip_backend_refuses_cpu():
    from models.vit_transformer_model import build_model

    m = build_model(W.VOCAB_SIZE, {"pretrained_vit": False, "backend": "hip"})
    with pytest.raises(RuntimeError):
        m.generate(torch.zeros(1, 3, 224, 224), W.START_TOKEN, W.END_TOKEN, max_len=3)


def test_stop_rules():
    E = W.END_TOKEN
    ids = torch.tensor([[107, 5, E, E, 7], [107, E, 3, E, 9]])
    assert apply_stop_rule(ids, E).shape[1] == 4  # first column where every row is <end>: col 3
    assert apply_stop_rule(torch.tensor([[107, 1, 2]]), E).shape[1] == 3
    from utils.scst_loss import masked_token_logp, sample_stop_length

    assert sample_stop_length(ids, E) == 3  # every row has emitted <end> by column 2
    logits = torch.zeros(2, 4, W.VOCAB_SIZE)
    lp = masked_token_logp(logits, ids, E)
    assert lp[0, :2].ne(0).all() and lp[0, 2:].eq(0).all() and lp[1, 0].ne(0) and lp[1, 1:].eq(0).all()


def test_cider_ids_match_string_restatement():
    from image_caption_amd.cider import cider_d
    from oracle.cider_ref import compute_score

    rng = np.random.Generator(np.random.PCG64(5))
    hyps, refs = [], []
    for i in range(40):
        hyps.append(list(rng.integers(1, 12, size=rng.integers(0, 9))))
        refs.append([list(rng.integers(1, 12, size=rng.integers(1, 10))) for _ in range(rng.integers(1, 3))])
    s = lambda t: " ".join(f"w{x}" for x in t)
    m1, per1 = cider_d(hyps, refs)
    m2, per2 = compute_score({i: [s(r) for r in rs] for i, rs in enumerate(refs)}, {i: [s(h)] for i, h in enumerate(hyps)})
    assert np.allclose(per1, per2, rtol=1e-12, atol=1e-12) and abs(m1 - m2) < 1e-12
    # identical caption and reference scores > 0; disjoint scores 0
    assert cider_d([[1, 2, 3], [4]], [[[1, 2, 3]], [[5]]])[1][1] == 0.0


def test_preprocess_matches_manual():
    from PIL import Image

    from scripts._io import MEAN, STD, center_crop, resize_shorter, to_normalized_tensor

    a = (np.arange(300 * 400 * 3) % 251).astype(np.uint8).reshape(300, 400, 3)
    img = Image.fromarray(a)
    r = resize_shorter(img, 256)
    assert r.size == (341, 256)
    c = center_crop(r, 224)
    assert c.size == (224, 224)
    t = to_normalized_tensor(c)
    ref = (np.asarray(c, dtype=np.float32) / 255.0 - MEAN) / STD
    assert np.allclose(t.numpy(), ref.transpose(2, 0, 1))


def test_shard_bounds():
    from image_caption_amd.parallel import shard_bounds

    for total in (0, 1, 7, 256, 2048, 1023):
        for ws in (1, 2, 3, 8):
            spans = [shard_bounds(total, ws, r) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(ws - 1))
            assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, ws, port, total, q):
    import torch.distributed as dist

    from image_caption_amd import parallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    parallel.init("gloo")
    sd = W.to_torch(W.vit_state_dict(0))
    mem_all = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).standard_normal((total, 20, 512)).astype(np.float32))
    s, e = parallel.shard_bounds(total, ws, rank)
    ids = O.greedy_from_memory(sd, mem_all[s:e], W.START_TOKEN, W.END_TOKEN, 6)
    full = torch.full((e - s, 6), W.END_TOKEN, dtype=torch.int32)
    full[:, : ids.shape[1]] = ids.int()
    g = parallel.gather_rows(full, total)
    if rank == 0:
        q.put(apply_stop_rule(g.long(), W.END_TOKEN).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_gather_matches_single_process():
    total, ws = 5, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, ws, port, total, q)) for r in range(ws)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sd = W.to_torch(W.vit_state_dict(0))
    mem_all = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).standard_normal((total, 20, 512)).astype(np.float32))
    ref = O.greedy_from_memory(sd, mem_all, W.START_TOKEN, W.END_TOKEN, 6)
    assert np.array_equal(got, ref.numpy())
