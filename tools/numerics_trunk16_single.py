"""CPU emulation (round 4, verdict r3 item 4): the fp16 Grid trunk with its layer3-4 residual stream as ONE fp16 plane
(instead of the built fp16 hi/lo pair, emulated as fp32) against the fp32 oracle: trunk features relative to the batch
maximum (the config-3 GPU test's 1e-3 bar), memory, teacher-forced logits, greedy ids.  B = 8 synthetic images
(seed 3, the config-3 test's), every branch one fp16 plane, layer3-4 conv1 on the hi plane (as built)."""
import sys

import torch

sys.path.insert(0, '/root/repo')
from image_caption_amd import weights as W
from oracle import captioner as O

torch.set_num_threads(8)
F = torch.nn.functional
sd = W.to_torch(W.grid_state_dict(0))
imgs = torch.from_numpy(W.synthetic_images(8, seed=3))
P = "encoder.cnn."


def bn(x, p):
    w, b, m, v = sd[p + ".weight"], sd[p + ".bias"], sd[p + ".running_mean"], sd[p + ".running_var"]
    sc = w / torch.sqrt(v + 1e-5)
    sh = b - m * sc
    return x * sc[None, :, None, None] + sh[None, :, None, None]


def q(x, dt):
    return x.to(dt).float()


def trunk(single_from):
    """residual stream one fp16 plane in layers < single_from... no: layers li >= 2 keep fp32 (hi/lo) unless
    li >= single_from; single_from = 2: all single, 4: the built form"""
    dt = torch.float16
    cw = lambda k: q(sd[k], dt)
    xdt = lambda li: dt if (li < 2 or li >= single_from) else torch.float32
    x = q(imgs, dt)
    x = q(torch.relu(bn(F.conv2d(x, cw(P + "0.weight"), stride=2, padding=3), P + "1")), xdt(0))
    x = F.max_pool2d(x, 3, 2, 1)
    mx = 0.0
    for li, nblk in enumerate((3, 4, 23, 3)):
        for b in range(nblk):
            p = P + f"{4 + li}.{b}."
            s = 2 if (b == 0 and li > 0) else 1
            y = q(torch.relu(bn(F.conv2d(q(x, dt), cw(p + "conv1.weight")), p + "bn1")), dt)
            y = q(torch.relu(bn(F.conv2d(y, cw(p + "conv2.weight"), stride=s, padding=1), p + "bn2")), dt)
            if b == 0:
                x = q(bn(F.conv2d(x, cw(p + "downsample.0.weight"), stride=s), p + "downsample.1"), xdt(li))
            x = q(torch.relu(x + bn(F.conv2d(y, cw(p + "conv3.weight")), p + "bn3")), xdt(li))
            mx = max(mx, x.abs().max().item())
    return x, mx


with torch.no_grad():
    ref = O.resnet101_trunk(sd, imgs)
    mem_o = O.grid_encode_tail(sd, ref)
    ids = O.greedy_from_memory(sd, mem_o, W.START_TOKEN, W.END_TOKEN, 30)
    a = O.teacher_forced_logits(sd, mem_o, ids.long())
    scale = ref.abs().max().item()
    for name, sf in (("built: layer3-4 residual hi/lo", 4), ("layer4 residual one fp16 plane", 3),
                     ("layer3-4 residual one fp16 plane", 2)):
        x, mx = trunk(sf)
        err = (x - ref).abs().flatten(1).amax(1)
        mem = O.grid_encode_tail(sd, x)
        b = O.teacher_forced_logits(sd, mem, ids.long())
        gid = O.greedy_from_memory(sd, mem, W.START_TOKEN, W.END_TOKEN, 30)
        print(f"{name}: features rel {max((err / scale).tolist()):.3e}  max |x| {mx:.1f}  memory "
              f"{(mem - mem_o).abs().max().item():.3e}  logits {(a - b).abs().max().item():.3e}  ids equal "
              f"{bool((gid == ids).all())}", flush=True)
