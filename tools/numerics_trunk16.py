import torch, numpy as np, sys
sys.path.insert(0, '/root/repo')
from image_caption_amd import weights as W
from oracle import captioner as O
torch.set_num_threads(8)
sd = W.to_torch(W.grid_state_dict(0))
imgs = torch.from_numpy(W.synthetic_images(4, seed=3))
F = torch.nn.functional
P = "encoder.cnn."
def bn(x, p):
    w, b, m, v = sd[p+".weight"], sd[p+".bias"], sd[p+".running_mean"], sd[p+".running_var"]
    sc = w / torch.sqrt(v + 1e-5); sh = b - m * sc
    return x * sc[None,:,None,None] + sh[None,:,None,None]
def q(x, dt): return x.to(dt).float()
def trunk(dt, wdt):
    cw = lambda k: q(sd[k], wdt)
    x = q(imgs, dt)
    mx = 0
    x = q(torch.relu(bn(F.conv2d(x, cw(P+"0.weight"), stride=2, padding=3), P+"1")), dt)
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate((3,4,23,3)):
        for b in range(nblk):
            p = P + f"{4+li}.{b}."
            s = 2 if (b == 0 and li > 0) else 1
            y = q(torch.relu(bn(F.conv2d(x, cw(p+"conv1.weight")), p+"bn1")), dt)
            y = q(torch.relu(bn(F.conv2d(y, cw(p+"conv2.weight"), stride=s, padding=1), p+"bn2")), dt)
            if b == 0:
                x = q(bn(F.conv2d(x, cw(p+"downsample.0.weight"), stride=s), p+"downsample.1"), dt)
            x = q(torch.relu(x + bn(F.conv2d(y, cw(p+"conv3.weight")), p+"bn3")), dt)
            mx = max(mx, x.abs().max().item(), y.abs().max().item())
    return x, mx
with torch.no_grad():
    ref = O.resnet101_trunk(sd, imgs)
    for name, dt, wdt in [("f16 act, f16 w", torch.float16, torch.float16), ("bf16 act/w", torch.bfloat16, torch.bfloat16), ("f16 act, fp32 w", torch.float16, torch.float32)]:
        x, mx = trunk(dt, wdt)
        scale = ref.abs().max().item()
        err = (x - ref).abs().flatten(1).amax(1)
        print(name, "max act", mx, "rel err per img", (err/scale).tolist())
        mem_o = O.grid_encode_tail(sd, ref); mem = O.grid_encode_tail(sd, x)
        print("   memory abs err", (mem-mem_o).abs().max().item())
def trunk2(dt, xdt, wdt=torch.float16):
    cw = lambda k: q(sd[k], wdt)
    x = q(imgs, dt)
    x = q(torch.relu(bn(F.conv2d(x, cw(P+"0.weight"), stride=2, padding=3), P+"1")), xdt)
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate((3,4,23,3)):
        for b in range(nblk):
            p = P + f"{4+li}.{b}."
            s = 2 if (b == 0 and li > 0) else 1
            y = q(torch.relu(bn(F.conv2d(x, cw(p+"conv1.weight")), p+"bn1")), dt)
            y = q(torch.relu(bn(F.conv2d(y, cw(p+"conv2.weight"), stride=s, padding=1), p+"bn2")), dt)
            if b == 0:
                x = q(bn(F.conv2d(x, cw(p+"downsample.0.weight"), stride=s), p+"downsample.1"), xdt)
            x = q(torch.relu(x + bn(F.conv2d(y, cw(p+"conv3.weight")), p+"bn3")), xdt)
    return x
with torch.no_grad():
    for name, xdt in [("x fp32, y f16", torch.float32)]:
        x = trunk2(torch.float16, xdt)
        scale = ref.abs().max().item()
        err = (x - ref).abs().flatten(1).amax(1)
        print(name, "rel err per img", (err/scale).tolist())
        mem = O.grid_encode_tail(sd, x)
        print("   memory abs err", (mem-mem_o).abs().max().item())
with torch.no_grad():
    x = trunk2(torch.float16, torch.float32)
    mem = O.grid_encode_tail(sd, x)
    ids = O.greedy_from_memory(sd, mem_o, W.START_TOKEN, W.END_TOKEN, 30)
    a = O.teacher_forced_logits(sd, mem_o, ids.long()); b = O.teacher_forced_logits(sd, mem, ids.long())
    print("logit err", (a-b).abs().max().item())
def trunk3(single_stages):
    dt = torch.float16
    cw = lambda k: q(sd[k], dt)
    x = q(imgs, dt)
    xdt = lambda li: dt if li in single_stages else torch.float32
    x = q(torch.relu(bn(F.conv2d(x, cw(P+"0.weight"), stride=2, padding=3), P+"1")), xdt(0))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate((3,4,23,3)):
        for b in range(nblk):
            p = P + f"{4+li}.{b}."
            s = 2 if (b == 0 and li > 0) else 1
            y = q(torch.relu(bn(F.conv2d(x, cw(p+"conv1.weight")), p+"bn1")), dt)
            y = q(torch.relu(bn(F.conv2d(y, cw(p+"conv2.weight"), stride=s, padding=1), p+"bn2")), dt)
            if b == 0:
                x = q(bn(F.conv2d(x, cw(p+"downsample.0.weight"), stride=s), p+"downsample.1"), xdt(li))
            x = q(torch.relu(x + bn(F.conv2d(y, cw(p+"conv3.weight")), p+"bn3")), xdt(li))
    return x
with torch.no_grad():
    for st in [(0,1,2)]:
        x = trunk3(st)
        scale = ref.abs().max().item()
        err = (x - ref).abs().flatten(1).amax(1)
        mem = O.grid_encode_tail(sd, x)
        b = O.teacher_forced_logits(sd, mem, ids.long())
        print("single-plane stages", st, "rel", max((err/scale).tolist()), "mem", (mem-mem_o).abs().max().item(), "logit", (a-b).abs().max().item())
