"""Host-side time of the graphed Res-ViT-B/16 bs 128 step (diagnostic): how long graph.replay() and the eager
optimizer tail take on the host against the GPU time per step, to see whether the host bounds the step."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "vit-of-pytorch_amd"))
from vitmi import resvit  # noqa: E402
from vitmi.optim import AdamW, get_cosine_schedule_with_warmup  # noqa: E402
from vitmi.resvit_train import GraphedTrainStep  # noqa: E402

a = dict(dim=768, mlp_dim=3072, n_layers=12, n_heads=12, n_kv_heads=12, norm_eps=1e-5, lora_rank=8,
         dynamic_active_target=0.6, dynamic_start_layer=2, dynamic_router_hdim=512, dynamic_reserve_initials=1,
         low_rank_dim=256, block_size=1, use_lora=True, use_reslr=True, image_size=(224, 224),
         patch_size=(16, 16), num_classes=100, device="cuda")
torch.manual_seed(42)
model = resvit.Transformer(resvit.ModelArgs(**a)).cuda().train()
opt = AdamW(model.parameters(), lr=1e-4, weight_decay=0.05, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=1.0)
sched = get_cosine_schedule_with_warmup(opt, 500, 15000)
g = torch.Generator(device="cuda").manual_seed(1000)
x = torch.randn(128, 3, 224, 224, device="cuda", generator=g)
y = torch.randint(0, 100, (128,), device="cuda", generator=g)
gs = GraphedTrainStep(model, x, y, opt, sched, 1e-4, 1e-2, 1.0, True)
for _ in range(3):
    gs.step()
torch.cuda.synchronize()
n = 10
t_zero, t_replay, t_tail = [], [], []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
for _ in range(n):
    a0 = time.perf_counter()
    gs.opt.zero_grad()
    a1 = time.perf_counter()
    gs.graph.replay()
    a2 = time.perf_counter()
    f = gs.opt.flat
    f.used_host = list(gs.used)
    import weakref
    for p, flag in gs.gates:
        gs._flat._GATES[id(p)] = (weakref.ref(p), flag)
    gs.opt.step()
    gs.sched.step()
    a3 = time.perf_counter()
    t_zero.append(a1 - a0)
    t_replay.append(a2 - a1)
    t_tail.append(a3 - a2)
e1.record()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / n
print(f"per step: wall {wall * 1e3:.2f} ms, GPU (events) {e0.elapsed_time(e1) / n:.2f} ms; host: zero_grad "
      f"{sum(t_zero) / n * 1e3:.3f} ms, graph.replay() {sum(t_replay) / n * 1e3:.3f} ms, optimizer tail "
      f"{sum(t_tail) / n * 1e3:.3f} ms", flush=True)
