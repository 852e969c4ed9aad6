#!/usr/bin/env python3
"""Where the Res-ViT-B/16 bs 128 step's ATen glue comes from: two eager train steps under torch.profiler with
Python stacks, ATen ops grouped by their calling vitmi frames, sorted by device time."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from vitmi import resvit  # noqa: E402
from vitmi.optim import AdamW, get_cosine_schedule_with_warmup  # noqa: E402
from vitmi.resvit_train import train_step  # noqa: E402

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
for _ in range(3):
    train_step(model, x, y, opt, sched, 1e-4, 1e-2, 1.0, True, None)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    for _ in range(2):
        train_step(model, x, y, opt, sched, 1e-4, 1e-2, 1.0, True, None)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=40, max_name_column_width=60), flush=True)
rows = [e for e in prof.key_averages(group_by_stack_n=8) if e.key in ("aten::add_", "aten::fill_", "aten::copy_",
                                                                     "aten::where", "aten::add", "aten::mul",
                                                                     "aten::zero_", "aten::sum", "aten::mean",
                                                                     "aten::_to_copy", "aten::div", "aten::sub")]
rows.sort(key=lambda e: -e.self_device_time_total)
for e in rows[:45]:
    frames = [f for f in e.stack if "vitmi" in f or "bench" in f][:4]
    print(f"{e.key:12s} n={e.count:4d} dev={e.self_device_time_total / 1e3:7.3f} ms  " + " <- ".join(
        f.split("/")[-1] for f in frames), flush=True)

# the glue ops by input shape (which tensors they touch: the backward's ops carry no Python frames)
shp = [e for e in prof.key_averages(group_by_input_shape=True) if e.key in ("aten::copy_", "aten::add", "aten::add_",
                                                                           "aten::fill_", "aten::mean", "aten::mul")]
shp.sort(key=lambda e: -e.self_device_time_total)
for e in shp[:40]:
    print(f"{e.key:12s} n={e.count:4d} dev={e.self_device_time_total / 1e3:7.3f} ms  {str(e.input_shapes)[:150]}", flush=True)
