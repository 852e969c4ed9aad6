"""Debug (not product code): which Res-ViT parameters differ between two gloo DP replicas after two train steps
(the setup of tests/test_resvit_train_gpu.py::test_resvit_data_parallel_two_ranks), and the reducer's mark counts."""
import os, sys, torch, torch.distributed as dist
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
from test_resvit_cpu import TINY
from vitmi import resvit
from vitmi.optim import AdamW
from vitmi.dist import FlatGradAllReducer
from vitmi.resvit_train import train_step
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
g = torch.Generator().manual_seed(5)
X = torch.randn(8, 3, 32, 32, generator=g); Y = torch.randint(0, 10, (8,), generator=g)
torch.manual_seed(42)
m = resvit.Transformer(resvit.ModelArgs(**dict(TINY, device="cuda"))).cuda().train()
gn = torch.Generator().manual_seed(9)
for l in [l for l in m.layers if hasattr(l, "router")]:
    noise = -torch.empty(8, 17, 2, 2).exponential_(generator=gn).log()
    l.router.gumbel_noise = (lambda nz: lambda logits: nz[rank * 4:(rank + 1) * 4])(noise.cuda())
opt = AdamW(m.parameters(), lr=1e-2, weight_decay=0.05, max_grad_norm=1.0)
red = FlatGradAllReducer(opt.flat, bucket_elems=2000).attach()
names = {id(p): n for n, p in m.named_parameters()}
marks = []
orig = red._on_grad
def spy(i):
    marks.append(i)
    orig(i)
opt.flat.on_grad = spy
x, y = X[rank * 4:(rank + 1) * 4].cuda(), Y[rank * 4:(rank + 1) * 4].cuda()
for step in range(2):
    marks.clear()
    train_step(m, x, y, opt, None, 0.0, 1e-2, 1.0, True, red)
    torch.cuda.synchronize()
    from collections import Counter
    c = Counter(marks)
    dup = {names.get(id(opt.flat.params[i]), i): n for i, n in c.items() if n > 1}
    print(f"rank {rank} step {step}: {len(marks)} marks, {len(c)} params, duplicates {dup}", flush=True)
    g_ = opt.flat.grad.clone()
    outg = [torch.zeros_like(g_) for _ in range(world)]
    dist.all_gather(outg, g_)
    if rank == 0:
        for i, (p, o) in enumerate(zip(opt.flat.params, opt.flat.offsets)):
            a, b = outg[0][o:o + p.numel()], outg[1][o:o + p.numel()]
            if not torch.equal(a, b):
                print(f"  step {step}: grad differs: {names.get(id(p), i)} bucket {red.bucket_of[i]} "
                      f"max {float((a - b).abs().max()):.3e}", flush=True)
dist.barrier()
dist.destroy_process_group()
