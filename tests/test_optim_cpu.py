"""Res-ViT training-step host logic on CPU: the cosine schedules (res-vit/train.py:280-291), the
config surface (res-vit/config.py), and the flat-gradient all-reduce ordering on a 2-rank gloo group."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _lrs(sched_fn, steps, lr=1e-4):
    opt = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=lr)
    s = sched_fn(opt)
    out = []
    for _ in range(steps):
        out.append(opt.param_groups[0]["lr"])
        opt.step()
        s.step()
    return out


@pytest.mark.parametrize("warmup,total", [(500, 15000), (2, 10), (0, 7), (10, 10)])
def test_cosine_warmup_schedule_matches_transformers(warmup, total):
    """vitmi.optim.get_cosine_schedule_with_warmup vs transformers' own (the reference's dependency,
    installed here), every step past the end"""
    tr = pytest.importorskip("transformers")
    from vitmi.optim import get_cosine_schedule_with_warmup
    mine = _lrs(lambda o: get_cosine_schedule_with_warmup(o, warmup, total), total + 3)
    ref = _lrs(lambda o: tr.get_cosine_schedule_with_warmup(o, warmup, total), total + 3)
    assert mine == ref


def test_schedule_matches_the_training_fixture(golden_dir):
    """the lr of each of the reference's three recorded steps (tests/golden/resvit_train3.npz)"""
    from vitmi.optim import get_cosine_schedule_with_warmup
    g = np.load(os.path.join(golden_dir, "resvit_train3.npz"))
    lr, _, _, _, _, warm, total = g["hparams"].tolist()[:7]
    mine = _lrs(lambda o: get_cosine_schedule_with_warmup(o, int(warm), int(total)), 3, lr)
    assert mine == [float(g[f"s{s}/lr"]) for s in range(3)]


def test_resvit_config_defaults_match_reference():
    """res-vit/config.py:122-184 defaults, including the type=bool switches (any non-empty string is True)"""
    from vitmi.resvit_train import config_to_model_args, get_train_config, set_model_architecture
    c = get_train_config([])
    assert (c.lr, c.wd, c.beta1, c.beta2, c.eps) == (1e-4, 0.05, 0.9, 0.999, 1e-8)
    assert (c.lr_scheduler, c.warmup_steps, c.train_steps, c.clip_grad_norm) == ("cosine_with_warmup", 500, 15000, True)
    assert (c.initial_lambda_active, c.initial_lambda_distill, c.initial_lambda_class) == (1e-4, 1e-2, 1)
    assert (c.use_lora, c.use_reslr, c.block_size, c.lora_rank, c.num_classes) == (True, True, 1, 8, 100)
    assert get_train_config(["--use_lora", "False"]).use_lora is True  # the reference's argparse quirk
    assert get_train_config(["--use_lora", ""]).use_lora is False
    a = set_model_architecture(config_to_model_args(c), "l16")
    assert (a.dim, a.mlp_dim, a.n_layers, a.n_heads, a.dynamic_start_layer) == (1024, 4096, 24, 16, 2)


class _FakeFlat:
    """stands in for vitmi.flat.FlatParams: CPU flat gradient, segments, used flags, hook slot"""

    def __init__(self, sizes):
        self.params = [torch.zeros(s) for s in sizes]
        self.offsets, off = [], 0
        for s in sizes:
            self.offsets.append(off)
            off += s
        self.numel, self.nseg = off, len(sizes)
        self.grad = torch.zeros(off)
        self.device = torch.device("cpu")
        self.used_host = [False] * self.nseg
        self.used = torch.zeros(self.nseg)
        self.used_reduced = False
        self.on_grad = None

    def upload_used(self):
        self.used.copy_(torch.tensor(self.used_host, dtype=torch.float32))
        return self.used

    def backward(self, rank, skip):
        for i in range(self.nseg):
            if i in skip:
                continue
            o = self.offsets[i]
            self.grad[o:o + self.params[i].numel()] = float(i + 1) * (rank + 1)
            self.used_host[i] = True
            self.on_grad(i)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vitmi.dist import FlatGradAllReducer
    f = _FakeFlat([5, 7, 3, 11, 2])
    red = FlatGradAllReducer(f, bucket_elems=8).attach()
    # rank 0 never touches segment 1 (an approximator no token was routed to), rank 1 never segment 3:
    # bucket completion differs between ranks, the collective order must not
    f.backward(rank, skip={1} if rank == 0 else {3})
    red.finish()
    q.put((rank, f.grad.clone(), f.used.clone(), f.used_reduced, len(red.buckets)))
    dist.barrier()
    dist.destroy_process_group()


def test_flat_grad_allreduce_gloo_world2_in_order():
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes, offs = [5, 7, 3, 11, 2], [0, 5, 12, 15, 26]
    expect = torch.zeros(28)
    for i, (o, s) in enumerate(zip(offs, sizes)):
        contrib = [(i + 1) * 1 if i != 1 else 0, (i + 1) * 2 if i != 3 else 0]
        expect[o:o + s] = sum(contrib) / world
    for r in range(world):
        grad, used, reduced, nb = res[r]
        assert torch.allclose(grad, expect), (r, grad)
        assert used.tolist() == [2.0, 1.0, 2.0, 1.0, 2.0] and reduced and nb >= 3
