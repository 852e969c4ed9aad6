"""Data-parallel gradient exchange (vitmi.dist.GradAllReducer) on a 2-rank gloo group (CPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _FakeLayout:
    def __init__(self, sizes):
        self.buckets = []
        off = 0
        names = ["head"] + [f"layer{i}" for i in reversed(range(len(sizes) - 2))] + ["embed"]
        for n, s in zip(names, sizes):
            self.buckets.append((n, off, off + s))
            off += s
        self.numel = off


class _FakeEngine:
    """Stands in for vitmi.engine.ViTEngine: a flat CPU grad buffer + bucket layout + hook slot."""

    def __init__(self, sizes):
        self.layout = _FakeLayout(sizes)
        self.grad = torch.zeros(self.layout.numel)
        self.dev = torch.device("cpu")
        self.grad_ready_hook = None

    def backward(self, rank):
        # fill each bucket as the real backward would, releasing it through the hook in order
        for name, s, e in self.layout.buckets:
            self.grad[s:e] = torch.arange(s, e, dtype=torch.float32) * (rank + 1)
            if self.grad_ready_hook:
                self.grad_ready_hook(self.grad, name, s, e)


def _worker(rank, world, port, sizes, average, q, compress=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vitmi.dist import GradAllReducer
    eng = _FakeEngine(sizes)
    red = GradAllReducer(eng, min_bucket_elems=50, average=average, compress=compress).attach()
    for _ in range(2):  # two steps: buckets re-used
        eng.backward(rank)
        red.finish()
    q.put((rank, eng.grad.clone()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("average,compress", [(True, None), (False, None), (True, "bf16")])
def test_grad_allreduce_gloo_world2(average, compress):
    world = 2
    sizes = [10, 100, 100, 100, 37]  # head (coalesced with layer2: below min_bucket), layers, embed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, average, q, compress)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = sum(sizes)
    base = torch.arange(n, dtype=torch.float32)
    expect = base * (1 + 2) / (world if average else 1)
    if compress == "bf16":  # each rank's bucket and the sum rounded to bf16
        expect = ((base.bfloat16().float() + (base * 2).bfloat16().float()).bfloat16().float()) / world
    for r in range(world):
        assert torch.allclose(res[r], expect), r
    assert torch.equal(res[0], res[1])  # replicas bit-identical


def _replica_worker(rank, world, port, differ, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    flat = torch.linspace(-3, 3, 10007)
    if differ and rank == 1:
        flat[5000] = torch.nextafter(flat[5000], torch.tensor(10.0))  # one ulp on one element
    out = bench.replica_check(flat, 1.0 + 0.5 * rank, 10, world, "gloo", torch.device("cpu"))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("differ", [False, True])
def test_bench_replica_check_gloo(differ):
    """bench.py's N > 1 self-check (2 gloo ranks on the CPU): every rank's time is gathered (the job's time is
    the max), and the flat-parameter fingerprints agree iff the replicas are bit-identical — a one-ulp
    difference on one element of one rank is caught."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_replica_worker, args=(r, 2, port, differ, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        o = res[r]
        assert o["ranks_seen"] == 2 and o["backend"] == "gloo"
        assert o["_dt_max"] == 1.5
        assert o["ms_per_step_per_rank"] == [100.0, 150.0]
        assert o["replicas_identical"] is (not differ)


def _exchange_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from vitmi.dist import GradAllReducer
    sizes = [10, 100, 100, 100, 37]
    eng = _FakeEngine(sizes)
    red = GradAllReducer(eng, min_bucket_elems=50).attach()

    def step():
        eng.backward(rank)
        red.finish()
    out = bench.exchange_check(step, red, 0.5, 10, world, torch.device("cpu"), lambda: None, solo_steps=3)
    attached = eng.grad_ready_hook is not None
    q.put((rank, out, attached))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_exchange_check_gloo():
    """bench.py's N > 1 exchange accounting (2 gloo ranks on the CPU): one step with the reducer's accounting on
    gives the all-reduced bytes of the whole flat buffer (four buckets: the head coalesced with the next layer),
    a solo timing with the reducer detached, the exposed time as their difference; the reducer is re-attached."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (o, a) for r, o, a in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        o, attached = res[r]
        assert attached
        assert o["allreduce_bytes_per_step"] == 4 * (10 + 100 + 100 + 100 + 37)
        assert o["allreduce_ms_per_step"] >= 0.0 and o["solo_ms_per_step"] >= 0.0
        assert abs(o["exposed_comm_ms_per_step"] - (50.0 - o["solo_ms_per_step"])) < 1e-2
