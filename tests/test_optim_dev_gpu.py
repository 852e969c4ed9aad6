"""The parameter update of bench.py's timed step: vit_sgd_step_dev driven by bench.onecycle_hyper_table.

Reference: torch.optim.SGD(momentum, weight_decay) + OneCycleLR as configured in src/train.py:154-163; the oracle
restates both (oracle/vit_oracle.py: sgd_step, OneCycle). The device-scalar kernel must be bit-identical to the
host-scalar one (one templated body, csrc/elementwise.hip) and follow the oracle's trajectory, including the first
step's buffer semantics (buf = d, whatever the buffer held) and the schedule's momentum cycling.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import onecycle_hyper_table  # noqa: E402
from oracle.vit_oracle import OneCycle, sgd_step  # noqa: E402
from vitmi import ops  # noqa: E402


@pytest.mark.parametrize("n,wd", [(1_000_003, 0.0), (4099, 1e-4)])
def test_sgd_dev_follows_bench_table_host_path_and_oracle(n, wd):
    dev = "cuda"
    table = onecycle_hyper_table(25, dev)  # bench.py's default warmup 5 + steps 20
    oc = OneCycle(0.03, 15000, 500 / 15000)
    gen = torch.Generator().manual_seed(7)
    p0 = torch.randn(n, generator=gen)
    grads = [torch.randn(n, generator=gen) for _ in range(3)]
    # device-scalar path (the bench's) and host-scalar path, each with a garbage initial momentum buffer
    p_d, p_h = p0.cuda(), p0.cuda()
    buf_d = torch.full((n,), 123.0, device=dev)
    buf_h = torch.full((n,), -7.0, device=dev)
    mir_d = torch.empty(n, device=dev, dtype=torch.bfloat16)
    mir_h = torch.empty(n, device=dev, dtype=torch.bfloat16)
    hyper = table[0].clone()
    ref, bufs = {"w": p0.clone()}, {}
    for k in range(3):
        lr32, mom32, first = (float(v) for v in table[k].cpu())
        lr, mom = oc.at(k)
        assert first == (1.0 if k == 0 else 0.0)
        assert abs(lr32 - lr) <= 1e-7 * lr and abs(mom32 - mom) <= 1e-7 * mom, (k, lr32, lr, mom32, mom)
        g = grads[k].cuda()
        ops.copy2d(hyper, 12, table[k], 12, 12, 1)  # the bench's per-step refresh
        ops.sgd_step_dev(p_d, g, buf_d, mir_d, n, hyper, wd)
        ops.sgd_step(p_h, g, buf_h, mir_h, n, lr32, mom32, wd, k == 0)
        ref, bufs = sgd_step(ref, {"w": grads[k]}, bufs, lr, mom, wd, first=(k == 0))
        torch.cuda.synchronize()
        assert torch.equal(p_d, p_h) and torch.equal(buf_d, buf_h) and torch.equal(mir_d, mir_h), k
        assert torch.equal(mir_d, p_d.bfloat16()), k
        # the oracle runs in fp32 with double scalars (and unfused multiply-add): agreement to fp32 rounding
        assert float((p_d.cpu().double() - ref["w"].double()).abs().max()) <= 1e-6 * (1 + float(ref["w"].abs().max()))
        assert float((buf_d.cpu().double() - bufs["w"].double()).abs().max()) <= 1e-6 * (1 + float(bufs["w"].abs().max()))
    # momentum cycles down during the warm-up (cycle_momentum: max 0.95 -> base 0.85)
    assert float(table[0, 1]) > float(table[2, 1])
