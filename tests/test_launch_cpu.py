"""Multi-GPU entry points honour their GPU-count flags (no GPU needed: the refusal / clamp paths, the
global-batch split and the cross-rank metric means on a 2-rank gloo group)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ, **kw)
    env.pop("WORLD_SIZE", None)
    env.pop("VITMI_SHARE_GPU", None)
    return env


@pytest.mark.skipif(torch.cuda.device_count() > 0, reason="checks the no-GPU refusal")
def test_bench_gpus_n_refuses_when_gpus_missing():
    """`bench.py --gpus 2` starts 2 ranks itself; with fewer GPUs visible it exits non-zero instead of
    silently running one GPU."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode != 0
    assert "2 ranks requested but 0 GPU(s) visible" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_bench_gpus_must_match_launcher_world():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300,
                       env=dict(_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "--gpus 4 but WORLD_SIZE=2" in r.stderr


@pytest.mark.skipif(torch.cuda.device_count() > 0, reason="checks the no-GPU clamp")
def test_train_n_gpu_is_not_silently_ignored():
    """vitmi.train --n-gpu 2: the reference's setup_device warning and clamp (src/utils.py:44-54) when the
    GPUs are not there, then the loud no-GPU refusal, never a silent one-GPU run."""
    r = subprocess.run([sys.executable, "-m", "vitmi.train", "--n-gpu", "2", "--synthetic", "--checkpoint-path", "",
                        "--no-save"], capture_output=True, text=True, timeout=300,
                       env=dict(_env(), PYTHONPATH=os.path.join(REPO, "vit-of-pytorch_amd")))
    assert r.returncode != 0
    assert "The number of GPU's configured to use is 2, but only 0 are available" in r.stdout
    assert "needs a ROCm GPU" in r.stderr


def test_train_batch_size_is_global():
    from vitmi.train import rank_batch
    assert rank_batch(512, 8) == 64 and rank_batch(256, 1) == 256
    with pytest.raises(SystemExit, match="global batch"):
        rank_batch(30, 4)


def test_train_launcher_world_mismatch(monkeypatch):
    from types import SimpleNamespace

    from vitmi.train import _launched_world
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert _launched_world(SimpleNamespace(n_gpu=1)) == (2, 1, 1)
    assert _launched_world(SimpleNamespace(n_gpu=2)) == (2, 1, 1)
    with pytest.raises(SystemExit, match="--n-gpu 4"):
        _launched_world(SimpleNamespace(n_gpu=4))


def _metric_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vitmi.train import MetricTracker, _rank_mean
    m = MetricTracker("loss", "acc1")
    for v in range(3):  # rank r sees losses r+0, r+1, r+2 (a device-like tensor and a float)
        m.update("loss", torch.tensor(float(rank + v)))
        m.update("acc1", 10.0 * (rank + 1))
    q.put((rank, m.result(), _rank_mean(torch.tensor(float(rank)), 4.0 * rank)))
    dist.barrier()
    dist.destroy_process_group()


def test_metric_means_over_ranks_gloo_world2():
    """train_epoch / valid_epoch results are the means over every rank's batches (the reference computes
    them on the gathered global batch)"""
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_metric_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        result, shown = res[r]
        assert result["loss"] == pytest.approx((0 + 1 + 2 + 1 + 2 + 3) / 6)
        assert result["acc1"] == pytest.approx(15.0)
        assert shown == pytest.approx([0.5, 2.0])
