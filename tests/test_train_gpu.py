"""The src/train.py-style driver on the GPU: single process and 2-rank data parallel (GPU only)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_train_main_b32_synthetic(capsys):
    from vitmi import train
    train.main(["--model-arch", "b32", "--batch-size", "16", "--synthetic", "--checkpoint-path", "",
                "--steps-per-epoch", "4", "--train-steps", "8", "--warmup-steps", "2", "--no-save",
                "--num-classes", "10"])
    out = capsys.readouterr().out
    assert "val_acc1" in out and "loss" in out


def test_train_main_u8_images_through_device_transform(capsys):
    """CIFAR-shaped uint8 32x32 images resized to 224 on the device (vitmi.data) feed the step."""
    from vitmi import train
    train.main(["--model-arch", "b32", "--batch-size", "8", "--synthetic", "--synthetic-source-size", "32",
                "--checkpoint-path", "", "--steps-per-epoch", "4", "--train-steps", "8", "--warmup-steps", "2",
                "--no-save", "--num-classes", "10"])
    out = capsys.readouterr().out
    assert "val_acc1" in out and "loss" in out


def test_device_image_loader_batches_match_oracle_transform():
    import numpy as np

    from oracle.preprocess import transform_batch
    from vitmi.train import DeviceImageLoader
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (10, 32, 32, 3), dtype=np.uint8)
    labels = np.arange(10)
    ld = DeviceImageLoader(imgs, labels, 4, 48, "cuda", train=False)
    got = [(x.cpu().numpy(), y.cpu().numpy()) for x, y in ld]
    assert [len(y) for _, y in got] == [4, 4, 2]
    x = np.concatenate([g[0] for g in got])
    assert np.array_equal(np.concatenate([g[1] for g in got]), labels)
    assert np.array_equal(x, transform_batch(imgs, 48))


@pytest.mark.parametrize("set_to_none", [True, False])
def test_data_parallel_two_ranks_replicas_identical(tmp_path, set_to_none):
    """2 ranks on one GPU over gloo (RCCL needs distinct GPUs): per-layer all-reduce overlapped with
    the backward; both replicas must end bit-identical and equal to one big-batch step. With
    zero_grad(set_to_none=False) the second step accumulates into existing .grad tensors, so the
    reduced buckets must be complete before autograd adds them."""
    script = tmp_path / "dp.py"
    script.write_text(r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.path.join(os.environ["REPO"], "vit-of-pytorch_amd")); sys.path.insert(0, os.environ["REPO"])
from vitmi.model import VisionTransformer, CrossEntropyLoss
from vitmi.optim import SGD
from vitmi.dist import GradAllReducer
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
torch.manual_seed(42)
m = VisionTransformer(image_size=(32, 32), patch_size=(4, 4), emb_dim=128, mlp_dim=256, num_heads=2, num_layers=2,
                      num_classes=10, dropout_rate=0.0).cuda()
eng = m.engine()
red = GradAllReducer(eng, min_bucket_elems=1).attach()
opt = SGD(m.parameters(), lr=0.05, momentum=0.9, model=m)
g = torch.Generator().manual_seed(3)
X = torch.randn(8, 3, 32, 32, generator=g); Y = torch.randint(0, 10, (8,), generator=g)
x, y = X[rank * 4:(rank + 1) * 4].cuda(), Y[rank * 4:(rank + 1) * 4].cuda()
for _ in range(2):
    opt.zero_grad(set_to_none=os.environ["SET_TO_NONE"] == "1")
    CrossEntropyLoss()(m(x), y).backward()
    red.finish()
    opt.step()
torch.cuda.synchronize()
flat = eng.flat.cpu()
out = [torch.zeros_like(flat) for _ in range(world)]
dist.all_gather(out, flat)
if rank == 0:
    assert torch.equal(out[0], out[1]), "replicas diverged"
    # single-process reference: the same 2 steps on the full batch of 8
    red.detach()
    torch.manual_seed(42)
    m2 = VisionTransformer(image_size=(32, 32), patch_size=(4, 4), emb_dim=128, mlp_dim=256, num_heads=2,
                           num_layers=2, num_classes=10, dropout_rate=0.0).cuda()
    opt2 = SGD(m2.parameters(), lr=0.05, momentum=0.9, model=m2)
    for _ in range(2):
        opt2.zero_grad()
        CrossEntropyLoss()(m2(X.cuda()), Y.cuda()).backward()
        opt2.step()
    ref = m2.engine().flat.cpu()
    rel = float((flat - ref).norm() / ref.norm())
    print("rel", rel)
    assert rel < 1e-3, rel
dist.barrier()
dist.destroy_process_group()
open(os.path.join(os.environ["OUTDIR"], f"rank{rank}.ok"), "w").write("ok")
''')
    port = "29533" if set_to_none else "29534"
    env = dict(os.environ, REPO=REPO, OUTDIR=str(tmp_path), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
               SET_TO_NONE="1" if set_to_none else "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", port, str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    # (the ranks' stdout interleaves: each rank leaves a marker file instead)
    assert (tmp_path / "rank0.ok").exists() and (tmp_path / "rank1.ok").exists()
