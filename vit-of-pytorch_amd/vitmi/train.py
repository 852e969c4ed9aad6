"""Training driver, mirroring reference src/train.py on the MI355X HIP engine.

    python -m vitmi.train --model-arch b16 --batch-size 256 --synthetic --checkpoint-path "" --no-save
    python -m vitmi.train --n-gpu 8 --batch-size 512 ...     # data parallel: starts 8 ranks (RCCL)
    torchrun --nproc-per-node 8 -m vitmi.train --n-gpu 8 ... # the same ranks under an outside launcher

Entry points keep the reference signatures: train_epoch (src/train.py:12-37), valid_epoch (:40-66),
save_model (:69-81), main (:84-194); MetricTracker / the step writer follow src/utils.py:79-100,
177-230. Differences, all on the execution side:
  * the model is vitmi.model.VisionTransformer (HIP engine), the optimizer vitmi.optim.SGD
    (torch.optim.SGD semantics, fused HIP update), the scheduler torch's OneCycleLR as configured
    by the reference (:159-163);
  * multi-GPU is one process per GPU with gradient all-reduce over RCCL overlapped with the
    backward (vitmi.dist, attached to the model's engine: the backward hands autograd reduced
    gradients), instead of single-process nn.DataParallel (:128-129). `--n-gpu k` keeps its meaning:
    main() starts k ranks itself (torch.distributed.run, before anything touches the GPU), after
    clamping k to the visible GPUs with the reference's warning (src/utils.py:44-54). `--batch-size`
    stays the GLOBAL batch, as under DataParallel (which scatters it): each rank takes batch/k
    images, and the per-rank mean loss averaged over ranks is the global-batch mean;
  * the printed loss and the returned {loss, acc1, acc5} means are averaged over ranks (what the
    reference computes on the gathered batch);
  * loss / top-1 / top-5 come from the fused cross-entropy kernel's per-row statistics and are
    accumulated on the device, read back when printed, instead of three .item() host syncs per
    step (:29-32); the reported means are the same.
"""
from __future__ import annotations

import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import checkpoint as _ckpt
from .config import get_train_config
from .dist import GradAllReducer
from .model import CrossEntropyLoss, VisionTransformer
from .optim import SGD


def set_seed(seed=42):
    """reference src/data_loaders.py:13-29"""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)


def accuracy(output, target, topk=(1,)):
    """top-k precision in percent (reference src/utils.py:28-41)."""
    maxk = max(topk)
    batch_size = target.size(0)
    _, pred = output.topk(maxk, 1, True, True)
    pred = pred.t()
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    return [correct[:k].reshape(-1).float().sum(0) / batch_size * 100.0 for k in topk]


class StepWriter:
    """The metrics writer interface train_epoch / valid_epoch drive (reference SwanLabWriter,
    src/utils.py:177-230, with SwanLab absent): set_step / add_scalar / log_metric, keeping the
    step, mode and steps_per_sec in memory. Device scalars are kept as detached device tensors (no
    host sync per step); `scalars_host()` reads them back in one batch."""

    def __init__(self, log_dir=None, enabled=False):
        if enabled:
            import warnings
            warnings.warn("StepWriter: no SwanLab / TensorBoard backend in this environment; scalars are kept "
                          "in memory only (log_dir=%r ignored)" % (log_dir,), stacklevel=2)
        self.enabled = False
        self.log_dir = log_dir
        self.step = 0
        self.mode = ""
        self.timer = time.perf_counter()
        self.scalars = []  # (step, tag, value)

    def set_step(self, step, mode="train"):
        self.mode = mode
        self.step = step
        now = time.perf_counter()
        if step != 0:
            # host-side rate between set_step calls: with asynchronous launches this is the rate at which
            # steps are issued, which tracks GPU throughput only once the launch queue is full
            self.log_metric("steps_per_sec", 1.0 / max(now - self.timer, 1e-9))
        self.timer = now

    def add_scalar(self, tag, data, *args, **kwargs):
        if torch.is_tensor(data):
            data = data.detach().clone()
        self.scalars.append((self.step, f"{tag}/{self.mode}" if self.mode else tag, data))
        if len(self.scalars) > 4096:
            del self.scalars[:2048]

    def log_metric(self, tag, data, *args, **kwargs):
        self.add_scalar(tag, data)

    def scalars_host(self):
        """[(step, tag, float)] with every device scalar read back in one transfer"""
        dev = [v for _, _, v in self.scalars if torch.is_tensor(v)]
        host = iter(torch.stack([v.reshape(()).double() for v in dev]).cpu().tolist()) if dev else iter(())
        return [(s, t, next(host) if torch.is_tensor(v) else float(v)) for s, t, v in self.scalars]


class MetricTracker:
    """Running means of named scalars (reference src/utils.py:79-100), device-resident."""

    def __init__(self, *keys, writer=None):
        self.writer = writer if writer is not None else StepWriter()
        self.keys = keys
        self.reset()

    def reset(self):
        self._total = {k: 0.0 for k in self.keys}
        self._count = {k: 0 for k in self.keys}

    def update(self, key, value, n=1):
        if self.writer is not None:
            self.writer.add_scalar(key, value)
        self._total[key] = self._total[key] + value * n
        self._count[key] += n

    def avg(self, key):
        t = self._total[key]
        t = float(t) if torch.is_tensor(t) else t
        return t / max(1, self._count[key])

    def result(self):
        if dist.is_initialized() and dist.get_world_size() > 1:
            return self._result_all_ranks()
        return {k: self.avg(k) for k in self.keys}

    def _result_all_ranks(self):
        """means over every rank's batches (equal per-rank batch sizes: the mean of rank means)"""
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
        tot = [self._total[k] for k in self.keys]
        t = torch.stack([(v.detach().double().to(dev) if torch.is_tensor(v) else torch.tensor(float(v), dtype=torch.float64,
                                                                                           device=dev)) for v in tot] +
                        [torch.tensor(float(self._count[k]), dtype=torch.float64, device=dev) for k in self.keys])
        dist.all_reduce(t)
        n = len(self.keys)
        return {k: float(t[i]) / max(1.0, float(t[n + i])) for i, k in enumerate(self.keys)}


def _step_accuracy(criterion, pred, target):
    """top-1 / top-5 (%) of the batch: from the fused CE kernel's per-row hit counts when the
    criterion is vitmi's CrossEntropyLoss (no extra pass), else src/utils.py:28-41's topk."""
    st = getattr(criterion, "last_row_stats", None)
    if st is not None and st.shape[0] == target.shape[0]:
        return st[:, 1].mean() * 100.0, st[:, 2].mean() * 100.0
    return accuracy(pred.detach(), target, topk=(1, 5))


class SyntheticDataLoader:
    """Synthetic N(0,1) images / uniform labels generated on the device (no host copies)."""

    def __init__(self, batch_size, image_size, num_classes, steps, device, seed=0):
        self.batch_size, self.image_size, self.num_classes, self.steps = batch_size, image_size, num_classes, steps
        g = torch.Generator(device=device).manual_seed(seed)
        self.x = torch.randn(batch_size, 3, image_size, image_size, device=device, generator=g)
        self.y = torch.randint(0, num_classes, (batch_size,), device=device, generator=g)

    def __len__(self):
        return self.steps

    def __iter__(self):
        for _ in range(self.steps):
            yield self.x, self.y


class DeviceImageLoader:
    """Batches of uint8 HWC images kept resident in HBM (CIFAR-100 train is 150 MB of uint8), run
    through the reference loader's transform on the device (vitmi.data.GPUTransform:
    Resize -> RandomHorizontalFlip -> ToTensor -> Normalize, src/data_loaders.py:66-80). Shuffled
    per epoch with a seeded generator like the reference's DataLoader (`:84-92`); a ragged last
    batch is kept (drop_last=False)."""

    def __init__(self, images_u8, labels, batch_size, image_size, device, train=True, seed=42):
        from .data import GPUTransform
        self.images = torch.as_tensor(images_u8, dtype=torch.uint8).to(device).contiguous()
        self.labels = torch.as_tensor(labels, dtype=torch.int64).to(device)
        if self.images.dim() != 4 or self.images.shape[3] != 3 or self.labels.numel() != self.images.shape[0]:
            raise ValueError("DeviceImageLoader: images uint8 [n, H, W, 3] and n labels")
        self.batch_size, self.train = batch_size, train
        self.generator = torch.Generator().manual_seed(seed)
        self.transform = GPUTransform(image_size, train=train, generator=self.generator)

    def __len__(self):
        return (self.images.shape[0] + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = self.images.shape[0]
        order = torch.randperm(n, generator=self.generator) if self.train else torch.arange(n)
        order = order.to(self.images.device)
        for s in range(0, n, self.batch_size):
            idx = order[s:s + self.batch_size]
            yield self.transform(self.images.index_select(0, idx)), self.labels.index_select(0, idx)


def _world():
    return dist.get_world_size() if dist.is_initialized() else 1


def _rank_mean(*vals):
    """host floats of device / host scalars, averaged over ranks when data parallel"""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [float(v) for v in vals]
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.stack([torch.as_tensor(v, dtype=torch.float64).to(dev).reshape(()) for v in vals])
    dist.all_reduce(t)
    return [float(v) / dist.get_world_size() for v in t]


def train_epoch(epoch, model, data_loader, criterion, optimizer, lr_scheduler, metrics, device=torch.device("cpu")):
    """reference src/train.py:12-37 (one optimizer step per batch)."""
    metrics.reset()
    for batch_idx, (batch_data, batch_target) in enumerate(data_loader):
        batch_data = batch_data.to(device, non_blocking=True)
        batch_target = batch_target.to(device, non_blocking=True)
        optimizer.zero_grad()
        batch_pred = model(batch_data)
        loss = criterion(batch_pred, batch_target)
        loss.backward()
        optimizer.step()
        lr_scheduler.step()
        acc1, acc5 = _step_accuracy(criterion, batch_pred, batch_target)
        metrics.writer.set_step((epoch - 1) * len(data_loader) + batch_idx)
        metrics.update("loss", loss.detach())
        metrics.update("acc1", acc1)
        metrics.update("acc5", acc5)
        if batch_idx % 100 == 0:
            shown = _rank_mean(loss.detach(), acc1, acc5)
            if not dist.is_initialized() or dist.get_rank() == 0:
                print("Train Epoch: {:03d} Batch: {:05d}/{:05d} Loss: {:.4f} Acc@1: {:.2f}, Acc@5: {:.2f}"
                      .format(epoch, batch_idx, len(data_loader), *shown), flush=True)
    return metrics.result()


def valid_epoch(epoch, model, data_loader, criterion, metrics, device=torch.device("cpu")):
    """reference src/train.py:40-66 (forward-only; means over batches)."""
    metrics.reset()
    losses, acc1s, acc5s = [], [], []
    with torch.no_grad():
        for batch_data, batch_target in data_loader:
            batch_data = batch_data.to(device)
            batch_target = batch_target.to(device)
            batch_pred = model(batch_data)
            loss = criterion(batch_pred, batch_target)
            acc1, acc5 = _step_accuracy(criterion, batch_pred, batch_target)
            losses.append(loss)
            acc1s.append(acc1)
            acc5s.append(acc5)
    metrics.writer.set_step(epoch, "valid")
    metrics.update("loss", float(torch.stack(losses).mean()))
    metrics.update("acc1", float(torch.stack(acc1s).mean()))
    metrics.update("acc5", float(torch.stack(acc5s).mean()))
    return metrics.result()


def save_model(save_dir, epoch, model, optimizer, lr_scheduler, device_ids=(), best=False):
    """Checkpoint format of reference src/train.py:69-81."""
    state = {
        "epoch": epoch,
        "state_dict": model.state_dict(),
        "optimizer": optimizer.state_dict(),
        "lr_scheduler": lr_scheduler.state_dict(),
    }
    torch.save(state, str(save_dir + "current.pth"))
    if best:
        torch.save(state, str(save_dir + "best.pth"))


def load_checkpoint(path):
    """Weights of a reference .pth or JAX .npz checkpoint (src/checkpoint.py:7-17)."""
    return _ckpt.load_checkpoint(path)


def build_model(config, device):
    return VisionTransformer(image_size=(config.image_size, config.image_size),
                             patch_size=(config.patch_size, config.patch_size), emb_dim=config.emb_dim,
                             mlp_dim=config.mlp_dim, num_heads=config.num_heads, num_layers=config.num_layers,
                             num_classes=config.num_classes, attn_dropout_rate=config.attn_dropout_rate,
                             dropout_rate=config.dropout_rate)


def _launched_world(config):
    """(world, rank, local rank) of this process. Under torch.distributed.run the environment says;
    --n-gpu must then be 1 (unset) or equal to WORLD_SIZE."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and config.n_gpu not in (1, world):
        raise SystemExit(f"--n-gpu {config.n_gpu} but the launcher started WORLD_SIZE={world} ranks")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def rank_batch(global_batch, world):
    """images per rank for a global --batch-size (DataParallel scatter semantics, src/train.py:128-129)"""
    if global_batch % world:
        raise SystemExit(f"--batch-size {global_batch} is the global batch and must divide evenly over {world} "
                         "GPUs (every rank's mean loss carries the same weight in the averaged gradient)")
    return global_batch // world


def main(argv=None):
    config = get_train_config(argv)
    if "WORLD_SIZE" not in os.environ and config.n_gpu > 1:
        # reference setup_device (src/utils.py:44-54): clamp to the visible GPUs with a warning;
        # then one rank per GPU, started here before any HIP call (device_count() makes none)
        n = torch.cuda.device_count()
        k = config.n_gpu
        if k > n and not os.environ.get("VITMI_SHARE_GPU"):
            print("Warning: The number of GPU's configured to use is {}, but only {} are available on this "
                  "machine.".format(k, n))
            k = n
        if k > 1:
            rank_batch(config.batch_size, k)
            import subprocess
            from socket import socket
            with socket() as s_:
                s_.bind(("127.0.0.1", 0))
                port = str(s_.getsockname()[1])
            args = list(sys.argv[1:] if argv is None else argv)
            args += ["--n-gpu", str(k)]  # (argparse: the last occurrence wins)
            pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            env = dict(os.environ, VITMI_EXP_STAMP=getattr(config, "exp_stamp", ""))
            env["PYTHONPATH"] = os.pathsep.join([pkg] + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
            rc = subprocess.call([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                                  f"--nproc-per-node={k}", "--master-addr", "127.0.0.1", "--master-port", port,
                                  "-m", "vitmi.train", *args], env=env)
            if rc:
                raise SystemExit(rc)
            return None
        config.n_gpu = k
    set_seed(config.seed)
    world, rank, local = _launched_world(config)
    if not torch.cuda.is_available():
        raise SystemExit("vitmi.train needs a ROCm GPU (MI355X)")
    if os.environ.get("VITMI_SHARE_GPU"):  # functional rehearsal of the N>1 path on fewer GPUs (gloo)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        from .dist import init_process_group
        init_process_group(device=device)
    batch = rank_batch(config.batch_size, world)

    model = build_model(config, device)
    if config.checkpoint_path:
        state_dict = load_checkpoint(config.checkpoint_path)
        if config.num_classes != state_dict["classifier.weight"].size(0):
            del state_dict["classifier.weight"]
            del state_dict["classifier.bias"]
            print("re-initialize fc layer")
            model.load_state_dict(state_dict, strict=False)
        else:
            model.load_state_dict(state_dict)
        print("Load pretrained weights from {}".format(config.checkpoint_path))
    model = model.to(device)
    engine = model.engine()
    if world > 1:
        dist.broadcast(engine.flat, 0)  # identical replicas
        GradAllReducer(engine).attach()  # the backward returns all-reduced (averaged) gradients

    if not config.synthetic:
        raise SystemExit("torchvision datasets are not available in this environment; use --synthetic "
                         "(the input pipeline is outside the MI355X hot path, SURVEY.md §2 row 5)")
    if config.synthetic_source_size > 0:
        # uint8 images (CIFAR-shaped when 32) through the device-side reference transform
        g = torch.Generator().manual_seed(config.seed + rank)
        n = batch * config.steps_per_epoch
        src = torch.randint(0, 256, (n, config.synthetic_source_size, config.synthetic_source_size, 3),
                            generator=g, dtype=torch.uint8)
        train_loader = DeviceImageLoader(src, torch.randint(0, config.num_classes, (n,), generator=g),
                                         batch, config.image_size, device, seed=config.seed + rank)
    else:
        train_loader = SyntheticDataLoader(batch, config.image_size, config.num_classes,
                                           config.steps_per_epoch, device, seed=config.seed + rank)
    valid_loader = SyntheticDataLoader(batch, config.image_size, config.num_classes,
                                       max(1, config.steps_per_epoch // 10), device, seed=10_000 + config.seed + rank)

    criterion = CrossEntropyLoss()
    optimizer = SGD(params=model.parameters(), lr=config.lr, weight_decay=config.wd, momentum=0.9, model=model)
    lr_scheduler = torch.optim.lr_scheduler.OneCycleLR(optimizer=optimizer, max_lr=config.lr,
                                                       pct_start=config.warmup_steps / config.train_steps,
                                                       total_steps=config.train_steps)
    writer = StepWriter(config.summary_dir, config.swanlab)
    metric_names = ["loss", "acc1", "acc5"]
    train_metrics = MetricTracker(*metric_names, writer=writer)
    valid_metrics = MetricTracker(*metric_names, writer=writer)
    best_acc = 0.0
    epochs = config.train_steps // len(train_loader)  # the reference's count (src/train.py:172): may be 0
    if rank == 0:
        print(config.train_steps, len(train_loader), epochs)
    for epoch in range(1, epochs + 1):
        log = {"epoch": epoch}
        model.train()
        log.update(train_epoch(epoch, model, train_loader, criterion, optimizer, lr_scheduler, train_metrics, device))
        model.eval()
        result = valid_epoch(epoch, model, valid_loader, criterion, valid_metrics, device)
        log.update(**{"val_" + k: v for k, v in result.items()})
        best = log["val_acc1"] > best_acc
        if best:
            best_acc = log["val_acc1"]
        if rank == 0 and not config.no_save:
            save_model(config.checkpoint_dir, epoch, model, optimizer, lr_scheduler, best=best)
        if rank == 0:
            for key, value in log.items():
                print("    {:15s}: {}".format(str(key), value), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return best_acc


if __name__ == "__main__":
    main(sys.argv[1:])
