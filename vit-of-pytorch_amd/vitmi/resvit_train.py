"""Res-ViT training driver, mirroring reference res-vit/train.py on the MI355X HIP path.

    python -m vitmi.resvit_train --synthetic --checkpoint-path "" --no-save
    python -m vitmi.resvit_train --n-gpu 8 --batch-size 256 --synthetic ...   # data parallel (RCCL)

The step is the reference's (res-vit/train.py:23-68): zero_grad, forward (teacher + routed student
paths, vitmi.resvit), total = lambda_class c_loss + lambda_active a_loss + lambda_distill d_loss,
backward, clip_grad_norm_(params, 1.0), AdamW.step(), the cosine schedule's step. Execution side:
  * the optimizer is vitmi.optim.AdamW: the trainable parameters live in one flat buffer and the
    clip + update are three launches (csrc/optim.hip); `fused_clip` folds the clip into the update;
  * data parallelism (new: the reference is single-device, res-vit/train.py:222,246): one process per
    GPU, the flat gradient buckets all-reduced over RCCL as the backward finishes them
    (vitmi.dist.FlatGradAllReducer), `--batch-size` global and split over the ranks;
  * losses / accuracies are accumulated on the device and read back when printed.
Flags are res-vit/config.py's (:122-184), including its `type=bool` switches (any non-empty value is
True), plus --synthetic / --steps-per-epoch / --no-save / --n-gpu.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.distributed as dist

from . import resvit
from .optim import AdamW, clip_grad_norm_, get_cosine_schedule_with_warmup
from .config import process_config
from .flat import sinks as _flat_sinks
from .train import MetricTracker, StepWriter, SyntheticDataLoader, _rank_mean, rank_batch, set_seed

METRICS = ["loss", "c_loss", "a_loss", "d_loss", "router_entropy", "acc1", "acc5", "active_ratio", "lr",
           "current_target"]


def _topk(logits, target):
    """top-1 / top-5 percent (res-vit/utils.py:30-43), device scalars"""
    k = min(5, logits.shape[1])
    _, pred = logits.topk(k, 1, True, True)
    correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
    b = target.numel()
    return correct[:1].reshape(-1).float().sum() / b * 100.0, correct[:k].reshape(-1).float().sum() / b * 100.0


def total_loss(model, c_loss, a_loss, d_loss, lambda_active, lambda_distill, lambda_class):
    """res-vit/train.py:54-58"""
    if model.use_reslr:
        return lambda_class * c_loss + lambda_active * a_loss + lambda_distill * d_loss
    return lambda_class * c_loss


def train_step(model, x, y, optimizer, lr_scheduler=None, lambda_active=10.0, lambda_distill=1.0, lambda_class=10.0,
               clip_grad_norm=True, reducer=None):
    """one batch of res-vit/train.py:23-68; returns (total, c, a, d, r_entropy, active_metric) as device values"""
    optimizer.zero_grad()
    c_loss, a_loss, d_loss, r_entropy, active_metric = model(x, y)
    total = total_loss(model, c_loss, a_loss, d_loss, lambda_active, lambda_distill, lambda_class)
    with _flat_sinks():
        total.backward()
    if reducer is not None:
        reducer.finish()
    if clip_grad_norm:
        if isinstance(optimizer, AdamW):
            if optimizer.max_grad_norm is None:
                clip_grad_norm_(None, max_norm=1.0, norm_type=2, flat=optimizer)
        else:
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0, norm_type=2)
    optimizer.step()
    if lr_scheduler is not None:
        lr_scheduler.step()
    return total, c_loss, a_loss, d_loss, r_entropy, active_metric


class GraphedTrainStep:
    """train_step with its forward + backward captured once in a HIP graph and replayed.

    The Res-ViT step is launch-bound when issued op by op (about 2,300 kernels at Res-ViT-B/16 bs 128, many
    of them the small routing / selection ops of the reference's model, res-vit/model.py:133-211,336-368):
    the host's issue rate leaves the GPU idle for a fifth of the step. Captured, the forward (teacher +
    routed student), the losses and the backward replay as one graph; zero_grad, the clip + AdamW update
    (three launches) and the LR schedule run eagerly after it, so the optimizer keeps reading its host
    hyper-parameters. The step's data-dependent decisions are all on the device already (routing masks,
    the approximators' participation flags of vitmi.flat.gate), so the graph computes exactly what
    train_step does; its inputs are the static `x` / `y` buffers (copy a new batch in with `step(x, y)`)
    and its outputs are static tensors overwritten by every replay.

    Data parallel (res-vit/train.py:23-68 on every rank): pass the rank's FlatGradAllReducer as `reducer`. Its
    per-parameter hooks stay detached (no collective is captured); after each replay the whole flat gradient is
    all-reduced bucket by bucket, with the used flags, by reducer.finish() before the clip + AdamW update. The
    trainable set is small (LoRA, routers, approximators, head: a few MB), so the exchange after the backward costs
    a fraction of a millisecond where the eager step's overlap would have hidden it, against the eager step's
    host-bound launch gaps. Without a reducer it raises when a torch.distributed group of more than one rank is
    initialised.

    Construction runs `warmup` forward + backward passes on `x` / `y` (no optimizer or scheduler step; the
    gradients are zeroed after them, and the torch CPU / CUDA RNG states are restored, so the Gumbel draws
    of the warm-up do not shift the run's random stream): the model's parameters, the optimizer's moments
    and the learning-rate schedule are exactly as they were before the constructor.
    """

    def __init__(self, model, x, y, optimizer, lr_scheduler=None, lambda_active=10.0, lambda_distill=1.0,
                 lambda_class=10.0, clip_grad_norm=True, warmup=1, reducer=None):
        from . import flat as _flat
        if not isinstance(optimizer, AdamW):
            raise TypeError("GraphedTrainStep: vitmi.optim.AdamW (flat gradients at fixed addresses) expected")
        if reducer is None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            raise RuntimeError("GraphedTrainStep with more than one rank needs the rank's FlatGradAllReducer "
                               "(reducer=...): the exchange runs after each replay")
        if reducer is not None:
            if reducer.flat is not optimizer.flat:
                raise ValueError("GraphedTrainStep: the reducer must own the optimizer's flat gradient buffer")
            reducer.detach()  # no collective inside the warm-up or the capture: finish() exchanges after the replay
        self.reducer = reducer
        self.model, self.opt, self.sched = model, optimizer, lr_scheduler
        self.lambdas = (lambda_active, lambda_distill, lambda_class)
        self.clip = clip_grad_norm
        self.x, self.y = x.clone(), y.clone()
        self._flat = _flat
        # eager warm-up (lazy initialisation, cached device constants, kernel attributes) on the side stream the
        # graph is then captured on: autograd runs each parameter's gradient accumulation on the stream its
        # AccumulateGrad node was created on, and the model keeps the warm-up's graph (and those nodes) alive
        # through `model.logits`; on any other stream the accumulation would escape the capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        rng = (torch.get_rng_state(), torch.cuda.get_rng_state())
        with torch.cuda.stream(s):
            for _ in range(warmup):  # forward + backward only: no parameter, moment or schedule changes
                optimizer.zero_grad()
                c_loss, a_loss, d_loss, r_entropy, active_metric = model(self.x, self.y)
                total = total_loss(model, c_loss, a_loss, d_loss, *self.lambdas)
                with _flat.sinks():
                    total.backward()
            optimizer.zero_grad()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        torch.set_rng_state(rng[0])
        torch.cuda.set_rng_state(rng[1])
        f = optimizer.flat
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            c_loss, a_loss, d_loss, r_entropy, active_metric = model(self.x, self.y)
            total = total_loss(model, c_loss, a_loss, d_loss, *self.lambdas)
            with _flat.sinks():
                total.backward()
        self.outputs = (total, c_loss, a_loss, d_loss, r_entropy, active_metric)
        # what the captured pass left on the host: the used flags (post-accumulate hooks) and the gated
        # parameters' device flags (graph outputs, refreshed by every replay)
        self.used = list(f.used_host)
        self.gates = [(p, e[1]) for p in f.params for e in [_flat._GATES.get(id(p))] if e is not None and e[0]() is p]

    def step(self, x=None, y=None):
        """one training step; returns train_step's tuple (static device tensors: clone what you keep)"""
        import weakref
        if x is not None:
            self.x.copy_(x)
            self.y.copy_(y)
        f = self.opt.flat
        self.opt.zero_grad()
        self.graph.replay()
        f.used_host = list(self.used)
        for p, flag in self.gates:
            self._flat._GATES[id(p)] = (weakref.ref(p), flag)
        if self.reducer is not None:
            self.reducer.finish()  # every bucket in order + the used flags over the ranks; the stream waits
        if self.clip and self.opt.max_grad_norm is None:
            clip_grad_norm_(None, max_norm=1.0, norm_type=2, flat=self.opt)
        self.opt.step()
        if self.sched is not None:
            self.sched.step()
        return self.outputs


def train_epoch(epoch, model, data_loader, optimizer, metrics, config, lr_scheduler=None, lambda_active=10.0,
                lambda_distill=1.0, lambda_class=10.0, device=torch.device("cpu"), save_routing_viz=False,
                reducer=None):
    """res-vit/train.py:11-104 (routing visualisation is not produced: no image writer here)"""
    metrics.reset()
    if metrics.writer is not None:
        metrics.writer.set_step(epoch * len(data_loader), mode="train")
    for batch_idx, (batch_data, batch_target) in enumerate(data_loader):
        batch_data = batch_data.to(device)
        batch_target = batch_target.to(device)
        total, c_loss, a_loss, d_loss, r_entropy, active_metric = train_step(
            model, batch_data, batch_target, optimizer, lr_scheduler, lambda_active, lambda_distill, lambda_class,
            getattr(config, "clip_grad_norm", True), reducer)
        if not model.use_reslr:
            a_loss = d_loss = r_entropy = torch.tensor(0.0)
            active_metric = {"non_low_rank_ratio": torch.tensor(0.0), "current_target": torch.tensor(0.0)}
        acc1, acc5 = _topk(model.logits.detach(), batch_target)
        metrics.writer.set_step(epoch * len(data_loader) + batch_idx, mode="train")
        for k, v in (("loss", total), ("c_loss", c_loss), ("a_loss", a_loss), ("d_loss", d_loss),
                     ("router_entropy", r_entropy), ("acc1", acc1), ("acc5", acc5),
                     ("active_ratio", active_metric["non_low_rank_ratio"]),
                     ("lr", optimizer.param_groups[0]["lr"]), ("current_target", active_metric["current_target"])):
            metrics.update(k, v.detach() if torch.is_tensor(v) else v)
        if batch_idx % getattr(config, "print_freq", 100) == 0:
            vals = _rank_mean(acc1, acc5, total.detach(), c_loss.detach(), torch.as_tensor(a_loss).detach(),
                              torch.as_tensor(d_loss).detach(), active_metric["non_low_rank_ratio"],
                              torch.as_tensor(r_entropy).detach())
            if not dist.is_initialized() or dist.get_rank() == 0:
                print(f"Train Epoch: {epoch:03d} Batch: {batch_idx:05d}/{len(data_loader):05d} Acc@1: {vals[0]:.2f}, "
                      f"Acc@5: {vals[1]:.2f} Loss: {vals[2]:.4f} C_Loss: {vals[3]:.4f} A_Loss: {vals[4]:.4f} "
                      f"D_Loss: {vals[5]:.4f} ActiveRatio: {vals[6]:.2f} "
                      f"CurrentTarget: {float(active_metric['current_target']):.2f} RouterEntropy: {vals[7]:.4f} "
                      f"LA: {lambda_active:.1e} LD: {lambda_distill:.1e} LC: {lambda_class:.1e}", flush=True)
    return metrics.result(), None, None


def valid_epoch(epoch, model, data_loader, optimizer, metrics, lambda_active=10.0, lambda_distill=1.0,
                lambda_class=10.0, device=torch.device("cpu"), save_routing_viz=False):
    """res-vit/train.py:107-216: means over the batches of the inference (ragged-attention) path"""
    metrics.reset()
    if metrics.writer is not None:
        metrics.writer.set_step(epoch, mode="valid")
    rows = []
    with torch.no_grad():
        for batch_data, batch_target in data_loader:
            batch_data, batch_target = batch_data.to(device), batch_target.to(device)
            c_loss, a_loss, d_loss, r_entropy, active_metric = model(batch_data, batch_target)
            total = total_loss(model, c_loss, a_loss, d_loss, lambda_active, lambda_distill, lambda_class)
            if not model.use_reslr:
                a_loss = d_loss = r_entropy = torch.tensor(0.0, device=device)
                active_metric = {"non_low_rank_ratio": torch.tensor(0.0, device=device), "current_target": 0.0}
            acc1, acc5 = _topk(model.logits, batch_target)
            rows.append(torch.stack([torch.as_tensor(v, device=device, dtype=torch.float32).reshape(()) for v in
                                     (total, c_loss, a_loss, d_loss, r_entropy, acc1, acc5,
                                      active_metric["non_low_rank_ratio"], active_metric["current_target"])]))
    means = torch.stack(rows).mean(0).tolist()
    for k, v in zip(("loss", "c_loss", "a_loss", "d_loss", "router_entropy", "acc1", "acc5", "active_ratio",
                     "current_target"), means):
        metrics.update(k, v)
    metrics.update("lr", optimizer.param_groups[0]["lr"])
    return metrics.result(), None, None


# ---- configuration (res-vit/config.py) ------------------------------------------------------------------
def set_model_architecture(model_args, model_arch):
    """res-vit/config.py:4-46"""
    presets = {"b16": (768, 3072, 12, 12, 16), "b32": (768, 3072, 12, 12, 32), "l16": (1024, 4096, 24, 16, 16),
               "l32": (1024, 4096, 24, 16, 32), "h14": (1280, 5120, 32, 16, 14)}
    if model_arch not in presets:
        raise ValueError(f"Unsupported model architecture: {model_arch}")
    d, m, nl, nh, p = presets[model_arch]
    model_args.dim, model_args.mlp_dim, model_args.n_layers, model_args.n_heads = d, m, nl, nh
    model_args.n_kv_heads = nh
    model_args.patch_size = (p, p)
    return model_args


def get_num_classes_for_dataset(name):
    """res-vit/config.py:48-66"""
    return {"CIFAR10": 10, "CIFAR100": 100, "ImageNet": 1000, "TinyImageNet": 200}.get(name, 1000)


def config_to_model_args(config):
    """res-vit/config.py:68-96"""
    a = resvit.ModelArgs()
    a.image_size = (config.image_size, config.image_size)
    a.patch_size = (config.patch_size, config.patch_size)
    for k in ("n_heads", "n_kv_heads", "norm_eps", "lora_rank", "dynamic_active_target", "dynamic_start_layer",
              "dynamic_router_hdim", "dynamic_reserve_initials", "low_rank_dim", "block_size", "use_lora",
              "use_reslr", "num_classes"):
        setattr(a, k, getattr(config, k))
    a.device = "cuda"
    return a


def get_train_config(argv=None):
    """res-vit/config.py:122-184 (+ --synthetic, --steps-per-epoch, --no-save, --n-gpu, --fused-clip)"""
    p = argparse.ArgumentParser("Visual Transformer Train/Fine-tune")
    a = p.add_argument
    a("--exp-name", type=str, default="reslr")
    a("--swanlab", default=True, action="store_true")
    a("--model-arch", type=str, default="b16", choices=["b16", "b32", "l16", "l32", "h14"])
    a("--checkpoint-path", type=str, default="../weights/pytorch/imagenet21k+imagenet2012_ViT-B_16-224.pth")
    a("--image-size", type=int, default=224, choices=[224, 384])
    a("--num-workers", type=int, default=1)
    a("--data-dir", type=str, default="../data/")
    a("--dataset", type=str, default="CIFAR100", choices=["CIFAR10", "CIFAR100", "ImageNet", "TinyImageNet"])
    a("--patch-size", type=int, default=16)
    a("--batch-size", type=int, default=32, help="batch size (global: split over --n-gpu ranks)")
    a("--train-steps", type=int, default=15000)
    a("--warmup-steps", type=int, default=500)
    a("--print-freq", type=int, default=100)
    a("--device", type=str, default="cuda:0")
    a("--seed", type=int, default=42)
    a("--lr", type=float, default=1e-4)
    a("--wd", type=float, default=0.05)
    a("--beta1", type=float, default=0.9)
    a("--beta2", type=float, default=0.999)
    a("--eps", type=float, default=1e-8)
    a("--lr-scheduler", type=str, default="cosine_with_warmup", choices=["cosine", "cosine_with_warmup"])
    a("--min-lr", type=float, default=1e-6)
    a("--clip-grad-norm", type=bool, default=True)
    a("--use_lora", type=bool, default=True)
    a("--use_reslr", type=bool, default=True)
    a("--initial-lambda-active", type=float, default=0.0001)
    a("--initial-lambda-distill", type=float, default=0.01)
    a("--initial-lambda-class", type=float, default=1)
    a("--dynamic_active_target", type=float, default=0.6)
    a("--n_heads", type=int, default=12)
    a("--n_kv_heads", type=int, default=12)
    a("--norm_eps", type=float, default=1e-5)
    a("--lora_rank", type=int, default=8)
    a("--dynamic_start_layer", type=int, default=2)
    a("--dynamic_router_hdim", type=int, default=512)
    a("--dynamic_reserve_initials", type=int, default=1)
    a("--low_rank_dim", type=int, default=256)
    a("--block_size", type=int, default=1)
    a("--save-routing-viz", default=False, type=bool)
    # MI355X path additions
    a("--synthetic", default=False, action="store_true", help="synthetic images / labels resident on the device")
    a("--steps-per-epoch", type=int, default=100)
    a("--no-save", default=False, action="store_true")
    a("--n-gpu", type=int, default=1, help="data-parallel ranks (one per GPU)")
    a("--fused-clip", default=False, action="store_true", help="fold clip_grad_norm_ into the AdamW update")
    config = p.parse_args(argv)
    config.num_classes = get_num_classes_for_dataset(config.dataset)
    return config


def save_model(save_dir, model, best=False):
    """res-vit/utils.py:149-155: current_model.pth every epoch, best_model.pth on a new best. The reference
    pickles the whole module (torch.save(model)); here the state_dict is saved, so the file loads with
    torch.load(weights_only=True) into resvit.Transformer(args).load_state_dict."""
    torch.save(model.state_dict(), str(save_dir + "current_model.pth"))
    if best:
        torch.save(model.state_dict(), str(save_dir + "best_model.pth"))


def build_model(config, device):
    args = set_model_architecture(config_to_model_args(config), config.model_arch)
    return resvit.Transformer(args).to(device)


def main(argv=None):
    # experiment dirs as res-vit/config.py:183 (process_config); ranks started below share the stamp
    config = process_config(get_train_config(argv))
    os.environ.setdefault("VITMI_EXP_STAMP", config.exp_stamp)
    if "WORLD_SIZE" not in os.environ and config.n_gpu > 1:
        rank_batch(config.batch_size, config.n_gpu)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        from bench import launch_ranks
        rc = launch_ranks(config.n_gpu, list(sys.argv[1:] if argv is None else argv), module="vitmi.resvit_train")
        if rc:
            raise SystemExit(rc)
        return None
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("vitmi.resvit_train needs a ROCm GPU (MI355X)")
    if os.environ.get("VITMI_SHARE_GPU"):
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        from .dist import init_process_group
        init_process_group(device=device)
    batch = rank_batch(config.batch_size, world)
    set_seed(config.seed)
    model = build_model(config, device)
    if config.checkpoint_path:
        raise SystemExit("load_pretrained_with_mapping (res-vit/utils.py:158-443) is outside the MI355X path; "
                         "pass --checkpoint-path ''")
    if not config.synthetic:
        raise SystemExit("torchvision datasets are not available in this environment; use --synthetic")
    optimizer = AdamW(model.parameters(), lr=config.lr, weight_decay=config.wd, betas=(config.beta1, config.beta2),
                      eps=config.eps, max_grad_norm=1.0 if (config.fused_clip and config.clip_grad_norm) else None)
    reducer = None
    if world > 1:
        from .dist import FlatGradAllReducer
        for p in model.parameters():
            dist.broadcast(p.data, 0)
        reducer = FlatGradAllReducer(optimizer.flat).attach()
    train_loader = SyntheticDataLoader(batch, config.image_size, config.num_classes, config.steps_per_epoch, device,
                                       seed=config.seed + rank)
    valid_loader = SyntheticDataLoader(batch, config.image_size, config.num_classes,
                                       max(1, config.steps_per_epoch // 10), device, seed=10_000 + config.seed + rank)
    epochs = config.train_steps // len(train_loader)
    if config.lr_scheduler == "cosine":
        lr_scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer=optimizer, T_max=max(1, epochs),
                                                                  eta_min=config.min_lr)
    else:
        lr_scheduler = get_cosine_schedule_with_warmup(optimizer, num_warmup_steps=config.warmup_steps,
                                                       num_training_steps=config.train_steps)
    writer = StepWriter()
    train_metrics = MetricTracker(*METRICS, writer=writer)
    valid_metrics = MetricTracker(*METRICS, writer=writer)
    la, ld, lc = config.initial_lambda_active, config.initial_lambda_distill, config.initial_lambda_class
    best_acc = 0.0
    if rank == 0:
        print(f"Training for {epochs} epochs based on {config.train_steps} steps")
    for epoch in range(epochs):
        log = {"epoch": epoch, "lambda_active": la, "lambda_distill": ld, "lambda_class": lc}
        model.train()
        res, _, _ = train_epoch(epoch, model, train_loader, optimizer, train_metrics, config,
                                lr_scheduler if config.lr_scheduler == "cosine_with_warmup" else None, la, ld, lc,
                                device, reducer=reducer)
        log.update(res)
        if config.lr_scheduler == "cosine":
            lr_scheduler.step()
        model.eval()
        res, _, _ = valid_epoch(epoch, model, valid_loader, optimizer, valid_metrics, la, ld, lc, device)
        log.update({"val_" + k: v for k, v in res.items()})
        best = log["val_acc1"] > best_acc
        if best:
            best_acc = log["val_acc1"]
        if rank == 0 and not config.no_save:
            save_model(config.checkpoint_dir, model, best)  # res-vit/train.py:335-341
        if rank == 0:
            for key, value in log.items():
                print("    {:15s}: {}".format(str(key), value), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return best_acc


if __name__ == "__main__":
    main(sys.argv[1:])
