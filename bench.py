#!/usr/bin/env python3
"""Throughput benchmark of the MI355X ViT training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--arch b16]

One step = forward + cross-entropy + backward + (N>1: gradient all-reduce over RCCL) + fused
SGD-momentum update with OneCycleLR scalars, on a synthetic batch already resident in HBM.
Weak scaling: every rank processes --batch images (256 = BASELINE config #2 per GPU).
For N>1 launch with torch.distributed.run (one process per GPU); rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2516.6  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; 256 CU x 2.4 GHz x 4096)
PEAK_HBM_GBS = 8000.0

ARCHS = {
    "b16": dict(patch_size=16, emb_dim=768, mlp_dim=3072, num_heads=12, num_layers=12),
    "b32": dict(patch_size=32, emb_dim=768, mlp_dim=3072, num_heads=12, num_layers=12),
    "l16": dict(patch_size=16, emb_dim=1024, mlp_dim=4096, num_heads=16, num_layers=24),
    "l32": dict(patch_size=32, emb_dim=1024, mlp_dim=4096, num_heads=16, num_layers=24),
    "h14": dict(patch_size=14, emb_dim=1280, mlp_dim=5120, num_heads=16, num_layers=32),
}


def train_flops_per_image(a, image_size, num_classes):
    D, M, P, L = a["emb_dim"], a["mlp_dim"], a["patch_size"], a["num_layers"]
    n = (image_size // P) ** 2
    N = n + 1
    patch = 2 * n * 3 * P * P * D
    fwd = patch + L * 2 * (3 * N * D * D + 2 * N * N * D + N * D * D + 2 * N * D * M) + 2 * D * num_classes
    return 3 * fwd - patch


def pmc_traffic(kernel_tag="gemm_pp2_kernel<true, true, 8,"):
    """HBM bytes per launch of a roofline kernel from the newest committed rocprofv3 PMC passes
    (tools/prof.sh: FETCH_SIZE and WRITE_SIZE in separate passes, FETCH_SIZE doubled per the gfx950
    correction of MI355X_MICROARCH.md). None when no pass of that kernel is committed."""
    import glob
    import re

    def version(path):  # profiles/rNN/<kernel>_traffic_vK.json: newest round, then newest pass
        m = re.search(r"r(\d+)[/\\]\w*?_traffic_v(\d+)", path)
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "*_traffic_v*.json")), key=version)
    for path in reversed(files):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if kernel_tag in d.get("kernel", ""):
            return {"bytes": round(d["traffic_bytes"]), "fetch": round(d["fetch_bytes_corrected"]),
                    "write": round(d["write_bytes"]), "source": os.path.relpath(path, REPO)}
    return None


def condition_init(model, seed=1):
    """The bench's weights: the reference constructor's seed-42 draw (src/model.py:161-194, reference RNG order) with
    the attention projections redrawn at N(0, 1/D) and the position embedding and classifier at N(0, 0.02^2), in
    named-parameter order from Generator(seed) (the rescale of SURVEY.md §8c's parity protocol). Under the raw std-1
    draw the first step's gradient norm is ~1e11 (layer 0's saturated attention) and the bf16 training step turns every
    parameter into NaN from step 1 on (tools/dbg/bench_loss_trace.py, profiles/r06/bench_loss_trace.txt): a throughput
    timed on NaN operands is not a training step (and DVFS runs constant bit patterns faster). VITMI_BENCH_INIT=reference
    keeps the raw draw for A/B."""
    import math
    g = torch.Generator().manual_seed(seed)
    sd = model.state_dict()
    new = {}
    for k, v in sd.items():
        if ".attn." in k and k.endswith(".weight"):
            D = v.shape[0] if not k.endswith("out.weight") else v.shape[-1]
            new[k] = torch.randn(v.shape, generator=g) / math.sqrt(D)
        elif k in ("transformer.pos_embedding.pos_embedding", "classifier.weight"):
            new[k] = 0.02 * torch.randn(v.shape, generator=g)
    model.load_state_dict(new, strict=False)


def onecycle_hyper_table(total_steps, dev):
    """{lr, momentum, first-step} of every bench step as a [steps][3] f32 device table: torch's OneCycleLR as the
    reference configures it (src/train.py:159-163: max_lr .03, 500 warm-up of 15000 steps, cycle_momentum) driving
    SGD(momentum .9). The SGD kernel of the timed step (vit_sgd_step_dev) reads its scalars from one row of it,
    refreshed by a 12-byte device copy before each step, so the step can be one HIP graph
    (tests/test_optim_dev_gpu.py pins this table and that kernel against the oracle)."""
    from torch.optim.lr_scheduler import OneCycleLR
    _p = torch.nn.Parameter(torch.zeros(1))
    _opt = torch.optim.SGD([_p], lr=0.03, momentum=0.9)
    sched = OneCycleLR(_opt, max_lr=0.03, pct_start=500 / 15000, total_steps=15000)
    hp = []
    for _ in range(total_steps):
        hp.append((_opt.param_groups[0]["lr"], _opt.param_groups[0]["momentum"]))
        _opt.step()
        sched.step()
    return torch.tensor([[lr_, mom_, 1.0 if k == 0 else 0.0] for k, (lr_, mom_) in enumerate(hp)],
                        device=dev, dtype=torch.float32)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """host cores this process may actually use: the affinity mask, capped by a cgroup CPU quota
    (cpu.max) and by OMP_NUM_THREADS when the launcher sets it (a GPU box shares its host: the mask
    lists every core of the machine, the quota grants ~16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_baseline(arch, image_size, num_classes, seconds_budget=20.0):
    """Time the CPU oracle (restatement of reference src/train.py:train_epoch's step) on the host, on
    every core this process may run on, under both init protocols: the tamed rescale
    (the parity protocol, = bench.condition_init: the weights the GPU line trains) and the reference's own std-1
    init (slower on CPU: saturated softmax -> subnormal floats). `value` is the tamed-init rate, the same weights
    as the GPU measurement (round 6; the GPU line moved off the std-1 draw, which trains on NaN from step 1);
    `value_reference_init` keeps the std-1 rate."""
    from oracle.vit_oracle import OneCycle, ViTConfig, init_params, loss_and_grads, sgd_step, tame_params
    cores = _cpu_share()
    torch.set_num_threads(cores)
    cfg = ViTConfig(image_size=image_size, num_classes=num_classes, **arch)
    sched = OneCycle(0.03, 15000, 500 / 15000)
    rates = {}
    for proto, bs in (("reference", 16), ("tamed", 16)):  # the config batch or bs 16-32
        print(f"cpu_baseline: {proto} init, batch {bs}, {cores} threads", file=sys.stderr, flush=True)
        g = torch.Generator().manual_seed(0)
        x = torch.randn(bs, 3, image_size, image_size, generator=g)
        y = torch.randint(0, num_classes, (bs,), generator=g)
        params = init_params(cfg, seed=42)
        if proto == "tamed":
            params = tame_params(params)
        bufs = {}
        _, _, grads = loss_and_grads(params, x, y, cfg)  # warm-up step (not timed)
        params, bufs = sgd_step(params, grads, bufs, *sched.at(0), 0.0, first=True)
        steps, t0 = 0, time.perf_counter()
        while True:
            _, _, grads = loss_and_grads(params, x, y, cfg)
            params, bufs = sgd_step(params, grads, bufs, *sched.at(steps + 1), 0.0, first=False)
            steps += 1
            if time.perf_counter() - t0 > seconds_budget / 2 or steps >= 20:
                break
        dt = time.perf_counter() - t0
        rates[proto] = (steps * bs / dt, steps, dt)
    r, t = rates["reference"], rates["tamed"]
    return dict(value=round(t[0], 3), unit="images/sec", cores=cores, kind="port", cpu_model=_cpu_model(),
                value_reference_init=round(r[0], 3),
                sample=f"oracle fp32 CPU train step (fwd+CE+bwd+SGD/OneCycleLR) on {cores} threads ({_cpu_model()}): "
                       f"tamed init (the GPU line's weights), batch 16, {t[1]} steps in {t[2]:.1f} s; reference std-1 "
                       f"init, batch 16, {r[1]} steps in {r[2]:.1f} s; each after 1 warm-up step")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, module=None, script=None):
    """Start n ranks of this program (one process per GPU, torch.distributed.run on 127.0.0.1) as a
    child process and return its exit code. Called before anything touches the GPU: only
    torch.cuda.device_count(), which does not initialise HIP on this image, is consulted. More ranks
    than visible GPUs is an error unless VITMI_SHARE_GPU=1 (functional rehearsal on one card)."""
    import subprocess
    visible = torch.cuda.device_count()
    if n > visible and not os.environ.get("VITMI_SHARE_GPU"):
        print(f"error: {n} ranks requested but {visible} GPU(s) visible "
              "(VITMI_SHARE_GPU=1 rehearses the multi-rank path on fewer GPUs)", file=sys.stderr)
        return 2
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    target = ["-m", module] if module else [script]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", port, *target, *argv]
    env = dict(os.environ)
    pp = [os.path.join(REPO, "vit-of-pytorch_amd"), REPO]
    env["PYTHONPATH"] = os.pathsep.join(pp + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks) of this node; >1 without a torch.distributed.run environment starts "
                         "that many ranks itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default 256; resvit_b16: 128)")
    ap.add_argument("--arch", default="b16", choices=sorted(ARCHS) + ["resvit_b16"],
                    help="resvit_b16: BASELINE config C5, the Res-ViT-B/16 training step (res-vit/train.py)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--grad-compress", choices=["none", "bf16"], default="none",
                    help="N>1: all-reduce the gradient buckets in bf16 (vitmi.dist compress='bf16')")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], script=os.path.abspath(__file__)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("VITMI_SHARE_GPU"):  # functional rehearsal of the N>1 path on fewer GPUs (gloo)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = None
    if world > 1:
        import torch.distributed as dist
        from vitmi.dist import init_process_group
        backend = init_process_group(device=dev)
    # torch's "nccl" backend is RCCL on ROCm; any other backend is named as itself
    comm = {None: None, "nccl": "RCCL"}.get(backend, backend)
    if args.arch == "resvit_b16":
        return bench_resvit(args, world, rank, dev, backend, comm)
    if args.batch is None:
        args.batch = 256

    from vitmi import ops
    from vitmi.dist import GradAllReducer
    from vitmi.model import VisionTransformer

    arch = ARCHS[args.arch]
    # random-init weights of the named architecture, drawn exactly like the reference ctor
    # (src/model.py:161-194, seed 42), then bound to the HIP engine on this GPU
    torch.manual_seed(42)
    model = VisionTransformer(image_size=(args.image_size, args.image_size),
                              patch_size=(arch["patch_size"], arch["patch_size"]), emb_dim=arch["emb_dim"],
                              mlp_dim=arch["mlp_dim"], num_heads=arch["num_heads"], num_layers=arch["num_layers"],
                              num_classes=args.num_classes, attn_dropout_rate=0.0, dropout_rate=0.0)
    init_kind = os.environ.get("VITMI_BENCH_INIT", "conditioned")
    if init_kind != "reference":
        condition_init(model)
    model = model.to(dev)
    eng = model.engine()
    eng.refresh_mirror()
    if os.environ.get("VITMI_ATTN_FWD_PATH"):  # A/B: 3 = the one-shot attention forward instead of the persistent one
        eng.attn_fwd_path = int(os.environ["VITMI_ATTN_FWD_PATH"])
    cfg = eng.cfg
    b = args.batch
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(b, 3, args.image_size, args.image_size, device=dev, generator=g)
    y = torch.randint(0, args.num_classes, (b,), device=dev, generator=g)
    mom_buf = torch.zeros_like(eng.flat)
    compress = None if args.grad_compress == "none" else args.grad_compress
    reducer = (GradAllReducer(eng, average=False, compress=compress).attach()  # CE pre-scaled by 1/(b*world)
               if world > 1 else None)
    total_steps = args.warmup + args.steps
    hyper_all = onecycle_hyper_table(total_steps, dev)
    hyper = hyper_all[0].clone()

    def step_body():
        eng.forward(x)
        dl, st = eng.cross_entropy(y, grad_scale=1.0 / (b * world))
        losses.append(st)
        eng.backward(dl)
        if reducer is not None:
            reducer.finish()
        ops.sgd_step_dev(eng.flat, eng.grad, mom_buf, eng.mirror, eng.layout.numel, hyper, 0.0)
        eng.refresh_mirror(full=False)

    # VITMI_BENCH_GRAPH=1 (one process on one GPU): the whole step (~450 launches on two streams) captured
    # once as a HIP graph and replayed. Off by default: the launch queue already runs ahead of the GPU, and
    # in a same-box A/B the replay was 0.5% slower than eager launches (7402 / 7417 vs 7452 / 7455 img/s)
    use_graph = world == 1 and os.environ.get("VITMI_BENCH_GRAPH", "0") != "0"
    graph = None

    losses = []  # the CE kernel's row-stats buffer (one persistent buffer, overwritten every step)
    first_timed = []

    def step(k):
        ops.copy2d(hyper, 12, hyper_all[k], 12, 12, 1)
        if graph is not None:
            graph.replay()
        else:
            step_body()
        if k == args.warmup and losses:  # the first timed step's mean loss, kept on the device (one tiny kernel)
            first_timed.append(losses[-1][:, 0].mean())

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    for k in range(args.warmup):
        step(k)
    barrier()
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step_body()
        barrier()
    t0 = time.perf_counter()
    for k in range(args.warmup, total_steps):
        step(k)
    barrier()
    dt = time.perf_counter() - t0
    loss_last = float(losses[-1][:, 0].mean()) if losses else float("nan")
    loss_first = float(first_timed[0]) if first_timed else float("nan")
    # HIP events around the roofline kernels' launches of one more (eager) step after the timed region,
    # on the stream the kernels run on (each event record costs the stream ~10 us of idle)
    probes = ([], [])
    eng.probe, eng.probe_wgrad = probes
    ops.copy2d(hyper, 12, hyper_all[total_steps - 1], 12, 12, 1)
    step_body()
    barrier()
    probe, probe_w = probes
    eng.probe = eng.probe_wgrad = None
    # a second eager probe step: HIP events around every forward / data-gradient GEMM call over all T rows
    # (the gemm_pp2 family and its wave-split remainder launches; kept apart from the probes above, whose
    # events would otherwise land inside these)
    T = b * cfg.tokens
    ops.GEMM_PROBE, ops.GEMM_PROBE_MIN_M = [], T
    ops.copy2d(hyper, 12, hyper_all[total_steps - 1], 12, 12, 1)
    step_body()
    barrier()
    probe_fd, ops.GEMM_PROBE = ops.GEMM_PROBE, None
    dist_check = None
    if world > 1:
        dist_check = replica_check(eng.flat, dt, args.steps, world, backend, dev)
        dt = dist_check.pop("_dt_max")
        ops.copy2d(hyper, 12, hyper_all[total_steps - 1], 12, 12, 1)
        dist_check["exchange"] = exchange_check(step_body, reducer, dt, args.steps, world, dev, barrier)
    fc1_ms = sum(s.elapsed_time(e) for s, e in probe) / max(1, len(probe))
    fd_ms = [s_.elapsed_time(e_) for s_, e_, _, _ in probe_fd]
    fd_flop = sum(p_[2] for p_ in probe_fd)
    fd_tflops = fd_flop / (sum(fd_ms) * 1e-3) / 1e12 if fd_ms else 0.0
    epi_names = {1: "bf16 (dgrads)", 2: "bias bf16 (qkv fwd)", 4: "bias + f32 residual (fc2 / out-proj fwd)",
                 6: "patch embed", 8: "bias + GELU + GELU' (fc1 fwd)", 9: "x GELU' (fc2 dgrad)"}
    fd_by_epi = {}
    for (s_, e_, fl, epi), ms in zip(probe_fd, fd_ms):
        d_ = fd_by_epi.setdefault(epi_names.get(epi, f"epilogue {epi}"), {"launches": 0, "ms": 0.0, "gflop": 0.0})
        d_["launches"] += 1
        d_["ms"] += ms
        d_["gflop"] += fl / 1e9
    for d_ in fd_by_epi.values():
        d_["frac"] = round(d_["gflop"] / d_["ms"] / PEAK_BF16_TFLOPS, 4) if d_["ms"] else None
        d_["ms"] = round(d_["ms"], 4)
        d_["gflop"] = round(d_["gflop"], 2)
    fc1_flop = 2.0 * T * cfg.emb_dim * cfg.mlp_dim
    fc1_tflops = fc1_flop / (fc1_ms * 1e-3) / 1e12
    # the step's dominant kernel by time: the split-K weight-gradient GEMMs (gemm_pp2_kernel<false, false, 7> and
    # the grouped gemm_pp2_group_kernel; ~20% of the step), every launch of the probe step; achieved = their
    # algorithmic FLOPs / their own time
    # headline: the launches over all T tokens (K = T rounded up to 64); the pruned last layer's
    # launches (K = the b cls rows padded to 64) are reported beside it, not averaged in
    full_w = [p_ for p_ in probe_w if p_[3] >= T]
    pr_w = [p_ for p_ in probe_w if p_[3] < T]
    wg_ms = [p_[0].elapsed_time(p_[1]) for p_ in full_w]
    n_group = sum(1 for p_ in full_w if p_[4])
    wg_flop = sum(p_[2] * T / p_[3] for p_ in full_w)  # algorithmic: the T real rows, not the padding
    wg_tflops = wg_flop / (sum(wg_ms) * 1e-3) / 1e12 if wg_ms else 0.0
    wg_avg_ms = sum(wg_ms) / max(1, len(wg_ms))
    pr_ms = sum(p_[0].elapsed_time(p_[1]) for p_ in pr_w)
    imgs = args.steps * b * world
    value = imgs / dt
    fpi = train_flops_per_image(arch, args.image_size, args.num_classes)
    # executed work: with the last layer pruned to its cls rows (engine.prune_last, only they reach
    # the classifier) its out-proj / fc1 / fc2 skip N-1 tokens per image in forward, dgrad and wgrad
    D_, M_, N_ = cfg.emb_dim, cfg.mlp_dim, cfg.tokens
    # (and its attention computes only the first 32-query pair: (N - 32) / N of QK^T / PV forward and
    # backward is skipped as well)
    q_kept = min(N_, 32)
    fpe = fpi - ((3 * 2 * (N_ - 1) * (D_ * D_ + 2 * D_ * M_) + 3 * 4 * (N_ - q_kept) * N_ * D_)
                 if eng.prune_last else 0)
    traffic = pmc_traffic() if args.arch == "b16" and b == 256 else None
    traffic_w = None
    if args.arch == "b16" and b == 256:
        # per-launch HBM bytes of the two weight-gradient kernels from their committed PMC passes, averaged over this
        # step's launches of each (fc1 / fc2: gemm_pp2_kernel; out-proj + q|k|v: the grouped kernel)
        t_pp2, t_grp = pmc_traffic("gemm_pp2_kernel<false, false, 7,"), pmc_traffic("gemm_pp2_group_kernel")
        n_all = len(full_w)
        if t_pp2 and (t_grp or n_group == 0) and n_all:
            tb = (t_pp2["bytes"] * (n_all - n_group) + (t_grp["bytes"] if t_grp else 0) * n_group) / n_all
            traffic_w = {"bytes": round(tb), "per_kernel": {"gemm_pp2_kernel<false, false, 7>": t_pp2,
                                                            "gemm_pp2_group_kernel": t_grp},
                         "launches": {"gemm_pp2_kernel<false, false, 7>": n_all - n_group,
                                      "gemm_pp2_group_kernel": n_group}}
    step_tflops_per_gpu = value / world * fpi / 1e12
    out = {
        "metric": "images/sec training step, ViT-B/16 224px bf16, 1/2/4/8 MI355X" if args.arch == "b16" and
        args.image_size == 224 else f"images/sec training step, ViT-{args.arch} {args.image_size}px bf16",
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": ("synthetic (N(0,1) images, uniform labels, seed-42 reference-order random init" +
                 (", attention projections at N(0,1/D) and pos-emb / classifier at N(0,0.02^2): bench.condition_init)"
                  if init_kind != "reference" else ")")),
        "loss_first_timed_step": round(loss_first, 5), "loss_last_timed_step": round(loss_last, 5),
        "config": {"workload": f"ViT-{args.arch.upper()} @{args.image_size} train step (fwd+CE+bwd+"
                               f"{comm + ' all-reduce+' if world > 1 else ''}SGD-momentum/OneCycleLR)",
                   "model": f"ViT-{args.arch.upper()}", "image_size": args.image_size, "per_gpu_batch": b,
                   "global_batch": b * world, "seq_len": cfg.tokens, "num_classes": args.num_classes,
                   "parallelism": f"dp{world}", "dist_backend": backend,
                   "step_launch": "one HIP graph per step" if use_graph else "eager",
                   **({"grad_allreduce_dtype": "bf16"} if compress and world > 1 else {})},
        "roofline": {"bound": "mfma", "kernel": "split-K weight-gradient GEMMs (the step's dominant kernel family): "
                                                f"the {len(wg_ms)} launches over all tokens of one step (HIP events, an "
                                                f"eager step after the timed region), K = {T} tokens padded to 64; fc1 "
                                                "and fc2 one gemm_pp2_kernel<false, false, 7> launch each, each layer's "
                                                "out-proj + q|k|v (three batched GEMMs) one gemm_pp2_group_kernel launch",
                     "achieved": round(wg_tflops, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(wg_tflops / PEAK_BF16_TFLOPS, 4), "traffic": (traffic_w or {}).get("bytes"),
                     "traffic_detail": traffic_w,
                     "algorithmic_flop_per_launch": round(wg_flop / max(1, len(wg_ms))),
                     "avg_launch_ms": round(wg_avg_ms, 4), "launches": len(wg_ms),
                     "pruned_layer_launches": {"launches": len(pr_w), "total_ms": round(pr_ms, 4),
                                               "note": "last layer's cls-row weight gradients (K = batch padded "
                                                       "to 64), excluded from achieved"}},
        "roofline_fc1_fwd": {"bound": "mfma", "kernel": "gemm fc1 fwd (bias + GELU + GELU' epilogue), "
                                                f"M={T} N={cfg.mlp_dim} K={cfg.emb_dim}",
                     "achieved": round(fc1_tflops, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(fc1_tflops / PEAK_BF16_TFLOPS, 4), "traffic": (traffic or {}).get("bytes"),
                     "traffic_detail": traffic,
                     "algorithmic_bytes": T * cfg.emb_dim * 2 + cfg.mlp_dim * cfg.emb_dim * 2 + 2 * T * cfg.mlp_dim * 2,
                     "avg_launch_ms": round(fc1_ms, 4), "launches": len(probe)},
        "roofline_fwd_dgrad": {"bound": "mfma", "kernel": "every forward and data-gradient GEMM call over all "
                                                      f"{T} token rows of one step (gemm_pp2_kernel family + the "
                                                      "wave-split 128x128 remainder launches; HIP events around each "
                                                      "vit_gemm_bf16 call, a separate eager probe step)",
                               "achieved": round(fd_tflops, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(fd_tflops / PEAK_BF16_TFLOPS, 4), "traffic": None,
                               "calls": len(fd_ms), "total_ms": round(sum(fd_ms), 4),
                               "gflop_per_step": round(fd_flop / 1e9, 2), "by_epilogue": fd_by_epi},
        "step_mfma_frac": round(value / world * fpe / 1e12 / PEAK_BF16_TFLOPS, 4),
        "step_mfma_frac_algorithmic": round(step_tflops_per_gpu / PEAK_BF16_TFLOPS, 4),
        "train_gflop_per_image": round(fpi / 1e9, 3),
        "executed_gflop_per_image": round(fpe / 1e9, 3),
    }
    if dist_check is not None:
        out["dist_check"] = dist_check
    if world == 1 and os.environ.get("VITMI_BENCH_TRAIN_EPOCH", "1") != "0":
        # the drop-in path (train_epoch + vitmi.optim.SGD + OneCycleLR + metrics) at the same shape, after the engine
        # loop: how much of `value` a user of the reference's entry point sees
        te, te_res = time_train_epoch(model, b, args.image_size, args.num_classes, args.steps, args.warmup, dev)
        out["train_epoch_img_s"] = round(te, 2)
        out["train_epoch_vs_value"] = round(te / value, 4)
        out["train_epoch_note"] = ("vitmi.train.train_epoch (src/train.py:12-37) + vitmi.optim.SGD + torch OneCycleLR + "
                                   f"loss/acc1/acc5 metrics, {args.steps} synthetic HBM-resident batches of {b} after a "
                                   f"{args.warmup}-batch epoch; last epoch loss {te_res['loss']:.4f}")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(arch, args.image_size, args.num_classes, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
        if not dist_check["replicas_identical"]:
            print("error: the data-parallel replicas' parameters differ after the run", file=sys.stderr)
            sys.exit(3)


def replica_hash(flat):
    """[2] int64 fingerprint of a flat f32 parameter buffer: the wrapped sum of its 32-bit patterns and a
    position-weighted wrapped sum (equal buffers give equal hashes, bit for bit; a permutation or any
    changed bit changes them)."""
    bits = flat.detach().reshape(-1).view(torch.int32).to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([bits.sum(), (bits * w).sum()])


def replica_check(flat, dt, steps, world, backend, dev):
    """After the timed run of an N-rank job: every rank's wall time (max = the job's), and an all-gather of
    replica_hash(flat) — data-parallel replicas must stay bit-identical (reference
    src/train.py:128-129 keeps one model)."""
    import torch.distributed as dist
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    ts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(ts, t)
    h = replica_hash(flat)
    hs = [torch.zeros_like(h) for _ in range(world)]
    dist.all_gather(hs, h)
    per = [float(x) / steps * 1e3 for x in ts]
    same = all(torch.equal(hs[0], x) for x in hs)
    return {"ranks_seen": dist.get_world_size(), "backend": backend,
            "ms_per_step_per_rank": [round(x, 3) for x in per],
            "ms_per_step_spread_pct": round((max(per) - min(per)) / min(per) * 100, 2),
            "replicas_identical": same, "param_hash_rank0": [int(x) for x in hs[0].tolist()],
            "_dt_max": max(float(x) for x in ts)}


def time_train_epoch(model, b, image_size, num_classes, steps, warmup, dev):
    """The drop-in user path at the bench's shape: vitmi.train.train_epoch (reference src/train.py:12-37) driving the
    model through autograd, vitmi.model.CrossEntropyLoss, vitmi.optim.SGD(momentum .9) + torch's OneCycleLR as
    src/train.py:151-163 configure them, and the loss / top-1 / top-5 metrics, on a synthetic HBM-resident batch.
    Returns images/s over `steps` batches after a `warmup`-batch epoch (its per-100-batch progress line goes to
    stderr, keeping stdout the one JSON line)."""
    import contextlib

    from vitmi.model import CrossEntropyLoss
    from vitmi.optim import SGD
    from vitmi.train import MetricTracker, SyntheticDataLoader, train_epoch
    crit = CrossEntropyLoss()
    opt = SGD(model.parameters(), lr=0.03, momentum=0.9, weight_decay=0.0, model=model)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=0.03, pct_start=500 / 15000, total_steps=15000)
    metrics = MetricTracker("loss", "acc1", "acc5")
    model.train()
    with contextlib.redirect_stdout(sys.stderr):
        train_epoch(1, model, SyntheticDataLoader(b, image_size, num_classes, warmup, dev, seed=7), crit, opt, sched,
                    metrics, dev)
        torch.cuda.synchronize()
        loader = SyntheticDataLoader(b, image_size, num_classes, steps, dev, seed=8)
        t0 = time.perf_counter()
        res = train_epoch(2, model, loader, crit, opt, sched, metrics, dev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return steps * b / dt, res


def exchange_check(step_fn, reducer, dt, steps, world, dev, sync, solo_steps=None):
    """N > 1: what the gradient exchange costs per step, for a reader of the driver's 8-GPU line (is the
    all-reduce hidden under the backward or serialised after it?). (1) One more step with the reducer's
    accounting on: the per-step all-reduce time (HIP events around every bucket's collective on the exchange
    stream, summed) and the bytes exchanged. (2) The same step WITHOUT the exchange (reducer detached, every rank
    computing alone at the same time, same job and clocks), timed like the main loop (max over ranks): exposed
    communication = the N-rank ms/step minus this solo ms/step. Runs after the replica check (the solo steps
    apply unreduced gradients, so the replicas diverge from here on). Reference: src/train.py:128-129."""
    import torch.distributed as dist
    reducer.timing = []
    step_fn()
    sync()
    ar_ms, buckets, elems = reducer.timing_summary()
    reducer.timing = None
    reducer.detach()
    n = solo_steps or steps
    step_fn()  # warm-up without the exchange
    sync()
    t0 = time.perf_counter()
    for _ in range(n):
        step_fn()
    sync()
    solo = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(solo, op=dist.ReduceOp.MAX)
    reducer.attach()
    solo_ms = float(solo) / n * 1e3
    step_ms = dt / steps * 1e3
    bpe = 2 if reducer.compress else 4
    return {"allreduce_ms_per_step": round(ar_ms, 3), "allreduce_buckets": buckets,
            "allreduce_bytes_per_step": int(elems) * bpe,
            "allreduce_algbw_gbs": round(int(elems) * bpe * 2 * (world - 1) / world / (ar_ms * 1e-3) / 1e9, 1)
            if ar_ms > 0 else None,
            "solo_ms_per_step": round(solo_ms, 3), "exposed_comm_ms_per_step": round(step_ms - solo_ms, 3),
            "note": "allreduce_ms: sum of the per-bucket collectives on the exchange stream (overlapped with the backward "
                    "where exposed_comm is small); solo: the same step with no exchange, every rank at once"}


def resvit_flops_per_image(a, image_size, block_heads, active_ratio):
    """executed matrix FLOPs per image of the Res-ViT training step (res-vit/model.py:590-702 under
    res-vit/train.py:23-68) with LoRA (frozen bases: no base weight gradients) and residual low-rank
    routing. Per layer, G = the q/k/v/o + FFN GEMMs, A = the two attention matmuls, of all N tokens:
    student forward every layer (computed on every token, then selected), teacher forward from
    dynamic_start_layer on, backward of the student path (data gradients G + attention 2A); router MLPs
    at block heads and LoRA: forward + data + weight gradients (3x); approximators on the
    (1 - active_ratio) routed rows (3x)."""
    D, M, L, P, r, h = a["dim"], a["mlp_dim"], a["n_layers"], a["patch"], a["lora_rank"], a["router_hdim"]
    s0, lr_dim, bs = a["dynamic_start_layer"], a["low_rank_dim"], a["block_size"]
    n = (image_size // P) ** 2
    N = n + 1
    G = 2 * N * (4 * D * D + 2 * D * M)
    A = 4 * N * N * D
    lora = 3 * 2 * N * 3 * (2 * D * r)
    router = 3 * 2 * N * (D * h + 2 * h * h + h * (h // 2) + (h // 2) * 2 * bs)
    approx = 3 * 2 * N * (2 * D * lr_dim) * (1.0 - active_ratio)
    patch = 2 * n * 3 * P * P * D
    return (patch + L * (G + A + lora) + (L - s0) * (G + A + lora) + L * (G + 2 * A + lora) +
            block_heads * router + (L - s0) * approx)


def bench_resvit(args, world, rank, dev, backend, comm):
    """BASELINE config C5: Res-ViT-B/16 @224 training step (res-vit/train.py:23-68) with the
    res-vit/config.py defaults (LoRA rank 8 over frozen bases, residual low-rank routing from layer 2,
    block size 1, active target 0.6, 100 classes, AdamW lr 1e-4 wd 0.05, clip 1.0, cosine warm-up
    schedule, lambdas class 1 / active 1e-4 / distill 1e-2), the clip folded into the HIP AdamW update;
    N > 1: one rank per GPU, flat gradient buckets all-reduced during the backward."""
    from vitmi import resvit
    from vitmi.optim import AdamW, get_cosine_schedule_with_warmup
    from vitmi.resvit_train import GraphedTrainStep, train_step
    b = args.batch or 128
    a = dict(dim=768, mlp_dim=3072, n_layers=12, n_heads=12, n_kv_heads=12, norm_eps=1e-5, lora_rank=8,
             dynamic_active_target=0.6, dynamic_start_layer=2, dynamic_router_hdim=512, dynamic_reserve_initials=1,
             low_rank_dim=256, block_size=1, use_lora=True, use_reslr=True, image_size=(args.image_size,) * 2,
             patch_size=(16, 16), num_classes=100, device="cuda")
    torch.manual_seed(42)
    model = resvit.Transformer(resvit.ModelArgs(**a)).to(dev).train()
    if os.environ.get("VITMI_RESVIT_PACK_EACH", "0") != "0":  # A/B: LoRA operands packed on every layer call
        from vitmi import resvit_fused
        resvit_fused.SHARE_PACK = False
    if os.environ.get("VITMI_RESVIT_NO_FUSED_EMBED", "0") != "0":  # A/B: conv, cat and position add as written
        resvit.FUSED_EMBED = False
    if os.environ.get("VITMI_RESVIT_NO_ROUTER_THROUGH", "0") != "0":  # A/B: autograd adds the block input's gradients
        resvit.ROUTER_THROUGH = False
    if os.environ.get("VITMI_RESVIT_NO_FUSED_SELECT", "0") != "0":  # A/B: isin / == / any per layer and approximator
        resvit.FUSED_SELECT = False
    if os.environ.get("VITMI_RESVIT_NO_FUSED_DISTILL", "0") != "0":  # A/B: cls_tap + torch's mse_loss per layer
        resvit.FUSED_DISTILL = False
    if os.environ.get("VITMI_RESVIT_NO_FUSED_HEAD", "0") != "0":  # A/B: the router head as separate ATen ops
        resvit.FUSED_HEAD = False
    if os.environ.get("VITMI_RESVIT_NO_CLS_TAP", "0") != "0":  # A/B: cls-row slices and the all-row final norm
        resvit.CLS_TAP = False
    if os.environ.get("VITMI_RESVIT_TEACHER_PASS", "0") != "0":  # A/B: a separate no-grad teacher pass everywhere
        resvit.SHARE_TEACHER = False
    if os.environ.get("VITMI_RESVIT_WHERE_OPS", "0") != "0":  # A/B: the routed row selection as torch.where
        resvit.FOLD_SELECT = False
    if os.environ.get("VITMI_RESVIT_ZERO_FULL", "0") != "0":  # A/B: padded operands cleared whole
        from vitmi import resvit_fused
        resvit_fused.ZERO_FULL = True
    if os.environ.get("VITMI_RESVIT_NO_SINK", "0") != "0":  # A/B: weight gradients through AccumulateGrad
        from vitmi import flat as vflat
        vflat.SINKS = False
    if os.environ.get("VITMI_RESVIT_APPROX_OPS", "0") != "0":  # A/B: the per-op approximator path
        for l in model.layers:
            if hasattr(l, "block_path_approximators"):
                l.block_path_approximators.fused = False
    if os.environ.get("VITMI_RESVIT_ROUTER_OPS", "0") != "0":  # A/B: the per-op router MLP
        for l in model.layers:
            if hasattr(l, "router"):
                l.router.fused_mlp = False
    opt = AdamW(model.parameters(), lr=1e-4, weight_decay=0.05, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=1.0)
    sched = get_cosine_schedule_with_warmup(opt, 500, 15000)
    reducer = None
    if world > 1:
        from vitmi.dist import FlatGradAllReducer
        reducer = FlatGradAllReducer(opt.flat).attach()
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(b, 3, args.image_size, args.image_size, device=dev, generator=g)
    y = torch.randint(0, 100, (b,), device=dev, generator=g)
    ratios = []
    # forward + backward replayed from a HIP graph (GraphedTrainStep), the optimizer eager; data parallel: the
    # flat gradient all-reduced after each replay (reducer.finish). VITMI_RESVIT_EAGER=1: op by op instead (the
    # all-reduce hooks then run during the backward) — the A/B of profiles/r06/resvit_eager_vs_graph.txt
    eager = os.environ.get("VITMI_RESVIT_EAGER", "0") != "0"
    graphed = None if eager else GraphedTrainStep(model, x, y, opt, sched, 1e-4, 1e-2, 1.0, True, reducer=reducer)

    totals = []

    def step():
        out = graphed.step() if graphed is not None else train_step(model, x, y, opt, sched, 1e-4, 1e-2, 1.0, True,
                                                                    reducer)
        ratios.append(out[5]["non_low_rank_ratio"].clone())
        totals.append(out[0].detach().clone())

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    dist_check = None
    if world > 1:  # the trainable flat buffer (LoRA, routers, approximators, head): the frozen bases never change
        dist_check = replica_check(opt.flat.data, dt, args.steps, world, backend, dev)
        dt = dist_check.pop("_dt_max")
    active = float(torch.stack(ratios[-args.steps:]).mean())
    value = args.steps * b * world / dt
    heads = sum(1 for l in model.layers if hasattr(l, "router"))
    fpi = resvit_flops_per_image(dict(a, patch=16, router_hdim=512), args.image_size, heads, active)
    achieved = value / world * fpi / 1e12
    out = {
        "metric": f"images/sec training step, Res-ViT-B/16 {args.image_size}px bf16",
        "value": round(value, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (N(0,1) images, uniform labels, seed-42 reference-order random init, Gumbel routing)",
        "config": {"workload": f"Res-ViT-B/16 @{args.image_size} train step (teacher+routed student fwd, 1c+1e-4a+"
                               f"1e-2d loss, bwd, {comm + ' all-reduce, ' if world > 1 else ''}clip 1.0 + AdamW, "
                               "cosine warm-up)" + (", fwd+bwd as one HIP graph" if graphed is not None else ""),
                   "model": "Res-ViT-B/16 (LoRA r8, reslr, block 1, 100 classes)", "image_size": args.image_size,
                   "per_gpu_batch": b, "global_batch": b * world, "seq_len": (args.image_size // 16) ** 2 + 1,
                   "parallelism": f"dp{world}", "dist_backend": backend},
        "roofline": {"bound": "mfma", "kernel": "whole step (executed matrix FLOPs, resvit_flops_per_image)",
                     "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": None},
        "executed_gflop_per_image": round(fpi / 1e9, 3),
        "active_ratio": round(active, 4),
        "loss_first_timed_step": round(float(totals[args.warmup]), 5),
        "loss_last_timed_step": round(float(totals[-1]), 5),
    }
    if dist_check is not None:
        out["dist_check"] = dist_check
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
        if not dist_check["replicas_identical"]:
            print("error: the data-parallel replicas' parameters differ after the run", file=sys.stderr)
            sys.exit(3)


if __name__ == "__main__":
    main()
