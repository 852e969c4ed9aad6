"""Command-line configuration, mirroring reference src/config.py.

Same flags, defaults and architecture presets (get_b16_config ... get_h14_config,
src/config.py:57-104). Additions for the MI355X path, all optional:
  --synthetic            synthetic N(0,1) images / uniform labels instead of torchvision datasets
  --steps-per-epoch      batches per synthetic epoch
  --synthetic-source-size  >0: synthetic uint8 HWC images of this size, resized / flipped /
                         normalised on the device like the reference's CIFAR transform (vitmi.data)
  --any-image-size       lift the reference's choices=[224, 384] on --image-size (src/config.py:37)
  --no-save              do not create experiments/ directories or checkpoints
  --precision            (eval) bf16 MFMA forward (default) or the reference's f32 arithmetic
"""
from __future__ import annotations

import argparse
import json
import os
from datetime import datetime


def _add_common(parser, train: bool):
    parser.add_argument("--n-gpu", type=int, default=1,
                        help="number of gpus to use (one rank per GPU; --batch-size is the global batch)")
    parser.add_argument("--model-arch", type=str, default="b16", help="model setting to use",
                        choices=["b16", "b32", "l16", "l32", "h14"])
    parser.add_argument("--batch-size", type=int, default=32, help="batch size")
    parser.add_argument("--data-dir", type=str, default="../data", help="data folder")
    parser.add_argument("--num-classes", type=int, default=100 if train else 1000, help="number of classes in dataset")
    parser.add_argument("--seed", type=int, default=42, help="random seed for reproducibility")
    parser.add_argument("--synthetic", default=False, action="store_true", help="synthetic data (MI355X benchmark)")
    parser.add_argument("--steps-per-epoch", type=int, default=100, help="batches per synthetic epoch")
    parser.add_argument("--synthetic-source-size", type=int, default=0,
                        help="synthetic uint8 images of this size through the device transform (0: f32 N(0,1))")
    parser.add_argument("--any-image-size", default=False, action="store_true", help="allow any --image-size")


def _image_size_arg(parser, default):
    parser.add_argument("--image-size", type=int, default=default, help="input image size")


def get_eval_config(argv=None):
    """reference src/config.py:5-25"""
    parser = argparse.ArgumentParser("Visual Transformer Evaluation")
    _add_common(parser, train=False)
    parser.add_argument("--checkpoint-path", type=str, default=None, help="model checkpoint to load weights")
    _image_size_arg(parser, 384)
    parser.add_argument("--num-workers", type=int, default=8, help="number of workers")
    parser.add_argument("--dataset", type=str, default="ImageNet", help="dataset for fine-tunning/evaluation")
    parser.add_argument("--precision", type=str, default="bf16", choices=["bf16", "fp32"],
                        help="bf16 MFMA forward or the reference's f32 arithmetic")
    config = parser.parse_args(argv)
    _check_image_size(config)
    config = globals()["get_{}_config".format(config.model_arch)](config)
    print_config(config)
    return config


def get_train_config(argv=None):
    """reference src/config.py:28-54"""
    parser = argparse.ArgumentParser("Visual Transformer Train/Fine-tune")
    _add_common(parser, train=True)
    parser.add_argument("--exp-name", type=str, default="ft", help="experiment name")
    parser.add_argument("--swanlab", default=False, action="store_true", help="flag of turning on swanlab")
    parser.add_argument("--checkpoint-path", type=str,
                        default="../weights/pytorch/imagenet21k+imagenet2012_ViT-B_16-224.pth",
                        help="model checkpoint to load weights")
    _image_size_arg(parser, 224)
    parser.add_argument("--num-workers", type=int, default=1, help="number of workers")
    parser.add_argument("--train-steps", type=int, default=15000, help="number of training/fine-tunning steps")
    parser.add_argument("--lr", type=float, default=0.03, help="learning rate")
    parser.add_argument("--wd", type=float, default=0.0, help="weight decay")
    parser.add_argument("--warmup-steps", type=int, default=500, help="learning rate warm up steps")
    parser.add_argument("--dataset", type=str, default="CIFAR100", help="dataset for fine-tunning/evaluation")
    parser.add_argument("--no-save", default=False, action="store_true", help="no experiment dirs / checkpoints")
    config = parser.parse_args(argv)
    _check_image_size(config)
    config = globals()["get_{}_config".format(config.model_arch)](config)
    process_config(config)
    print_config(config)
    return config


def _check_image_size(config):
    if not config.any_image_size and config.image_size not in (224, 384):
        raise SystemExit(f"--image-size {config.image_size}: choose 224 or 384 (reference src/config.py:37), "
                         "or pass --any-image-size")


def get_b16_config(config):
    """ViT-B/16 configuration (reference src/config.py:57-66)"""
    config.patch_size = 16
    config.emb_dim = 768
    config.mlp_dim = 3072
    config.num_heads = 12
    config.num_layers = 12
    config.attn_dropout_rate = 0.0
    config.dropout_rate = 0.0
    return config


def get_b32_config(config):
    """ViT-B/32 configuration (reference src/config.py:69-73)"""
    config = get_b16_config(config)
    config.patch_size = 32
    return config


def get_l16_config(config):
    """ViT-L/16 configuration (reference src/config.py:76-85)"""
    config.patch_size = 16
    config.emb_dim = 1024
    config.mlp_dim = 4096
    config.num_heads = 16
    config.num_layers = 24
    config.attn_dropout_rate = 0.0
    config.dropout_rate = 0.0
    return config


def get_l32_config(config):
    """ViT-L/32 configuration (reference src/config.py:88-92)"""
    config = get_l16_config(config)
    config.patch_size = 32
    return config


def get_h14_config(config):
    """ViT-H/14 configuration (reference src/config.py:95-104)"""
    config.patch_size = 14
    config.emb_dim = 1280
    config.mlp_dim = 5120
    config.num_heads = 16
    config.num_layers = 32
    config.attn_dropout_rate = 0.0
    config.dropout_rate = 0.0
    return config


def process_config(config):
    """Experiment directories + config.json (reference src/utils.py:56-76)."""
    # (ranks started by `--n-gpu k` inherit their launcher's stamp, so all share one experiment dir)
    timestamp = os.environ.get("VITMI_EXP_STAMP") or datetime.now().strftime("%y%m%d_%H%M%S")
    config.exp_stamp = timestamp
    exp_name = config.exp_name + "_{}_bs{}_lr{}_wd{}".format(config.dataset, config.batch_size, config.lr, config.wd)
    exp_name += "_" + timestamp
    config.summary_dir = os.path.join("experiments", "tb", exp_name)
    config.checkpoint_dir = os.path.join("experiments", "save", exp_name, "checkpoints/")
    config.result_dir = os.path.join("experiments", "save", exp_name, "results/")
    if getattr(config, "no_save", False):
        return config
    for d in (config.summary_dir, config.checkpoint_dir, config.result_dir):
        os.makedirs(d, exist_ok=True)
    with open(os.path.join("experiments", "save", exp_name, "config.json"), "w") as f:
        json.dump(vars(config), f, indent=4)
    return config


def print_config(config):
    message = "----------------- Config ---------------\n"
    for k, v in sorted(vars(config).items()):
        message += "{:>35}: {:<30}\n".format(str(k), str(v))
    message += "----------------- End -------------------"
    print(message)
