"""vitmi — MI355X-native (gfx950 HIP) training path for the ViT of sea-with-sakura/ViT-of-Pytorch.

Drop-in surface: vitmi.model (src/model.py classes), vitmi.config (src/config.py), vitmi.train
(src/train.py entrypoints), vitmi.optim.SGD. Compute runs in libvit_hip.so (C ABI in
include/vit_hip.h) through vitmi.engine.
"""
from .engine import ArchConfig, ViTEngine  # noqa: F401
from .model import (CrossEntropyLoss, Encoder, EncoderBlock, LinearGeneral, MlpBlock, MLPBlock,  # noqa: F401
                    PositionEmbs, SelfAttention, VisionTransformer)

__version__ = "0.1.0"
