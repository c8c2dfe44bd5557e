"""vitcnn_amd — MI355X-native ViT-CNN ("Multimodality_Mamba") training hot path.

Python mirror of the reference's plugin surface (model_utils.get_model / train / test / val)
over hand-written gfx950 HIP kernels behind the C ABI in include/vitcnn.h.
"""
from .model import Multimodality_Mamba  # noqa: F401
from .losses import CrossEntropyLoss  # noqa: F401
from .optim import AdamW  # noqa: F401
from .step import fused_train_step  # noqa: F401

__all__ = ["Multimodality_Mamba", "CrossEntropyLoss", "AdamW", "fused_train_step"]
