"""ugpg -- MI355X-native (gfx950) Uncertainty-Guided Progressive U-Net.

Drop-in for the reference modules (tridang04022004/UG-PG-UNet):
  UG_unet_parts.py             -> ugpg.unet_parts   (alias module ugpg.UG_unet_parts)
  UG_unet.py                   -> ugpg.unet, ugpg.loss (alias module ugpg.UG_unet)
  uncertainty_guided_trainer.py-> ugpg.trainer      (alias ugpg.uncertainty_guided_trainer)
  Herlev/train_herlev.py model -> ugpg.herlev
  MoNuSegImprove/test_monuseg.py evaluation -> ugpg.evaluation
All hot-path arithmetic runs in libugpg.so (hand-written HIP kernels, C-ABI in
include/ugpg.h); there is no CPU fallback.
"""
from .unet_parts import DoubleConv, Down, InConv, OutConv, Up  # noqa: F401
from .unet import (PGUNet1, PGUNet2, PGUNet3, PGUNet4, ProgressiveUNet,  # noqa: F401
                   STAGE_RESOLUTIONS, transfer_state)
from .loss import UncertaintyGuidedLoss  # noqa: F401
from .optim import RMSprop  # noqa: F401
from .trainer import UncertaintyGuidedProgressiveTrainer  # noqa: F401
from .evaluation import MoNuSegTester, evaluate_logits, predict_masks  # noqa: F401
from .augment import AugMoNuSegDataset, MoNuSegAugmenter, MoNuSegDataset  # noqa: F401

__version__ = "0.1.0"
