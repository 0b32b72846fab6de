"""Alias of the reference module name uncertainty_guided_trainer (drop-in import path)."""
from .trainer import UncertaintyGuidedProgressiveTrainer  # noqa: F401
from .unet import PGUNet1, PGUNet2, PGUNet3, PGUNet4, ProgressiveUNet  # noqa: F401
from .loss import UncertaintyGuidedLoss  # noqa: F401
