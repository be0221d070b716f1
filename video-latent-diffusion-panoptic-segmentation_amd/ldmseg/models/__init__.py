from .unet import UNet, UNetOutput  # noqa: F401
from .vae import GeneralVAESeg, DiagonalGaussianDistribution, LayerNorm2d  # noqa: F401
