from .ddp import FlatParams, GradBucketer  # noqa: F401
from .ldm import LDMTrainStep, unet_backward_order  # noqa: F401
