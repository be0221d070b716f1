"""ldmseg — MI355X-native drop-in for the latent-diffusion denoising path of
weentiaan/Video-latent-diffusion-panoptic-segmentation.

Same import paths as the reference package (``ldmseg.models.UNet``,
``ldmseg.models.GeneralVAESeg``, ``ldmseg.schedulers.DDIMNoiseScheduler``,
``ldmseg.utils.OutputDict``); every op of the path runs through the gfx950 HIP library
``lib/libldmseg_hip.so`` (C ABI: include/ldmseg_hip.h).
"""
__version__ = "0.1.0"
