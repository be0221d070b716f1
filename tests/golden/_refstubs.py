"""Import shims for loading the *reference* ldmseg package in the build container.

Used ONLY by ``make_golden.py`` (fixture generation, run in the survey/build
container where /root/reference exists).  The reference package imports several
third-party libraries that are not installed here (detectron2, diffusers,
torchvision, easydict, termcolor, wandb, tabulate).  None of them sits on the
code paths we take golden vectors from (bit codec, DDIM scheduler, GeneralVAESeg
with ``num_mid_blocks=0``, ``vpq_eval``), so each is registered as an inert
module.  Recipe: SURVEY.md Appendix C.
"""
import importlib.machinery as _im
import sys
import types

import torch.nn as nn

REFERENCE_ROOT = "/root/reference"


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = _im.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Unavailable:
    def __init__(self, *a, **k):
        raise RuntimeError("third-party class is stubbed in the fixture generator")


def install():
    """Register the stubs and put the reference on sys.path (idempotent)."""
    if "detectron2" not in sys.modules:
        _mod("detectron2")
        _mod("detectron2.utils")
        _mod("detectron2.utils.comm")
        _mod("detectron2.utils.visualizer", Visualizer=object, _PanopticPrediction=_Unavailable,
             ColorMode=_Unavailable, _OFF_WHITE=(1.0, 1.0, 1.0),
             _create_text_labels=lambda *a, **k: None)
        _mod("detectron2.utils.file_io", PathManager=object)
        _mod("detectron2.data")
        _mod("detectron2.data.datasets")
        _mod("detectron2.data.datasets.builtin_meta", COCO_CATEGORIES=[])
        _mod("detectron2.evaluation")
        _mod("detectron2.evaluation.evaluator", DatasetEvaluator=object)
        sys.modules["detectron2.utils"].comm = sys.modules["detectron2.utils.comm"]
    if "diffusers" not in sys.modules:
        _mod("diffusers", AutoencoderKL=_Unavailable, UNet2DConditionModel=nn.Module)
        _mod("diffusers.models")
        _mod("diffusers.models.unet_2d_blocks", UNetMidBlock2D=_Unavailable)
        _mod("diffusers.training_utils", EMAModel=object)
    if "torchvision" not in sys.modules:
        tv = _mod("torchvision")
        tv.transforms = _mod("torchvision.transforms", Compose=lambda x: x,
                             Resize=lambda *a, **k: None, ToTensor=lambda *a, **k: None,
                             Normalize=lambda *a, **k: None)
    for name, attrs in (("easydict", dict(EasyDict=dict)),
                        ("tabulate", dict(tabulate=lambda *a, **k: "")),
                        ("termcolor", dict(colored=lambda s, *a, **k: s)),
                        ("wandb", {})):
        if name not in sys.modules:
            _mod(name, **attrs)
    # CLIP descriptors are off-path (image_descriptors: remove) and would fetch remote weights.
    _mod("ldmseg.models.descriptors", get_image_descriptor_model=None)
    if REFERENCE_ROOT not in sys.path:
        sys.path.insert(0, REFERENCE_ROOT)
