"""Drop-in ``DDIMNoiseScheduler`` (ldmseg/schedulers/ddim_scheduler.py:26-291).

Schedule tables are built once on the host in fp32 exactly as the reference does
(:51-95, :97-117, :119-131).  The per-step arithmetic — ``step`` (:218-269),
``add_noise`` (:155-187), ``remove_noise`` (:189-216) — runs as one fused HIP kernel on
GPU tensors, reading the timestep and the alphas_cumprod table on the device: the
reference's per-step host sync (CPU table indexed by a device scalar) is gone, and a
python-int timestep is served from a device-resident table without any H2D copy.
"""
import math
from typing import Optional, Union

import numpy as np
import torch

from ..ops import native as K
from ..utils import OutputDict


class DDIMNoiseSchedulerOutput(OutputDict):
    prev_sample: torch.FloatTensor
    pred_original_sample: Optional[torch.FloatTensor] = None


def _alpha_bar_betas(n, max_beta=0.999):
    """GLIDE cosine schedule discretisation (:138-153)."""
    f = lambda s: math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
    return torch.tensor([min(1.0 - f((i + 1) / n) / f(i / n), max_beta) for i in range(n)], dtype=torch.float32)


_BETAS = {
    "linear": lambda n, b0, b1: torch.linspace(b0, b1, n, dtype=torch.float32),
    "scaled_linear": lambda n, b0, b1: torch.linspace(b0 ** 0.5, b1 ** 0.5, n, dtype=torch.float32) ** 2,
    "squaredcos_cap_v2": lambda n, b0, b1: _alpha_bar_betas(n),
    "sigmoid": lambda n, b0, b1: torch.sigmoid(torch.linspace(-6, 6, n)) * (b1 - b0) + b0,
}


class DDIMNoiseScheduler(object):
    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.0001, beta_end: float = 0.02,
                 beta_schedule: str = "linear", clip_sample: bool = True, set_alpha_to_one: bool = True,
                 steps_offset: int = 0, prediction_type: str = "epsilon", thresholding: bool = False,
                 dynamic_thresholding_ratio: float = 0.995, clip_sample_range: float = 1.0,
                 sample_max_value: float = 1.0, weight: str = "none", max_snr: float = 5.0,
                 device: Union[str, torch.device] = None, verbose: bool = True):
        if beta_schedule not in _BETAS:
            raise NotImplementedError(f"{beta_schedule} does is not implemented for {self.__class__}")
        self.betas = _BETAS[beta_schedule](num_train_timesteps, beta_start, beta_end)
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.compute_loss_weights(mode=weight, max_snr=max_snr)
        self.weights = self.weights.to(device)
        self.num_train_timesteps = num_train_timesteps
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, num_train_timesteps)[::-1].copy().astype(np.int64))
        self.clip_sample = clip_sample
        self.clip_sample_range = clip_sample_range
        self.prediction_type = prediction_type
        self.thresholding = thresholding
        self.dynamic_thresholding_ratio = dynamic_thresholding_ratio
        self.steps_offset = steps_offset
        self.beta_schedule = beta_schedule
        self.beta_start = beta_start
        self.beta_end = beta_end
        self.init_noise_sigma = 1.0
        self.verbose = verbose
        self._dev_tables = {}

    # ---------------------------------------------------------------- host-side tables
    def compute_loss_weights(self, mode="max_clamp_snr", max_snr=5.0):
        assert mode in ["inverse_log_snr", "max_clamp_snr", "linear", "fixed", "none"]
        self.weight_mode = mode
        snr = self.alphas_cumprod / (1 - self.alphas_cumprod)
        if mode == "inverse_log_snr":
            # the reference's in-place `w /= w[-1]` raises on torch>=2 (self-aliasing); this is its intent
            w = torch.log(1.0 / snr).clamp(min=1)
            self.weights = w / w[-1].clone()
        elif mode == "max_clamp_snr":
            self.weights = snr.clamp(max=max_snr) / snr
        elif mode == "fixed":
            self.weights = snr.clone()
            self.weights[: len(self.weights) // 4] = 0.1
        elif mode == "linear":
            self.weights = torch.arange(1, len(snr) + 1) / len(snr)
        else:
            self.weights = torch.ones_like(snr)

    def set_timesteps_inference(self, num_inference_steps: int, device: Union[str, torch.device] = None,
                                tmin: int = 0):
        self.num_inference_steps = num_inference_steps
        ratio = self.num_train_timesteps // self.num_inference_steps
        self.steps_offset = ratio - 1
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
        ts = torch.from_numpy(ts) + self.steps_offset
        self.timesteps = ts[ts >= tmin].to(device)

    def move_timesteps_to(self, device: Union[str, torch.device]):
        self.timesteps = self.timesteps.to(device)

    def get_betas_for_alpha_bar(self, num_diffusion_timesteps, max_beta=0.999) -> torch.Tensor:
        return _alpha_bar_betas(num_diffusion_timesteps, max_beta)

    # ---------------------------------------------------------------- device residency
    def _tables(self, device):
        key = str(device)
        tab = self._dev_tables.get(key)
        if tab is None:
            tab = (self.alphas_cumprod.to(device).contiguous(),
                   torch.arange(self.num_train_timesteps, dtype=torch.int64, device=device))
            self._dev_tables[key] = tab
        return tab

    def _t_device(self, timestep, device):
        """A one-element int64 device tensor for `timestep` without a host<->device round trip."""
        ac, ar = self._tables(device)
        if torch.is_tensor(timestep) and timestep.is_cuda:
            t = timestep.reshape(-1)[:1]
            return t if t.dtype == torch.int64 else t.to(torch.int64)
        t = int(timestep)
        if not 0 <= t < self.num_train_timesteps:
            raise IndexError(f"timestep {t} outside [0, {self.num_train_timesteps})")
        return ar[t:t + 1]

    # ---------------------------------------------------------------- per-step arithmetic (HIP)
    def step(self, model_output: torch.FloatTensor, timestep: int, sample: torch.FloatTensor,
             use_clipped_model_output: bool = False) -> DDIMNoiseSchedulerOutput:
        if self.thresholding:
            raise NotImplementedError
        if self.prediction_type not in K.PRED:
            raise NotImplementedError
        dev = sample.device
        ac, _ = self._tables(dev)
        t = self._t_device(timestep, dev)
        out_dtype = torch.promote_types(model_output.dtype, sample.dtype)
        prev, x0 = K.ddim_step(model_output.contiguous(), sample.contiguous(), t, ac,
                               float(self.final_alpha_cumprod), self.num_train_timesteps // self.num_inference_steps,
                               self.prediction_type, self.clip_sample, self.clip_sample_range,
                               use_clipped_model_output, out_dtype)
        return DDIMNoiseSchedulerOutput(prev_sample=prev, pred_original_sample=x0)

    def fused_step_args(self, timestep, sample: torch.FloatTensor, model_output_dtype, use_clipped_model_output=False,
                        prev_out=None):
        """The step() arguments as the device-side dict a producer kernel that fuses the step takes
        (ldm_unet_tail: the UNet's conv_out epilogue runs this same arithmetic on its output), or None
        when this configuration has no fused form.  prev_out: where prev_sample goes (may be sample
        itself, updated in place)."""
        if self.thresholding or self.prediction_type not in K.PRED:
            return None
        dev = sample.device
        ac, _ = self._tables(dev)
        return dict(sample=sample.contiguous(), t=self._t_device(timestep, dev), alphas_cumprod=ac,
                    final_alpha=float(self.final_alpha_cumprod),
                    step_ratio=self.num_train_timesteps // self.num_inference_steps,
                    prediction_type=self.prediction_type, clip_sample=self.clip_sample,
                    clip_range=self.clip_sample_range, use_clipped=use_clipped_model_output,
                    out_dtype=torch.promote_types(model_output_dtype, sample.dtype), prev_out=prev_out)

    def add_noise(self, original_samples: torch.FloatTensor, noise: torch.FloatTensor, timesteps: torch.IntTensor,
                  scale: float = 1.0, mask_noise_perc: Optional[float] = None) -> torch.FloatTensor:
        dev = original_samples.device
        ac, _ = self._tables(dev)
        if mask_noise_perc is not None:
            mask = torch.rand_like(original_samples) < mask_noise_perc
            noise *= mask                                     # in place, as the reference (:184)
        t = timesteps.reshape(-1).to(device=dev, dtype=torch.int64)
        return K.ddim_add_noise(original_samples.contiguous(), noise.to(original_samples.dtype).contiguous(), t, ac,
                                scale)

    @torch.no_grad()
    def remove_noise(self, noisy_samples: torch.FloatTensor, noise: torch.FloatTensor, timesteps: torch.IntTensor,
                     scale: float = 1.0) -> torch.FloatTensor:
        dev = noisy_samples.device
        ac, _ = self._tables(dev)
        t = timesteps.reshape(-1).to(device=dev, dtype=torch.int64)
        return K.ddim_remove_noise(noisy_samples.contiguous(), noise.to(noisy_samples.dtype).contiguous(), t, ac,
                                   scale)

    def __str__(self) -> str:
        w = self.weights if self.verbose else "VerboseDisabled"
        return (f"DDIMScheduler(num_inference_steps={self.num_inference_steps}, "
                f"num_train_timesteps={self.num_train_timesteps}, prediction_type={self.prediction_type}, "
                f"beta_start={self.beta_start}, beta_end={self.beta_end}, beta_schedule={self.beta_schedule}, "
                f"clip_sample={self.clip_sample}, clip_sample_range={self.clip_sample_range}, "
                f"thresholding={self.thresholding}, dynamic_thresholding_ratio={self.dynamic_thresholding_ratio}, "
                f"steps_offset={self.steps_offset}, weight_mode={self.weight_mode}, weights={w})")

    __repr__ = __str__

    def __len__(self) -> int:
        return self.num_train_timesteps
