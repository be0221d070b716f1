"""DDIM noise scheduler arithmetic — torch fp32 CPU restatement (test infrastructure only).

Follows ldmseg/schedulers/ddim_scheduler.py:
  schedule tables  :51-75    loss weights :97-117    inference timesteps :119-131
  add_noise        :155-187  remove_noise :189-216   step                :218-269
"""
import math

import numpy as np
import torch


def betas_for(schedule, n, beta_start, beta_end):
    if schedule == "linear":                                               # :52
        return torch.linspace(beta_start, beta_end, n, dtype=torch.float32)
    if schedule == "scaled_linear":                                        # :53-57
        return torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=torch.float32) ** 2
    if schedule == "squaredcos_cap_v2":                                    # :138-153
        f = lambda s: math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
        return torch.tensor([min(1 - f((i + 1) / n) / f(i / n), 0.999) for i in range(n)],
                            dtype=torch.float32)
    if schedule == "sigmoid":                                              # :61-64
        return torch.sigmoid(torch.linspace(-6, 6, n)) * (beta_end - beta_start) + beta_start
    raise NotImplementedError(schedule)


def tables(schedule="linear", n=1000, beta_start=0.0001, beta_end=0.02, set_alpha_to_one=True):
    betas = betas_for(schedule, n, beta_start, beta_end)
    ac = torch.cumprod(1.0 - betas, dim=0)                                 # :68-69
    final = torch.tensor(1.0) if set_alpha_to_one else ac[0]               # :75
    return betas, ac, final


def loss_weights(ac, mode, max_snr):                                       # :97-117
    snr = ac / (1 - ac)
    if mode == "max_clamp_snr":
        return snr.clamp(max=max_snr) / snr
    if mode == "fixed":
        w = snr.clone()
        w[: len(w) // 4] = 0.1
        return w
    if mode == "linear":
        return torch.arange(1, len(snr) + 1) / len(snr)
    if mode == "inverse_log_snr":
        w = torch.log(1.0 / snr).clamp(min=1)
        return w / w[-1].clone()
    return torch.ones_like(snr)


def inference_timesteps(n_train, n_inf, tmin=0):                           # :119-131
    ratio = n_train // n_inf
    ts = (np.arange(0, n_inf) * ratio).round()[::-1].astype(np.int64) + (ratio - 1)
    return ts[ts >= tmin]


def step(ac, final, n_train, n_inf, model_output, t, sample, prediction_type="epsilon",
         clip_sample=False, clip_range=1.0, use_clipped_model_output=False):  # :218-269
    prev_t = t - n_train // n_inf
    a_t = ac[t]
    a_prev = ac[prev_t] if prev_t >= 0 else final
    b_t = 1 - a_t
    if prediction_type == "epsilon":
        x0 = (sample - b_t ** 0.5 * model_output) / a_t ** 0.5
        eps = model_output
    elif prediction_type == "sample":
        x0 = model_output
        eps = (sample - a_t ** 0.5 * x0) / b_t ** 0.5
    elif prediction_type == "v_prediction":
        x0 = a_t ** 0.5 * sample - b_t ** 0.5 * model_output
        eps = a_t ** 0.5 * model_output + b_t ** 0.5 * sample
    else:
        raise NotImplementedError(prediction_type)
    if clip_sample:
        x0 = x0.clamp(-clip_range, clip_range)
    if use_clipped_model_output:
        eps = (sample - a_t ** 0.5 * x0) / b_t ** 0.5
    prev = a_prev ** 0.5 * x0 + (1 - a_prev) ** 0.5 * eps
    return prev, x0


def _bcast(v, ref):
    v = v.flatten()
    while v.ndim < ref.ndim:
        v = v.unsqueeze(-1)
    return v


def add_noise(ac, x0, noise, t, scale=1.0):                                # :155-187
    a = ac[t]
    return _bcast(a ** 0.5, x0) * scale * x0 + _bcast((1 - a) ** 0.5, x0) * noise


def remove_noise(ac, xt, noise, t, scale=1.0):                             # :189-216
    a = ac[t]
    return (xt - _bcast((1 - a) ** 0.5, xt) * noise) / (_bcast(a ** 0.5, xt) * scale)
