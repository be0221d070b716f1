"""The denoising sampler: TrainerDiffusion.sample (ldmseg/trainers/trainers_ldm_cond.py:1048-1173)
as a host loop over HIP-only steps.

Same semantics as the reference loop:
  latents ~ N(0, 1) from a CPU torch.Generator(seed), moved to the GPU (:1091-1095)
  per t: inputs = [x_t || rgb_latents (|| x0_prev if self_condition)]  (:1134-1141)
         eps = unet(inputs, t); condition = step(eps, t, x_t).x0       (:1144, :1152-1153)
         x_t = step(eps, t, x_t).prev_sample, or .pred_original_sample at the last t (:1157-1162)
Differences that change no number: the input concat is folded into the UNet's conv_in
gather, the two identical ``scheduler.step`` calls share one fused kernel launch, and
timesteps are read from device-resident tables (no host sync per step).  With
``use_graph=True`` one step (UNet + DDIM) is captured once as a HIP graph and replayed.
"""
import torch

from ..ops import native as K


class DenoiseStep:
    """One denoising step on static buffers, optionally captured into a HIP graph."""

    def __init__(self, unet, scheduler, rgb_latents, self_condition, use_graph):
        self.unet, self.sched = unet, scheduler
        dev = rgb_latents.device
        B, _, L, Lw = rgb_latents.shape
        self.rgb = rgb_latents.contiguous()
        self.lat = torch.zeros(B, 4, L, Lw, dtype=torch.float32, device=dev)
        self.cond = torch.zeros_like(self.rgb) if self_condition else None
        # the timestep as int64 (DDIM) and float32 (time embedding) in one 16-byte buffer, so one copy
        # from a per-timestep device table sets both before a replay
        self._tb = torch.zeros(16, dtype=torch.uint8, device=dev)
        self.t_int = self._tb[0:8].view(torch.int64)
        self.t_f = self._tb[8:12].view(torch.float32)
        ac, ar = scheduler._tables(dev)
        tab = torch.zeros(ar.numel(), 16, dtype=torch.uint8, device=dev)
        tab[:, 0:8] = ar.to(torch.int64).view(-1, 1).view(torch.uint8)
        tab[:, 8:12] = ar.to(torch.float32).view(-1, 1).view(torch.uint8)
        self._tab = tab
        self.graph = None
        self.prev = self.x0 = None
        unet.prepare()
        if use_graph:
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self._body()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.prev, self.x0 = self._body()

    def _body(self):
        srcs = [self.lat, self.rgb] + ([self.cond] if self.cond is not None else [])   # conv_in gather casts
        if hasattr(self.unet, "forward_ddim_step"):
            # UNet + scheduler.step, the step fused into the UNet tail's launch where it can be
            # prev_sample written over the latents in place (the tail reads each element first)
            return self.unet.forward_ddim_step(srcs, self.t_f, self.sched, self.t_int, self.lat, prev_out=self.lat)
        eps = self.unet.forward_sources(srcs, self.t_f)
        r = self.sched.step(eps, self.t_int, self.lat)
        return r.prev_sample, r.pred_original_sample

    def set_latents(self, latents):
        self.lat.copy_(latents)
        if self.cond is not None:
            self.cond.zero_()

    def run(self, t: int, last: bool):
        self._tb.copy_(self._tab[t])
        if self.graph is not None:
            self.graph.replay()
            prev, x0 = self.prev, self.x0
        else:
            prev, x0 = self._body()
        if self.cond is not None:
            self.cond.copy_(x0)
        if last:
            return x0
        if prev.data_ptr() != self.lat.data_ptr():
            self.lat.copy_(prev)
        return self.lat


@torch.no_grad()
def sample_latents(unet, scheduler, rgb_latents, num_inference_steps=50, seed=0, self_condition=False,
                   use_graph=False, return_all_latents=False, stepper=None):
    scheduler.set_timesteps_inference(num_inference_steps)
    B, _, L, Lw = rgb_latents.shape
    gen = torch.Generator().manual_seed(seed) if seed is not None else None
    latents = torch.randn((B, 4, L, Lw), generator=gen).to(rgb_latents.device) * scheduler.init_noise_sigma
    step = stepper or DenoiseStep(unet, scheduler, rgb_latents, self_condition, use_graph)
    step.set_latents(latents)
    ts = [int(t) for t in scheduler.timesteps]
    outs = []
    x = None
    for i, t in enumerate(ts):
        x = step.run(t, last=i == len(ts) - 1)
        if return_all_latents:
            outs.append(x.clone())
    if return_all_latents:
        return torch.cat(outs, dim=0)
    return x.clone()
