#!/usr/bin/env python3
"""UNet denoising steps/sec (T=8, 4x64x64 latent) on MI355X — BASELINE.json's headline metric.

One "step" = one denoising step of the reference sampler (trainers_ldm_cond.py:1130-1166)
on one T=8 clip: the SD-1.4 UNet forward over B=8 frames of [x_t || rgb] (8x64x64,
cross-attention removed, 815.5 M params, random init) + one fused DDIM step, replayed as
one captured HIP graph per step.  Frames are independent (no temporal layers),
so N GPUs run N independent clips: no collective on the data path, weak scaling;
``value`` = N x K steps / max-over-ranks wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  It carries a "roofline" object for the dominant kernel
family (HIP events around every launch of an instrumented step, algorithmic FLOPs/bytes)
and, at N=1, a "cpu_baseline" timed on the host cores with the oracle restatement.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "UNet denoising steps/sec (T=8, 4×64×64 latent)"
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3      # fp32 MFMA = vector rate
PEAK_FP8_TFLOPS = 5000.0      # dense fp8 MFMA (2x bf16; the headline figures with sparsity are not used)
PEAK_HBM_GBS = 8000.0


def build_unet(dev, dtype):
    from ldmseg.models import UNet
    torch.manual_seed(0)
    with torch.device(dev):
        u = UNet()                                        # SD-1.4 UNet2DConditionModel config
    u.remove_cross_attention()                            # base.yaml:71 image_descriptors: remove
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")   # base.yaml:37-45
    return u.to(dtype=dtype).eval()


def make_scheduler(dev):
    from ldmseg.schedulers import DDIMNoiseScheduler
    s = DDIMNoiseScheduler(prediction_type="epsilon", beta_schedule="scaled_linear", num_train_timesteps=1000,
                           beta_start=0.00085, beta_end=0.012, steps_offset=1, clip_sample=False,
                           set_alpha_to_one=False, device=dev, verbose=False)          # base.yaml:48-62
    s.set_timesteps_inference(50)
    return s


def parse_latent(spec):
    """'64' -> (64, 64); '32x64' -> (32, 64)."""
    parts = str(spec).lower().split("x")
    if len(parts) == 1:
        return int(parts[0]), int(parts[0])
    if len(parts) == 2:
        return int(parts[0]), int(parts[1])
    raise SystemExit(f"--latent: expected L or HxW, got {spec!r}")


def roofline(unet, stepper, ts, nsteps, dtype, fp8=False):
    from ldmseg.ops import native as K
    prof = K.LaunchProfiler()
    K.set_profiler(prof)
    try:
        for i in range(nsteps):
            t = ts[i % len(ts)]
            stepper._tb.copy_(stepper._tab[t])
            stepper._body()
    finally:
        K.set_profiler(None)
    fam = prof.summary()
    if os.environ.get("LDM_OPLOG"):
        # the profiled steps' launches in order (tools/traffic_table.py aligns them with the
        # per-dispatch PMC counters of the same run to attribute HBM traffic per op)
        with open(os.environ["LDM_OPLOG"], "w") as f:
            json.dump({"steps": nsteps, "ops": [{"family": r[0], "flops": r[1], "bytes": r[2], "detail": r[5]}
                                                for r in prof.records]}, f)
    if os.environ.get("LDM_BENCH_DETAIL"):
        det = prof.summary(by_detail=True)
        print(f"{'kernel':10s} {'shape':44s} {'n':>3s} {'ms':>8s} {'TF/s':>7s} {'GB/s':>7s}", file=sys.stderr)
        for (f, s), v in sorted(det.items(), key=lambda kv: -kv[1]["ms"])[:40]:
            ms = v["ms"] / nsteps
            print(f"{f:10s} {s:44s} {v['launches'] // nsteps:3d} {ms:8.3f} "
                  f"{v['flops'] / nsteps / ms / 1e9:7.1f} {v['bytes'] / nsteps / ms / 1e6:7.1f}", file=sys.stderr)
    peak_tf = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_FP32_TFLOPS
    per_step = {}
    for k, v in fam.items():
        # eager_event_ms: HIP events around every launch of eager (non-graph) steps — it carries ~5-7 us of
        # dispatch per launch, so the families sum to more than the graph-replayed ms_per_step
        e = dict(launches=v["launches"] // nsteps, eager_event_ms=round(v["ms"] / nsteps, 4),
                 gflop=round(v["flops"] / nsteps / 1e9, 2), mb=round(v["bytes"] / nsteps / 1e6, 2))
        sec = v["ms"] * 1e-3
        if v["flops"] > 0:      # MFMA-bound family: fraction of the dense MFMA peak
            pk = PEAK_FP8_TFLOPS if (fp8 and k == "attention") else peak_tf
            e["tflops"] = round(v["flops"] / sec / 1e12, 1)
            e["frac_mfma"] = round(v["flops"] / sec / 1e12 / pk, 4)
            if pk != peak_tf:
                e["peak_tflops"] = pk
        e["gbs"] = round(v["bytes"] / sec / 1e9, 1)
        e["frac_hbm"] = round(v["bytes"] / sec / 1e9 / PEAK_HBM_GBS, 4)
        per_step[k] = e
    dom = max(fam, key=lambda k: fam[k]["ms"])
    d = fam[dom]
    if d["flops"] > 0:
        achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
        peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_FP32_TFLOPS
        rl = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
              "frac": round(achieved / peak, 4)}
    else:
        achieved = d["bytes"] / (d["ms"] * 1e-3) / 1e9
        rl = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
              "frac": round(achieved / PEAK_HBM_GBS, 4)}
    rl["pmc_workload"] = pmc_key = f"B={unet_batch(stepper)} {stepper.lat.shape[-2]}x{stepper.lat.shape[-1]} " \
        f"{str(dtype).replace('torch.', '')}{' fp8' if fp8 else ''}"
    rl["traffic"], rl["traffic_source"] = pmc_traffic(dom, pmc_key)
    rl["avg_launch_ms"] = round(d["ms"] / d["launches"], 5)
    rl["launches_per_step"] = d["launches"] // nsteps
    rl["algorithmic_flops_per_launch"] = round(d["flops"] / d["launches"], 1)
    rl["algorithmic_bytes_per_launch"] = round(d["bytes"] / d["launches"], 1)
    rl["kernels_per_step"] = per_step
    return rl


def unet_batch(stepper):
    return stepper.lat.shape[0]


def pmc_traffic(family, workload):
    """HBM bytes per launch of `family` from the newest committed PMC summary of the SAME workload
    (profiles/rNN_families.json, written by tools/profile_bench.sh from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes over this same command, tagged with the bench line's
    `pmc_workload`).  A live bench run cannot read PMC counters itself; None when no summary of
    this workload exists (a B=1 or config-5 line never borrows the B=8 figure)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_families.json")))
    for f in reversed(files):
        try:
            meta = json.load(open(f))
            if meta.get("workload") != workload:
                continue
            fam = meta["families"].get(family, {})
        except (OSError, ValueError, KeyError):
            continue
        if "traffic_bytes_per_call" in fam:
            return fam["traffic_bytes_per_call"], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(unet, budget_s=25.0, frames=8, lh=64, lw=64):
    """Oracle restatement (oracle/unet.py + oracle/ddim.py, fp32 torch on the host cores),
    bounded sample: whole frames of the T=`frames` step until ~budget_s, scaled to steps/s."""
    from oracle import ddim as oddim
    from oracle import unet as ounet
    host = host_cores()
    threads = host["usable"]
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu() for k, v in unet.state_dict().items()}
    cfg = dict(unet.config)
    _, ac, final = oddim.tables("scaled_linear", 1000, 0.00085, 0.012, False)
    g = torch.Generator().manual_seed(5)
    T = frames
    frames, elapsed = 0, 0.0
    with torch.no_grad():
        while elapsed < budget_s and frames < T:
            x = torch.randn(1, 4, lh, lw, generator=g)
            rgb = torch.randn(1, 4, lh, lw, generator=g)
            t0 = time.perf_counter()
            eps = ounet.forward(sd, cfg, torch.cat([x, rgb], 1), torch.tensor(979))
            oddim.step(ac, final, 1000, 50, eps, 979, x)
            elapsed += time.perf_counter() - t0
            frames += 1
    per_step = elapsed / frames * T
    return {"value": round(1.0 / per_step, 5), "unit": "steps/s", "cores": threads, "kind": "port",
            "host": host,
            "sample": f"{frames} frame(s) of one T={T} denoising step (UNet fwd + DDIM, fp32, {lh}x{lw}), "
                      f"{elapsed:.1f} s, scaled x{T / frames:g} to one {T}-frame step"}


def host_cores():
    """The CPU baseline's thread count: os.cpu_count(), capped by what this process
    may actually run on — its CPU affinity and its cgroup CPU quota (a GPU box shares a large host:
    os.cpu_count() there counts the whole machine, and oversubscribing a 16-core quota would
    understate the CPU).  Everything is reported."""
    n = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:   # noqa: BLE001
        phys = None
    usable = min(n, aff, quota or n)
    return {"os_cpu_count": n, "affinity": aff, "cgroup_quota_cpus": quota, "physical_cores": phys, "usable": usable}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=8, help="T: frames per clip (folded into the batch)")
    ap.add_argument("--latent", default="64", help="latent side L (LxL) or HxW, e.g. 32x64 for config 5's 256x512 frames")
    ap.add_argument("--fp8", action="store_true",
                    help="config 5: self-attention on the fp8 (e4m3) MFMA path (UNet.set_attention_fp8)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="compute dtype (default: bf16, the reference's fp16-autocast width; --mode ae: fp32, config "
                         "1's reference precision, trainers_ae.py:279-389)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=2)
    ap.add_argument("--repeats", type=int, default=5, help="timed windows of --steps steps; value from the median")
    ap.add_argument("--mode", default="denoise", choices=["denoise", "train", "sample", "ae"],
                    help="denoise: the headline metric; train: config 3's DDP training iteration; "
                         "sample: config 4's full clip sampling (encode -> 50 DDIM steps -> decode -> panoptic); "
                         "ae: config 1's VAE (autoencoder) training iteration")
    ap.add_argument("--clips", type=int, default=2, help="train mode: clips of T frames per GPU")
    ap.add_argument("--zero", action="store_true",
                    help="train mode: ZeRO-1 sharded AdamW (train_diffusion.sh:27 optimizer_zero_redundancy)")
    args = ap.parse_args()
    if args.dtype is None:
        args.dtype = "fp32" if args.mode == "ae" else "bf16"
    if args.mode == "train":
        return main_train(args)
    if args.mode == "sample":
        return main_sample(args)
    if args.mode == "ae":
        return main_ae(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)   # RCCL; used only for barrier + timing reduce
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    from ldmseg.pipelines import DenoiseStep
    unet = build_unet(dev, dtype)
    if args.fp8:
        if dtype != torch.bfloat16:
            raise SystemExit("--fp8 needs --dtype bf16")
        unet.set_attention_fp8(True)
    sched = make_scheduler(dev)
    B = args.frames
    LH, LW = parse_latent(args.latent)
    g = torch.Generator().manual_seed(1 + rank)                    # each rank: its own clip
    rgb = torch.randn(B, 4, LH, LW, generator=g).to(dev)
    stepper = DenoiseStep(unet, sched, rgb, self_condition=False, use_graph=not args.no_graph)
    stepper.set_latents(torch.randn(B, 4, LH, LW, generator=g).to(dev))
    ts = [int(t) for t in sched.timesteps]

    for i in range(args.warmup):
        stepper.run(ts[i % len(ts)], last=False)
    from ldmseg.utils import max_over_ranks

    def window():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            stepper.run(ts[k % len(ts)], last=False)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return max_over_ranks(time.perf_counter() - t0, device=dev)
    windows = [window() for _ in range(args.repeats)]
    elapsed = sorted(windows)[len(windows) // 2]          # median window (median of 5)
    finite = bool(torch.isfinite(stepper.lat).all().item())

    rl = roofline(unet, stepper, ts, args.profile_steps, dtype, fp8=args.fp8) if rank == 0 else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(unet, frames=B, lh=LH, lw=LW)
    if rank == 0:
        headline = (B, LH, LW) == (8, 64, 64) and not args.fp8
        workload = f"UNet fwd (B={B} frames = one T={B} clip, 8x{LH}x{LW} input) + DDIM step, HIP graph per step"
        if args.fp8:
            workload += ", self-attention on the fp8 e4m3 MFMA (BASELINE config 5)"
        line = {
            "metric": METRIC if headline else f"UNet denoising steps/sec (T={B}, 4x{LH}x{LW} latent)", "value": round(world * args.steps / elapsed, 4), "unit": "steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": f"synthetic: random-init SD-1.4 UNet weights, N(0,1) KITTI-shaped 4x{LH}x{LW} latents",
            "config": {"workload": workload,
                       "model": "SD-1.4 UNet2DConditionModel, cross-attn removed, 8-ch conv_in (815.5M)",
                       "global_batch": B * world, "seq_len": LH * LW,
                       "parallelism": f"replicas x{world} (independent clips, no data-path collective)"},
            "outputs_finite": finite,
            "windows_ms_per_step": [round(w / args.steps * 1e3, 3) for w in windows],
            "roofline": rl,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


SAMPLE_METRIC = "full panoptic sampling clips/sec (T=8 KITTI frames 192x640, 50 DDIM steps, K=128)"


def main_sample(args):
    """Config 4: per clip, RGB encode (SD VAE encoder at 192x192) -> 50 DDIM steps of the UNet ->
    seg-VAE decode to K=128 logits at 512x512 -> resize to the frame -> panoptic head.  `steps`
    clips are timed after `warmup` untimed clips; every rank samples its own clips."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    from ldmseg.models import GeneralVAESeg
    from ldmseg.models.autoencoder_kl import GeneralVAEImage
    from ldmseg.pipelines import DenoiseStep
    from ldmseg.pipelines.sample import sample_panoptic
    from ldmseg.utils import max_over_ranks
    torch.manual_seed(0)
    unet = build_unet(dev, dtype)
    sched = make_scheduler(dev)
    vae_image = GeneralVAEImage().to(dev, dtype).eval()
    vae_seg = GeneralVAESeg(in_channels=16, int_channels=256, out_channels=128, block_out_channels=(32, 64, 128, 256),
                            num_upscalers=2, scaling_factor=0.2)
    # random-init logits are too flat for any segment to pass mask_th / count_th: sharpen the last
    # conv as tests/test_gpu_fullsize.py does, so the timed head runs its keep / relabel work
    # (trainers_ldm_cond.py:1274-1336) on surviving segments
    with torch.no_grad():
        vae_seg.decoder[10].weight.mul_(20.0)
        vae_seg.decoder[10].bias.sub_(1.0).mul_(20.0)
    vae_seg = vae_seg.to(dev, dtype).eval()
    B, L = args.frames, parse_latent(args.latent)[0]
    steps = args.steps if args.steps != 20 else 3        # default: 3 timed clips
    warm = min(args.warmup, 1)
    g = torch.Generator().manual_seed(1 + rank)
    clip = torch.rand(B, 3, 192, 640, generator=g).to(dev)
    stepper = DenoiseStep(unet, sched, torch.zeros(B, 4, L, L, device=dev), self_condition=False,
                          use_graph=not args.no_graph)
    run = lambda: sample_panoptic(clip, vae_image, vae_seg, unet, sched, latent_size=L, stepper=stepper)  # noqa
    for _ in range(warm):
        run()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, device=dev)
    if rank == 0:
        print(json.dumps({
            "metric": SAMPLE_METRIC, "value": round(world * steps / elapsed, 4), "unit": "clips/s", "n_gpus": world,
            "steps": steps, "warmup": warm, "ms_per_step": round(elapsed / steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic: random-init SD-1.4 UNet / SD VAE encoder / seg-VAE (K=128) weights, U(0,1) frames",
            "config": {"workload": f"clip of T={B} frames: encode + 50 DDIM steps + decode + panoptic head",
                       "global_batch": B * world, "parallelism": f"replicas x{world}"},
            "segments_frame0": len(res[0]["panoptic_seg"][1])}), flush=True)
    if world > 1:
        dist.destroy_process_group()


AE_METRIC = "VAE (autoencoder) training iterations/sec (4 semKITTI frames 10x192x640, point losses)"


def main_ae(args):
    """Config 1 (main_worker_ae.py): GeneralVAESeg (KITTI: 10 bits in, 30 classes out) train
    iteration on 4 synthetic frames: forward with posterior sampling, CE + BCE/dice point losses
    (12544 points, oversample 3), backward, clip 3.0, AdamW."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    from ldmseg.models import GeneralVAESeg
    from ldmseg.trainers.ae import AETrainStep
    torch.manual_seed(0)
    vae = GeneralVAESeg(in_channels=10, int_channels=256, out_channels=30, block_out_channels=(32, 64, 128, 256),
                        num_upscalers=2, scaling_factor=0.2).to(dev, dtype).train()
    g = torch.Generator().manual_seed(1)
    lo = torch.randn(4, 20, 12, 40, generator=g)
    targets = torch.nn.functional.interpolate(lo, size=(192, 640), mode="bilinear").argmax(1).to(dev)
    bits = torch.stack([(targets >> i) & 1 for i in range(5)] * 2, 1).float()
    st = AETrainStep(vae, lr=1e-4, clip_grad=3.0, ignore_label=0)
    steps = args.steps
    for _ in range(args.warmup):
        st.train_step(bits, targets)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss, ce, mask = st.train_step(bits, targets)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    print(json.dumps({
        "metric": AE_METRIC, "value": round(steps / elapsed, 4), "unit": "iterations/s", "n_gpus": 1,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic: blobby 20-class KITTI-shaped targets, their 5+5 bit planes; random-init VAE (1.80 M)",
        "config": {"workload": "AE train iteration, B=4 frames 192x640", "global_batch": 4},
        "loss": round(loss.item(), 5),
        "cpu_baseline": None if args.no_cpu_baseline else cpu_baseline_ae(vae, bits, targets)}),
        flush=True)


def cpu_baseline_ae(vae, bits, targets, budget_s=20.0):
    """Config 1 on the host cores: the oracle AE iteration (oracle/ae.py: the reference's VAE
    forward with posterior sampling + point losses, autograd backward) + clip 3.0 + torch AdamW,
    fp32, the same B=4 x 10 x 192 x 640 batch; whole iterations until ~budget_s."""
    from oracle import ae as oae
    host = host_cores()
    torch.set_num_threads(host["usable"])
    sd = {k: v.detach().float().cpu() for k, v in vae.state_dict().items()}
    cfg = dict(in_channels=10, int_channels=256, out_channels=30, block_out_channels=(32, 64, 128, 256),
               latent_channels=4, num_latents=2, num_upscalers=2, norm_num_groups=32)
    b, t = bits.float().cpu(), targets.cpu()
    g = torch.Generator().manual_seed(0)
    rand = lambda *shape: torch.rand(*shape, generator=g)          # noqa: E731
    randn = lambda shape: torch.randn(shape, generator=g)          # noqa: E731
    params = {k: v.clone() for k, v in sd.items()}
    opt_state = {}
    iters, elapsed = 0, 0.0
    while elapsed < budget_s and iters < 5:
        t0 = time.perf_counter()
        _, _, _, grads = oae.train_iteration(params, cfg, b, t, rand, randn)
        gl = [grads[k] for k in params if grads.get(k) is not None]
        torch.nn.utils.clip_grad_norm_(gl, 3.0)
        if not opt_state:
            ps = [torch.nn.Parameter(params[k]) for k in params]
            opt_state["opt"] = torch.optim.AdamW(ps, lr=1e-4)
            opt_state["ps"] = ps
        for p_, k in zip(opt_state["ps"], params):
            p_.grad = grads.get(k)
        opt_state["opt"].step()
        params = {k: p_.detach() for p_, k in zip(opt_state["ps"], params)}
        elapsed += time.perf_counter() - t0
        iters += 1
    return {"value": round(iters / elapsed, 4), "unit": "iterations/s", "cores": host["usable"], "kind": "port",
            "host": host, "sample": f"{iters} AE iteration(s) (fwd + point losses + bwd + clip + AdamW, fp32, B=4 "
                                    f"10x192x640), {elapsed:.1f} s"}


TRAIN_METRIC = "LDM training iterations/sec (2 clips x T=8 per GPU, 4x64x64 latents, self-conditioning)"


def main_train(args):
    """BASELINE config 3 (tools/main_ldm.py + train_diffusion.sh): per GPU 2 clips x T=8 = 16
    frames of [x_t || rgb || self-cond] (12x64x64), SD-1.4 UNet with fp32 master weights
    computing in bf16 (the reference: fp32 weights + fp16 autocast), self-conditioning forward,
    SNR-weighted masked L2, hand-written backward, grad clip 1.0, AdamW (lr 1e-4, wd 0.05).
    N > 1: one process per GPU, gradients summed by bucketed RCCL all-reduces overlapped with
    the backward (ldmseg/trainers/ddp.py).  value = N x steps / max-over-ranks time."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from ldmseg.models import UNet
    from ldmseg.schedulers import DDIMNoiseScheduler
    from ldmseg.trainers import LDMTrainStep
    from ldmseg.utils import max_over_ranks
    torch.manual_seed(0)                                   # identical init on every rank (DDP broadcast)
    with torch.device(dev):
        u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero", cond_channels=4,
                     init_mode_cond="zero")                 # train_diffusion.sh: self_condition, cond_channels 4
    u.freeze_layers(["time_embedding"])
    u.train()
    sched = DDIMNoiseScheduler(prediction_type="epsilon", beta_schedule="scaled_linear", beta_start=0.00085,
                               beta_end=0.012, steps_offset=1, clip_sample=False, set_alpha_to_one=False,
                               weight="max_clamp_snr", max_snr=2.0, device=dev, verbose=False)
    step = LDMTrainStep(u, sched, lr=1e-4, weight_decay=0.05, clip_grad=1.0, self_condition=True,
                        compute_dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32, seed=1 + rank,
                        zero_redundancy=args.zero)
    B, L = args.clips * args.frames, parse_latent(args.latent)[0]
    g = torch.Generator().manual_seed(100 + rank)
    lat = (torch.randn(B, 4, L, L, generator=g)).to(dev)
    rgb = (torch.randn(B, 4, L, L, generator=g)).to(dev)
    mask = (torch.rand(B, L, L, generator=g) > 0.05).float().to(dev)
    for _ in range(args.warmup):
        step.train_step(lat, rgb, mask)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = step.train_step(lat, rgb, mask)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, device=dev)
    lv = float(loss.item())
    if rank == 0:
        tflop = 4 * 6.17 * B / 8          # fwd + bwd (2x fwd) + self-cond fwd; 6.17 TFLOP per 8-frame fwd
        line = {
            "metric": TRAIN_METRIC, "value": round(world * args.steps / elapsed, 4), "unit": "iterations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic: random-init SD-1.4 UNet weights, N(0,1) latents, 5% ignore mask",
            "config": {"workload": f"train iteration: self-cond fwd + fwd + bwd + clip + AdamW, {B} frames/GPU",
                       "model": "SD-1.4 UNet2DConditionModel, cross-attn removed, 12-ch conv_in (815.5M)",
                       "global_batch": B * world, "seq_len": L * L,
                       "parallelism": f"dp{world} (RCCL bucketed all-reduce overlapped with backward)"
                                      + (", ZeRO-1 sharded AdamW" if args.zero and world > 1 else "")},
            "loss": round(lv, 6),
            "algorithmic_tflop_per_iter_per_gpu": round(tflop, 2),
            "achieved_tflops_per_gpu": round(tflop * args.steps / elapsed, 1),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
