"""One rank of the world-2 data-parallel training check (tests/test_gpu_train_full.py).

Launched as a plain subprocess per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment), both ranks on cuda:0 with the gloo backend (RCCL refuses two ranks on one GPU).
Each rank builds the reduced-width UNet from a DIFFERENT seed — LDMTrainStep's rank-0 broadcast
(DDP's construction-time broadcast, tools/main_ldm.py:184-197) must make them start equal — then
runs two training iterations on its half of the batch and saves its final flat parameters.

    python tests/ddp_train_worker.py <inputs.pt> <out_prefix>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    inputs, out_prefix = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    from golden_utils import DDIM_CONFIGS, build_loop_unet
    from ldmseg.models import UNet
    from ldmseg.schedulers import DDIMNoiseScheduler
    from ldmseg.trainers import LDMTrainStep
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = torch.load(inputs, weights_only=True)
    u = build_loop_unet(UNet, cond=4, seed=10 + rank).to(dev)
    sched = DDIMNoiseScheduler(**DDIM_CONFIGS["script"], device=dev, verbose=False)
    st = LDMTrainStep(u, sched, lr=1e-3, weight_decay=0.05, clip_grad=1.0, self_condition=True,
                      compute_dtype=torch.float32, bucket_mb=1)
    init = st.flat.data.detach().cpu().clone()
    frozen = torch.cat([q.detach().reshape(-1).float().cpu() for q in u.parameters() if not q.requires_grad])
    n = d["latents"].shape[1] // world
    sl = slice(rank * n, (rank + 1) * n)
    losses = []
    for i in range(d["latents"].shape[0]):
        g = lambda k: d[k][i, sl].to(dev)        # noqa: E731
        losses.append(st.train_step(g("latents"), g("rgb"), g("mask"), timesteps=g("t"), noise=g("noise")).item())
    torch.cuda.synchronize()
    torch.save({"init": init, "frozen": frozen, "final": st.flat.data.detach().cpu(), "losses": torch.tensor(losses),
                "buckets": len(st.bucketer.buckets)}, f"{out_prefix}{rank}.pt")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
