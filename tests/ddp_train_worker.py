"""One rank of the world-2 data-parallel training check (tests/test_gpu_train_full.py).

Launched as a plain subprocess per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment), both ranks on cuda:0 with the gloo backend (RCCL refuses two ranks on one GPU).
Each rank builds the reduced-width UNet from a DIFFERENT seed — LDMTrainStep's rank-0 broadcast
(DDP's construction-time broadcast, tools/main_ldm.py:184-197) must make them start equal — then
runs two training iterations on its half of the batch and saves its final flat parameters.

    python tests/ddp_train_worker.py <inputs.pt> <out_prefix> [zero]

With ``zero`` the optimizer is ZeRO-1 sharded (LDMTrainStep(zero_redundancy=True)); the rank also
saves its shard bounds and the consolidated (collective) optimizer state.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _moments(st):
    if st.zero:                                           # collective per call; rank `to` keeps the moments
        for dst in range(st.world):
            st.consolidate_state_dict(to=dst)
            if st.rank == dst:
                sd = st.state_dict()
    else:
        sd = st.state_dict()
    return torch.cat([torch.cat([v["exp_avg"].reshape(-1), v["exp_avg_sq"].reshape(-1)]).cpu()
                      for _, v in sorted(sd["state"].items())])


def main():
    inputs, out_prefix = sys.argv[1], sys.argv[2]
    zero = len(sys.argv) > 3 and sys.argv[3] == "zero"
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
                      compute_dtype=torch.float32, bucket_mb=1, zero_redundancy=zero)
    init = st.flat.data.detach().cpu().clone()
    frozen = torch.cat([q.detach().reshape(-1).float().cpu() for q in u.parameters() if not q.requires_grad])
    n = d["latents"].shape[1] // world
    sl = slice(rank * n, (rank + 1) * n)
    losses = []
    for i in range(d["latents"].shape[0]):
        g = lambda k: d[k][i, sl].to(dev)        # noqa: E731
        losses.append(st.train_step(g("latents"), g("rgb"), g("mask"), timesteps=g("t"), noise=g("noise")).item())
    torch.cuda.synchronize()
    moments = _moments(st)                                # collective under ZeRO (consolidation)
    # the optimizer alone on identical state and gradients on both ranks (no clip: no reduction
    # order in the arithmetic), so ZeRO and unsharded runs must agree bit for bit
    u2 = build_loop_unet(UNet, cond=4, seed=30).to(dev)
    st2 = LDMTrainStep(u2, sched, lr=1e-3, weight_decay=0.05, clip_grad=0.0, compute_dtype=torch.float32,
                       zero_redundancy=zero)
    gg = torch.Generator().manual_seed(5)
    for _ in range(2):
        st2.flat.grad.copy_(torch.randn(st2.flat.numel, generator=gg))
        st2.optimizer_step()
    torch.cuda.synchronize()
    torch.save({"init": init, "frozen": frozen, "final": st.flat.data.detach().cpu(), "losses": torch.tensor(losses),
                "buckets": len(st.bucketer.buckets), "shard": torch.tensor(st.shard),
                "moment_numel": st.exp_avg.numel(), "moments": moments,
                "opt_final": st2.flat.data.detach().cpu(), "opt_moments": _moments(st2)}, f"{out_prefix}{rank}.pt")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
