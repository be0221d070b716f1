"""BASELINE config 3 on the GPU (tools/main_ldm.py + trainers_ldm_cond.py:792-900).

* The full SD-1.4 UNet (815.5 M, 12-channel conv_in for self-conditioning) trained at the
  config's per-GPU workload: 2 clips x T=8 = 16 frames of 4x64x64 latents, bf16 compute with fp32
  master weights, self-conditioning, SNR weights, clip 1.0, AdamW — loss and every parameter
  update finite, the trainable parameters (all but the frozen time_embedding) updated.
* fp32 parameter gradients of the full SD-1.4 UNet at B=1, 64x64 against torch autograd through
  the CPU oracle (oracle/unet.py; diffusers parity unpinned) for a named subset spanning every
  block type, bar 1e-3 (max-abs error relative to the tensor's max-abs).
* Data parallel, world 2 (two processes on this GPU, gloo): ranks start from different seeds,
  LDMTrainStep's rank-0 broadcast makes them equal (DDP's construction broadcast,
  tools/main_ldm.py:184-197); after two iterations on half batches with the bucketed, overlapped
  all-reduce (1 MB buckets: ~50 collectives per step, the time_emb_proj buckets last), both ranks
  hold bit-identical weights, equal (update rel L2 < 1e-2) to one process stepping on the
  concatenated batch.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

from golden_utils import DDIM_CONFIGS, build_loop_unet
from ldmseg.models import UNet
from ldmseg.schedulers import DDIMNoiseScheduler
from ldmseg.trainers import LDMTrainStep
from oracle import unet as ounet

pytestmark = pytest.mark.gpu
DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))


def _sched(dev):
    return DDIMNoiseScheduler(**DDIM_CONFIGS["script"], device=dev, verbose=False)


def _sd14(cond):
    torch.manual_seed(0)
    with torch.device(DEV):
        u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero", cond_channels=cond,
                     init_mode_cond="zero")
    u.freeze_layers(["time_embedding"])
    return u.train()


def test_full_sd14_train_step_config3_bf16():
    u = _sd14(4)
    st = LDMTrainStep(u, _sched(DEV), lr=1e-4, weight_decay=0.05, clip_grad=1.0, self_condition=True,
                      compute_dtype=torch.bfloat16, seed=1)
    assert st.flat.numel == sum(p.numel() for p in u.parameters() if p.requires_grad)
    assert abs(st.flat.numel - 813.4e6) < 0.5e6                       # 813.4 M trainable
    B, L = 16, 64
    g = torch.Generator().manual_seed(2)
    lat = torch.randn(B, 4, L, L, generator=g).to(DEV)
    rgb = torch.randn(B, 4, L, L, generator=g).to(DEV)
    mask = (torch.rand(B, L, L, generator=g) > 0.05).float().to(DEV)
    w0 = st.flat.data.clone()
    losses = [st.train_step(lat, rgb, mask).item() for _ in range(2)]
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert torch.isfinite(st.flat.data).all() and torch.isfinite(st.exp_avg_sq).all()
    moved = (st.flat.data != w0)
    assert moved.float().mean().item() > 0.99                        # AdamW moves (almost) every weight
    for n, p in u.named_parameters():
        if p.requires_grad:
            assert (p.detach() != w0[st.flat.offsets[st.flat.index[id(p)]]:][:p.numel()].view_as(p)).any(), n


SUBSET = ("conv_in.weight", "down_blocks.0.resnets.0.conv1.weight", "down_blocks.0.resnets.0.time_emb_proj.weight",
          "down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q.weight",
          "down_blocks.0.attentions.0.transformer_blocks.0.ff.net.0.proj.weight",
          "down_blocks.1.resnets.0.conv_shortcut.weight", "down_blocks.2.downsamplers.0.conv.weight",
          "mid_block.attentions.0.transformer_blocks.0.attn1.to_out.0.weight", "mid_block.resnets.1.norm2.weight",
          "up_blocks.0.resnets.2.conv1.weight", "up_blocks.1.upsamplers.0.conv.bias",
          "up_blocks.3.attentions.2.proj_out.weight", "up_blocks.3.attentions.2.transformer_blocks.0.norm3.bias",
          "conv_norm_out.weight", "conv_out.weight")


def test_full_sd14_grads_fp32_b1_match_oracle():
    u = _sd14(0)
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 8, 64, 64, generator=g)
    gy = torch.randn(1, 4, 64, 64, generator=g)
    t = torch.tensor([437])
    # oracle autograd on the CPU, gradients for the subset only
    sd = {k: v.detach().cpu().clone() for k, v in u.state_dict().items() if not k.startswith("new_conv.")}
    for k in SUBSET:
        sd[k].requires_grad_(True)
    torch.set_num_threads(16)
    ref_out = ounet.forward(sd, dict(u.config), x, t)
    (ref_out * gy).sum().backward()
    out = u(x.to(DEV), t.to(DEV)).sample
    (out * gy.to(DEV)).sum().backward()
    assert ((out.detach().cpu() - ref_out.detach()).abs().max() / ref_out.detach().abs().max()).item() < 1e-3
    named = dict(u.named_parameters())
    worst = []
    for k in SUBSET:
        ref = sd[k].grad
        e = ((named[k].grad.cpu() - ref).abs().max() / ref.abs().max().clamp_min(1e-20)).item()
        worst.append((e, k))
    worst.sort(reverse=True)
    assert worst[0][0] < 1e-3, worst[:5]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(tmp_path):
    g = torch.Generator().manual_seed(4)
    I, B, L = 2, 4, 16
    d = {"latents": torch.randn(I, B, 4, L, L, generator=g), "rgb": torch.randn(I, B, 4, L, L, generator=g),
         "mask": (torch.rand(I, B, L, L, generator=g) > 0.1).float(), "noise": torch.randn(I, B, 4, L, L, generator=g),
         "t": torch.randint(0, 1000, (I, B), generator=g)}
    torch.save(d, tmp_path / "in.pt")
    return d, I


def _run_world2(tmp_path, tag, *extra):
    """Two ranks of tests/ddp_train_worker.py on this GPU (gloo); returns their saved records."""
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "ddp_train_worker.py"), str(tmp_path / "in.pt"),
                               str(tmp_path / tag), *extra], env=dict(env, RANK=str(r)))
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    return [torch.load(tmp_path / f"{tag}{r}.pt", weights_only=True) for r in range(2)]


def test_ddp_world2_equals_single_process_on_concatenated_batch(tmp_path):
    d, I = _inputs(tmp_path)
    r0, r1 = _run_world2(tmp_path, "rank")
    assert r0["buckets"] > 10
    assert torch.equal(r0["init"], r1["init"])                      # the rank-0 broadcast ...
    assert torch.equal(r0["frozen"], r1["frozen"])                  # ... of the frozen time_embedding too
    assert torch.equal(r0["final"], r1["final"])                    # one averaged update on both ranks
    # single process, same initial weights (rank 0's seed), whole batch per iteration
    u = build_loop_unet(UNet, cond=4, seed=10).to(DEV)
    st = LDMTrainStep(u, _sched(DEV), lr=1e-3, weight_decay=0.05, clip_grad=1.0, self_condition=True,
                      compute_dtype=torch.float32)
    assert torch.equal(st.flat.data.cpu(), r0["init"])
    for i in range(I):
        loss = st.train_step(d["latents"][i].to(DEV), d["rgb"][i].to(DEV), d["mask"][i].to(DEV),
                             timesteps=d["t"][i].to(DEV), noise=d["noise"][i].to(DEV)).item()
        # step 0 runs on identical weights; step 1 after one AdamW update, whose normalised step
        # turns ~1e-6 gradient differences of near-zero gradients into O(lr) weight differences
        tol = 1e-6 if i == 0 else 1e-3
        assert abs(loss - 0.5 * (r0["losses"][i] + r1["losses"][i]).item()) / loss < tol, i
    single = st.flat.data.cpu()
    worst = []
    for p in st.flat.params:
        o, k = st.flat.offsets[st.flat.index[id(p)]], p.numel()
        dref = single[o:o + k] - r0["init"][o:o + k]
        dm = r0["final"][o:o + k] - r0["init"][o:o + k]
        worst.append(((dm - dref).norm() / dref.norm().clamp_min(1e-30)).item())
    assert max(worst) < 1e-2, sorted(worst)[-5:]


def test_zero1_world2_matches_unsharded_ddp(tmp_path):
    """ZeRO stage 1 (optim.py:71-78, train_diffusion.sh:27): each rank keeps the AdamW moments of
    half the flat buffer, updates that half and all-gathers it.  The optimizer alone (identical
    state and gradients) equals the unsharded run bit for bit, weights and consolidated state; and
    since every reduction of the backward is deterministic (slab reductions summed in a fixed
    order: bias / time-embedding column sums, LayerNorm dgamma / dbeta, the loss and the gradient
    norm; split-K weight gradients), two full training iterations do too."""
    _inputs(tmp_path)
    z0, z1 = _run_world2(tmp_path, "zero", "zero")
    r0, _ = _run_world2(tmp_path, "plain")
    n = r0["final"].numel()
    (a0, b0), (a1, b1) = z0["shard"].tolist(), z1["shard"].tolist()
    assert a0 == 0 and b0 == a1 and b1 == n                         # disjoint shards covering the buffer
    assert z0["moment_numel"] == b0 - a0 and z1["moment_numel"] == b1 - a1 and r0["moment_numel"] == n
    assert torch.equal(z0["final"], z1["final"]) and torch.equal(z0["opt_final"], z1["opt_final"])
    assert torch.equal(z0["opt_final"], r0["opt_final"])
    assert torch.equal(z0["opt_moments"], r0["opt_moments"]) and torch.equal(z1["opt_moments"], r0["opt_moments"])
    assert torch.equal(z0["moments"], z1["moments"])
    assert torch.equal(z0["init"], r0["init"])
    assert torch.equal(z0["losses"], r0["losses"])
    assert torch.equal(z0["final"], r0["final"])                    # full iterations, bit for bit
    assert torch.equal(z0["moments"], r0["moments"])


def test_training_iterations_are_deterministic():
    """Two identical runs of two full LDM training iterations (self-conditioning forward, HIP
    backward, clip, AdamW) give bit-identical weights, moments and losses: no reduction of the step
    depends on atomic ordering."""
    g = torch.Generator().manual_seed(11)
    B, L = 4, 16
    data = [dict(latents=torch.randn(B, 4, L, L, generator=g), rgb=torch.randn(B, 4, L, L, generator=g),
                 mask=(torch.rand(B, L, L, generator=g) > 0.1).float(), noise=torch.randn(B, 4, L, L, generator=g),
                 t=torch.randint(0, 1000, (B,), generator=g)) for _ in range(2)]

    def run():
        u = build_loop_unet(UNet, cond=4, seed=12).to(DEV)
        st = LDMTrainStep(u, _sched(DEV), lr=1e-3, weight_decay=0.05, clip_grad=1.0, self_condition=True,
                          compute_dtype=torch.bfloat16)
        losses = [st.train_step(d["latents"].to(DEV), d["rgb"].to(DEV), d["mask"].to(DEV),
                                timesteps=d["t"].to(DEV), noise=d["noise"].to(DEV)).item() for d in data]
        torch.cuda.synchronize()
        return losses, st.flat.data.cpu().clone(), st.exp_avg.cpu().clone(), st.exp_avg_sq.cpu().clone()
    a, b = run(), run()
    assert a[0] == b[0]
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)
