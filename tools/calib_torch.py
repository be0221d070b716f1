#!/usr/bin/env python3
"""Calibration only (never on the product path): time the vendor libraries (hipBLASLt via
torch.matmul, MIOpen via F.conv2d channels_last, torch SDPA) on the UNet's largest shapes, to
see how far the hand-written kernels are from what the chip's libraries reach."""
import torch
import torch.nn.functional as F

DEV = "cuda"
BF = torch.bfloat16


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best


def main():
    for (M, N, Kd) in [(32768, 320, 2880), (32768, 2560, 320), (32768, 320, 320), (2048, 1280, 11520),
                       (512, 1280, 11520), (8192, 5120, 640), (2048, 10240, 1280), (8192, 8192, 8192)]:
        a = torch.randn(M, Kd, device=DEV, dtype=BF)
        b = torch.randn(Kd, N, device=DEV, dtype=BF)
        ms = timeit(lambda: a @ b)
        print(f"matmul M={M:6d} N={N:6d} K={Kd:6d}  {ms * 1e3:8.1f} us  {2 * M * N * Kd / ms / 1e9:7.1f} TF/s", flush=True)
    for (B, H, C, Co) in [(8, 64, 320, 320), (8, 32, 640, 640), (8, 16, 1280, 1280), (8, 8, 1280, 1280)]:
        x = torch.randn(B, C, H, H, device=DEV, dtype=BF).to(memory_format=torch.channels_last)
        w = torch.randn(Co, C, 3, 3, device=DEV, dtype=BF).to(memory_format=torch.channels_last)
        ms = timeit(lambda: F.conv2d(x, w, padding=1))
        print(f"conv3x3 B={B} H={H} C={C}->{Co}  {ms * 1e3:8.1f} us  {2 * B * H * H * C * Co * 9 / ms / 1e9:7.1f} TF/s",
              flush=True)
    for (B, N, h, d) in [(8, 4096, 8, 40), (8, 1024, 8, 80), (8, 256, 8, 160), (8, 4096, 8, 64)]:
        q = torch.randn(B, h, N, d, device=DEV, dtype=BF)
        ms = timeit(lambda: F.scaled_dot_product_attention(q, q, q))
        print(f"sdpa B={B} N={N} h={h} d={d}  {ms * 1e3:8.1f} us  {4 * B * h * N * N * d / ms / 1e9:7.1f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()
