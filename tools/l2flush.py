#!/usr/bin/env python3
"""Isolate an op's own HBM writes from lines another launch left dirty in L2 (VERDICT r05 item 7:
"test the inherited-dirty-lines claim for gemm_wide / feedforward with an L2-flushing opbench").

    python tools/l2flush.py --case ff_po_l0 --prev flush|producer|none [--iters 30]

Runs --iters rounds of [prev, case] on one stream, each case an opbench case (tools/opbench.py CASES):
  none      the case back to back (its own previous launch is the only writer before it);
  flush     a 1 GiB read-only sweep (torch sum) before each launch: it evicts L2 and the MALL, so
            every dirty line the previous launch left is written back inside the sweep's window and
            the case's WRITE_SIZE is its own stores only;
  producer  the op that precedes it in the UNet step (PRODUCER below) before each launch, as in the
            step: dirty lines of the producer's output evicted during the case are charged to it.
Run under `rocprofv3 --pmc WRITE_SIZE` (and FETCH_SIZE in its own pass); tools/l2flush.sh does the
passes and tools/l2flush_summary.py reads them.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import opbench  # noqa: E402
import torch  # noqa: E402

# the op before each case in the B = 8 step (profiles/r08_step_trace.txt): to_out 320 before the
# 64x64 feed-forward + proj_out; to_out 1280 before the 16x16 LN-folded GEGLU on gemm_wide
PRODUCER = {"ff_po_l0": "gemm_proj_320", "gemm_ln_geglu_1280": "gemm_proj_1280_l2",
            "gemm_geglu_1280_l2": "gemm_proj_1280_l2",
            # the 32x32 level: proj_in -> LN-folded QKV, GEGLU -> FF2, to_out -> GEGLU
            "gemm_ln_qkv_640": "gemm_proj_640", "gemm_ff2_2560": "gemm_ln_geglu_640",
            "gemm_ln_geglu_640": "gemm_proj_640", "gemm_proj_640": "gemm_ff2_2560"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True)
    ap.add_argument("--prev", choices=["none", "flush", "producer"], required=True)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    run, _, _ = opbench.CASES[a.case]()
    if a.prev == "producer":
        prev, _, _ = opbench.CASES[PRODUCER[a.case]]()
    elif a.prev == "flush":
        big = torch.ones(1 << 28, device="cuda")          # 1 GiB fp32

        def prev():
            return big.sum()
    else:
        def prev():
            return None
    for _ in range(a.iters):
        prev()
        run()
    torch.cuda.synchronize()
    print(f"{a.case} prev={a.prev} iters={a.iters} done", flush=True)


if __name__ == "__main__":
    main()
