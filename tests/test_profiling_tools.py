"""CPU tests of the profiling tools whose output DESIGN.md and bench.py cite: the kernel -> (family,
role) table (tools/kernel_families.py), the per-op traffic table's strict op <-> dispatch alignment
(tools/traffic_table.py) and the step splitter (tools/step_trace.py).

The traffic table is fed synthetic rocprofv3 counter files and op logs of the shapes
tools/profile_bench.sh produces: an aligned step gives one row per op with the split-K reduction
charged to its conv and the GroupNorm statistics kernel to the GroupNorm after it; a kernel the
family table does not know, or one op too many, must stop the tool instead of shifting the kernel
column against the ops ("the per-op traffic evidence is broken").
"""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")
sys.path.insert(0, TOOLS)

from kernel_families import kind_of  # noqa: E402


@pytest.mark.parametrize("name,fam,role", [
    ("void (anonymous namespace)::conv_in_kernel<5>(...)", "igemm", "p"),
    ("void (anonymous namespace)::igemm_kernel<unsigned short, 128, 160, true, 2, false>(...)", "igemm", "p"),
    ("void (anonymous namespace)::conv3_halo_kernel<64, 4, false>(...)", "igemm", "p"),
    ("void (anonymous namespace)::gemm_ring_kernel<128, 80, 4, 1, 5, 3, false>(...)", "igemm", "p"),
    ("(anonymous namespace)::unet_tail_kernel((anonymous namespace)::TailArgs)", "igemm", "p"),
    ("void (anonymous namespace)::splitk_gn_kernel<64, 4>(...)", "igemm", "post"),
    ("void (anonymous namespace)::splitk_epilogue_kernel<unsigned short, 64, 64>(...)", "igemm", "post"),
    ("void (anonymous namespace)::attn_d40_kernel<8, 1, 64, 40, 2, false, false, false, true>(...)", "attention", "p"),
    ("(anonymous namespace)::attn_kv_combine(...)", "attention", "post"),
    ("(anonymous namespace)::attn_f8_prep(...)", "attention", "pre"),
    ("void (anonymous namespace)::gn_apply<unsigned short, 1>(...)", "group_norm", "p"),
    ("void (anonymous namespace)::gn_stats<unsigned short>(...)", "group_norm", "pre"),
    ("(anonymous namespace)::linear_rows_kernel(...)", "linear_rows", "p"),
    ("void (anonymous namespace)::nchw_to_nhwc_kernel(...)", None, None),
    ("__amd_rocclr_copyBuffer", None, None),
])
def test_kernel_families(name, fam, role):
    assert kind_of(name) == (fam, role)


def test_every_profiled_kernel_is_classified():
    """Every kernel of the committed final-tree profile that is not layout glue or a torch / copy
    kernel has a family (a new kernel missing from the table would be silently dropped)."""
    path = os.path.join(ROOT, "profiles", "r08z_kernel_stats.csv")
    names = [r["Name"] for r in csv.DictReader(open(path))]
    glue = ("nchw_to_nhwc", "at::native", "__amd_rocclr", "elementwise", "copy", "fill", "reduce_kernel",
            "rocblas", "Cijk_")                        # (torch / library kernels of the bench's setup)
    missing = [n for n in names if kind_of(n)[0] is None and not any(g in n for g in glue)]
    assert not missing, missing


def _write_pmc(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for did, (name, val) in enumerate(rows):
            w.writerow(dict(Dispatch_Id=did, Kernel_Name=name, Grid_Size=256, Counter_Name=counter, Counter_Value=val))


def _run_table(tmp_path, kernels, ops):
    _write_pmc(str(tmp_path / "fetch"), "FETCH_SIZE", [(k, 1000.0) for k in kernels])
    _write_pmc(str(tmp_path / "write"), "WRITE_SIZE", [(k, 500.0) for k in kernels])
    json.dump({"ops": ops}, open(tmp_path / "oplog.json", "w"))
    return subprocess.run([sys.executable, os.path.join(TOOLS, "traffic_table.py"), "--fetch", str(tmp_path / "fetch"),
                           "--write", str(tmp_path / "write"), "--oplog", str(tmp_path / "oplog.json"),
                           "--json", str(tmp_path / "t.json")], capture_output=True, text=True)


def _op(fam, detail, nbytes=1_000_000):
    return dict(family=fam, bytes=nbytes, detail=detail)


STEP = [  # an earlier eager step, then the profiled one
    "void (anonymous namespace)::conv_in_kernel<5>(...)",
    "void (anonymous namespace)::gn_apply<unsigned short, 1>(...)",
    "void (anonymous namespace)::conv_in_kernel<5>(...)",
    "void (anonymous namespace)::nchw_to_nhwc_kernel(...)",
    "void (anonymous namespace)::igemm_kernel<unsigned short, 64, 160, true, 2, true>(...)",
    "void (anonymous namespace)::splitk_epilogue_kernel<unsigned short, 64, 64>(...)",
    "void (anonymous namespace)::gn_stats<unsigned short>(...)",
    "void (anonymous namespace)::gn_apply<unsigned short, 1>(...)",
    "void (anonymous namespace)::attn_d40_kernel<8, 1, 64, 40, 2, false, false, false, true>(...)",
    "(anonymous namespace)::unet_tail_kernel((anonymous namespace)::TailArgs)",
]
OPS = [_op("igemm", "conv_in"), _op("igemm", "k3 split"), _op("group_norm", "gn"), _op("attention", "attn"),
       _op("igemm", "tail")]


def test_traffic_table_aligned(tmp_path):
    r = _run_table(tmp_path, STEP, OPS)
    assert r.returncode == 0, r.stderr
    rows = json.load(open(tmp_path / "t.json"))["ops"]
    assert [x["detail"] for x in rows] == ["conv_in", "k3 split", "gn", "attn", "tail"]
    kern = {x["detail"]: x["kernels"] for x in rows}
    assert "splitk_epilogue_kernel" in kern["k3 split"] and "igemm_kernel" in kern["k3 split"]
    assert "gn_stats" in kern["gn"] and "gn_apply" in kern["gn"]
    # 2 x FETCH + WRITE per dispatch, KB -> bytes: the split conv has two dispatches
    split = next(x for x in rows if x["detail"] == "k3 split")
    assert split["hbm_mb"] == pytest.approx(2 * (2 * 1000 + 500) * 1024 / 1e6)


def test_traffic_table_refuses_unknown_kernel(tmp_path):
    bad = list(STEP)
    bad[8] = "void (anonymous namespace)::brand_new_gemm_kernel<1>(...)"   # attention op has no dispatch now
    r = _run_table(tmp_path, bad, OPS)
    assert r.returncode != 0 and "traffic_table" in (r.stderr + r.stdout)


def test_traffic_table_refuses_extra_op(tmp_path):
    r = _run_table(tmp_path, STEP, [_op("igemm", "phantom")] + OPS[:1] + OPS)
    assert r.returncode != 0


def test_step_trace_splits_at_either_entry_kernel(tmp_path):
    """tools/step_trace.py cuts steps at ldm_conv_in (B = 8) or at the NCHW gather (B = 1)."""
    for entry in ("conv_in_kernel<5>", "nchw_to_nhwc_kernel"):
        path = tmp_path / f"trace_{entry[:4]}.csv"
        with open(path, "w", newline="") as f:
            cols = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z",
                    "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z", "LDS_Block_Size", "VGPR_Count",
                    "Accum_VGPR_Count", "Dispatch_Id"]
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            t, did = 0, 0
            for _ in range(6):
                for k in (entry, "gn_apply<bf16, 1>", "igemm_kernel<bf16, 64, 160>"):
                    w.writerow(dict(Kernel_Name=k, Start_Timestamp=t, End_Timestamp=t + 1000, Grid_Size_X=256 * 64,
                                    Grid_Size_Y=1, Grid_Size_Z=1, Workgroup_Size_X=64, Workgroup_Size_Y=1,
                                    Workgroup_Size_Z=1, LDS_Block_Size=0, VGPR_Count=64, Accum_VGPR_Count=0,
                                    Dispatch_Id=did))
                    t += 1100
                    did += 1
        r = subprocess.run([sys.executable, os.path.join(TOOLS, "step_trace.py"), str(path)], capture_output=True,
                           text=True)
        assert r.returncode == 0, r.stderr
        assert "sequences of 3 launches" in r.stdout, r.stdout[:400]
