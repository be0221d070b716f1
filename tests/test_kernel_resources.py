"""Register budgets of the occupancy-critical kernels, read from the built library's gfx950 code
object (no GPU needed).

The head_dim-40 attention kernel only runs two 8-wave blocks per CU (four waves per SIMD) at
<= 128 VGPRs; one register more silently halves its occupancy (223 -> 251 us per launch at B = 8,
DESIGN tuning log), and a small source change elsewhere in the kernel can cost exactly that.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd", "lib", "libldmseg_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# (mangled-name regex, max VGPRs): the planner's head_dim-40 forms
BUDGETS = [
    (r"attn_d40_kernelILi8ELi2ELi64ELi40ELi1ELb0ELb0E", 128),   # B >= 2: two 8-wave blocks per CU
    (r"attn_d40_kernelILi8ELi2ELi64ELi40ELi1ELb0ELb1E", 128),   # split-KV form (B = 1)
    (r"attn_d40_kernelILi4ELi2ELi64ELi40ELi1ELb0ELb0E", 128),   # few-block fallback
]
# kernels allowed to spill: the generic 16x16x16 attention (tuning / fallback only)
SPILL_OK = re.compile(r"attn_kernelI")


def _kernel_metadata(tmp_path):
    for tool in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            pytest.skip(f"{tool} not available")
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    fb, co = str(tmp_path / "fb.bin"), str(tmp_path / "co.elf")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "x")],
                   check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"],
                   check=True, capture_output=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    rows, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"^    \.name:\s+(\S+)", line)
        if m:
            cur = rows.setdefault(m.group(1), {})
            continue
        m = re.match(r"^    \.(vgpr_count|vgpr_spill_count|private_segment_fixed_size):\s+(\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return rows


def test_attention_register_budgets(tmp_path):
    rows = _kernel_metadata(tmp_path)
    assert len(rows) > 50
    for pat, cap in BUDGETS:
        hits = {k: v for k, v in rows.items() if re.search(pat, k)}
        assert hits, pat
        for name, v in hits.items():
            assert v["vgpr_count"] <= cap, (name, v)


def test_no_spills_on_the_path(tmp_path):
    rows = _kernel_metadata(tmp_path)
    bad = {k: v for k, v in rows.items() if v.get("vgpr_spill_count", 0) and not SPILL_OK.search(k)}
    assert not bad, bad
