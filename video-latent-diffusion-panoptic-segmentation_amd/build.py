"""Build the gfx950 HIP library (lib/libldmseg_hip.so) in-tree.

    python video-latent-diffusion-panoptic-segmentation_amd/build.py [--force] [--jobs N]

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU container and the
resulting .so travels to the GPU box with the repo snapshot.  Objects are rebuilt only
when their source (or a shared header) is newer.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libldmseg_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-I" + os.path.join(ROOT, "include")]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, obj):
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force=False, jobs=None, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = _headers()
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, [s, *hdrs]):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 1, max(1, len(todo)))
    if todo:
        if verbose:
            print(f"[build] compiling {len(todo)} HIP sources for {ARCH} ({jobs} jobs)", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda so: _compile(*so), todo))
    if force or todo or _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(LIB + ".tmp", LIB)
        if verbose:
            print(f"[build] linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args()
    try:
        build(a.force, a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
