"""Build the gfx950 HIP kernels into one C-ABI shared library, in-tree.

    python -m onetrainer_amd.build            # incremental
    python -m onetrainer_amd.build --force

Output: onetrainer_amd/_lib/libotamd.so (git-ignored; travels to the GPU box with the
snapshot).  Every exported symbol is declared in include/otamd.h.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG.parent / "build" / "obj"
LIB_DIR = PKG / "_lib"
LIB = LIB_DIR / "libotamd.so"
ARCH = "gfx950"

# per-source extra flags: the optimizer restates torch's CPU rounding sequence exactly,
# so no fp contraction beyond the explicit fmaf calls
EXTRA = {
    "adamw.hip": ["-ffp-contract=off"],
    "diffusion.hip": ["-ffp-contract=off"],
    # no NaN canonicalisation (v_max_f32 x, x) in front of every fmaxf on an MFMA result: one extra
    # VALU per softmax score; the kernels never produce or test NaNs (masked keys are -inf)
    "attention.hip": ["-fno-honor-nans"],
}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the onetrainer_amd kernels need ROCm's hipcc (gfx950)")


def _compile(src: Path, force: bool) -> Path:
    obj = OBJ / (src.stem + ".o")
    deps = [src] + sorted(CSRC.glob("*.h"))
    if not force and obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return obj
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
           "-I", str(CSRC), "-c", str(src), "-o", str(obj)] + EXTRA.get(src.name, [])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    print(build(a.force, a.j))
    sys.exit(0)
