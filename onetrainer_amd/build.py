"""Build the gfx950 HIP kernels into one C-ABI shared library, in-tree.

    python -m onetrainer_amd.build            # incremental
    python -m onetrainer_amd.build --force

Output: onetrainer_amd/_lib/libotamd.so and the native host layer _lib/_otamd_host.so (git-ignored;
travel to the GPU box with the snapshot).  Every exported symbol of libotamd.so is declared in
include/otamd.h.
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
    # no SLP packing of the softmax's f32 math into v_pk_*_f32, which costs more than two single-issue ops
    # beside MFMAs (MI355X_MICROARCH.md, per-instruction cycle constants)
    "attention.hip": ["-fno-honor-nans", "-fno-slp-vectorize"],
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


HOST_SRC = CSRC / "host" / "ops_host.cpp"
HOST_LIB = LIB_DIR / "_otamd_host.so"
INCLUDE = PKG.parent / "include"


def build_host(force: bool = False) -> Path:
    """The native host layer (csrc/host/ops_host.cpp -> _lib/_otamd_host.so): a CPython extension over torch's
    C++ tensor API that calls libotamd.so's C ABI (rpath $ORIGIN).  Host code only: plain g++."""
    import sysconfig

    import torch
    import torch.utils.cpp_extension as ce
    deps = [HOST_SRC, INCLUDE / "otamd.h", LIB]
    if not force and HOST_LIB.exists() and HOST_LIB.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return HOST_LIB
    cxx = shutil.which("g++") or "c++"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", str(HOST_SRC),
           "-o", str(HOST_LIB.with_suffix(".so.tmp")), f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-DTORCH_EXTENSION_NAME=_otamd_host", "-DTORCH_API_INCLUDE_EXTENSION_H",
           "-I", str(INCLUDE), "-I", "/opt/rocm/include", "-I", sysconfig.get_paths()["include"]]
    for d in ce.include_paths():
        cmd += ["-isystem", d]
    for d in ce.library_paths():
        cmd += ["-L", d, f"-Wl,-rpath,{d}"]
    cmd += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-L", str(LIB_DIR), "-lotamd", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host layer build failed:\n{r.stderr[-6000:]}")
    os.replace(HOST_LIB.with_suffix(".so.tmp"), HOST_LIB)
    return HOST_LIB


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
    build_host(force)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    print(build(a.force, a.j))
    sys.exit(0)
