"""In-tree native build: hipcc (gfx950) for csrc/**/*.hip, the host compiler for the C++ runtime and
bindings, linked into ``pytorch_distributed_examples_amd/_C*.so`` against the HIP runtime and RCCL that
torch itself loads (torch ships its own libamdhip64.so.7 / librccl.so.1 with the same
sonames as /opt/rocm, so the extension binds to the already-loaded copies).

No hipify step runs: sources are written in HIP directly, and ``torch.utils.cpp_extension`` is not
used to compile them (it would hipify on ROCm).  Objects are rebuilt only when their source or a header
changed.  ``python -m pytorch_distributed_examples_amd._build`` builds from the command line.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PDE_OFFLOAD_ARCH", "gfx950")

EXTENSIONS = {
    # module name -> (hip sources, host C++ sources)
    "_C": (
        ["kernels/gemm.hip", "kernels/gemm_dma_tt.hip", "kernels/gemm_dma_tf.hip", "kernels/gemm_dma_ft.hip",
         "kernels/gemm_dma_ff.hip", "kernels/gemm_dma_pair.hip", "kernels/elementwise.hip", "kernels/loss.hip", "kernels/optim.hip",
         "kernels/norm_pool.hip", "kernels/cnn_fused.hip", "kernels/mlp_fused.hip"],
        ["bindings.cpp"],
    ),
    "_comm": (
        ["comm/pack.hip", "comm/xgmi_allreduce.hip", "comm/p2p_ring.hip"],
        ["comm/comm_manager.cpp", "comm/fusion_engine.cpp", "comm/comm_bindings.cpp"],
    ),
}


# Per-source device flags.  cnn_fused.hip gathers 8 consecutive bf16 values from 2-byte-aligned LDS
# addresses: with gfx950's unaligned-access mode the compiler merges them into one 16-byte ds_read that the
# LDS replays as an unaligned access (64 cycles; measured SQ_LDS_UNALIGNED_STALL), so that mode is off there.
# (The host compiler ignores the device target feature with a warning.)
HIP_FLAGS = {
    "kernels/cnn_fused.hip": ["-Xclang", "-target-feature", "-Xclang", "-unaligned-access-mode"],
}
# GEMM ring depth / K-tiles per barrier / DMA ring slots / default core sweeps (gemm_common.h / gemm_ring.h / gemm_dma.h)
_GEMM_SRCS = ("kernels/gemm.hip", "kernels/gemm_dma_tt.hip", "kernels/gemm_dma_tf.hip", "kernels/gemm_dma_ft.hip",
              "kernels/gemm_dma_ff.hip", "kernels/gemm_dma_pair.hip")
for _knob in ("PDE_FAST_STAGES", "PDE_GEMM_SUB", "PDE_GEMM_WPE", "PDE_DMA_STAGES", "PDE_GEMM_CORE_DEFAULT"):
    if os.environ.get(_knob):
        for _src in _GEMM_SRCS:
            HIP_FLAGS.setdefault(_src, []).append(f"-D{_knob}={int(os.environ[_knob])}")


def _torch_paths():
    import torch  # noqa: WPS433

    tdir = Path(torch.__file__).resolve().parent
    return tdir, tdir / "include", tdir / "lib", bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _headers() -> list[Path]:
    return sorted(CSRC.rglob("*.h")) + sorted(CSRC.rglob("*.cuh"))


_INC_DIRS = [CSRC / "include", CSRC / "kernels", CSRC / "comm"]


def _deps(src: Path, seen: set | None = None) -> set:
    """In-tree headers ``src`` includes (``#include "..."``, recursively) -- an object is rebuilt only
    when one of ITS headers changed, not any header of the tree."""
    seen = set() if seen is None else seen
    try:
        text = src.read_text(errors="ignore")
    except OSError:
        return seen
    for line in text.splitlines():
        line = line.strip()
        if not line.startswith("#include \""):
            continue
        name = line.split('"')[1]
        for d in [src.parent, *_INC_DIRS]:
            h = (d / name).resolve()
            if h.exists():
                if h not in seen:
                    seen.add(h)
                    _deps(h, seen)
                break
    return seen


def _stale(obj: Path, src: Path, headers: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    return any(h.stat().st_mtime > t for h in _deps(src))


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("native build failed:\n  " + " ".join(cmd) + "\n" + res.stdout + res.stderr)


def build(verbose: bool = False, jobs: int | None = None) -> list[Path]:
    """Compile every extension; returns the paths of the built shared objects."""
    tdir, tinc, tlib, cxx11 = _torch_paths()
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    cxx = os.environ.get("CXX", "g++")
    py_inc = sysconfig.get_paths()["include"]
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = _headers()
    abi = f"-D_GLIBCXX_USE_CXX11_ABI={1 if cxx11 else 0}"
    common_inc = [f"-I{CSRC / 'include'}", f"-I{CSRC / 'kernels'}", f"-I{CSRC / 'comm'}"]
    torch_inc = [f"-I{tinc}", f"-I{tinc / 'torch/csrc/api/include'}", f"-I{py_inc}", f"-I{ROCM / 'include'}"]

    jobs = jobs or min(8, os.cpu_count() or 4)
    outputs = []
    for name, (hip_srcs, cpp_srcs) in EXTENSIONS.items():
        objs: list[Path] = []
        tasks = []
        for rel in hip_srcs:
            src = CSRC / rel
            obj = BUILD / (rel.replace("/", "_") + ".o")
            objs.append(obj)
            if _stale(obj, src, headers):
                tasks.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", abi,
                              "-munsafe-fp-atomics", *HIP_FLAGS.get(rel, []), *common_inc,
                              *([f"-I{ROCM / 'include'}"]), "-c", str(src), "-o", str(obj)])
        for rel in cpp_srcs:
            src = CSRC / rel
            obj = BUILD / (rel.replace("/", "_") + ".o")
            objs.append(obj)
            if _stale(obj, src, headers):
                tasks.append([cxx, "-O2", "-std=c++17", "-fPIC", abi, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                              f"-DTORCH_EXTENSION_NAME={name}", "-DTORCH_API_INCLUDE_EXTENSION_H",
                              "-Wno-deprecated-declarations", *common_inc, *torch_inc, "-c", str(src), "-o", str(obj)])
        if tasks:
            with cf.ThreadPoolExecutor(jobs) as ex:
                for cmd in tasks:
                    if verbose:
                        print(" ".join(cmd), flush=True)
                list(ex.map(_run, tasks))
        so = PKG_DIR / f"{name}{_ext_suffix()}"
        if not so.exists() or any(o.stat().st_mtime > so.stat().st_mtime for o in objs):
            link = [cxx, "-shared", "-o", str(so), *map(str, objs), f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch",
                    "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lrccl",
                    f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"]
            if verbose:
                print(" ".join(link), flush=True)
            _run(link)
        outputs.append(so)
    return outputs


if __name__ == "__main__":
    for p in build(verbose="-v" in sys.argv):
        print(p)
