"""Build the native extensions in-tree.

* ``_k8sllm_ops``      - gfx950 HIP kernels (hipcc, one object per ``csrc/*.hip``, no torch
                          headers) + a thin PyTorch binding (``csrc/bindings.cpp``, g++).
* ``_k8sllm_runtime``  - the C++ serving runtime (paged-KV block manager, continuous-batching
                          scheduler, byte-level BPE tokenizer), pybind11, no torch / HIP.

Both land next to their Python packages so the GPU box sees them in the repo snapshot.
Objects are rebuilt only when a source (or a header) is newer than the shared library.
Run:  python -m k8s_llm_monitor_amd.ops.build   [--force] [--only ops|runtime]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent
OPS_DIR = PKG / "ops"
OPS_SRC = OPS_DIR / "csrc"
RT_DIR = PKG / "runtime"
RT_SRC = RT_DIR / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

OPS_SO = OPS_DIR / ("_k8sllm_ops" + sysconfig.get_config_var("EXT_SUFFIX"))
RT_SO = RT_DIR / ("_k8sllm_runtime" + sysconfig.get_config_var("EXT_SUFFIX"))


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"native build failed: {cmd[0]} {cmd[-1]}")


def _stale(target: Path, sources: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources)


def _torch_flags() -> tuple[list[str], list[str]]:
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths()]
    libdir = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = inc + [
        f"-I{sysconfig.get_paths()['include']}",
        f"-I{ROCM / 'include'}",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_k8sllm_ops",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
    ]
    # link against torch's own HIP runtime (same SONAME as /opt/rocm's) so one runtime is loaded
    ldflags = [
        f"-L{libdir}",
        f"-Wl,-rpath,{libdir}",
        "-lc10",
        "-lc10_hip",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_hip",
        "-ltorch_python",
        "-lamdhip64",
    ]
    return cflags, ldflags


def build_ops(force: bool = False, jobs: int = 8) -> Path:
    hips = sorted(OPS_SRC.glob("*.hip"))
    cpps = sorted(OPS_SRC.glob("*.cpp"))
    hdrs = sorted(OPS_SRC.glob("*.h"))
    if not force and not _stale(OPS_SO, hips + cpps + hdrs + [Path(__file__)]):
        return OPS_SO
    if shutil.which("hipcc") is None and not (ROCM / "bin" / "hipcc").exists():
        raise RuntimeError("hipcc not found: cannot build the gfx950 kernels")
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    out = BUILD / "ops"
    out.mkdir(parents=True, exist_ok=True)
    cflags, ldflags = _torch_flags()

    def hip_obj(src: Path) -> Path:
        obj = out / (src.stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
                  "-munsafe-fp-atomics", "-c", str(src), "-o", str(obj)])
        return obj

    def cpp_obj(src: Path) -> Path:
        obj = out / (src.stem + ".o")
        if force or _stale(obj, [src]):
            _run(["g++", "-O2", "-std=c++17", "-fPIC", *cflags, "-c", str(src), "-o", str(obj)])
        return obj

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(hip_obj, hips)) + list(ex.map(cpp_obj, cpps))
    tmp = OPS_SO.with_suffix(".tmp.so")
    _run(["g++", "-shared", "-o", str(tmp), *map(str, objs), *ldflags])
    os.replace(tmp, OPS_SO)
    return OPS_SO


def build_runtime(force: bool = False) -> Path:
    srcs = sorted(RT_SRC.glob("*.cpp"))
    hdrs = sorted(RT_SRC.glob("*.h"))
    if not srcs:
        raise RuntimeError("runtime sources missing")
    if not force and not _stale(RT_SO, srcs + hdrs + [Path(__file__)]):
        return RT_SO
    import pybind11

    out = BUILD / "runtime"
    out.mkdir(parents=True, exist_ok=True)
    tmp = RT_SO.with_suffix(".tmp.so")
    _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
          f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
          f"-I{RT_SRC}", *map(str, srcs), "-o", str(tmp), "-lrt"])
    os.replace(tmp, RT_SO)
    return RT_SO


def build_all(force: bool = False) -> list[Path]:
    return [build_runtime(force), build_ops(force)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["ops", "runtime"], default=None)
    a = ap.parse_args()
    if a.only in (None, "runtime"):
        print(build_runtime(a.force))
    if a.only in (None, "ops"):
        print(build_ops(a.force))


if __name__ == "__main__":
    main()
