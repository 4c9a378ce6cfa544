"""Builds the in-tree native extension ``mipipe/_C.so`` for gfx950.

    python -m mipipe.build            # incremental
    python -m mipipe.build --clean    # from scratch

Every source is compiled directly with ``hipcc --offload-arch=gfx950`` (no
hipify, no CUDA path): the HIP kernels (``csrc/kernels/*.hip``) see only HIP
headers, the runtime (``csrc/runtime``) only HIP + roctx, and a single
bindings TU includes torch.  The objects are linked against the libtorch that
``import torch`` loads, so the extension shares torch's HIP runtime, caching
allocator and generators.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
import time
from typing import List, Optional, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(os.path.dirname(HERE), "build", "mipipe")
OUT = os.path.join(HERE, "_C.so")
ARCH = os.environ.get("MIPIPE_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found")
    return p


def _torch_paths() -> Tuple[List[str], str]:
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(root, "lib")


def _newest(paths: List[str]) -> float:
    return max((os.path.getmtime(p) for p in paths if os.path.exists(p)), default=0.0)


def _sources() -> List[Tuple[str, str]]:
    out = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        out.append((src, "kernel"))
    for src in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))):
        out.append((src, "runtime"))
    out.append((os.path.join(CSRC, "bindings.cpp"), "bindings"))
    return out


def _flags(kind: str) -> List[str]:
    common = ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1"]
    if kind == "kernel":
        # Fully unrolled epilogues keep MFMA accumulators in registers (an
        # unroll refused for size spills them to scratch).
        return common + ["-O3", "-ffp-contract=fast", "-munsafe-fp-atomics", "-mllvm", "-pragma-unroll-threshold=1000000"]
    if kind == "runtime":
        return common + ["-O2", f"-I{ROCM}/include"]
    tinc, _ = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return common + [
        "-O2",
        "-DUSE_ROCM=1",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"-I{py_inc}",
        f"-I{CSRC}",
        "-Wno-deprecated-declarations",
        "-Wno-unused-result",
    ] + [f"-I{p}" for p in tinc]


def _compile(src: str, kind: str, verbose: bool) -> Optional[str]:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    obj = os.path.join(BUILD, rel + ".o")
    deps = [src] + glob.glob(os.path.join(CSRC, "kernels", "*.h")) + glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest(deps):
        return obj
    cmd = [_hipcc()] + _flags(kind) + ["-c", src, "-o", obj]
    if src.endswith(".cpp") and kind != "bindings":
        cmd.insert(1, "-xhip")
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {src}")
    if verbose:
        print(f"  [{time.time() - t0:5.1f}s] {os.path.relpath(src, HERE)}", flush=True)
    return obj


def build(clean: bool = False, verbose: bool = True, jobs: Optional[int] = None) -> str:
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(BUILD, exist_ok=True)
    sources = _sources()
    jobs = jobs or min(len(sources), int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 4, 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s[0], s[1], verbose), sources))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= _newest(objs):
        return OUT
    _, tlib = _torch_paths()
    cmd = (
        [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT + ".tmp"]
        + objs
        + [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
        + [f"-L{ROCM}/lib", "-lrocprofiler-sdk-roctx"]
        + [f"-Wl,-rpath,{tlib}", f"-Wl,-rpath,{ROCM}/lib"]
    )
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError("link failed")
    os.replace(OUT + ".tmp", OUT)
    if verbose:
        print(f"built {OUT}", flush=True)
    return OUT


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-q", "--quiet", action="store_true")
    args = ap.parse_args()
    build(clean=args.clean, verbose=not args.quiet, jobs=args.jobs)


if __name__ == "__main__":
    main()
