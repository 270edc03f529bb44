"""In-tree native build: HIP kernels (gfx950) + host runtime, no torch headers, no JIT cache.

Two extension modules land in ``llm_consensus_amd/_lib`` (git-ignored, but shipped to the GPU
box by the gpurun snapshot):

* ``_llmc_rt``  — host C++ runtime (tokenizer, paged-KV allocator, Go JSON), g++ + pybind11.
* ``_llmc_hip`` — every HIP kernel in ``csrc/kernels/*.hip`` compiled with
  ``hipcc --offload-arch=gfx950`` plus a pybind11 launcher table. Launchers take raw device
  pointers and a ``hipStream_t`` (torch's current stream), so they are capturable by
  ``torch.cuda.graph`` and carry no torch ABI dependency.

Incremental: an object is rebuilt only when its source or any header in its directory is
newer.  ``python -m llm_consensus_amd._build [--force]`` builds both.
"""

from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "llm_consensus_amd")
LIB = os.path.join(PKG, "_lib")
BUILD = os.path.join(ROOT, "build")
CSRC = os.path.join(ROOT, "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("LLMC_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> List[str]:
    import pybind11

    return ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]


def _newer(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)


def _jobs() -> int:
    return max(1, min(16, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))


def runtime_path() -> str:
    return os.path.join(LIB, "_llmc_rt" + _ext_suffix())


def kernels_path() -> str:
    return os.path.join(LIB, "_llmc_hip" + _ext_suffix())


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    src_dir = os.path.join(CSRC, "runtime")
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(src_dir, "*.h")))
    out = runtime_path()
    if not force and not _newer(out, srcs + hdrs + [__file__]):
        return out
    os.makedirs(LIB, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", *_py_includes(),
           *srcs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    os.replace(out + ".tmp", out)
    return out


def _hip_flags() -> List[str]:
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-ffp-contract=fast", "-Wno-unused-result"]


def build_kernels(force: bool = False, verbose: bool = False) -> str:
    kdir = os.path.join(CSRC, "kernels")
    hips = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(kdir, "*.h")))
    bind = os.path.join(kdir, "bindings.cpp")
    out = kernels_path()
    objdir = os.path.join(BUILD, "kernels")
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")

    jobs = []
    objs = []
    for src in hips:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + hdrs + [__file__]):
            jobs.append([hipcc, *_hip_flags(), "-c", src, "-o", obj])
    bobj = os.path.join(objdir, "bindings.o")
    objs.append(bobj)
    if force or _newer(bobj, [bind] + hdrs + [__file__]):
        jobs.append([hipcc, "-O2", "-std=c++17", "-fPIC", "-x", "c++", "-D__HIP_PLATFORM_AMD__",
                     "-I" + os.path.join(ROCM, "include"), *_py_includes(), "-c", bind, "-o", bobj])
    if jobs:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            for cmd in jobs:
                if verbose:
                    print(" ".join(cmd), flush=True)
            list(ex.map(_run, jobs))
    if force or jobs or _newer(out, objs):
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        os.replace(out + ".tmp", out)
    return out


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_runtime(force, verbose)
    build_kernels(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
    print("built:", runtime_path(), kernels_path())
