"""In-tree build of determined_amd's native code.

Two shared objects are produced next to the sources (so they travel with the repo
snapshot to a GPU box; nothing is installed into site-packages):

* ``determined_amd/ops/_hip_ops*.so`` -- the CDNA4 kernels (``csrc/*.hip``, compiled
  with ``hipcc --offload-arch=gfx950``) plus the torch bindings (``csrc/bindings.cpp``).
  Device translation units include only ``hip_runtime.h`` so they compile in seconds;
  the single host TU carries the torch headers.
* ``determined_amd/_native/_native*.so`` -- the C++ control plane (search methods,
  scheduler) bound with pybind11; no torch or HIP dependency.

Object files are cached under ``build/`` and rebuilt only when a source or header is
newer (a tiny make).  Usage: ``python -m determined_amd._build [--force] [-j N]``.
"""

import argparse
import concurrent.futures
import os
import pathlib
import shlex
import subprocess
import sys
import sysconfig
from typing import List, Optional, Sequence

PKG = pathlib.Path(__file__).resolve().parent
ROOT = PKG.parent
BUILD = ROOT / "build" / "native"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = os.environ.get("DAMD_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["optim.hip", "norm.hip", "bn.hip", "attention.hip", "fused.hip", "conv_stem.hip", "conv_igemm.hip", "conv3x3v2.hip"]
# MFMA kernels whose accumulators are also touched by VALU code (online softmax, rescales):
# keep them in the unified VGPR file instead of AGPRs, which otherwise costs a
# v_accvgpr_read/write pair per element per tile (attention: 450 copies per kv tile) and
# lowers occupancy.
HIP_EXTRA_FLAGS = {
    "attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
    "conv_stem.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}
HOST_SOURCES = ["bindings.cpp"]
NATIVE_SOURCES = ["searcher.cpp", "scheduler.cpp", "loader.cpp", "module.cpp"]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def hip_ops_path() -> pathlib.Path:
    return PKG / "ops" / f"_hip_ops{_ext_suffix()}"


def native_path() -> pathlib.Path:
    return PKG / "_native" / f"_native{_ext_suffix()}"


def _torch_paths():
    import torch  # noqa: F401  (only needed for paths)
    import torch.utils.cpp_extension as ce

    tdir = pathlib.Path(torch.__file__).resolve().parent
    incs = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return incs, tdir / "lib", int(torch._C._GLIBCXX_USE_CXX11_ABI), ce


def _newer(target: pathlib.Path, deps: Sequence[pathlib.Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.exists() and d.stat().st_mtime > t for d in deps)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build command failed:\n{shlex.join(cmd)}\n{r.stdout}")


def build_hip_ops(force: bool = False, jobs: int = 8) -> pathlib.Path:
    csrc = PKG / "csrc"
    headers = list(csrc.glob("*.h"))
    incs, tlib, abi, _ = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    BUILD.mkdir(parents=True, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1"]
    jobs_list = []
    objs = []
    for src in HIP_SOURCES:
        s = csrc / src
        if not s.exists():
            continue
        o = BUILD / (src + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            jobs_list.append([HIPCC, *common, "-munsafe-fp-atomics", *HIP_EXTRA_FLAGS.get(src, []), "-c", str(s),
                              "-o", str(o)])
    for src in HOST_SOURCES:
        s = csrc / src
        o = BUILD / (src + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            flags = [
                "-DUSE_ROCM=1",
                "-DTORCH_EXTENSION_NAME=_hip_ops",
                "-DTORCH_API_INCLUDE_EXTENSION_H",
                f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                *[f"-I{p}" for p in incs],
                f"-I{py_inc}",
                "-I/opt/rocm/include",
                "-Wno-unused-result",
            ]
            jobs_list.append([HIPCC, "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", *flags,
                              "-c", str(s), "-o", str(o)])
    with concurrent.futures.ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    out = hip_ops_path()
    if force or jobs_list or _newer(out, objs):
        libs = ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
        # Link against torch's bundled HIP runtime so only one runtime is ever loaded.
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out), f"-L{tlib}", *libs,
              f"-Wl,-rpath,{tlib}"])
    return out


SANITIZERS = {"address": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"],
              "thread": ["-fsanitize=thread"]}


def sanitizer_runtime(kind: str) -> str:
    """The gcc runtime to LD_PRELOAD into the (uninstrumented) python that loads a sanitizer build."""
    lib = {"address": "libasan.so", "thread": "libtsan.so"}[kind]

    def where(name: str) -> str:
        return subprocess.run([CXX, f"-print-file-name={name}"], stdout=subprocess.PIPE, text=True,
                              check=True).stdout.strip()

    # libstdc++ preloaded too: python itself does not link it, and the runtime's __cxa_throw interceptor
    # must find the real symbol at start-up (C++ exceptions thrown by the module otherwise abort)
    return f"{where(lib)}:{where('libstdc++.so.6')}"


def build_native(force: bool = False, jobs: int = 8, sanitize: Optional[str] = None) -> pathlib.Path:
    """The C++ control plane.  ``sanitize`` ("address" = ASan+UBSan, "thread" = TSan) builds an
    instrumented copy under build/sanitize-<kind>/ instead of the in-tree module (load it with
    DAMD_NATIVE_PATH=<path> and LD_PRELOAD=<sanitizer_runtime(kind)>; tests/test_native_sanitizers.py)."""
    import pybind11

    src_dir = PKG / "_native"
    srcs = [src_dir / s for s in NATIVE_SOURCES if (src_dir / s).exists()]
    headers = list(src_dir.glob("*.h"))
    bdir = BUILD if sanitize is None else ROOT / "build" / f"sanitize-{sanitize}"
    bdir.mkdir(parents=True, exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    opt = ["-O3"] if sanitize is None else ["-O1", "-g", *SANITIZERS[sanitize]]
    objs, jobs_list = [], []
    for s in srcs:
        o = bdir / ("native_" + s.name + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            jobs_list.append([CXX, *opt, "-fPIC", "-std=c++17", "-Wall", "-pthread", f"-I{pybind11.get_include()}",
                              f"-I{py_inc}", f"-I{src_dir}", "-c", str(s), "-o", str(o)])
    with concurrent.futures.ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    out = native_path() if sanitize is None else bdir / native_path().name
    if objs and (force or jobs_list or _newer(out, objs)):
        _run([CXX, "-shared", "-pthread", *([] if sanitize is None else SANITIZERS[sanitize]), *map(str, objs),
              "-o", str(out)])
    return out


def build_all(force: bool = False, jobs: int = 8) -> None:
    build_native(force=force, jobs=jobs)
    build_hip_ops(force=force, jobs=jobs)


def main(argv: Sequence[str] = ()) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--force", action="store_true")
    p.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    p.add_argument("--only", choices=["hip", "native"], default=None)
    p.add_argument("--sanitize", choices=sorted(SANITIZERS), default=None,
                   help="build an instrumented copy of the native control plane only")
    a = p.parse_args(list(argv))
    if a.sanitize:
        print("built", build_native(a.force, a.jobs, sanitize=a.sanitize))
        return 0
    if a.only in (None, "native"):
        print("built", build_native(a.force, a.jobs))
    if a.only in (None, "hip"):
        print("built", build_hip_ops(a.force, a.jobs))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
