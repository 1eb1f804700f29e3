"""Native build driver for the framework's HIP/C++ extension (``_C``).

The extension is built *in-tree* (``pytorch_distributed_rnn_amd/_C*.so``) so it
travels with the repository snapshot to the GPU box.  Two toolchains are used on
purpose:

* ``hipcc --offload-arch=gfx950`` compiles the device code in
  ``csrc/kernels/*.hip``.  These translation units do not include any torch
  header; they export plain ``extern "C"`` launchers that take raw pointers and
  a ``hipStream_t``.  Keeping torch out of them makes kernel rebuilds take
  seconds.
* ``g++`` compiles the host runtime (``csrc/runtime/*.cpp``: RCCL communicator,
  bucketed gradient reducer, fusion buffer, ...) and the pybind11/torch bindings
  with the same compiler torch itself was built with, so torch's pybind11 types
  (``c10d::ProcessGroup`` and friends) interoperate.

The link step uses ``hipcc`` so the fat binaries register with the HIP runtime.
At import time torch has already loaded ``libamdhip64.so.7`` and ``librccl.so.1``
from ``torch/lib``; our ``NEEDED`` entries resolve to those same objects (same
SONAME), so there is exactly one HIP runtime and one RCCL in the process.

Usage::

    python -m pytorch_distributed_rnn_amd._build          # incremental
    PDRNN_DEBUG_BUILD=1 python -m pytorch_distributed_rnn_amd._build   # -O1 -g + device asserts
    python -m pytorch_distributed_rnn_amd._build --clean  # full rebuild
    PDRNN_SANITIZE=address,undefined python -m pytorch_distributed_rnn_amd._build
        # host runtime (comm.cpp, reducer.cpp, bindings) under ASan + UBSan (or
        # PDRNN_SANITIZE=thread: TSan) into build_native_san_<flavour>/; load it
        # with PDRNN_EXT_SO=<that .so> and the sanitizer runtime preloaded
        # (tools/sanitize_host.sh).  Device code is built as usual.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR / "build_native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PDRNN_OFFLOAD_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def sanitize_flavour() -> str:
    return os.environ.get("PDRNN_SANITIZE", "").strip()


def _san_dir() -> Path:
    tag = sanitize_flavour().replace(",", "_")
    return PKG_DIR / f"build_native_san_{tag}"


def ext_path() -> Path:
    if sanitize_flavour():
        return _san_dir() / ("_C" + _ext_suffix())
    return PKG_DIR / ("_C" + _ext_suffix())


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    lib = Path(torch.__file__).resolve().parent / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _sources():
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    runtime = sorted((CSRC / "runtime").glob("*.cpp")) + [CSRC / "bindings.cpp"]
    headers = sorted(CSRC.rglob("*.h")) + sorted(CSRC.rglob("*.hpp"))
    return kernels, runtime, headers


def _digest(paths, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in paths:
        h.update(str(p).encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(
            f"native build step failed ({r.returncode}):\n{' '.join(map(str, cmd))}\n"
            f"{r.stdout}\n{r.stderr}"
        )
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    return r


# per-file device flags.  lstm_sw: the backward's weight-gradient waves
# (mode 4) keep their MFMA accumulators in VGPRs -- in AGPRs they would be
# allocated beside the BPTT waves' VGPRs (one kernel, one register budget)
# and the workgroup would drop to one wave per SIMD.
_FILE_FLAGS = {"lstm_sw": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def build(verbose: bool = False, clean: bool = False, jobs: int | None = None) -> Path:
    """Compile every HIP kernel for gfx950 plus the host runtime; link ``_C``."""
    inc, torch_lib, abi = _torch_paths()
    kernels, runtime, headers = _sources()
    san = sanitize_flavour()
    build_dir = _san_dir() if san else BUILD_DIR
    if clean and build_dir.exists():
        shutil.rmtree(build_dir)
    build_dir.mkdir(exist_ok=True)
    hipcc = ROCM / "bin" / "hipcc"
    py_inc = sysconfig.get_paths()["include"]
    common_inc = [f"-I{CSRC / 'include'}"]
    debug = os.environ.get("PDRNN_DEBUG_BUILD", "0") == "1"
    hip_opt = ["-O1", "-g", "-DPDRNN_DEBUG=1"] if debug else ["-O3"]
    host_opt = ["-O0", "-g", "-DPDRNN_DEBUG=1"] if debug else ["-O2"]
    if san:  # the host TUs only (g++): device code has no sanitizer on this pool
        host_opt = ["-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
    hip_flags = [
        "-c", *hip_opt, "-fPIC", "-std=c++17", f"--offload-arch={ARCH}",
        "-munsafe-fp-atomics", "-Wno-unused-result", *common_inc,
        # diagnostic / A-B builds only (e.g. -DPDRNN_GEMM_AB=3); part of the build signature
        *os.environ.get("PDRNN_HIP_EXTRA_FLAGS", "").split(),
    ]
    host_flags = [
        "-c", *host_opt, "-fPIC", "-fvisibility=hidden", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations",
        *common_inc, *[f"-I{p}" for p in inc], f"-I{ROCM / 'include'}", f"-I{py_inc}",
    ]
    hdr_sig = _digest(headers, ARCH)

    jobs_list = []
    for src in kernels:
        obj = BUILD_DIR / (src.stem + ".hip.o")  # device code: shared with the plain build
        flags = hip_flags + _FILE_FLAGS.get(src.stem, [])
        sig = _digest([src], hdr_sig + " ".join(flags))
        jobs_list.append((src, obj, sig, [hipcc, *flags, src, "-o", obj]))
    for src in runtime:
        obj = build_dir / (src.stem + ".cpp.o")
        sig = _digest([src], hdr_sig + " ".join(host_flags))
        jobs_list.append((src, obj, sig, ["g++", *host_flags, src, "-o", obj]))

    def compile_one(job):
        src, obj, sig, cmd = job
        stamp = obj.with_suffix(obj.suffix + ".sig")
        if obj.exists() and stamp.exists() and stamp.read_text() == sig:
            return obj, False
        _run(cmd, verbose)
        stamp.write_text(sig)
        return obj, True

    n = jobs or min(8, max(1, (os.cpu_count() or 4)))
    n = min(n, 16)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        results = list(ex.map(compile_one, jobs_list))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    out = ext_path()
    if rebuilt or not out.exists():
        link = [
            hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out,
            f"-L{torch_lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10_hip", "-ltorch_hip", f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl",
            f"-Wl,-rpath,{torch_lib}", f"-Wl,-rpath,{ROCM / 'lib'}",
        ]
        _run(link, verbose)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    out = build(verbose=a.verbose, clean=a.clean, jobs=a.jobs)
    print(f"built {out}")


if __name__ == "__main__":
    main()
