"""In-tree build of the native extensions (no JIT cache outside the repo).

Two extensions are produced next to the package sources so they travel with the
repository snapshot to a GPU box:

* ``fasttalk_llm_microservice_amd/_C.so``  -- the gfx950 HIP kernels in
  ``csrc/kernels/*.hip`` (compiled with ``hipcc --offload-arch=gfx950``) plus the
  torch bindings ``csrc/bindings.cpp``.
* ``fasttalk_llm_microservice_amd/_rt.so`` -- the host runtime in
  ``csrc/runtime/*.cpp`` (KV block manager, detokenizer, JSON-schema token FSM,
  batch metadata builder), plain C++17 + pybind11, no torch / HIP dependency so
  CPU-only hosts can use it.

Each translation unit is compiled separately (kernels do not include torch
headers, which keeps a kernel rebuild at seconds) and cached by a content hash
of the source, the headers it can include, and the flags.

Usage: ``python -m fasttalk_llm_microservice_amd.ops.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parents[1]
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
ARCH = os.environ.get("FT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _ext_suffix() -> str:
    return ".so"


def _hash(parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        if isinstance(p, Path):
            h.update(p.read_bytes())
        else:
            h.update(str(p).encode())
    return h.hexdigest()[:24]


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(map(str, cmd))}\n{r.stdout}")
    return r.stdout


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [
        f"-I{sysconfig.get_paths()['include']}",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_C",   # _C_checked for the checked build (build_kernels)
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-fPIC",
        "-O3",
        "-std=c++17",
    ]
    ldflags = [f"-L{lib}", f"-Wl,-rpath,{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-ltorch_python"]
    return cflags, ldflags


def _compile(src: Path, obj: Path, cmd: list, deps: list, force: bool) -> bool:
    key = _hash([src, *deps, " ".join(cmd)])
    stamp = obj.with_suffix(obj.suffix + ".hash")
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == key:
        return False
    obj.parent.mkdir(parents=True, exist_ok=True)
    _run(cmd + ["-c", str(src), "-o", str(obj)])
    stamp.write_text(key)
    return True


# Per-kernel extra flags.  The attention kernels keep their MFMA accumulators in
# VGPRs (gfx950's unified register file): in the AGPR form hipcc copied the O
# accumulator AGPR -> VGPR -> AGPR around every online-softmax rescale (64 extra
# instructions per KV tile in the decode kernel); and without NaN semantics fmaxf
# on MFMA results needs no canonicalising v_max first.
KERNEL_FLAGS = {
    "attn_decode": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-honor-nans"],
    "attn_prefill": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-honor-nans"],
    # W4: the per-group scale / zero correction reads every MFMA result on the VALU
    "w4a16": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = True,
                  checked: bool = False) -> Path:
    """``checked``: the bounds-checked debug build (``-DFT_KERNEL_CHECKS=1``,
    csrc/include/ft_common.h) as a separate extension ``_C_checked.so``, loaded by
    ``ops.native()`` when ``FT_KERNEL_CHECKS=1``."""
    headers = sorted((CSRC / "include").glob("*.h")) + sorted((CSRC / "kernels").glob("*.h"))
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    name = "_C_checked" if checked else "_C"
    extra = ["-DFT_KERNEL_CHECKS=1"] if checked else []
    bdir = BUILD / ("checked" if checked else "")
    kflags = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
              f"-I{CSRC / 'include'}", "-munsafe-fp-atomics"] + extra
    tflags, ldflags = _torch_flags()
    tflags = [f for f in tflags if not f.startswith("-DTORCH_EXTENSION_NAME=")] + \
        [f"-DTORCH_EXTENSION_NAME={name}"]
    bflags = [HIPCC, f"--offload-arch={ARCH}"] + tflags + [f"-I{CSRC / 'include'}"] + extra
    jobs_list = [(k, bdir / "kernels" / (k.stem + ".o"), kflags + KERNEL_FLAGS.get(k.stem, []), headers)
                 for k in kernels]
    jobs_list.append((CSRC / "bindings.cpp", bdir / "bindings.o", bflags + ["-x", "hip"], headers))
    changed = False
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(_compile, s, o, c, d, force): s for s, o, c, d in jobs_list}
        for f in cf.as_completed(futs):
            if f.result():
                changed = True
                if verbose:
                    print(f"[build] compiled {futs[f].name}", flush=True)
    out = PKG_DIR / (name + _ext_suffix())
    objs = [str(o) for _, o, _, _ in jobs_list]
    if changed or force or not out.exists():
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(out), *ldflags])
        if verbose:
            print(f"[build] linked {out.relative_to(REPO)}", flush=True)
    return out


def build_runtime(force: bool = False, jobs: int = 8, verbose: bool = True) -> Path:
    import pybind11

    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    headers = sorted((CSRC / "runtime").glob("*.h"))
    flags = [CXX, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
             f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
             f"-I{CSRC / 'runtime'}"]
    jobs_list = [(s, BUILD / "runtime" / (s.stem + ".o"), flags, headers) for s in srcs]
    changed = False
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(_compile, s, o, c, d, force): s for s, o, c, d in jobs_list}
        for f in cf.as_completed(futs):
            if f.result():
                changed = True
                if verbose:
                    print(f"[build] compiled {futs[f].name}", flush=True)
    out = PKG_DIR / ("_rt" + _ext_suffix())
    if changed or force or not out.exists():
        _run([CXX, "-shared", "-fPIC", *[str(o) for _, o, _, _ in jobs_list], "-o", str(out)])
        if verbose:
            print(f"[build] linked {out.relative_to(REPO)}", flush=True)
    return out


def build_all(force: bool = False, jobs: int = 8, verbose: bool = True, checked: bool = True):
    """Runtime, release kernels and (``checked``) the bounds-checked kernel build."""
    rt = build_runtime(force=force, jobs=jobs, verbose=verbose)
    k = build_kernels(force=force, jobs=jobs, verbose=verbose)
    if checked:
        build_kernels(force=force, jobs=jobs, verbose=verbose, checked=True)
    return k, rt


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=["kernels", "checked", "runtime"], default=None)
    a = ap.parse_args(argv)
    if a.only == "kernels":
        build_kernels(a.force, a.jobs)
    elif a.only == "checked":
        build_kernels(a.force, a.jobs, checked=True)
    elif a.only == "runtime":
        build_runtime(a.force, a.jobs)
    else:
        build_all(a.force, a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
