"""Sanitizer runs of the host side (SURVEY.md §5 "race detection / sanitizers";
VERDICT r1 #6):

* the C++ runtime (``csrc/runtime/*.cpp``: KV block manager, detokenizer, JSON
  token FSM) built with AddressSanitizer + UndefinedBehaviorSanitizer into an
  executable that embeds CPython (``csrc/tools/rt_sanitize.cpp``), running the
  runtime's own unit tests plus the guided-decoding and engine CPU tests through
  it -- any heap overflow, use-after-free or UB aborts the run;
* the asyncio service paths (WebSocket protocol, OpenAI facade) under asyncio
  debug mode with never-awaited coroutines as errors.

CPU only; the instrumented binary is cached under build/sanitize by a hash of
its sources and flags."""
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[2]
OUT = REPO / "build" / "sanitize"


def _build() -> Path:
    import pybind11

    srcs = sorted((REPO / "csrc" / "runtime").glob("*.cpp")) + [REPO / "csrc/tools/rt_sanitize.cpp"]
    flags = ["-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-DFTRT_EMBEDDED",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
             f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
             f"-I{REPO / 'csrc' / 'runtime'}"]
    h = hashlib.sha256()
    for p in srcs + sorted((REPO / "csrc" / "runtime").glob("*.h")):
        h.update(p.read_bytes())
    h.update(" ".join(flags).encode())
    exe = OUT / f"rt_sanitize_{h.hexdigest()[:16]}"
    if not exe.exists():
        OUT.mkdir(parents=True, exist_ok=True)
        libdir = sysconfig.get_config_var("LIBDIR")
        ver = f"{sys.version_info.major}.{sys.version_info.minor}"
        cmd = ["g++", *flags, *map(str, srcs), "-o", str(exe), f"-L{libdir}", f"-lpython{ver}",
               "-ldl", "-lpthread", "-lutil"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-4000:]
    return exe


def test_runtime_under_asan_ubsan():
    exe = _build()
    env = dict(os.environ)
    env.update(FT_RT_MODULE="_rt_san", PYTHONPATH=str(REPO), FT_AUTOBUILD="0",
               # CPython's arena allocator keeps memory until exit: leak reports are noise
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    tests = ["tests/unit/test_runtime_native.py", "tests/unit/test_engine_cpu.py",
             "tests/unit/test_kv_swap.py"]
    r = subprocess.run([str(exe), "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu", *tests],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert r.returncode == 0, out[-6000:]
    assert " passed" in out


def test_service_paths_under_asyncio_debug():
    env = dict(os.environ, PYTHONASYNCIODEBUG="1", PYTHONPATH=str(REPO))
    r = subprocess.run([sys.executable, "-X", "dev", "-m", "pytest", "-q", "-x", "-p",
                        "no:cacheprovider", "-W", "error::RuntimeWarning", "-m", "not gpu",
                        "tests/protocol"], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    for bad in ("was never awaited", "Task was destroyed but it is pending",
                "Task exception was never retrieved"):
        assert bad not in out, out[-6000:]
