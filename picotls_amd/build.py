"""Builds the engine's shared objects in-tree (they travel to the GPU box with the repo snapshot).

  picotls_amd/_lib/libptls_mi355x.so          HIP kernels + C ABI (include/picotls/mi355x.h), hipcc --offload-arch=gfx950
  picotls_amd/_lib/libptls_mi355x_picotls.so  the ptls_aead_algorithm_t objects (C, gcc), only where picotls.h exists
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_DIR = os.path.join(PKG, "_lib")
ENGINE_SO = os.path.join(LIB_DIR, "libptls_mi355x.so")
PICOTLS_SO = os.path.join(LIB_DIR, "libptls_mi355x_picotls.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
PICOTLS_INCLUDE = os.environ.get("PICOTLS_INCLUDE", "/root/reference/include")

# The machine scheduler's iterative-ILP strategy keeps more of each round's LDS lookups in flight than the default
# occupancy-driven one (+5 % seal+open on 16 KiB and 1200 B records, interleaved A/B with tools/ab.py).
ENGINE_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
ENGINE_SRCS = [os.path.join(PKG, "csrc", "aesgcm_engine.hip")]
PICOTLS_SRCS = [os.path.join(PKG, "csrc", "ptls_mi355x.c")]
HEADERS = [os.path.join(ROOT, "include", "picotls", h) for h in ("mi355x.h", "mi355x_picotls.h", "mi355x_debug.h")]
ENGINE_PARTS = sorted(os.path.join(PKG, "csrc", "engine", f) for f in os.listdir(os.path.join(PKG, "csrc", "engine"))
                      if f.endswith(".h"))  # included by aesgcm_engine.hip (one translation unit)


def source_digest(files: list[str], extra: str = "") -> str:
    """SHA-256 over the sources' paths and contents (and the compile settings): a built library carries the digest of
    what it was built from (<lib>.sha256 beside it), so a rebuild is decided by content, not by file times, and
    load_library refuses an in-tree library whose sources changed since (picotls_amd/__init__.py)."""
    h = hashlib.sha256(extra.encode())
    for f in sorted(files):
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def engine_digest() -> str:
    return source_digest(ENGINE_SRCS + ENGINE_PARTS + HEADERS, " ".join([ARCH, *ENGINE_FLAGS]))


def picotls_digest() -> str:
    return source_digest(PICOTLS_SRCS + HEADERS, engine_digest())


def _stamp(lib: str) -> str | None:
    try:
        with open(lib + ".sha256") as fh:
            return fh.read().strip()
    except OSError:
        return None


def _stale(lib: str, digest: str) -> bool:
    return not os.path.exists(lib) or _stamp(lib) != digest


def _install(tmp: str, lib: str, digest: str) -> None:
    os.replace(tmp, lib)
    with open(lib + ".sha256", "w") as fh:
        fh.write(digest + "\n")


def build_engine(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    digest = engine_digest()
    if force or _stale(ENGINE_SO, digest):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result",
               "-Wno-unused-value", *ENGINE_FLAGS, "-I", os.path.join(ROOT, "include"), *ENGINE_SRCS,
               "-o", ENGINE_SO + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        _install(ENGINE_SO + ".tmp", ENGINE_SO, digest)
    return ENGINE_SO


def build_picotls_backend(force: bool = False, verbose: bool = False) -> str | None:
    """The picotls vtable adapter needs picotls.h at build time (a picotls installation; here the reference tree)."""
    if not os.path.exists(os.path.join(PICOTLS_INCLUDE, "picotls.h")):
        return PICOTLS_SO if os.path.exists(PICOTLS_SO) else None
    digest = picotls_digest()
    if force or _stale(PICOTLS_SO, digest):
        cc = shutil.which("gcc") or "cc"
        cmd = [cc, "-std=gnu99", "-O2", "-fPIC", "-shared", "-Wall", "-I", os.path.join(ROOT, "include"), "-I",
               PICOTLS_INCLUDE, *PICOTLS_SRCS, "-L", LIB_DIR, "-lptls_mi355x", "-Wl,-rpath,$ORIGIN",
               "-o", PICOTLS_SO + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        _install(PICOTLS_SO + ".tmp", PICOTLS_SO, digest)
    return PICOTLS_SO


def build(force: bool = False, verbose: bool = False) -> None:
    build_engine(force, verbose)
    build_picotls_backend(force, verbose)


if __name__ == "__main__":
    build(force=True, verbose=True)
