"""In-tree build of ``libflipchain.so`` for gfx950 (``hipcc``; no JIT cache, no CMake).

The shared library lands next to this file so that it travels to the GPU box with the
repository snapshot.  ``python -m flipcomplexityempirical_amd.build`` rebuilds it.
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
# FC_LIB_VARIANT selects a diagnostic build under its own file name: "_"-separated tokens, each a
# -D flag (prof: per-phase s_memtime counters; sync: each stamp drains outstanding memory first).
# Such a build (and any with FC_HIPCC_FLAGS) also gets -DFC_VARIANT_BUILD: fc_build_flags()
# reports it and _lib.load() refuses it unless called with allow_variant=True (tools only).
VARIANT = os.environ.get("FC_LIB_VARIANT", "")
VARIANT_FLAGS = {"prof": "-DFC_PHASE_PROF", "sync": "-DFC_PHASE_SYNC"}
LIB = os.environ.get("FC_LIB_OUT") or os.path.join(PKG, f"libflipchain_{VARIANT}.so" if VARIANT else "libflipchain.so")
SOURCES = ["fc_flip2.hip", "fc_deal.hip", "fc_kernels.hip", "fc_series.hip", "fc_recom.hip", "fc_capi.cpp", "fc_graph.cpp"]
HEADERS = ["fc_internal.h", "fc_philox.h", "fc_device.h", "fc_ring.h", os.path.join("..", "..", "include", "flipchain.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("FC_OFFLOAD_ARCH", "gfx950")


def _flags() -> list:
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
    for tok in filter(None, VARIANT.split("_")):
        if tok not in VARIANT_FLAGS:
            raise ValueError(f"FC_LIB_VARIANT token {tok!r} (known: {', '.join(VARIANT_FLAGS)})")
        flags.append(VARIANT_FLAGS[tok])
    # FC_HIPCC_FLAGS: extra compiler flags for experiment builds (with FC_LIB_OUT naming the output)
    extra = os.environ.get("FC_HIPCC_FLAGS", "").split()
    flags += extra
    if VARIANT or extra:
        flags.append("-DFC_VARIANT_BUILD")
    return flags


def source_id() -> str:
    """SHA-256 over every source and header (name and bytes) and the compiler flags: the id the
    library is built with (``fc_build_id()``) and the one a current library must carry."""
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        h.update(f.encode() + b"\0")
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(_flags()).encode())
    return h.hexdigest()[:32]


def library_id(path: str = None) -> str:
    """The build id embedded in a built library (the ``FC_BUILD_ID=`` marker), or "" if none."""
    path = path or LIB
    try:
        with open(path, "rb") as fh:
            m = re.search(rb"FC_BUILD_ID=([0-9a-f]{32})", fh.read())
    except OSError:
        return ""
    return m.group(1).decode() if m else ""


def _stale() -> bool:
    """Rebuild when the library is missing or was built from other sources / flags (by content
    hash, not file times: a snapshot copy or checkout resets mtimes)."""
    return not os.path.exists(LIB) or library_id(LIB) != source_id()


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    if verbose and res.stderr:
        print(res.stderr, file=sys.stderr)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every source to an object in parallel (the kernel files dominate: ~45 s each),
    then link the shared library."""
    if not force and not _stale():
        return LIB
    flags = _flags() + [f'-DFC_BUILD_ID="{source_id()}"']
    with tempfile.TemporaryDirectory(prefix="fc_build_") as tmp:
        objs = [os.path.join(tmp, os.path.splitext(src)[0] + ".o") for src in SOURCES]
        jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(SOURCES), os.cpu_count() or 1, 8)
        with ThreadPoolExecutor(max_workers=jobs) as pool:
            futs = [pool.submit(_run, [HIPCC, *flags, "-c", "-o", obj, os.path.join(CSRC, src)], verbose)
                    for src, obj in zip(SOURCES, objs)]
            for f in futs:
                f.result()
        _run([HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", LIB, *objs], verbose)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
