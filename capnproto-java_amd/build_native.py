"""Builds the MI355X codec library in-tree (hipcc, gfx950):
capnproto-java_amd/lib/libcapnp_packed_hip.so.  Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
SRC = PKG / "csrc" / "packed_codec.hip"
HDR = PKG.parent / "include" / "capnp_packed.h"
# every source the library is built from: packed_codec.hip #includes the
# other csrc/*.hip files, so any of them (or the header) being newer rebuilds
DEPS = sorted((PKG / "csrc").glob("*.hip")) + [HDR]
LIB = PKG / "lib" / "libcapnp_packed_hip.so"
# the same sources with diagnostics counters compiled in (tests only)
DIAG_LIB = PKG / "lib" / "libcapnp_packed_hip_diag.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CPK_OFFLOAD_ARCH", "gfx950")


def _build_one(lib: Path, extra: list[str], force: bool, verbose: bool) -> Path:
    if (not force and lib.exists()
            and lib.stat().st_mtime >= max(d.stat().st_mtime for d in DEPS)):
        return lib
    lib.parent.mkdir(parents=True, exist_ok=True)
    cmd = [HIPCC, "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-value", "-Wno-unused-result", *extra, "-o", str(lib), str(SRC)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return lib


def build(force: bool = False, verbose: bool = False) -> Path:
    return _build_one(LIB, [], force, verbose)


def build_diag(force: bool = False, verbose: bool = False) -> Path:
    """The diagnostics library (-DCPK_DEC_CNT=1: the dense decoder form's
    window counters, cpk_ctx_dense_windows) -- loaded by tests only."""
    return _build_one(DIAG_LIB, ["-DCPK_DEC_CNT=1"], force, verbose)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_diag(force="--force" in sys.argv, verbose=True))
