"""Build libdfq_hip.so (gfx950) in-tree with hipcc.

The library is the product: plain C ABI (include/dfq_hip.h), loaded by
``data_free_quantization_amd._lib`` through ctypes.  Built artefacts stay in the
package directory so they travel to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libdfq_hip.so"
SOURCES = ["dfq_lib.hip", "dfq_sweep.hip", "dfq_transform.hip", "dfq_cle.hip", "dfq_cle_relation.hip"]
# Diagnostics build (bench.py's ceiling probes, scripts/ A/B runs): the same
# sources with -DDFQ_DIAGNOSTICS (the sweep's A/B variants and environment
# switches) plus the probes (include/dfq_diag.h).  Never loaded by the product path.
DIAG_LIB = PKG / "libdfq_diag.so"
DIAG_SOURCES = SOURCES + ["dfq_probe.hip"]
# linker version script: the dynamic symbol table holds dfq_* and nothing else
EXPORTS = CSRC / "exports.map"
ARCH = os.environ.get("DFQ_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: no FMA contraction (bit parity with torch CPU eager ops).
# Correctly-rounded fp32 divide/sqrt is hipcc's default; keep it explicit.
FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
    # only the C ABI is exported, and each library binds to its own internals
    # (libdfq_hip.so and libdfq_diag.so loaded together must not interpose)
    "-fvisibility=hidden", "-fvisibility-inlines-hidden",
]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or Path(c).exists()):
            return c
    raise RuntimeError("hipcc not found")


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _build_one(out: Path, sources, defines, force: bool, verbose: bool) -> Path:
    deps = [CSRC / s for s in sources] + [CSRC / "dfq_common.h", CSRC / "dfq_cle_common.h", ROOT / "include" / "dfq_hip.h",
                                          ROOT / "include" / "dfq_diag.h", EXPORTS, Path(__file__)]
    if not force and not _stale(out, deps):
        return out
    tag = out.stem
    objs, cmds = [], []
    for s in sources:
        obj = CSRC / f"{Path(s).stem}.{tag}.o"
        cmds.append([hipcc(), *FLAGS, *defines, "-I", str(ROOT / "include"), "-I", str(CSRC), "-c", str(CSRC / s),
                     "-o", str(obj)])
        objs.append(str(obj))
    if verbose:
        for cmd in cmds:
            print(" ".join(cmd), file=sys.stderr)
    # translation units compile in parallel (one hipcc each)
    with ThreadPoolExecutor(max_workers=min(len(cmds), max(1, (os.cpu_count() or 1) // 2), 8)) as ex:
        for f in [ex.submit(subprocess.run, cmd, check=True) for cmd in cmds]:
            f.result()
    tmp = out.with_suffix(".so.tmp")
    cmd = [hipcc(), "-shared", f"--offload-arch={ARCH}", "-Wl,-Bsymbolic", f"-Wl,--version-script={EXPORTS}",
           "-o", str(tmp), *objs]
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    for o in objs:
        os.remove(o)
    return out


def build(force: bool = False, verbose: bool = False, diagnostics: bool = True) -> Path:
    """Build libdfq_hip.so (the product) and, by default, libdfq_diag.so."""
    _build_one(LIB, SOURCES, [], force, verbose)
    if diagnostics:
        _build_one(DIAG_LIB, DIAG_SOURCES, ["-DDFQ_DIAGNOSTICS"], force, verbose)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
