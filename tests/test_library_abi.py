"""libdfq_hip.so loads (no GPU needed) and exports exactly what include/dfq_hip.h
declares; the ctypes binding covers every symbol."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "dfq_hip.h"
LIB = ROOT / "data_free_quantization_amd" / "libdfq_hip.so"


DIAG_HEADER = ROOT / "include" / "dfq_diag.h"
DIAG_LIB = ROOT / "data_free_quantization_amd" / "libdfq_diag.so"


def declared(header=HEADER):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dfq_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_functions():
    names = declared()
    assert "dfq_sweep_plan_create" in names and "dfq_cle_relation" in names
    assert len(names) >= 20


@pytest.fixture(scope="module")
def lib():
    if not LIB.exists():
        pytest.skip("libdfq_hip.so not built (run __graft_entry__.build())")
    return ctypes.CDLL(str(LIB))


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (dfq_[a-z0-9_]+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    for n in declared():
        assert hasattr(lib, n)


def test_python_binding_covers_header():
    from data_free_quantization_amd import _lib
    assert sorted(_lib.EXPORTS) == declared()
    assert sorted(_lib.DIAG_EXPORTS) == [n for n in declared(DIAG_HEADER) if n not in declared()]


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True, check=True).stdout
    return set(re.findall(r" T (dfq_[a-z0-9_]+)", out))


def test_product_library_carries_no_diagnostics():
    """The probes, the timeline and the A/B variants live in libdfq_diag.so only."""
    if not LIB.exists() or not DIAG_LIB.exists():
        pytest.skip("libraries not built (run __graft_entry__.build())")
    prod, diag = _exports(LIB), _exports(DIAG_LIB)
    diag_only = [n for n in declared(DIAG_HEADER) if n not in declared()]
    assert diag_only and not (set(diag_only) & prod)
    assert set(declared(DIAG_HEADER)) <= diag
    assert LIB.stat().st_size < DIAG_LIB.stat().st_size


def _dynsyms(path, *flags):
    out = subprocess.run(["nm", "-D", *flags, str(path)], capture_output=True, text=True, check=True).stdout
    return [ln.split()[-1] for ln in out.splitlines() if ln.strip()]


@pytest.mark.parametrize("path", [LIB, DIAG_LIB], ids=["product", "diagnostics"])
def test_only_the_c_abi_is_exported(path):
    """csrc/exports.map: the dynamic symbol table of each library holds its dfq_*
    entry points and nothing else (no kernel stub handles, templates or inline
    helpers that a second library loaded in the process could interpose)."""
    if not path.exists():
        pytest.skip("libraries not built (run __graft_entry__.build())")
    defined = _dynsyms(path, "--defined-only")
    assert defined and all(n.startswith("dfq_") for n in defined), [n for n in defined if not n.startswith("dfq_")]


def test_product_library_reads_no_environment():
    """The A/B switches (DFQ_SWEEP_*, DFQ_CLE_*) are read by libdfq_diag.so only:
    the product library does not even import getenv."""
    if not LIB.exists() or not DIAG_LIB.exists():
        pytest.skip("libraries not built (run __graft_entry__.build())")
    assert not any(n.split("@")[0] in ("getenv", "secure_getenv") for n in _dynsyms(LIB, "--undefined-only"))
    assert any(n.split("@")[0] == "getenv" for n in _dynsyms(DIAG_LIB, "--undefined-only"))


def test_version_and_errors(lib):
    from data_free_quantization_amd import _lib
    L = _lib.load()
    assert L.dfq_abi_version() == 1
    assert L.dfq_error_string(-5) == b"shape mismatch"
    # argument validation runs on the host, no device needed
    d = _lib.TensorDesc()
    import ctypes as C
    nbytes = C.c_size_t(0)
    assert L.dfq_quantize_ws_bytes(C.byref(d), C.byref(nbytes)) == _lib.DFQ_ERR_INVALID   # src NULL
    d.src = 16
    d.rows, d.row_len, d.khw, d.bits, d.mode = 4, 64, 1, 8, _lib.DFQ_TENSOR_ASYM
    assert L.dfq_quantize_ws_bytes(C.byref(d), C.byref(nbytes)) == 0
    assert nbytes.value > 0
    d.bits = 17
    assert L.dfq_quantize_ws_bytes(C.byref(d), C.byref(nbytes)) == _lib.DFQ_ERR_INVALID
    d.bits, d.khw = 8, 3
    d.esum = 32
    assert L.dfq_quantize_ws_bytes(C.byref(d), C.byref(nbytes)) == _lib.DFQ_ERR_SHAPE   # 64 % 3


def test_product_rejects_cpu_tensors():
    import torch
    from data_free_quantization_amd.utils.quantize import quantize
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        quantize(torch.randn(4, 4), 8, -1.0, 1.0)


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: a missing libdfq_hip.so raises instead of degrading."""
    from data_free_quantization_amd import _lib
    with pytest.raises(_lib.DFQLibraryError, match="no CPU fallback"):
        _lib.load(tmp_path / "libdfq_hip.so")


def _header_constants():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    consts = {k: int(v, 0) for k, v in re.findall(r"#define (DFQ_[A-Z0-9_]+)\s+(-?(?:0x[0-9a-fA-F]+|\d+))", text)}
    for body in re.findall(r"enum\s*\{([^}]*)\}", text):
        for k, v in re.findall(r"(DFQ_[A-Z0-9_]+)\s*=\s*(-?(?:0x[0-9a-fA-F]+|\d+))", body):
            consts[k] = int(v, 0)
    return consts


def test_python_constants_match_header():
    """Every DFQ_* constant the Python layer defines has the header's value."""
    from data_free_quantization_amd import _lib
    consts = _header_constants()
    mine = {k: getattr(_lib, k) for k in dir(_lib) if k.startswith("DFQ_") and isinstance(getattr(_lib, k), int)}
    assert len(mine) >= 15
    for k, v in mine.items():
        assert k in consts, k
        assert consts[k] == v, (k, consts[k], v)


def _struct_fields(name):
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    body = re.search(r"typedef struct " + name + r"\s*\{(.*?)\}\s*" + name + ";", text, flags=re.S).group(1)
    return re.findall(r"([A-Za-z_][A-Za-z0-9_]*)\s*;", body)


@pytest.mark.parametrize("cname,pyname", [("dfq_tensor_desc", "TensorDesc"), ("dfq_bn_fold_desc", "BnFoldDesc"),
                                          ("dfq_bc_op", "BcOp")])
def test_ctypes_structs_follow_header_field_order(cname, pyname):
    """The ctypes mirrors (and the numpy record tables built on them) list the
    header's fields in the header's order."""
    from data_free_quantization_amd import _lib
    want = _struct_fields(cname)
    got = [f for f, _ in getattr(_lib, pyname)._fields_]
    assert got == want, (got, want)


def test_numpy_tables_match_ctypes_layouts():
    from data_free_quantization_amd import _lib
    from data_free_quantization_amd.sweep import _DESC
    from data_free_quantization_amd.utils.layer_transform import _BN_DESC
    from data_free_quantization_amd.bias_correction import _BC_OP
    for dt, st in ((_DESC, _lib.TensorDesc), (_BN_DESC, _lib.BnFoldDesc), (_BC_OP, _lib.BcOp)):
        assert dt.itemsize == ctypes.sizeof(st)
