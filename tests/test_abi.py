"""CPU-side checks of the drop-in boundary: the shared objects load and export exactly what include/ declares.

No compute calls (no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import pytest

import picotls_amd as pa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header: str) -> set:
    text = open(os.path.join(ROOT, "include", "picotls", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(ptls_mi355x_\w+)\s*\(", text))


def exported(so: str) -> set:
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_engine_library_loads_and_exports_header():
    lib = pa.load_library()
    assert isinstance(lib, ctypes.CDLL)
    decl = declared("mi355x.h")
    assert decl == set(pa.ABI_FUNCTIONS)
    missing = decl - exported(pa.LIB_PATH)
    assert not missing, missing


def test_engine_library_exports_debug_hooks():
    """include/picotls/mi355x_debug.h (test and measurement hooks, outside the picotls boundary) is exported too."""
    decl = declared("mi355x_debug.h")
    assert decl == set(pa.DEBUG_FUNCTIONS)
    assert not decl & set(pa.ABI_FUNCTIONS)
    missing = decl - exported(pa.LIB_PATH)
    assert not missing, missing


def test_picotls_backend_exports_algorithms():
    if not os.path.exists(pa.PICOTLS_LIB_PATH):
        pytest.skip("picotls headers were not available at build time")
    syms = exported(pa.PICOTLS_LIB_PATH)
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "picotls", "mi355x_picotls.h")).read(), flags=re.S)
    objects = set()
    for decl in re.findall(r"extern\s+ptls_\w+_algorithm_t\s+([^;]+);", text):
        objects |= {n.strip() for n in decl.split(",")}
    assert objects == {"ptls_mi355x_aes128ctr", "ptls_mi355x_aes256ctr", "ptls_mi355x_quiclb", "ptls_mi355x_aes128gcm",
                       "ptls_mi355x_aes256gcm", "ptls_mi355x_non_temporal_aes128gcm", "ptls_mi355x_non_temporal_aes256gcm"}
    assert objects <= syms
    assert declared("mi355x_picotls.h") <= syms


def test_kernels_are_gfx950_code_objects():
    # the fat binary embeds a gfx950 code object (target id hipv4-amdgcn-amd-amdhsa--gfx950) and nothing else
    data = open(pa.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_record_descriptor_layout_matches_header():
    text = open(os.path.join(ROOT, "include", "picotls", "mi355x.h")).read()
    assert "#define PTLS_MI355X_RECORD_SIZE 40" in text
    assert pa.RECORD_DTYPE.itemsize == 40
    names = list(pa.RECORD_DTYPE.names)
    assert names == ["in_off", "out_off", "seq", "aad_off", "len", "key_idx", "aad_len", "flags"]
    # the oracle's ctypes view must agree with the engine's
    import oracle

    assert oracle.RECORD_DTYPE == pa.RECORD_DTYPE


def test_side_descriptor_layouts_match_header():
    text = open(os.path.join(ROOT, "include", "picotls", "mi355x.h")).read()
    # ptls_mi355x_cid_t (QUIC-LB), ptls_mi355x_hp_t (header protection), ptls_mi355x_tls_result_t
    assert re.search(r"uint64_t in_off;\s*uint64_t out_off;\s*uint32_t key_idx;\s*uint8_t len;\s*uint8_t encrypt;", text)
    assert list(pa.CID_DTYPE.names) == ["in_off", "out_off", "key_idx", "len", "encrypt", "reserved"]
    assert pa.CID_DTYPE.itemsize == 24 and pa.HP_DTYPE.itemsize == 16 and pa.TLS_RESULT_DTYPE.itemsize == 8
    assert "#define PTLS_MI355X_QUICLB_MIN_LEN 7" in text and "#define PTLS_MI355X_QUICLB_MAX_LEN 19" in text


def test_no_cpu_fallback_when_library_missing(tmp_path):
    # the product path fails loudly instead of falling back to any CPU implementation
    saved = pa._lib
    try:
        pa._lib = None
        with pytest.raises(pa.EngineError):
            pa.load_library(str(tmp_path / "missing.so"))
    finally:
        pa._lib = saved


def test_in_tree_library_is_built_from_the_current_sources(tmp_path):
    """build.py stamps each library with the SHA-256 of its sources and compile settings (<lib>.sha256), so a rebuild
    follows content rather than file times; the in-tree engine library carries the digest of the sources beside it
    (load_library refuses it otherwise), and the digest moves with any source byte."""
    from picotls_amd import build as b

    if os.environ.get("PTLS_MI355X_LIB"):
        pytest.skip("a variant library is loaded instead of the in-tree build")
    assert b._stamp(b.ENGINE_SO) == b.engine_digest()
    if os.path.exists(b.PICOTLS_SO + ".sha256"):
        assert b._stamp(b.PICOTLS_SO) == b.picotls_digest()
    f = tmp_path / "x.h"
    f.write_text("int a;\n")
    d0 = b.source_digest([str(f)])
    f.write_text("int b;\n")
    assert b.source_digest([str(f)]) != d0
    assert b.source_digest([str(f)], "gfx950") != b.source_digest([str(f)], "gfx942")
