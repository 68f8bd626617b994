"""C-ABI checks that need no GPU: every symbol the public headers declare is
exported by the built libraries; parameter validation; and the product path
fails loudly (no CPU fallback) when no HIP device is present."""
import ctypes as C
import pathlib
import re
import subprocess

import numpy as np
import pytest

import kbin

from conftest import gpu_available

REPO = pathlib.Path(__file__).resolve().parent.parent


def declared(header: str, prefix: str):
    txt = (REPO / "include" / header).read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"\w+)\s*\(", txt)))


def exported(lib: pathlib.Path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], check=True,
                         capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_kbin_exports_every_declared_symbol():
    decl = declared("kbin.h", "kb_")
    assert decl, "no kb_ declarations parsed"
    ex = exported(kbin.LIB_PATH)
    missing = [d for d in decl if d not in ex]
    assert not missing, missing
    assert sorted(kbin.EXPORTED) == decl


def test_host_exports_reference_surface():
    ex = exported(kbin.HOST_LIB_PATH)
    for sym in ["process_read", "prune_data"] + declared("binning_gpu.h", "kbh_"):
        assert sym in ex, sym
    # clean-room container API (zhash.h / llist.h names)
    for sym in declared("kb_zhash.h", "z") + ["create_node_num", "create_node_item", "free_llist"]:
        assert sym in ex, sym
    # the drop-in archive must NOT define the containers (they come from the caller)
    arch = subprocess.run(["nm", "--defined-only", str(kbin.LIB_DIR / "libkbin_host.a")],
                          check=True, capture_output=True, text=True).stdout
    assert " zhash_set" not in arch and " create_node_num" not in arch
    assert " T process_read" in arch and " T prune_data" in arch


def test_abi_version():
    assert kbin.load_library().kb_abi_version() == 3


def test_struct_layouts_match_header(tmp_path):
    """the ctypes mirrors of kb_params / kb_csr / kb_timing have the C layout
    of include/kbin.h (size and every field offset, compiled here with gcc)"""
    structs = {"kb_params": kbin.kb_params, "kb_csr": kbin.kb_csr, "kb_timing": kbin.kb_timing}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "kbin.h"', "int main(void) {"]
    for name, cls in structs.items():
        lines.append(f'printf("{name} %zu\\n", sizeof({name}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{name}.{f} %zu\\n", offsetof({name}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(kbin.INCLUDE_DIR), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    for name, cls in structs.items():
        assert int(got[name]) == C.sizeof(cls), name
        for f, _ in cls._fields_:
            assert int(got[f"{name}.{f}"]) == getattr(cls, f).offset, f"{name}.{f}"


# (K < 2M is accepted since round 5: the binned engine walks the reference's
# incremental branch, test_gpu_parity.py::test_k_below_2m_vs_oracle)
@pytest.mark.parametrize("K,M,code", [(64, 7, kbin.KB_EINVAL), (31, 9, kbin.KB_EINVAL), (31, 0, kbin.KB_EINVAL),
                                      (5, 7, kbin.KB_EINVAL), (0, 3, kbin.KB_EINVAL), (-1, 1, kbin.KB_EINVAL)])
def test_param_validation(K, M, code):
    with pytest.raises(kbin.KbError) as ei:
        kbin.Engine(K, M)
    assert ei.value.code == code


def test_no_silent_cpu_fallback():
    if gpu_available():
        pytest.skip("GPU present")
    with pytest.raises(kbin.KbError) as ei:
        kbin.Engine(31, 7)
    assert ei.value.code == kbin.KB_EDEVICE


def test_missing_library_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        kbin.load_library(tmp_path / "nope.so")


@pytest.mark.parametrize("M", range(1, 9))
def test_bucket_map_guard(M):
    """a record whose mmer code is below 2^(2M-1) (no entry
    in the bucket map, which covers canonical codes only) takes the hash
    route; the map is indexed only for canonical codes.  The kernels and this
    CPU hook share the predicate (kbin_internal.h bm_has_entry)."""
    lib = kbin.load_library()
    f = lib.kb_internal_map_dest
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.c_int, C.c_uint32]
    half, NB = 1 << (2 * M - 1), 97
    poison = np.full(half, 0xFFFFFFFF, dtype=np.uint32)
    mp = np.arange(half, dtype=np.uint32) % NB
    nomap = [f(None, c, M, NB) for c in range(half)]
    for c in range(0, half, max(1, half // 512)):
        assert f(poison.ctypes.data_as(C.POINTER(C.c_uint32)), c, M, NB) == nomap[c]  # hash route, map untouched
        assert nomap[c] < NB
    for c in range(half, 2 * half, max(1, half // 512)):
        assert f(mp.ctypes.data_as(C.POINTER(C.c_uint32)), c, M, NB) == (c - half) % NB
