"""INTEGRATION.md's ctypes stub, executed verbatim (the documented binding must be
the tested code path).  CPU only: the stub's fc_params / fc_chain_stats match the header's
layout field for field (names, offsets, size), and fc_run_create rejects -- before touching any
device -- a struct whose struct_size or abi_version is not this library's, e.g. a binding written
against the round-2 header (no tune_* fields, no chain_pop_bounds)."""
import ctypes
import os
import re

import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import graphs as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stub_namespace():
    """Run the code block between INTEGRATION.md's stub markers and return its globals."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"<!-- stub:begin -->\s*```python\n(.*?)```\s*<!-- stub:end -->", text, flags=re.S)
    assert m, "INTEGRATION.md lost its stub markers"
    ns = {"__name__": "integration_stub"}
    exec(compile(m.group(1), "INTEGRATION.md:stub", "exec"), ns)
    return ns


def _layout(struct):
    return [(name, getattr(struct, name).offset, getattr(struct, name).size) for name, _ in struct._fields_]


def test_stub_layout_matches_header_binding():
    ns = stub_namespace()
    assert _layout(ns["fc_params"]) == _layout(_lib.Params)
    assert ctypes.sizeof(ns["fc_params"]) == ctypes.sizeof(_lib.Params)
    assert _layout(ns["fc_chain_stats"]) == _layout(_lib.ChainStats)
    hdr = open(os.path.join(ROOT, "include", "flipchain.h")).read()
    assert f"#define FC_ABI_VERSION {_lib.FC_ABI_VERSION}u" in hdr
    assert f"FC_ABI_VERSION {_lib.FC_ABI_VERSION})" in open(os.path.join(ROOT, "INTEGRATION.md")).read()


def test_header_struct_fields_in_order():
    """The stub's field names are exactly the header's fc_params members, in order."""
    ns = stub_namespace()
    hdr = open(os.path.join(ROOT, "include", "flipchain.h")).read()
    body = hdr[hdr.index("typedef struct fc_params {"):hdr.index("} fc_params;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";")[:-1]:
        decl = decl.split("{", 1)[-1].strip()
        if not decl:
            continue
        typ_and_first, *rest = decl.split(",")
        first = re.sub(r"\[.*?\]", "", typ_and_first).split()[-1].lstrip("*")
        names.append(first)
        names += [re.sub(r"\[.*?\]", "", x).strip().lstrip("*") for x in rest]
    assert names == [f for f, _ in ns["fc_params"]._fields_]


def _graph(lib, ns):
    spec = G.grid_graph(10, 10)
    P = lambda a, t: a.ctypes.data_as(ctypes.POINTER(t))  # noqa: E731
    row = np.ascontiguousarray(spec.row_ptr, np.int32)
    col = np.ascontiguousarray(spec.col_idx, np.int32)
    pop = np.ascontiguousarray(spec.pop, np.int32)
    pos = np.ascontiguousarray(spec.pos, np.float64).reshape(-1)
    g = ctypes.c_void_p()
    ns["check"](lib, lib.fc_graph_create(ctypes.c_int32(spec.n), P(row, ctypes.c_int32), P(col, ctypes.c_int32),
                                         P(pop, ctypes.c_int32), P(pos, ctypes.c_double), ctypes.c_uint32(0),
                                         ctypes.byref(g)), "fc_graph_create")
    a0 = spec.assignment_array(G.threshold_plan(spec.nodes, 0, 5), [-1, 1])
    return spec, g, np.ascontiguousarray(a0[None, :], np.int8)


@pytest.mark.parametrize("case", ["truncated", "version", "round2_layout"])
def test_mismatched_struct_rejected(case):
    ns = stub_namespace()
    lib = ns["load"](_lib.lib_path())
    spec, g, init = _graph(lib, ns)
    try:
        prm = ns["fc_params"]()
        ns["check"](lib, lib.fc_params_init(ctypes.byref(prm), ctypes.c_uint32(ctypes.sizeof(prm))), "init")
        assert prm.struct_size == ctypes.sizeof(prm) and prm.abi_version == _lib.FC_ABI_VERSION
        arg = ctypes.byref(prm)
        if case == "truncated":     # a caller whose struct ends early says so in struct_size
            prm.struct_size -= 8
        elif case == "version":
            prm.abi_version -= 1
        else:                       # a binding of the round-2 header: k first, no size / version
            class Old(ctypes.Structure):
                _fields_ = [("k", ctypes.c_int32), ("proposal", ctypes.c_int32), ("base", ctypes.c_double)]
            old = Old(k=2, proposal=0, base=1.0)
            arg = ctypes.byref(old)
        r = ctypes.c_void_p()
        rc = lib.fc_run_create(g, arg, ctypes.c_int32(1), init.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), None,
                               ctypes.byref(r))
        assert rc == ns["FC_ERR_ARG"], rc
        assert b"struct_size" in lib.fc_last_error()
        assert not r.value
    finally:
        lib.fc_graph_destroy(g)


def test_params_init_rejects_other_size():
    ns = stub_namespace()
    lib = ns["load"](_lib.lib_path())
    prm = ns["fc_params"]()
    assert lib.fc_params_init(ctypes.byref(prm), ctypes.c_uint32(ctypes.sizeof(prm) + 8)) == ns["FC_ERR_ARG"]
    assert lib.fc_params_init(ctypes.byref(prm), ctypes.c_uint32(ctypes.sizeof(prm))) == 0
    assert prm.base == 1.0 and prm.hit_lo > prm.hit_hi and prm.pop_hi == 2 ** 31 - 1
