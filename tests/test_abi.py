"""The C-ABI library loads and exports every entry point include/flipchain.h declares
(no compute calls: these run without a GPU)."""
import ctypes
import os
import re

from flipcomplexityempirical_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "flipchain.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fc_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_api():
    names = declared_functions()
    assert set(names) == set(_lib.EXPORTED), (set(names) ^ set(_lib.EXPORTED))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.lib_path())
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_last_error_is_thread_local_string():
    L = _lib.load()
    rc = L.fc_graph_create(0, None, None, None, None, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == _lib.FC_ERR_ARG
    assert b"graph" in L.fc_last_error()


def test_error_mapping():
    import pytest
    with pytest.raises(ValueError):
        _lib.check(_lib.FC_ERR_INVALID_STATE)
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.FC_ERR_UNSUPPORTED)
    with pytest.raises(_lib.FlipChainError):
        _lib.check(_lib.FC_ERR_HIP)


def test_product_library_has_no_experiment_build_flags():
    """the default library is the product build (fc_build_flags() = 0), and
    the kernel sources hold no timing-only experiment blocks."""
    assert _lib.build_flags() == 0
    csrc = os.path.join(os.path.dirname(HEADER), "..", "flipcomplexityempirical_amd", "csrc")
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        assert "FC_EXP_" not in text and "FC_MASKED_STORES" not in text, f


def test_loader_refuses_variant_libraries():
    """A variant selected by the environment is refused unless the caller allows it."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from flipcomplexityempirical_amd import _lib\n"
            "try:\n    _lib.load()\nexcept ImportError as e:\n    print('refused', e)\n"
            "else:\n    print('loaded')\n" % root)
    env = dict(os.environ, FC_LIB_PATH=_lib.lib_path())
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.startswith("refused") and "FC_LIB_PATH" in out.stdout, out.stdout + out.stderr
    code2 = code.replace("_lib.load()", "_lib.load(allow_variant=True)")
    out = subprocess.run([sys.executable, "-c", code2], env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.startswith("loaded"), out.stdout + out.stderr
