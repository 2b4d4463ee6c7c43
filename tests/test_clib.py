"""CPU: the C ABI library loads and exports exactly what include/dfk.h declares
(no compute calls — there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dfk.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t)\s+(dfk_\w+)\s*\(", src, flags=re.M)))


def test_header_matches_binding_table():
    from deepfake_amd import _lib
    assert header_symbols() == sorted(_lib.SIGNATURES), "include/dfk.h and deepfake_amd/_lib.py disagree"


def test_library_exports_every_symbol():
    from deepfake_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdfk.so not built (run python -m deepfake_amd.build)")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    _lib.lib()  # binds argtypes for every symbol


def test_struct_layouts_match_header():
    """ctypes mirrors of the ABI structs have the field order / sizes of include/dfk.h."""
    from deepfake_amd import _lib
    src = open(HEADER).read()
    for cname, cls in (("dfk_drop", _lib.Drop), ("dfk_view", _lib.View), ("dfk_gemm_args", _lib.GemmArgs),
                       ("dfk_wattn_args", _lib.WattnArgs), ("dfk_patch_embed_args", _lib.PatchEmbedArgs),
                       ("dfk_conv2d_geo", _lib.Conv2dGeo),
                       ("dfk_wattn_bwd_args", _lib.WattnBwdArgs), ("dfk_im2col_args", _lib.Im2colArgs)):
        body = re.search(r"typedef struct \{([^{}]*)\}\s*" + cname + ";", src, flags=re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            for part in decl.split(","):
                names.append(re.sub(r"[^\w]", "", part.strip().split()[-1]))
        assert names == [f[0] for f in cls._fields_], (cname, names, [f[0] for f in cls._fields_])


def test_product_has_no_cpu_fallback():
    """Calling an op with CPU tensors must raise, never compute on the host."""
    import torch
    from deepfake_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.ptr(torch.zeros(4))


def test_header_parameter_counts_match_binding():
    """Every prototype of include/dfk.h has as many parameters as its ctypes argtypes entry (a changed C
    signature — e.g. dfk_w2v_conv0_bwd's scratch_bytes — cannot drift from the binding)."""
    from deepfake_amd import _lib
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = re.findall(r"^(?:int|int64_t)\s+(dfk_\w+)\s*\(([^;]*)\)\s*;", src, flags=re.M | re.S)
    assert protos
    for name, params in protos:
        n = 0 if params.strip() in ("", "void") else params.count(",") + 1
        assert n == len(_lib.SIGNATURES[name]), (name, n, len(_lib.SIGNATURES[name]))
