"""The C-ABI library loads and exports every symbol include/dpvo_hot.h
declares (no GPU work)."""
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "dpvo_hot.h")
LIB = os.path.join(PKG, "libdpvo_hot.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dpvo_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG, "libdpvo_hot.so"])


def test_header_declares_the_expected_surface():
    names = declared()
    for must in ["dpvo_corr_forward", "dpvo_corr_forward_pyramid", "dpvo_corr_backward", "dpvo_patchify_forward",
                 "dpvo_patchify_backward", "dpvo_ba_forward", "dpvo_ba_workspace_bytes", "dpvo_reproject",
                 "dpvo_neighbors", "dpvo_lie_forward", "dpvo_lie_backward", "dpvo_transform", "dpvo_point_cloud", "dpvo_motion_mag"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_ctypes_binding_covers_header_and_loads():
    import _dpvo_hot as H
    assert sorted(H.EXPORTED) == declared()
    lib = H.lib()  # dlopen without touching the GPU
    assert lib.dpvo_hot_abi_version() == 2
    assert lib.dpvo_ba_workspace_bytes(95424, 2048 * 192, 10) > 0
    assert lib.dpvo_neighbors_workspace_bytes(95424) > 0


def test_shims_refuse_cpu_tensors():
    import torch
    import cuda_ba
    import cuda_corr
    import lietorch_backends
    with pytest.raises(RuntimeError, match="GPU"):
        lietorch_backends.inv(3, torch.zeros(2, 7))
    with pytest.raises(RuntimeError, match="GPU"):
        cuda_ba.neighbors(torch.zeros(3, dtype=torch.long), torch.zeros(3, dtype=torch.long))
    with pytest.raises(RuntimeError, match="GPU"):
        cuda_corr.patchify_forward(torch.zeros(1, 2, 4, 4), torch.zeros(1, 1, 2), 1)


def prototypes():
    """name -> [parameter type class] for every function the header declares"""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for name, params in re.findall(r"\b(dpvo_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
        ps = [q.strip() for q in params.split(",") if q.strip() and q.strip() != "void"]
        out[name] = [klass(q) for q in ps]
    return out


def klass(c_param):
    if "*" in c_param:
        return "ptr"
    t = c_param.rsplit(" ", 1)[0].replace("const ", "").strip()
    return {"int64_t": "i64", "size_t": "size", "int": "int", "float": "float", "double": "double"}[t]


def test_ctypes_signatures_match_the_header():
    """every ctypes binding has the header's arity and argument classes (a
    miscounted binding fails here instead of as a ctypes error on the GPU)"""
    import ctypes
    import _dpvo_hot as H
    cls = {ctypes.c_void_p: "ptr", ctypes.c_char_p: "ptr", ctypes.c_int64: "i64", ctypes.c_size_t: "size",
           ctypes.c_int: "int", ctypes.c_float: "float", ctypes.c_double: "double"}
    protos = prototypes()
    bad = {}
    for name, (_, argtypes) in H._SIGNATURES.items():
        got = [cls[a] for a in argtypes]
        if protos.get(name) != got:
            bad[name] = (protos.get(name), got)
    assert not bad, bad
