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


def test_library_provenance_matches_the_shipped_sources():
    """The loaded library was compiled from the csrc/ beside it, as the product
    (not the stamped diagnostic) build."""
    import _dpvo_hot as H
    H.lib()
    assert H.build_info["flavour"] == "product"
    assert H.build_info["sha"] == H.source_sha()


def test_stale_or_stamped_library_is_refused():
    import _dpvo_hot as H
    sha = H.source_sha()
    stale = "0" * 16 if sha != "0" * 16 else "1" * 16
    with pytest.raises(ImportError, match="stale"):
        H.verify_build(f"sha={stale} flavour=product", sha)
    with pytest.raises(ImportError, match="diagnostic"):
        H.verify_build(f"sha={sha} flavour=stamps", sha)
    assert H.verify_build(f"sha={sha} flavour=stamps", sha, diag=True)["flavour"] == "stamps"
    # an experiment build (scripts/build_exp.sh) from other sources: only with DPVO_DIAG=1
    with pytest.raises(ImportError, match="stale"):
        H.verify_build(f"sha={stale} flavour=cbase", sha)
    assert H.verify_build(f"sha={stale} flavour=cbase", sha, diag=True)["flavour"] == "cbase"
    with pytest.raises(ImportError, match="stale"):   # never the product
        H.verify_build(f"sha={stale} flavour=product", sha, diag=True)
    with pytest.raises(ImportError, match="provenance"):
        H.verify_build("", sha)


def test_stale_library_fails_at_load(tmp_path):
    """A library whose recorded sha differs from the tree's sources fails when
    a fresh interpreter loads it (sources edited after the build)."""
    import shutil
    import sys
    csrc = tmp_path / "csrc"
    shutil.copytree(os.path.join(PKG, "csrc"), csrc)
    with open(csrc / "common.hpp", "a") as f:
        f.write("\n// edited after the build\n")
    code = ("import sys; sys.path.insert(0, %r); import _dpvo_hot as H; H.source_sha = "
            "(lambda f: (lambda *a, **k: f(%r)))(H.source_sha); H.lib()") % (PKG, str(csrc))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert r.returncode != 0 and "stale" in r.stderr
