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
    assert lib.dpvo_hot_abi_version() == 1
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
