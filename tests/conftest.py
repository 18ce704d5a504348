"""Shared pytest configuration.

Markers:
  gpu  -- needs an MI355X (runs through the C-ABI library on cuda:0).
Tests without the marker run on CPU in the build container and must not touch
/root/reference (it does not exist on the GPU box).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "wild-video-3d-reconstruction_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU (HIP path through the C-ABI)")


def pytest_report_header(config):
    """which libdpvo_hot.so the run loads (its source sha and flavour)."""
    try:
        import _dpvo_hot as H
        H.lib()
        return [f"libdpvo_hot: {H.LIB_PATH} {H.build_info} (tree sources sha={H.source_sha()})"]
    except Exception as e:  # pragma: no cover - reported, the tests then fail on their own
        return [f"libdpvo_hot: not loadable: {e}"]


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def poisoned():
    """Every buffer the shims allocate uninitialised (outputs, workspaces) is
    filled with 0xff -- NaN in every float type, -1 in the integer types --
    for the test's duration (_dpvo_hot.set_poison): a kernel that reads memory
    it never wrote shows up as NaNs or as bits that differ between patterns."""
    import _dpvo_hot as H
    old = H.poison()
    H.set_poison(0xFF)
    yield 0xFF
    H.set_poison(old)
