"""Host-side logic of bench.py and the boundary shims that needs no GPU:
per-rank core pinning, the counter-record gate, and the torch_scatter shim's
refusal of host tensors (no CPU fallback)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import PKG, REPO


def test_core_string():
    import bench
    assert bench._core_str([0, 1, 2, 3]) == "0-3"
    assert bench._core_str([0, 1, 4, 5, 7]) == "0-1,4-5,7"
    assert bench._core_str(None) is None


def test_pin_host_cores_splits_the_allowed_cpus():
    """rank r of W keeps the r-th contiguous block of the allowed CPUs (run in
    a child so this process keeps its affinity)"""
    code = ("import os, sys; sys.path.insert(0, %r); import bench; "
            "allowed = sorted(os.sched_getaffinity(0)); mine = bench.pin_host_cores(1, 2); "
            "per = len(allowed) // 2; assert mine == allowed[per:2 * per], (mine, allowed); "
            "assert sorted(os.sched_getaffinity(0)) == mine; print('ok')") % REPO
    if len(os.sched_getaffinity(0)) < 2:
        pytest.skip("one CPU")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr


def test_counter_record_only_for_current_sources(tmp_path):
    import bench
    p = tmp_path / "c.json"
    rec = {"edges": 100, "sha": {"corr": bench.source_sha(*bench.CORR_SOURCES), "update_op": "stale"},
           "corr": {"hbm_bytes_per_launch": 1}, "update_op": {"hbm_bytes_per_update": 2}}
    p.write_text(json.dumps(rec))
    got, ok = bench.load_counters(str(p), 100)
    assert ok == {"corr": True, "update_op": False}
    assert bench.load_counters(str(p), 101) is None
    assert bench.load_counters(str(tmp_path / "missing.json"), 100) is None


def test_torch_scatter_shim_refuses_host_tensors():
    import torch_scatter
    assert os.path.dirname(torch_scatter.__file__) == PKG
    src, idx = torch.randn(1, 10, 4), torch.zeros(10, dtype=torch.long)
    with pytest.raises(RuntimeError, match="GPU"):
        torch_scatter.scatter_sum(src, idx, dim=1)
    with pytest.raises(RuntimeError, match="GPU"):
        torch_scatter.scatter_softmax(src, idx, dim=1)
    with pytest.raises(ValueError):
        torch_scatter.scatter_sum(torch.zeros(3, dtype=torch.long), torch.zeros(3, dtype=torch.long))
