"""Fused projective ops (transform, point cloud) on the GPU vs the reference
Python's outputs (golden) and the oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def run_transform(g, flags, with_valid=False):
    import _dpvo_hot as H
    E, P = len(g["ii"]), 3
    od = 3 if flags & 1 else 2
    out = torch.empty(E, P, P, od, device="cuda:0")
    valid = torch.empty(E, P, P, device="cuda:0") if with_valid else None
    poses, patches, intr = T(g["poses"]), T(g["patches"]), T(g["intrinsics"])
    ii, jj, kk = T(g["ii"]), T(g["jj"]), T(g["kk"])
    H.check(H.lib().dpvo_transform(H.ptr(poses), H.ptr(patches), P, H.ptr(intr), H.ptr(ii), H.ptr(jj), H.ptr(kk),
                                   E, flags, H.ptr(out), H.ptr(valid), H.stream_of(poses)))
    return out.cpu().numpy()[None], (valid.cpu().numpy()[None] if with_valid else None)


def test_transform_matches_reference_python():
    g = np.load(os.path.join(GOLDEN, "pops_ref.npz"))
    c, _ = run_transform(g, 0)
    np.testing.assert_allclose(c, g["coords"], rtol=1e-5, atol=2e-4)
    cd, v = run_transform(g, 1, with_valid=True)
    np.testing.assert_allclose(cd, g["coords_depth"], rtol=1e-5, atol=2e-4)
    np.testing.assert_array_equal(v, g["valid"])
    ct, _ = run_transform(g, 2)
    np.testing.assert_allclose(ct, g["coords_tonly"], rtol=1e-5, atol=2e-4)


def test_point_cloud_matches_reference_python():
    import _dpvo_hot as H
    g = np.load(os.path.join(GOLDEN, "pops_ref.npz"))
    poses, patches, intr, ix = T(g["poses"]), T(g["patches"]), T(g["intrinsics"]), T(g["ix"])
    m = ix.numel()
    full = torch.empty(m, 3, 3, 4, device="cuda:0")
    centre = torch.empty(m, 3, device="cuda:0")
    for out, c in ((full, 0), (centre, 1)):
        H.check(H.lib().dpvo_point_cloud(H.ptr(poses), H.ptr(patches), 3, H.ptr(intr), H.ptr(ix), m, c, H.ptr(out),
                                         H.stream_of(poses)))
    np.testing.assert_allclose(full.cpu().numpy(), g["point_cloud"][0], rtol=1e-5, atol=1e-5)
    pc = g["point_cloud"][0]
    np.testing.assert_allclose(centre.cpu().numpy(), pc[:, 1, 1, :3] / pc[:, 1, 1, 3:], rtol=1e-5, atol=1e-5)
