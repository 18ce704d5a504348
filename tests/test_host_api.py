"""Host-side API checks (no GPU): tracker config presets and refusals, the
quaternion helper behind PatchGraph.init_from_prior, argument validation of
the native shims."""
import numpy as np
import pytest
import torch


def test_presets_match_reference_yaml_values():
    """dpvo_configs/*.yaml restated as data (values as in the reference files)."""
    from dpvo.config import make_cfg
    tum = make_cfg("tum_default")
    assert (tum.PATCHES_PER_FRAME, tum.REMOVAL_WINDOW, tum.OPTIMIZATION_WINDOW, tum.PATCH_LIFETIME) == (384, 22, 10, 13)
    assert tum.KEYFRAME_THRESH == 30.0 and tum.GRADIENT_BIAS is False and tum.MIXED_PRECISION is True
    c2 = make_cfg("default", PATCHES_PER_FRAME=96)
    assert c2.PATCHES_PER_FRAME == 96 and c2.KEYFRAME_THRESH == 15.0
    assert make_cfg("dpvo_2k").PATCHES_PER_FRAME == 192


def test_loop_closure_refused_not_ignored():
    """cfg.loop_enabled builds a loop closer in the reference (dpvo.py:101-102);
    here it is out of scope and must raise rather than be ignored."""
    from dpvo.config import make_cfg
    from dpvo.dpvo import DPVO
    with pytest.raises(NotImplementedError, match="loop"):
        DPVO(make_cfg("fast", loop_enabled=True), None, device="cpu")


def test_matrix_to_quaternion_matches_rotation_algebra():
    from scipy.spatial.transform import Rotation
    from dpvo.utils import matrix_to_quaternion
    r = Rotation.random(500, random_state=0)
    mats = r.as_matrix()
    # include the four branch regimes: near-identity and 180-degree turns about each axis
    extra = np.stack([np.eye(3), np.diag([1.0, -1.0, -1.0]), np.diag([-1.0, 1.0, -1.0]), np.diag([-1.0, -1.0, 1.0])])
    mats = np.concatenate([mats, extra])
    q = matrix_to_quaternion(torch.tensor(mats)).numpy()
    ref = Rotation.from_matrix(mats).as_quat()[:, [3, 0, 1, 2]]
    ref = np.where(ref[:, :1] < 0, -ref, ref)
    # 180-degree turns: w = 0 and the sign of the vector part is arbitrary
    same = np.minimum(np.abs(q - ref).max(1), np.abs(q + ref).max(1))
    assert same.max() < 1e-12
    assert np.all(q[:, 0] >= 0)
    with pytest.raises(ValueError):
        matrix_to_quaternion(torch.zeros(2, 3, 4))


def test_group_by_key_bits_validated():
    import update_ops
    assert update_ops.key_bits_for(2048 * 192) == 19
    assert update_ops.key_bits_for(1) == 1
    with pytest.raises(RuntimeError, match="key_bits"):
        update_ops.group_by(torch.zeros(4, dtype=torch.int64), key_bits=65)
