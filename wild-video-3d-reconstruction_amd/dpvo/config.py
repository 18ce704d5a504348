"""Tracker configuration: the reference's yacs defaults (dpvo/config.py:6-35)
with YAML overrides (dpvo_configs/*.yaml).  yacs is not a dependency here,
so a small attribute-dict CfgNode with the same merge API stands in."""
import copy

import yaml


class CfgNode(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def clone(self):
        return copy.deepcopy(self)

    def merge_from_dict(self, d):
        for k, v in d.items():
            if k not in self:
                raise KeyError(f"Non-existent config key: {k}")
            self[k] = type(self[k])(v) if isinstance(self[k], (int, float)) and not isinstance(self[k], bool) else v

    def merge_from_file(self, path):
        with open(path) as f:
            self.merge_from_dict(yaml.safe_load(f) or {})

    def merge_from_list(self, kv):
        for k, v in zip(kv[0::2], kv[1::2]):
            self.merge_from_dict({k: yaml.safe_load(str(v))})


_C = CfgNode()
_C.BUFFER_SIZE = 2048
_C.GRADIENT_BIAS = True
_C.PATCHES_PER_FRAME = 80
_C.REMOVAL_WINDOW = 20
_C.OPTIMIZATION_WINDOW = 12
_C.PATCH_LIFETIME = 12
_C.KEYFRAME_INDEX = 4
_C.KEYFRAME_THRESH = 12.5
_C.MOTION_MODEL = "DAMPED_LINEAR"
_C.MOTION_DAMPING = 0.5
_C.MIXED_PRECISION = True
_C.loop_enabled = False
_C.LOOP_CLOSE_WINDOW_SIZE = 3
_C.LOOP_RETR_THRESH = 0.50
_C.ENABLE_GLOBAL_BA = False
_C.DISTANCE_THRESH = 3.0
_C.USE_DISTANCE_EDGES = True
# MI355X build additions
_C.BA_ITERATIONS = 2          # the reference hard-codes 2 (dpvo.py:734)
_C.CHANNEL_LAST_FMAPS = True  # keep the feature rings channel-contiguous (altcorr fast path)
_C.EXACT_CORR = False         # True: the bit-exact fp16-chain altcorr instead of the matrix-core kernel
_C.DEFER_BA_CHECK = True      # BA's Cholesky status read at keyframe()'s host read, not inside update()
_C.DEFER_KEYFRAME = False     # keyframe()'s decision applied by the next __call__ (its host read overlaps that frame's encoders)

cfg = _C

# the reference's dpvo_configs/*.yaml, as data
PRESETS = {
    "default": dict(PATCHES_PER_FRAME=384, REMOVAL_WINDOW=22, OPTIMIZATION_WINDOW=10, PATCH_LIFETIME=13,
                    KEYFRAME_THRESH=15.0, MOTION_MODEL="DAMPED_LINEAR", MOTION_DAMPING=0.5, MIXED_PRECISION=True,
                    GRADIENT_BIAS=False),
    "dpvo_2k": dict(PATCHES_PER_FRAME=192, REMOVAL_WINDOW=22, OPTIMIZATION_WINDOW=10, PATCH_LIFETIME=13,
                    KEYFRAME_THRESH=65.0, MOTION_MODEL="DAMPED_LINEAR", MOTION_DAMPING=0.5, MIXED_PRECISION=True,
                    GRADIENT_BIAS=False),
    "tum_default": dict(PATCHES_PER_FRAME=384, REMOVAL_WINDOW=22, OPTIMIZATION_WINDOW=10, PATCH_LIFETIME=13,
                        KEYFRAME_THRESH=30.0, MOTION_MODEL="DAMPED_LINEAR", MOTION_DAMPING=0.5,
                        MIXED_PRECISION=True, GRADIENT_BIAS=False),
    "fast": dict(PATCHES_PER_FRAME=48, REMOVAL_WINDOW=16, OPTIMIZATION_WINDOW=7, PATCH_LIFETIME=11,
                 KEYFRAME_THRESH=15.0, MOTION_MODEL="DAMPED_LINEAR", MOTION_DAMPING=0.5, MIXED_PRECISION=True,
                 GRADIENT_BIAS=False),
}


def make_cfg(preset=None, **overrides):
    c = cfg.clone()
    if preset:
        c.merge_from_dict(PRESETS[preset])
    c.merge_from_dict(overrides)
    return c
