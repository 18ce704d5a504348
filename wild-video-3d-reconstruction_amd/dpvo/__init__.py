"""MI355X-native mirror of the reference's ``dpvo`` package (hot path only).

Same module layout as the reference (dpvo/altcorr, dpvo/fastba,
dpvo/lietorch, dpvo/projective_ops.py, dpvo/dpvo.py ...): code written
against the reference's operator surfaces runs unchanged on the HIP kernels
behind cuda_corr / cuda_ba / lietorch_backends.
"""
