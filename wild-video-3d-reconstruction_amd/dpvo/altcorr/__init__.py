from .correlation import corr, corr_pyramid, corr_pyramid_mfma, patchify
